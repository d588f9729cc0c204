/*
 * flexar — MI355X-native allreduce library (C API).
 *
 * Capability parity with the reference's public entry `MPI_Allreduce_FT`
 * (reference: allreduce_over_mpi/mpi_mod.hpp:1167-1221) and its FT_TOPO
 * topology selection (mpi_mod.hpp:880-929), re-designed for GPU-resident
 * buffers moved peer-to-peer over xGMI by CU-issued loads/stores into
 * IPC-mapped workspaces, with the local reduction fused into the transfer.
 *
 * Lifecycle (no MPI dependency — the bootstrap is pluggable):
 *   flexar_comm_create()  -> allocate workspace/flags on `device`
 *   flexar_comm_export()  -> opaque handle bytes (IPC handles) of this rank
 *   <application all-gathers the handle bytes: MPI_Allgather, torch store, ...>
 *   flexar_comm_connect() -> map every peer's workspace
 *   flexar_allreduce()    -> stream-ordered, graph-capturable collective
 *   flexar_comm_destroy()
 */
#ifndef FLEXAR_FLEXAR_H
#define FLEXAR_FLEXAR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLEXAR_VERSION_MAJOR 0
#define FLEXAR_VERSION_MINOR 1
#define FLEXAR_VERSION_PATCH 0

typedef enum {
  FLEXAR_FLOAT32 = 0,
  FLEXAR_FLOAT16 = 1,
  FLEXAR_BFLOAT16 = 2,
  FLEXAR_FLOAT64 = 3,
  FLEXAR_FP8_E4M3 = 4, /* OCP e4m3fn (gfx950 native), saturating */
  FLEXAR_FP8_E5M2 = 5, /* OCP e5m2, saturating */
  FLEXAR_INT8 = 6,
  FLEXAR_UINT8 = 7,
  FLEXAR_INT16 = 8,
  FLEXAR_UINT16 = 9,
  FLEXAR_INT32 = 10,
  FLEXAR_UINT32 = 11,
  FLEXAR_INT64 = 12,
  FLEXAR_UINT64 = 13,
  FLEXAR_BOOL = 14,
  FLEXAR_NUM_DTYPES = 15
} flexar_dtype_t;

typedef enum {
  FLEXAR_SUM = 0,
  FLEXAR_PROD = 1,
  FLEXAR_MAX = 2,
  FLEXAR_MIN = 3,
  FLEXAR_AVG = 4, /* SUM followed by a fused 1/N post-scale */
  FLEXAR_BAND = 5,
  FLEXAR_BOR = 6,
  FLEXAR_BXOR = 7,
  FLEXAR_NUM_OPS = 8
} flexar_op_t;

/* Error codes (0 = success). */
enum {
  FLEXAR_OK = 0,
  FLEXAR_ERR_INVALID = 1,
  FLEXAR_ERR_UNSUPPORTED = 2,
  FLEXAR_ERR_HIP = 3,
  FLEXAR_ERR_TIMEOUT = 4,
  FLEXAR_ERR_STATE = 5,
  FLEXAR_ERR_NOMEM = 6,
  FLEXAR_ERR_RCCL = 7
};

typedef struct flexar_comm* flexar_comm_t;

/* ---- version / errors ---------------------------------------------------- */
const char* flexar_version(void);
const char* flexar_last_error(void); /* thread-local message of the last failure */
size_t flexar_dtype_size(int dtype);

/* ---- communicator ------------------------------------------------------- */
/* workspace_bytes: staging capacity (both parities); 0 = default (FLEXAR_WORKSPACE_BYTES or 512 MiB). */
int flexar_comm_create(int rank, int nranks, int device, size_t workspace_bytes, flexar_comm_t* out);
size_t flexar_handle_size(void);
int flexar_comm_export(flexar_comm_t comm, void* handle_out);
/* all_handles: nranks * flexar_handle_size() bytes, rank-major. */
int flexar_comm_connect(flexar_comm_t comm, const void* all_handles);
/* Collective teardown (every rank of a connected communicator): drains this rank's work, agrees with
 * every peer (a host shared-memory page) that all calls have finished, closes the peer mappings, agrees
 * that every rank has unmapped, then frees. A peer that does not arrive within FLEXAR_TIMEOUT_MS leaves
 * this rank's exported buffers allocated and returns FLEXAR_ERR_TIMEOUT (the communicator is gone). */
int flexar_comm_destroy(flexar_comm_t comm);
/* The same teardown when the host page is gone (flexar_comm_host_page_drop, or a host agreement timed out):
 * `agree(ctx)` is called twice, where the page's two agreements would be (all calls finished; all peers
 * unmapped), and must return 1 only once every rank has called it (e.g. a barrier over the caller's
 * bootstrap). With the page present it is not called. Without either agreement the exported buffers stay
 * allocated and the call returns non-zero (FLEXAR_ERR_STATE) with a named error. */
int flexar_comm_destroy_agreed(flexar_comm_t comm, int (*agree)(void*), void* ctx);
/* Bytes of exported buffers this process keeps allocated because a teardown could not agree (diagnostic). */
uint64_t flexar_parked_bytes(void);
/* Non-collective teardown (garbage collection): no agreement; exported buffers stay allocated. */
int flexar_comm_destroy_local(flexar_comm_t comm);
/* Collective host-side agreement (shared-memory page of a connected communicator): *out = the maximum
 * (op 0) or bitwise OR (op 1) of `mine` over the ranks. FLEXAR_ERR_STATE when the communicator has no page. */
int flexar_comm_host_agree(flexar_comm_t comm, uint64_t mine, int op, uint64_t* out);
/* Connect-time check that the host page is shared by every rank (call on every rank after a bootstrap
 * barrier that follows flexar_comm_connect): *shared = 1, or 0 and the page is dropped on this rank. If any
 * rank reports 0, every rank calls flexar_comm_host_page_drop: teardown then parks exported buffers instead
 * of waiting out FLEXAR_TIMEOUT_MS, and host agreements report FLEXAR_ERR_STATE. */
int flexar_comm_host_page_check(flexar_comm_t comm, int* shared);
int flexar_comm_host_page_drop(flexar_comm_t comm);
int flexar_comm_rank(flexar_comm_t comm);
int flexar_comm_size(flexar_comm_t comm);

/* Algorithm spec strings:
 *   "auto"                 cost-model selection (default)
 *   "ring" | "ring:C"      ring (C channels over link-disjoint Hamiltonian cycles)
 *   "flat"                 one-stage tree = direct reduce-scatter + all-gather (FT_TOPO unset)
 *   "rhd" | "rhd:C"        tree 2,2,...,2 (recursive halving / doubling), optionally on C channels
 *   "tree:a,b,c" | "tree:a,b,c:C"  mixed-radix FlexTree with the given stage widths; ":C" runs it on C
 *                          link-balanced channels (disjoint slices, relabelled ranks: every stage covers the
 *                          xGMI links evenly, "rhd:7" at N = 8 drives all 7 links in every stage)
 *   "oneshot"              every rank reduces the full buffer (small messages)
 *   "ft"                   honour FT_TOPO exactly like the reference (any 1 = ring)
 * Optional suffixes: "+pull" (all-gather pulls from owners) / "+push" (owners push), "+nts" (streaming
 * stores), "+wt" (write-through protocol), "+f32" / "+rw" (typed staging of 16/8-bit multi-hop schedules),
 * "+rccl" (message transport), "+zc" (flat only: zero copy over registered buffers, flexar_reg_*).
 */
int flexar_comm_set_algo(flexar_comm_t comm, const char* spec);
int flexar_comm_set_grid(flexar_comm_t comm, int grid_blocks, int block_threads); /* 0 = auto */
/* Executor work split of large spans: 0 = one contiguous slice per workgroup (default), else chunks of `elems`
 * elements (a multiple of 8192) dealt round-robin to the workgroups. Every rank must set the same. */
int flexar_comm_set_xfer_chunk(flexar_comm_t comm, uint64_t elems);
/* Replace the communicator's measured tune table ("nranks bytes spec" lines, FLEXAR_TUNE_FILE format;
 * a row covers sizes >= bytes). NULL or "" clears it (back to the cost model). */
int flexar_comm_set_tune_table(flexar_comm_t comm, const char* text);

/* sendbuf == NULL or sendbuf == recvbuf => in place. count is size_t (no 2^31 cap). */
int flexar_allreduce(flexar_comm_t comm, const void* sendbuf, void* recvbuf, size_t count, int dtype,
                     int op, void* hip_stream);
/* Same, with an explicit algorithm spec (NULL = communicator default) and a fused
 * post-scale applied to the reduced value (1.0f = none; AVG multiplies 1/N on top). */
int flexar_allreduce_ex(flexar_comm_t comm, const void* sendbuf, void* recvbuf, size_t count, int dtype,
                        int op, void* hip_stream, const char* algo, float scale);
/* Compressed allreduce: fp32 / bf16 / fp16 buffers, OCP fp8 (wire_dtype FLEXAR_FP8_E4M3 / _E5M2) on the
 * links. amax_parts: FLEXAR_AMAX_PARTIALS device floats from flexar_amax(sendbuf) on the same stream; the
 * pre-scale fp8_max / (N * global amax) and the post-scale are fused into the flat schedule's transfers
 * (every contribution and every result is rounded to fp8 once; all ranks get identical results).
 * op: SUM or AVG. algo: NULL = "flat+pull"; "+wt" selects the write-through protocol.
 * The OCP MX form needs no amax pass: flexar_allreduce_ex with algo "flat+mxe4m3" / "flat+mxe5m2" (one
 * e8m0 scale per 32-element block, computed inside the executor; docs/DESIGN.md §9.2). */
int flexar_allreduce_fp8(flexar_comm_t comm, const void* sendbuf, void* recvbuf, size_t count, int dtype, int op,
                         void* hip_stream, int wire_dtype, const float* amax_parts, const char* algo);
/* Reduce-scatter: sendbuf holds nranks blocks of `count` elements, recvbuf receives this rank's
 * reduced block (count elements). All-gather: sendbuf has `count` elements, recvbuf nranks*count.
 * algo: "ring" or the direct exchange ("flat", default). Used by FSDP/ZeRO-style sharded DP and by
 * the hierarchical multi-node allreduce of the MPI layer. */
int flexar_reduce_scatter(flexar_comm_t comm, const void* sendbuf, void* recvbuf, size_t count, int dtype, int op,
                          void* hip_stream, const char* algo);
int flexar_all_gather(flexar_comm_t comm, const void* sendbuf, void* recvbuf, size_t count, int dtype,
                      void* hip_stream, const char* algo);
/* All-to-all with equal splits (expert parallelism): sendbuf holds nranks blocks of `count` elements,
 * block p goes to rank p; recvbuf receives nranks blocks, block q from rank q. One direct exchange. */
int flexar_all_to_all(flexar_comm_t comm, const void* sendbuf, void* recvbuf, size_t count, int dtype,
                      void* hip_stream);
/* Same with an algorithm spec: NULL = the direct exchange through staging, "flat+zc" = zero copy (every rank
 * writes straight into its peers' registered recvbuf). */
int flexar_all_to_all_ex(flexar_comm_t comm, const void* sendbuf, void* recvbuf, size_t count, int dtype,
                         void* hip_stream, const char* algo);
/* Broadcast `count` elements from `root`: the root reads sendbuf (NULL = recvbuf), every rank writes
 * recvbuf. algo: "oneshot" = direct multicast from the root; "flat" (or any other spec) = scatter +
 * all-gather (~2 S / N per link); NULL/"auto" = direct up to 256 KiB, scatter + all-gather above. */
int flexar_broadcast(flexar_comm_t comm, const void* sendbuf, void* recvbuf, size_t count, int dtype, int root,
                     void* hip_stream, const char* algo);
/* Non-blocking health check: returns FLEXAR_ERR_TIMEOUT (and fills flexar_last_error)
 * if a device-side wait timed out in any previous call. */
int flexar_comm_check(flexar_comm_t comm);
/* Clear a recorded timeout once every rank has synchronised (collective use: all ranks call it). */
int flexar_comm_clear_error(flexar_comm_t comm);
/* Readiness (collective, after connect): run three exact integer allreduces per protocol family in
 * `families` (1 = fence executor, 2 = write-through executor, 4 = LL, 8 = copy engines) with a short
 * watchdog; *failed_out = families that failed on THIS rank. OR the masks of all ranks and install
 * them with flexar_comm_set_disabled: calls then move to a verified family (ll -> oneshot,
 * fence -> +wt -> dma) or fail with FLEXAR_ERR_UNSUPPORTED when none is left. */
int flexar_comm_selftest(flexar_comm_t comm, uint32_t families, uint32_t* failed_out);
/* Why families failed on this rank in the last self-test (HIP errors named); "" = none failed. */
int flexar_comm_selftest_note(flexar_comm_t comm, char* buf, size_t buflen);
/* Collective protocol reset (every rank, between two agreements that no call is in flight / every rank
 * has reset): flags, epochs, staging and the error word back to their state after connect. */
int flexar_comm_resync(flexar_comm_t comm);
int flexar_comm_set_disabled(flexar_comm_t comm, uint32_t families);
/* Message transport (RCCL ncclSend/ncclRecv + local executor segments; family 16): algorithm suffix "+rccl",
 * or every call when IPC mapping is unavailable. RCCL is resolved at run time (the process's librccl). */
int flexar_rccl_available(void);
int flexar_rccl_unique_id(void* out, size_t len);                       /* rank 0; len >= 128 */
int flexar_comm_init_msg(flexar_comm_t comm, const void* unique_id);    /* collective */
int flexar_comm_connect_msg_only(flexar_comm_t comm);                   /* no IPC: all calls over RCCL */
uint32_t flexar_comm_disabled(flexar_comm_t comm);
/* Registered buffers for zero-copy allreduce (algorithm suffix "+zc", flat schedule): the reduce-scatter
 * reads every peer's input and the all-gather every peer's output directly over IPC, with no staging.
 * Registration is collective: every rank exports its buffer of the same size (flexar_reg_export), the
 * blobs are all-gathered rank-major, and every rank opens them (flexar_reg_open). A "+zc" call then takes
 * buffers that lie inside registrations, at the same offsets on every rank. */
#define FLEXAR_REG_HANDLE_BYTES 128
size_t flexar_reg_handle_size(void);
int flexar_reg_export(flexar_comm_t comm, const void* ptr, size_t bytes, void* out);
int flexar_reg_open(flexar_comm_t comm, const void* ptr, size_t bytes, const void* all_blobs, int* id_out);
int flexar_reg_close(flexar_comm_t comm, int id);
int flexar_reg_count(flexar_comm_t comm);
int flexar_reg_ids(flexar_comm_t comm, int* ids_out, int max); /* current registration ids; returns the count */
/* Registration holding [ptr, ptr + bytes): its id, 0 if none, -1 if its allocation was freed and the address
 * reused (stale peer mappings). A new registration replaces the old ones it contains or that are stale. */
int flexar_reg_find(flexar_comm_t comm, const void* ptr, size_t bytes);
/* The zero-copy policy (zc_policy.hpp) applied to a concrete spec, for tests and tools: writes the spec a call
 * runs and sets *decision (1 switched to "+zc+push", -1 fell back to staging, 0 unchanged). flags: 1 buffers
 * registered, 2 the call named the spec, 4 automatic choice, 8 FLEXAR_ZC_AUTO, 16 a tune table is installed. */
int flexar_zc_decide(const char* spec, int nranks, double bytes, int flags, uint32_t disabled, int* decision,
                     char* out, size_t outlen);
/* JSON: per-peer PCI bus id, device ordinal, link class (same-device / xgmi / pcie / unknown) and hop
 * count from the connect-time probe; links used by the cost model; self-test state. */
int flexar_comm_topology(flexar_comm_t comm, char* buf, size_t buflen);
/* Cost-model estimate (us) of spec ("auto" = the model's own choice) on this communicator's model. */
double flexar_comm_predict_us(flexar_comm_t comm, const char* spec, double bytes);
/* Install fitted cost-model parameters on this communicator (auto selection then uses them; links from
 * the connect-time probe unless links > 0). Collective in effect: every rank must install the same. */
int flexar_comm_set_model(flexar_comm_t comm, double alpha_launch_us, double alpha_sync_us, double link_gbps,
                          double hbm_gbps, int links);
/* Probe agreement (collective in effect, after connect): every rank exports its topology-probe summary
 * (flexar_probe_blob_size() bytes), the application all-gathers them, every rank agrees: the minimum link
 * count is installed everywhere, asymmetric link classes or settings fail with a message naming the ranks. */
size_t flexar_probe_blob_size(void);
int flexar_comm_probe_export(flexar_comm_t comm, void* out);
int flexar_comm_probe_agree(flexar_comm_t comm, const void* all_blobs);
int flexar_probe_agree(const void* all_blobs, int nranks, int* links_out); /* host-only check of the blobs */
int flexar_probe_agree_resident(const void* all_blobs, int nranks, int* links_out, int* resident_out);
uint64_t flexar_settings_fingerprint(int with_calib); /* env settings hash (1 = connect form, 0 = cache form) */
/* Connect-time calibration (collective, after the self-test): mode 0 off, 1 cached-or-measure, 2 measure.
 * Times fixed executor schedules, max over ranks, fits and installs the cost model; caches it on disk per
 * (arch, N, links, link classes, disabled families, version). Writes a JSON report. */
int flexar_comm_calibrate(flexar_comm_t comm, int mode, char* json, size_t jlen);
int flexar_comm_calibration(flexar_comm_t comm, char* json, size_t jlen); /* the last report */
int flexar_comm_reset_model(flexar_comm_t comm);   /* FLEXAR_MODEL / defaults, agreed links kept */
uint64_t flexar_comm_model_hash(flexar_comm_t comm);
/* JSON statistics (calls, bytes; per-algorithm device time when FLEXAR_PROFILE=1). */
int flexar_comm_stats(flexar_comm_t comm, char* buf, size_t buflen);
/* Describe the algorithm the communicator would run for (count, dtype). */
int flexar_comm_describe(flexar_comm_t comm, size_t count, int dtype, char* buf, size_t buflen);
/* The schedule the last allreduce on this communicator ran (after the zero-copy decision), "" before any. */
int flexar_comm_last_spec(flexar_comm_t comm, char* buf, size_t buflen);
/* Whether automatic choices may switch to zero copy on registered buffers (FLEXAR_ZC_AUTO at creation).
 * Every rank must set the same value before a call; the MPI layer sets it per call from an agreement. */
int flexar_comm_set_zc_auto(flexar_comm_t comm, int on);

/* ---- in-process group: nranks ranks on ONE device in ONE process ---------------
 * Every rank's workgroups run in a single launch (rank = blockIdx / grid), so the
 * complete multi-rank device protocol (flags, parity, staging, all algorithms) runs
 * on one GPU without IPC — used by tests and by calibration sweeps. */
int flexar_group_create(int nranks, int device, size_t workspace_bytes, flexar_comm_t* comms_out);
int flexar_group_allreduce(flexar_comm_t* comms, int nranks, const void* const* ins, void* const* outs, size_t count,
                           int dtype, int op, void* hip_stream, const char* algo, float scale);
/* fp8-wire allreduce for the group (amax_parts: nranks device pointers of FLEXAR_AMAX_PARTIALS floats). */
int flexar_group_allreduce_fp8(flexar_comm_t* comms, int nranks, const void* const* ins, void* const* outs,
                               size_t count, int dtype, int op, void* hip_stream, int wire_dtype,
                               const float* const* amax_parts);
/* coll: 1 = reduce-scatter, 2 = all-gather, 4 = all-to-all (count = elements per rank block). */
int flexar_group_collective(flexar_comm_t* comms, int nranks, int coll, const void* const* ins, void* const* outs,
                            size_t count, int dtype, int op, void* hip_stream, const char* algo);
int flexar_group_broadcast(flexar_comm_t* comms, int nranks, int root, const void* const* ins, void* const* outs,
                           size_t count, int dtype, void* hip_stream, const char* algo);

/* ---- standalone device reduction kernel ----------------------------------- */
/* dst[i] = scale * OP_k srcs[k][i], k < nsrc (1..64), fp32 accumulation for 16/8-bit floats. */
int flexar_reduce(void* dst, const void* const* srcs, int nsrc, size_t count, int dtype, int op, float scale,
                  void* hip_stream);
/* Same on host memory (OpenMP-free vectorised loop) — the CPU path's reduction. */
int flexar_reduce_host(void* dst, const void* const* srcs, int nsrc, size_t count, int dtype, int op,
                       float scale);

/* ---- fp8 (OCP e4m3) gradient compression (one HBM pass each) --------------- */
#define FLEXAR_AMAX_PARTIALS 256
/* parts_out: FLEXAR_AMAX_PARTIALS device floats of per-workgroup max |x| (their max = amax). */
int flexar_amax(const void* x, size_t n, int dtype, float* parts_out, void* hip_stream);
/* q = e4m3(clamp(x * num / amax, +-448)); amax = max over the partials (device pointer, no host sync). */
int flexar_quantize_fp8(const void* x, int dtype, void* q, size_t n, const float* amax_parts, float num,
                        void* hip_stream);
/* x = q * amax / num (dtype: float32, bfloat16 or float16). */
int flexar_dequantize_fp8(const void* q, void* x, int dtype, size_t n, const float* amax_parts, float num,
                          void* hip_stream);

/* ---- OCP MX fp8 message codec (hierarchical cross-node step) --------------- */
/* msg = n fp8 values then ceil(n/32) e8m0 block-scale bytes; wire 4 = e4m3, 5 = e5m2 (x: f32/bf16/f16). */
int flexar_mx_pack(const void* x, int dtype, void* msg, size_t n, int wire, void* hip_stream);
/* out[i] = sum over nmsg messages (msg_stride bytes apart), in order, of q_k[i] * 2^X_k (fp32). */
int flexar_mx_unpack_sum(const void* msgs, size_t msg_stride, int nmsg, size_t n, int wire, float* out,
                         void* hip_stream);
/* Same, times `post` (AVG's 1 / world fused into the pass; 1 = none). */
int flexar_mx_unpack_sum_scaled(const void* msgs, size_t msg_stride, int nmsg, size_t n, int wire, float post,
                                float* out, void* hip_stream);

/* ---- helpers --------------------------------------------------------------- */
int flexar_pointer_is_device(const void* p); /* 1 if p is device memory */
int flexar_current_device(void);
int flexar_copy_device_host(void* dst, const void* src, size_t bytes); /* synchronous, any direction */
int flexar_device_synchronize(void); /* hipDeviceSynchronize of the current device */
void* flexar_device_alloc(size_t bytes);
void flexar_device_free(void* p);

/* Kernel facts for a (dtype, op) instantiation: kind 0 = executor (proto 0 fence, 1 +nts, 2 +wt),
 * 1 = LL, 2 = standalone reduce, 3/4/5 = typed executor with fp32 partials / e4m3 wire / e5m2 wire,
 * 6/7 = typed executor with an OCP MX block-scaled e4m3 / e5m2 wire.
 * Writes workgroups resident per CU (512 threads) and VGPRs; the _ex form also the scratch (private segment)
 * bytes per lane. */
int flexar_kernel_info(int dtype, int op, int kind, int proto, int* blocks_per_cu, int* vgprs);
int flexar_kernel_info_ex(int dtype, int op, int kind, int proto, int* blocks_per_cu, int* vgprs, int* scratch_bytes);

/* ---- fault attribution (crumbs.hpp) ------------------------------------------ */
/* Every launch, copy, RCCL group and phase is appended to a per-process ring of breadcrumbs; on a fatal
 * signal or std::terminate the ring and each live communicator's device progress (epoch started / finished
 * by executor workgroup 0, host-mapped) are written to stderr. Installed once per process by the Python
 * layer and at the first communicator; FLEXAR_CRASH_REPORT=0 disables it. */
void flexar_crash_report_install(void);
void flexar_crash_report_dump(const char* why); /* write the report now */
/* A phase breadcrumb (start-up phases of bench.py / the Python communicator). */
void flexar_crumb(const char* what, const char* label, int rank, int nranks, uint64_t epoch, uint64_t bytes);
void flexar_test_fatal(int kind); /* tests only: 0 = std::terminate(), 1 = abort() */

/* ---- host-only planning utilities (no GPU needed) ------------------------ */
/* The collective-teardown agreement alone (tests): `phases` host barriers of `nranks` processes on the
 * shared-memory page `name`. 0, or FLEXAR_ERR_TIMEOUT with the straggler in flexar_last_error(). */
int flexar_host_barrier_run(const char* name, int rank, int nranks, int phases, uint64_t timeout_ms, int delay_ms);
/* The connect-time shared-page check alone (tests): open = join + mark; shared = every rank's mark present
 * (call after a barrier of the caller's); close = unlink + release. */
void* flexar_host_page_open(const char* name, int rank, int nranks, uint64_t token);
int flexar_host_page_shared(void* page, uint64_t token, int* missing);
void flexar_host_page_close(void* page);
/* Readiness downgrade chain (see flexar_comm_selftest) applied to `spec` for nranks with the given
 * failed-family mask; writes the spec a call would run, or returns FLEXAR_ERR_UNSUPPORTED. */
int flexar_downgrade_spec(const char* spec, int nranks, uint32_t disabled, int allow_dma, char* out, size_t outlen);
/* Concurrent-link count the cost model uses for a peer list of link classes / hops (probe results). */
int flexar_direct_links(const int32_t* link_classes, const int32_t* hops, int nranks, int self_rank);
/* Parse an FT_TOPO string for nranks with the reference's rules (any 1 -> ring, unset -> flat,
 * product must equal nranks; trailing/duplicate separators tolerated). Writes a canonical spec
 * ("ring" or "tree:a,b,c") into out. Returns FLEXAR_ERR_INVALID on a bad topology. */
int flexar_parse_ft_topo(const char* ft_topo, int nranks, char* out, size_t outlen);
/* Number of ordered factorizations H(n) (reference topo_count/factor_count.py). */
uint64_t flexar_count_factorizations(int n);
int flexar_ring_order(int n, int channel, int C, int* order);
/* Enumerate candidate plans for nranks as newline separated specs. */
int flexar_enumerate_plans(int nranks, char* out, size_t outlen);
/* Cost-model estimate (microseconds) of spec for (nranks, bytes). */
double flexar_model_cost_us(const char* spec, int nranks, double bytes);
/* Linear cost features of spec (see XgmiModel::features): 4 doubles, cost = f . (alpha_launch_us,
 * alpha_sync_us, 1/link_gbps, 1/hbm_gbps). links <= 0: the model's default link count. */
int flexar_model_features(const char* spec, int nranks, double bytes, int links, double* out);
/* Same for elements of `esize` bytes (typed staging of a 16/8-bit dtype prices at its real sizes). */
int flexar_model_features_ex(const char* spec, int nranks, double bytes, int links, int esize, double* out);
/* Cost of rank's compiled program (cost_model.hpp program_cost): out[5] = {handoffs, link_bytes,
 * link_time_bytes (busiest link, per phase), hbm_read, hbm_write}. links <= 0: the model's default. */
int flexar_program_cost(const char* spec, int rank, int nranks, size_t count, int dtype, int links, double* out);
/* Cost-model choice for (nranks, bytes) written to out. */
int flexar_select_plan(int nranks, double bytes, char* out, size_t outlen);
/* The typed form spec runs for a call of dtype / op (FLEXAR_PARTIALS: fp32 partials "+f32", per-hop "+rw"). */
int flexar_apply_partials(const char* spec, int nranks, double bytes, int dtype, int op, char* out, size_t outlen);
/* Cost-model choice for a call of dtype / op (the typed form it runs included; FLEXAR_PARTIALS applies). */
int flexar_select_plan_ex(int nranks, double bytes, int dtype, int op, int links, char* out, size_t outlen);
/* Calibration helpers (calibration.hpp): fit theta to rows (specs newline-separated; out[7] = alpha_launch_us,
 * alpha_sync_us, link_gbps, hbm_gbps, median / max relative error, rows used), the cache key / path / file,
 * and the measurement set ("spec bytes" lines) of flexar_comm_calibrate. */
int flexar_calib_fit(int nrows, const char* specs_nl, const double* bytes, const double* us, int nranks, int links,
                     int esize, double* out);
int flexar_calib_key(const char* arch, int nranks, int links, const char* classes, uint32_t disabled, char* out,
                     size_t outlen);
int flexar_calib_path(const char* key, char* out, size_t outlen);
int flexar_calib_load(const char* path, const char* key, double* theta); /* 1 loaded, 0 miss */
int flexar_calib_store(const char* path, const char* key, const double* theta, int nrows, const char* specs_nl,
                       const double* bytes, const double* us);
int flexar_calib_points(int nranks, char* out, size_t outlen);
/* Reference cost model (cost_model/CostModel.h) score, fixed: returns the argmin spec and cost. */
double flexar_legacy_cost(const char* widths_csv, int nranks, double chunk);
/* Human-readable dump of rank's op program (like Operations::print_ops). */
int flexar_plan_dump(const char* spec, int rank, int nranks, size_t count, int dtype, char* out, size_t outlen);
/* Execute the exact op programs the GPU runs, on host memory with one thread per (rank, grid block).
 * inputs/outputs: nranks host pointers each. in_place: outputs[r] already holds the input.
 * Returns 0 on success. Used to validate every algorithm/topology without a GPU. */
/* Same for coll = 0 allreduce, 1 reduce-scatter (inputs nranks*count, outputs count), 2 all-gather
 * (inputs count, outputs nranks*count). */
int flexar_simulate_coll(int coll, const char* spec, int nranks, size_t count, int dtype, int op,
                         const void* const* inputs, void* const* outputs, int grid, int ncalls, float scale);
int flexar_simulate(const char* spec, int nranks, size_t count, int dtype, int op, const void* const* inputs,
                    void* const* outputs, int grid, int ncalls, int in_place, float scale);
/* Typed-staging programs (spec suffix "+f32", "+e4m3", "+e5m2", "+mxe4m3", "+mxe5m2"; float dtype, SUM/AVG)
 * with the fp8 pre-scale `pre` given explicitly (the device derives it from the global amax; the MX wire
 * modes have per-block scales and ignore it). */
int flexar_simulate_typed(const char* spec, int nranks, size_t count, int dtype, int op, const void* const* inputs,
                          void* const* outputs, int grid, int ncalls, float scale, float pre);
/* Message-transport plans (msg_plan.hpp: the schedule as local executor segments + grouped send/recv,
 * what the RCCL transport runs) on host memory through in-order per-pair mailboxes. */
int flexar_simulate_msg(const char* spec, int nranks, size_t count, int dtype, int op, const void* const* inputs,
                        void* const* outputs, int ncalls, float scale);
/* JSON summary of rank's message plan: steps (executor ops / group sends+receives with peer, bytes, source). */
int flexar_msg_plan_dump(const char* spec, int rank, int nranks, size_t count, int dtype, char* out, size_t outlen);
/* Broadcast programs from `root` (inputs: root's source; outputs: every rank's destination). */
int flexar_simulate_bcast(const char* spec, int nranks, size_t count, int dtype, int root, const void* const* inputs,
                          void* const* outputs, int grid, int ncalls);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* FLEXAR_FLEXAR_H */
