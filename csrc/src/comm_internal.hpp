// Internal state of the flexar device communicator, shared by its translation units:
//   comm.hip          call resolution (spec, programs, grid) and the collective entry points
//   comm_connect.hip  create / export / connect (readiness gate, probe agreement), self-test,
//                     calibration, configuration setters, destroy
//   comm_reg.hip      registered buffers (zero copy)
//   comm_msg.hip      the message transport (schedules over RCCL send/recv)
//   comm_dma.hip      the copy-engine allreduce and the standalone reduction chain
//   comm_group.hip    in-process groups (N ranks on one device in one launch)
#pragma once

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <tuple>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "crumbs.hpp"
#include "host_barrier.hpp"
#include "launch.hpp"
#include "flexar/calibration.hpp"
#include "flexar/cost_model.hpp"
#include "flexar/flexar.h"
#include "flexar/log.hpp"
#include "flexar/msg_plan.hpp"
#include "flexar/zc_policy.hpp"
#include "flexar/planner.hpp"
#include "flexar/readiness.hpp"
#include "flexar/timer.hpp"
#include "internal.hpp"

namespace flexar {

#define FX_HIP(call)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess) {                                                                        \
      set_error(std::string(#call) + ": " + hipGetErrorString(e_));                                \
      return FLEXAR_ERR_HIP;                                                                       \
    }                                                                                              \
  } while (0)

static const uint32_t kHandleMagic = 0xF1E8A11Du;

struct CommHandle {
  uint32_t magic;
  uint32_t version;
  int32_t rank;
  int32_t nranks;
  uint64_t ws_bytes;
  hipIpcMemHandle_t stg;
  hipIpcMemHandle_t flags;
  int32_t pid;
  int32_t device;
  char host[64];
  char bus[32];          // PCI bus id of the rank's GPU (hipDeviceGetPCIBusId): resolves the peer device
  uint64_t fingerprint;  // settings every rank must agree on (readiness.hpp env_fingerprint)
  uint64_t nonce;        // random per communicator: rank 0's names the teardown agreement page
};

struct DevProgram {
  std::string spec;  // the schedule it runs (breadcrumb tag)
  Program prog;
  Op* d_ops = nullptr;
  uint32_t* d_chan = nullptr;
};

static const uint32_t kGroupMaxBlocks = 256;

// Optional roctx ranges (FLEXAR_ROCTX=1): resolved with dlopen so libflexar has no hard dependency.
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    const char* e = getenv("FLEXAR_ROCTX");
    if (!e || *e != '1') return;
    void* h = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
    pop = (int (*)())dlsym(h, "roctxRangePop");
    if (!push || !pop) push = nullptr, pop = nullptr;
  }
};
inline Roctx& roctx() {
  static Roctx r;
  return r;
}

// Per-call device timing (FLEXAR_PROFILE=1): hipEvent pairs resolved lazily by flexar_comm_stats.
struct ProfRec {
  std::string algo;
  uint64_t bytes;
  std::unique_ptr<DeviceTimer> t;
};

// RCCL entry points for the message transport, resolved at run time from the process's RCCL (the one
// torch already mapped, else /opt/rocm's): libflexar has no link-time RCCL dependency and a process never
// holds two RCCL instances.
struct RcclApi {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool ok = false;
  RcclApi() {
    void* h = nullptr;
    for (const char* n : {"librccl.so.1", "librccl.so"})
      if (!h) h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so"})
      if (!h) h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    GetUniqueId = (decltype(GetUniqueId))dlsym(h, "ncclGetUniqueId");
    CommInitRank = (decltype(CommInitRank))dlsym(h, "ncclCommInitRank");
    CommDestroy = (decltype(CommDestroy))dlsym(h, "ncclCommDestroy");
    Send = (decltype(Send))dlsym(h, "ncclSend");
    Recv = (decltype(Recv))dlsym(h, "ncclRecv");
    GroupStart = (decltype(GroupStart))dlsym(h, "ncclGroupStart");
    GroupEnd = (decltype(GroupEnd))dlsym(h, "ncclGroupEnd");
    GetErrorString = (decltype(GetErrorString))dlsym(h, "ncclGetErrorString");
    ok = GetUniqueId && CommInitRank && CommDestroy && Send && Recv && GroupStart && GroupEnd && GetErrorString;
  }
};
inline RcclApi& rccl() {
  static RcclApi a;
  return a;
}

// A message plan with its executor segments uploaded.
struct DevMsgPlan {
  std::string spec;  // breadcrumb tag ("msg:" + schedule)
  MsgPlan plan;
  std::vector<Op*> d_ops;
  std::vector<uint32_t*> d_chan;
};

inline uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* e = getenv(name);
  if (!e || !*e) return dflt;
  return strtoull(e, nullptr, 0);
}

// Caller buffers at any byte offset take the 16-B vector path (device_exec.hpp ld16/st16: unaligned
// dwordx4 accesses); FLEXAR_SCALAR_MISALIGNED=1 restores the round-3 policy (a base that is not 16-B
// aligned runs the whole span through 4-byte scalar code) for A/B measurements.
inline bool vec_any_alignment() {
  static const bool v = env_u64("FLEXAR_SCALAR_MISALIGNED", 0) == 0;
  return v;
}
inline bool vec_ok_for(uintptr_t addr_bits) { return vec_any_alignment() || (addr_bits & 15) == 0; }

}  // namespace flexar

using namespace flexar;

constexpr int kCalAgreeMax = 256;  // doubles in one calibration agreement (flexar_comm_calibrate)

struct flexar_comm {
  int rank = 0, nranks = 1, device = 0;
  size_t ws_bytes = 0, half_bytes = 0;
  size_t ll_bytes = 0;    // LL granule region at the end of each parity half (0 = LL disabled)
  size_t exec_half = 0;   // part of each half available to op programs
  char* stg = nullptr;
  uint64_t* flags = nullptr;
  uint64_t* epochs = nullptr;
  uint32_t* err_host = nullptr;
  uint32_t* err_dev = nullptr;
  char* peer_stg[kMaxRanks] = {};
  uint64_t* peer_flags[kMaxRanks] = {};
  bool opened[kMaxRanks] = {};
  bool connected = false;
  bool group_member = false;  // in-process group: peers' pointers are direct device pointers
  AlgoSpec spec;              // communicator default
  int grid_override = 0;
  // XFER work split (DevCtx::ichunk): 0 = per-workgroup slices; else elements per round-robin chunk (a multiple
  // of kXferChunk). FLEXAR_EXEC_INTERLEAVE=1 (in the settings fingerprint) or flexar_comm_set_xfer_chunk
  uint64_t xfer_chunk = 0;
  int max_grid = 256;
  uint64_t min_block_bytes = 32 * 1024;
  uint64_t chunk_bytes = 0;  // FLEXAR_CHUNK_BYTES: cap on the bytes of one launch (0 = workspace-bound only)
  int nchannels = 0;         // FLEXAR_NCHANNELS: channels of a plain "ring" spec (0 = 1)
  uint64_t timeout_ticks = 0;
  uint32_t fi_kind = 0, fi_slot = 0;
  uint64_t fi_ticks = 0;
  XgmiModel model;
  TuneTable tune;
  bool have_tune = false;
  std::map<std::string, std::unique_ptr<DevProgram>> cache;
  std::mutex mu;
  bool profile = false;
  std::vector<ProfRec> prof_pending;
  struct Agg { uint64_t calls = 0, bytes = 0; double ms = 0; };
  std::map<std::string, Agg> prof;
  uint64_t calls = 0, bytes = 0;
  // host mirror of the device epoch: every executor/LL launch and every dma call advances it by one
  uint64_t launches = 0;
  // copy-engine (dma) engine: one stream per peer (created on first use) and fork/join events
  // copy-engine (dma) engine: per peer one reduce-scatter stream and one all-gather stream (created on
  // first use), the call's fork event, per peer and staging parity the "all-gather copy done" event the
  // reduce-scatter copy two pieces later waits on, and the streams' end-of-call events
  bool dma_ready = false;
  hipStream_t dma_st[kMaxRanks] = {};   // reduce-scatter copies + RS flags
  hipStream_t dma_ag[kMaxRanks] = {};   // AG flag waits + all-gather copies
  hipEvent_t dma_fork = nullptr, dma_join[kMaxRanks] = {}, dma_rs_end[kMaxRanks] = {};
  hipEvent_t dma_ag_done[kMaxRanks][2] = {};
  // call ordering across streams: calls share epochs/staging, so two calls of one communicator must never
  // run concurrently (NCCL semantics). A call on a new stream waits for everything enqueued so far on the
  // previous call's stream (an event recorded lazily, only when the stream changes).
  hipStream_t last_st = nullptr;
  bool have_last = false;
  hipEvent_t order_ev = nullptr;
  bool unordered = false;  // FLEXAR_UNORDERED_CALLS=1: test-only, shows the race the ordering prevents
  // A call of this communicator was captured into a graph. Replays advance the device epochs without the
  // host seeing them, and the copy-engine path (dma) bakes the host mirror of the epoch into its copies
  // and flag writes, so from then on a dma request runs the executor's flat exchange instead.
  bool captured = false;
  // Plan memo of the allreduce hot path: what a (algo, count, dtype, op, scale) call resolved to last
  // time — spec, piece size, program, grid — so a repeated call skips spec parsing, key formatting and
  // the program-cache lookup. Every setter that changes what a call resolves to bumps memo_gen.
  struct CallMemo {
    uint64_t gen = 0;  // == memo_gen when valid
    uint64_t count = 0;
    int dtype = -1, op = -1;
    uint32_t fsb = 0;  // scale bits
    std::string algo;
    AlgoSpec s;
    uint64_t piece = 0;
    DevProgram* dp = nullptr;  // program of a one-piece call
    int grid = 0;
    bool zc_auto = true;  // the zero-copy policy the decision was made under (flexar_comm_set_zc_auto)
  };
  CallMemo memo[16];
  uint64_t memo_gen = 1;
  // the selector's choice per (bytes, element size, call kind) under the current model (memo_gen): pricing every
  // candidate program costs tens of us, and the 16-slot call memo above can miss when many sizes alternate
  std::mutex sel_mu;
  uint64_t sel_gen = 0;
  std::map<std::tuple<double, uint32_t, int>, AlgoSpec> sel_memo;
  // readiness (readiness.hpp): protocol families that failed the connect-time self-test, per-peer
  // link classes from the topology probe, residency of the executor kernel
  uint32_t disabled = 0;
  uint32_t selftested = 0;  // families the self-test ran
  int32_t link_cls[kMaxRanks] = {};
  int32_t link_hops[kMaxRanks] = {};
  int32_t peer_dev[kMaxRanks] = {};  // peer's device ordinal in THIS process (-1 = not visible)
  char peer_bus[kMaxRanks][32] = {};
  bool links_from_env = false;  // FLEXAR_MODEL fixed the link count: the probe does not override it
  int links_local = 0;          // this rank's own probe result (model.links = the ranks' agreed minimum)
  bool links_agreed = false;    // flexar_comm_probe_agree ran
  std::string calib_json;       // the connect-time calibration's report (flexar_comm_calibrate)
  double* cal_dev = nullptr;    // agreement scratch of the calibration (device, kCalAgreeMax doubles)
  int resident = 0;             // executor workgroups resident at once on this GPU (occupancy x CUs)
  // message transport (msg_plan.hpp over RCCL): its own staging arena (never the IPC workspace, whose
  // parity halves peers may still read), the RCCL communicator, plans per call shape
  bool ipc = true;              // peer workspaces mapped (false: every call runs the message transport)
  ncclComm_t nccl = nullptr;
  char* msg_ws = nullptr;
  // the message transport's executor segments are local-only programs whose number differs between ranks
  // for tiny calls (empty blocks): they count calls in their own epoch array, never in `epochs`, which
  // must advance in lockstep on every rank for the peer-memory protocols
  uint64_t* msg_epochs = nullptr;
  size_t msg_ws_bytes = 0;
  std::map<std::string, std::unique_ptr<DevMsgPlan>> msg_cache;
  // registered caller buffers (zero-copy "+zc"): every rank registered its buffer of the same size in
  // the same order; peer[p] is rank p's buffer mapped into this process. IPC mappings of one peer
  // allocation are shared by every registration inside it (torch's allocator carves tensors out of
  // larger segments).
  struct Reg {
    int id;
    char* base;
    size_t bytes;
    bool aligned;
    uint64_t bufid;  // HIP's unique id of the local allocation at registration (0 = unknown)
    char* peer[kMaxRanks];
    std::string key[kMaxRanks];
  };
  std::vector<Reg> regs;
  int next_reg = 1;
  std::map<std::string, std::pair<char*, int>> ipc_maps;  // (peer, handle) -> mapped base, references
  bool zc_auto = true;  // FLEXAR_ZC_AUTO=0: automatic choices never switch to zero copy
  AlgoSpec last_spec;     // the schedule the last allreduce ran (after the zero-copy decision)
  bool have_last_spec = false;
  int* st_buf = nullptr;        // self-test buffers (device)
  uint32_t* st_bad = nullptr;   // self-test mismatch counter (host-mapped)
  uint32_t* st_bad_dev = nullptr;
  std::string selftest_note;    // why a family failed on this rank (HIP errors named), last self-test
  uint32_t test_hip_fail = 0;   // FLEXAR_TEST_SELFTEST_HIP: families whose self-test launch fails here
  // collective teardown (host_barrier.hpp): joined at connect, agreed on in flexar_comm_destroy
  uint64_t nonce = 0;
  std::unique_ptr<HostBarrier> hb;
  int crumb_slot = -1;  // live-communicator slot of the crash report (crumbs.hpp)
  uint64_t hb_token = 0;  // rank 0's nonce: the identity every rank writes into the page (HostBarrier::mark)
  int hb_shared = -1;     // the page verified shared by every rank: 1 yes, 0 no (dropped), -1 not checked
};

namespace flexar {

// ---- functions shared by the communicator's translation units ------------------------------------
// comm.hip: call resolution, programs, launch contexts
int order_call(flexar_comm* c, hipStream_t st);
CallKind call_kind(int dtype, int op);
int resolve_spec(flexar_comm* c, const char* algo, double bytes, AlgoSpec* out, const CallKind& k = CallKind());
int typed_spec(flexar_comm* c, AlgoSpec* s, int dtype, int op, bool have_amax, double bytes);
int executor_proto(flexar_comm* c, AlgoSpec* s);
bool ll_usable(flexar_comm* c, uint64_t count, uint32_t es);
int ll_grid(flexar_comm* c, uint64_t count, uint32_t es);
void mark_barriers(Program& P, uint32_t rank);
int get_program(flexar_comm* c, const AlgoSpec& s, uint64_t count, uint32_t esize, float fscale, DevProgram** out,
                Coll coll = Coll::ALLREDUCE, uint64_t stride = 0);
int proto_of(const AlgoSpec& s);
const flexar_comm::Reg* reg_lookup(flexar_comm* c, const void* p, uint64_t bytes);
int zc_bind(flexar_comm* c, const Program& P, const void* in, uint64_t in_bytes, const void* out, uint64_t out_bytes,
            DevCtx* x);
int choose_grid(flexar_comm* c, uint64_t bytes, uint32_t nchan);
void fill_ctx(flexar_comm* c, DevProgram* dp, const void* in, void* out, DevCtx* x, uint64_t bytes = ~0ull);
bool zc_registered(flexar_comm* c, const void* in, const void* out, uint64_t bytes);
int plan_pieces(flexar_comm* c, const AlgoSpec& s, uint64_t count, uint32_t esize, float fs, uint64_t* piece,
                Coll coll = Coll::ALLREDUCE, uint64_t stride = 0);
int run_rs_ag(flexar_comm* c, Coll coll, const void* in, void* out, size_t count, int dtype, int op, hipStream_t st,
              const char* algo, float scale);
int bcast_spec(flexar_comm* c, const char* algo, uint64_t bytes, AlgoSpec* out);
int run_bcast(flexar_comm* c, const void* in, void* out, size_t count, int dtype, int root, hipStream_t st,
              const char* algo);
// comm_msg.hip: the message transport (msg_plan.hpp over RCCL)
int rccl_check(ncclResult_t r, const char* what);
int get_msg_plan(flexar_comm* c, const AlgoSpec& s, uint64_t count, uint32_t es, float fs, Coll coll, uint64_t stride,
                 DevMsgPlan** out);
int run_msg(flexar_comm* c, const AlgoSpec& s, Coll coll, const void* in, void* out, uint64_t count, int dtype, int op,
            float fs, uint64_t stride, hipStream_t st);
// comm_dma.hip: copy-engine allreduce and the standalone reduction chain
int reduce_chain(char* dst, char* dst2, const char* const* srcs, int nsrc, uint64_t count, int dtype, int op, float fs,
                 hipStream_t st, int proto);
int run_dma(flexar_comm* const* cs, int ncomm, const char* const* ins, char* const* outs, uint64_t count, int dtype,
            int op, float fs, hipStream_t st);
// comm_connect.hip: lifecycle, readiness, calibration
uint64_t comm_fingerprint(flexar_comm* c, bool with_calib = true);
int resident_blocks(int device);
int check_err(flexar_comm* c);
int validate_call(flexar_comm* c, int dtype, int op, float scale);
int alloc_workspace(flexar_comm* c, size_t ws);
void init_defaults(flexar_comm* c);

}  // namespace flexar
