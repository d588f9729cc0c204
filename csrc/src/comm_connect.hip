// flexar communicator lifecycle: create, export, connect (readiness gate), self-test, configuration
// setters, topology report, destroy. Reference counterpart: FlexTree_Context and the lazily created
// scratch buffer (allreduce_over_mpi/mpi_mod.hpp:216-243, 931-950).
#include <atomic>
#include <chrono>
#include <random>

#include "comm_internal.hpp"

namespace flexar {

// Settings fingerprint exchanged in the handle (readiness.hpp): environment knobs + workspace size +
// the loaded tune table.
uint64_t comm_fingerprint(flexar_comm* c, bool with_calib) {
  std::string extra = "ws=" + std::to_string(c->ws_bytes) + ";";
  for (auto& n : c->tune.rows)
    for (auto& row : n.second) extra += std::to_string(n.first) + " " + std::to_string(row.first) + " " + row.second + ";";
  return env_fingerprint(extra, with_calib);
}

// Self-test pattern (flexar_comm_selftest): rank r contributes (r + 1) * p(i), p(i) in [1, 1000], so
// the exact sum is N (N + 1) / 2 * p(i); OUT is poisoned so an element nobody wrote is caught too.
__device__ FX_INLINE int selftest_pattern(uint64_t i, uint32_t salt) { return (int)((i * 7 + salt) % 1000) + 1; }
static __global__ void selftest_fill(int* in, int* out, uint64_t n, int rank, uint32_t salt) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    in[i] = (rank + 1) * selftest_pattern(i, salt);
    out[i] = -1;
  }
}
static __global__ void selftest_check(const int* out, uint64_t n, int nranks, uint32_t salt, uint32_t* bad) {
  uint32_t mine = 0;
  const int tri = nranks * (nranks + 1) / 2;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    mine += out[i] != tri * selftest_pattern(i, salt);
  if (mine) __hip_atomic_fetch_add(bad, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Executor workgroups resident at once on this device: occupancy of the fp32 fence executor (the
// largest register footprint among the hot instantiations is within one workgroup of it) x CUs.
int resident_blocks(int device) {
  LaunchArgs la;
  la.kind = LAUNCH_QUERY;
  int occ = 0, regs = 0;
  la.occ_out = &occ;
  la.regs_out = &regs;
  if (launch_dtype(FLEXAR_FLOAT32, FLEXAR_SUM, la) != 0 || occ < 1) return 0;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return occ * cus;
}

int check_err(flexar_comm* c) {
  uint32_t e = __atomic_load_n(c->err_host, __ATOMIC_ACQUIRE);
  if ((e & 0x40000000u) && ((e >> 8) & 0xffffu) == 0xfdu) {
    set_error("rank " + std::to_string(c->rank) + ": internal: a typed transfer with an operand pattern the "
              "executor does not run (planner/executor mismatch)");
    return FLEXAR_ERR_STATE;
  }
  if (e & 0x40000000u) {
    char buf[200];
    snprintf(buf, sizeof(buf), "rank %d: protocol violation — peer %u is more than one call ahead (slot %u): "
             "two calls of this communicator overlapped", c->rank, e & 0xffu, (e >> 8) & 0xffffu);
    set_error(buf);
    return FLEXAR_ERR_STATE;
  }
  if (e) {
    char buf[160];
    snprintf(buf, sizeof(buf), "rank %d: device wait timed out (slot %u, peer %u) — a peer stopped participating",
             c->rank, (e >> 8) & 0xffffu, e & 0xffu);
    set_error(buf);
    return FLEXAR_ERR_TIMEOUT;
  }
  return 0;
}

int validate_call(flexar_comm* c, int dtype, int op, float scale) {
  if (!c) { set_error("null communicator"); return FLEXAR_ERR_INVALID; }
  if (!c->connected) { set_error("communicator not connected"); return FLEXAR_ERR_STATE; }
  if (!op_supported(dtype, op)) {
    set_error(std::string("unsupported dtype/op: ") + dtype_name(dtype) + "/" + op_name(op));
    return FLEXAR_ERR_UNSUPPORTED;
  }
  if (scale != 1.0f && !(dtype_is_float(dtype) && (op == FLEXAR_SUM || op == FLEXAR_AVG))) {
    set_error("a post-scale needs a float dtype with SUM/AVG");
    return FLEXAR_ERR_INVALID;
  }
  return 0;
}

int alloc_workspace(flexar_comm* c, size_t ws) {
  FX_HIP(hipSetDevice(c->device));
  c->ws_bytes = (ws + 511) / 512 * 512;
  c->half_bytes = c->ws_bytes / 2 / kStageAlignBytes * kStageAlignBytes;
  FX_HIP(hipMalloc(&c->stg, c->ws_bytes));
  FX_HIP(hipMemset(c->stg, 0, c->ws_bytes));  // LL granules: zero = epoch 0, never matches a live call
  c->ll_bytes = (size_t)(2 * kLLMaxBytes) * c->nranks;
  if (c->ll_bytes * 2 > c->half_bytes) c->ll_bytes = 0;
  // each parity half: [op-program staging | amax granules (fp8 wire) | LL granules]
  c->exec_half = c->half_bytes - c->ll_bytes - kAmaxRegion;
  FX_HIP(hipExtMallocWithFlags((void**)&c->flags, kFlagWords * sizeof(uint64_t), hipDeviceMallocUncached));
  FX_HIP(hipMemset(c->flags, 0, kFlagWords * sizeof(uint64_t)));
  FX_HIP(hipMalloc(&c->epochs, kMaxGridBlocks * sizeof(uint64_t)));
  FX_HIP(hipMemset(c->epochs, 0, kMaxGridBlocks * sizeof(uint64_t)));
  FX_HIP(hipHostMalloc((void**)&c->err_host, 64, hipHostMallocMapped));
  memset(c->err_host, 0, 64);
  FX_HIP(hipHostGetDevicePointer((void**)&c->err_dev, c->err_host, 0));
  // the calibration's agreement vector: allocated here, so no collective step of flexar_comm_calibrate
  // can be skipped by one rank's allocation failure (its peers would advance an epoch it never reaches)
  FX_HIP(hipMalloc(&c->cal_dev, kCalAgreeMax * sizeof(double)));
  FX_HIP(hipDeviceSynchronize());
  return 0;
}

void init_defaults(flexar_comm* c) {
  c->model = XgmiModel::from_env();
  if (const char* m = getenv("FLEXAR_MODEL")) c->links_from_env = std::count(m, m + strlen(m), ',') >= 4;
  c->have_tune = c->tune.load(getenv("FLEXAR_TUNE_FILE"));
  c->timeout_ticks = env_u64("FLEXAR_TIMEOUT_MS", 20000) * 100000ull;  // 100 MHz s_memrealtime
  c->zc_auto = env_u64("FLEXAR_ZC_AUTO", 1) != 0;
  c->xfer_chunk = env_u64("FLEXAR_EXEC_INTERLEAVE", 0) ? kXferChunk : 0;
  c->max_grid = (int)env_u64("FLEXAR_MAX_GRID", 256);
  if (c->max_grid < 1) c->max_grid = 1;
  if (c->max_grid > (int)kMaxGridBlocks) c->max_grid = kMaxGridBlocks;
  c->min_block_bytes = env_u64("FLEXAR_MIN_BLOCK_BYTES", 32 * 1024);
  c->chunk_bytes = env_u64("FLEXAR_CHUNK_BYTES", 0);
  c->nchannels = (int)env_u64("FLEXAR_NCHANNELS", 0);
  c->profile = env_u64("FLEXAR_PROFILE", 0) != 0;
  c->unordered = env_u64("FLEXAR_UNORDERED_CALLS", 0) != 0;
  if (!c->min_block_bytes) c->min_block_bytes = 1;
  // FLEXAR_FAULT_INJECT=delay:RANK:SLOT:MICROSECONDS | drop:RANK:SLOT  (tests / race hunting)
  if (const char* fi = getenv("FLEXAR_FAULT_INJECT")) {
    char kind[16] = {0};
    int rk = -1, slot = 0;
    double us = 0;
    if (sscanf(fi, "%15[a-z]:%d:%d:%lf", kind, &rk, &slot, &us) >= 3 && rk == c->rank) {
      c->fi_kind = strcmp(kind, "drop") == 0 ? 2 : 1;
      c->fi_slot = (uint32_t)slot;
      c->fi_ticks = (uint64_t)(us * 100.0);  // 100 MHz s_memrealtime
    }
  }
  const char* a = getenv("FLEXAR_ALGO");
  std::string err;
  if (a && *a && strcmp(a, "rccl") != 0) {  // "rccl" is routed by the Python layer / c10d backend
    if (!parse_algo(a, c->nranks, &c->spec, &err)) logf(LOG_WARN, c->rank, "ignoring FLEXAR_ALGO: %s", err.c_str());
    if (c->spec.kind == AlgoKind::RING && c->nchannels > 1 && !strchr(a, ':')) c->spec.channels = c->nchannels;
  } else if (getenv("FT_TOPO")) {  // reference compatibility: FT_TOPO selects the algorithm
    if (!parse_ft_topo(getenv("FT_TOPO"), c->nranks, &c->spec, &err))
      logf(LOG_WARN, c->rank, "ignoring FT_TOPO: %s", err.c_str());
  }
}

}  // namespace flexar

extern "C" {

int flexar_comm_create(int rank, int nranks, int device, size_t workspace_bytes, flexar_comm_t* out) {
  if (!out || nranks < 1 || nranks > (int)kMaxRanks || rank < 0 || rank >= nranks) {
    set_error("invalid rank/nranks (nranks must be 1..16)");
    return FLEXAR_ERR_INVALID;
  }
  crash_report_install();  // once per process; FLEXAR_CRASH_REPORT=0 disables it
  crumb_phase("comm_create", "workspace + flags + error page", rank, nranks);
  std::unique_ptr<flexar_comm> c(new flexar_comm);
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  init_defaults(c.get());
  size_t ws = workspace_bytes ? workspace_bytes : env_u64("FLEXAR_WORKSPACE_BYTES", 512ull << 20);
  int rc = alloc_workspace(c.get(), ws);
  if (rc) return rc;
  c->crumb_slot = crumb_register_comm(rank, nranks, device, reinterpret_cast<const volatile uint64_t*>(c->err_host) + 1);
  c->resident = resident_blocks(device);
  c->model.stg_cap = (double)c->exec_half;  // the selector prices pieces of programs larger than a half
  c->peer_stg[rank] = c->stg;
  c->peer_flags[rank] = c->flags;
  if (nranks == 1) c->connected = true;
  {
    std::random_device rd;
    c->nonce = ((uint64_t)rd() << 32) ^ rd() ^ ((uint64_t)getpid() << 17) ^
               (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
  }
  // FLEXAR_TEST_SELFTEST_HIP="RANK:FAMILIES[:COMMS]" (tests only): the self-test launches of those families
  // fail with a real HIP launch error on that rank (an invalid block size: not sticky, the device stays
  // usable), in the first COMMS multi-rank communicators this process creates (default: all of them)
  static std::atomic<int> created{0};
  const int serial = nranks > 1 ? created.fetch_add(1) : -1;
  if (const char* t = getenv("FLEXAR_TEST_SELFTEST_HIP")) {
    int rk = -1, comms = 1 << 30;
    unsigned fams = 0;
    if (sscanf(t, "%d:%u:%d", &rk, &fams, &comms) >= 2 && rk == rank && serial >= 0 && serial < comms)
      c->test_hip_fail = fams;
  }
  *out = c.release();
  return 0;
}

size_t flexar_handle_size(void) { return sizeof(CommHandle); }

// The IPC handle of a communicator buffer. On ROCm 7 with dmabuf IPC, exporting a fresh allocation that
// landed at the virtual address of an earlier, exported and since freed allocation (a previous
// communicator of this process) intermittently fails with "invalid argument" (seen once in a 4-process
// test on one GPU). The buffer is then replaced by a new allocation made while the old one is still held -
// so it cannot come back at the same address - and the export is retried.
static int exportable(flexar_comm* c, char** buf, size_t bytes, bool uncached, hipIpcMemHandle_t* h, const char* what) {
  std::vector<char*> held;
  hipError_t e = hipSuccess;
  for (int attempt = 0; attempt < 4; ++attempt) {
    e = hipIpcGetMemHandle(h, *buf);
    if (e == hipSuccess) break;
    (void)hipGetLastError();
    logf(LOG_WARN, c->rank, "export: hipIpcGetMemHandle(%s) failed (%s); re-allocating the %s", what,
         hipGetErrorString(e), what);
    crumb_phase("comm_export", "re-allocating a buffer whose export failed", c->rank, c->nranks);
    char* nb = nullptr;
    hipError_t a = uncached ? hipExtMallocWithFlags((void**)&nb, bytes, hipDeviceMallocUncached) : hipMalloc(&nb, bytes);
    if (a != hipSuccess || hipMemset(nb, 0, bytes) != hipSuccess) {
      (void)hipGetLastError();
      if (nb) (void)hipFree(nb);
      break;
    }
    held.push_back(*buf);
    *buf = nb;
  }
  (void)hipDeviceSynchronize();
  for (char* p : held) (void)hipFree(p);
  if (e != hipSuccess) {
    set_error(std::string("comm_export: hipIpcGetMemHandle(") + what + "): " + hipGetErrorString(e));
    return FLEXAR_ERR_HIP;
  }
  return 0;
}

int flexar_comm_export(flexar_comm_t c, void* handle_out) {
  if (!c || !handle_out) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  FX_HIP(hipSetDevice(c->device));
  crumb_phase("comm_export", "hipIpcGetMemHandle of workspace and flags", c->rank, c->nranks);
  CommHandle h;
  memset(&h, 0, sizeof(h));
  h.magic = kHandleMagic;
  h.version = FLEXAR_VERSION_MAJOR * 100 + FLEXAR_VERSION_MINOR;
  h.rank = c->rank;
  h.nranks = c->nranks;
  h.ws_bytes = c->ws_bytes;
  int rc = exportable(c, &c->stg, c->ws_bytes, false, &h.stg, "workspace");
  if (!rc) rc = exportable(c, (char**)&c->flags, kFlagWords * sizeof(uint64_t), true, &h.flags, "flags");
  if (rc) return rc;
  c->peer_stg[c->rank] = c->stg;
  c->peer_flags[c->rank] = c->flags;
  h.pid = (int32_t)getpid();
  h.device = c->device;
  gethostname(h.host, sizeof(h.host) - 1);
  if (hipDeviceGetPCIBusId(h.bus, sizeof(h.bus) - 1, c->device) != hipSuccess) {
    (void)hipGetLastError();
    snprintf(h.bus, sizeof(h.bus), "dev%d", c->device);
  }
  h.fingerprint = comm_fingerprint(c);
  h.nonce = c->nonce;
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

// Readiness gate (readiness.hpp), before any peer memory is mapped: every handle comes from this host,
// the same library version and the same settings; every peer GPU that this process can see is
// reachable peer-to-peer (hipDeviceCanAccessPeer) and its link class / hop count is recorded
// (hipExtGetLinkTypeAndHopCount) and feeds the cost model's concurrent-link count. A failure names
// the rank and the reason instead of surfacing as a raw hipIpcOpenMemHandle error or a device hang.
int flexar_comm_connect(flexar_comm_t c, const void* all) {
  if (!c || !all) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  FX_HIP(hipSetDevice(c->device));
  const CommHandle* hs = (const CommHandle*)all;
  const CommHandle& me = hs[c->rank];
  crumb_phase("comm_connect", "host page join, probe, hipIpcOpenMemHandle of every peer", c->rank, c->nranks);
  // Join the teardown agreement first (every rank gets the same handle bytes, so every rank that reaches
  // connect joins, whatever fails below): flexar_comm_destroy is collective from here on.
  if (!c->hb && c->nranks > 1 && hs[0].magic == kHandleMagic && hs[0].nranks == c->nranks) {
    char name[128];
    snprintf(name, sizeof(name), "/flexar.%d.%016llx", (int)hs[0].pid, (unsigned long long)hs[0].nonce);
    // FLEXAR_TEST_PAGE_PRIVATE=1 (tests only): every rank joins a page of its own, as with one container per
    // rank (a private /dev/shm) - what flexar_comm_host_page_check must detect
    if (env_u64("FLEXAR_TEST_PAGE_PRIVATE", 0))
      snprintf(name + strlen(name), sizeof(name) - strlen(name), ".r%d", c->rank);
    std::unique_ptr<HostBarrier> hb(new HostBarrier);
    std::string err;
    if (hb->join(name, c->rank, c->nranks, &err)) {
      c->hb = std::move(hb);
      c->hb_token = hs[0].nonce;
      c->hb_shared = -1;
      c->hb->mark(c->hb_token);  // checked by flexar_comm_host_page_check after the caller's next barrier
    } else {
      logf(LOG_WARN, c->rank, "connect: %s: teardown falls back to deferred frees", err.c_str());
    }
  }
  for (int r = 0; r < c->nranks; ++r) {
    const CommHandle& h = hs[r];
    const std::string who = "rank " + std::to_string(r);
    if (h.magic != kHandleMagic || h.rank != r || h.nranks != c->nranks) {
      set_error("bad handle from " + who + " (mismatched ranks or version)");
      return FLEXAR_ERR_INVALID;
    }
    if (h.version != me.version) {
      set_error(who + " runs another flexar version (" + std::to_string(h.version) + " vs " +
                std::to_string(me.version) + ")");
      return FLEXAR_ERR_INVALID;
    }
    if (h.ws_bytes != c->ws_bytes) {
      set_error("workspace size differs across ranks (" + who + ": " + std::to_string(h.ws_bytes) + " B, rank " +
                std::to_string(c->rank) + ": " + std::to_string(c->ws_bytes) + " B)");
      return FLEXAR_ERR_INVALID;
    }
    if (strncmp(h.host, me.host, sizeof(h.host)) != 0) {
      set_error(who + " is on host '" + std::string(h.host) + "', rank " + std::to_string(c->rank) + " on '" +
                std::string(me.host) + "': the device transport is intra-node (IPC over xGMI); use the "
                "hierarchical allreduce or RCCL across nodes");
      return FLEXAR_ERR_UNSUPPORTED;
    }
    if (h.fingerprint != me.fingerprint) {
      std::string vars;
      for (const char* const* v = fingerprint_vars(); *v; ++v) vars += std::string(vars.empty() ? "" : ", ") + *v;
      set_error(who + " resolves calls with different settings than rank " + std::to_string(c->rank) +
                " (one of " + vars + " or the tune table differs): every rank must pick the same schedule");
      return FLEXAR_ERR_INVALID;
    }
    memcpy(c->peer_bus[r], h.bus, sizeof(c->peer_bus[r]));
    c->peer_bus[r][sizeof(c->peer_bus[r]) - 1] = 0;
    c->peer_dev[r] = -1;
    if (r == c->rank) {
      c->peer_dev[r] = c->device;
      c->link_cls[r] = LINK_SAME;
      continue;
    }
    int pd = -1;
    if (hipDeviceGetByPCIBusId(&pd, c->peer_bus[r]) != hipSuccess) {
      (void)hipGetLastError();
      pd = -1;
    }
    c->peer_dev[r] = pd;
    if (pd < 0) {
      c->link_cls[r] = LINK_UNKNOWN;  // not visible here (HIP_VISIBLE_DEVICES): IPC still maps it
    } else if (pd == c->device) {
      c->link_cls[r] = LINK_SAME;
    } else {
      int can = 0;
      FX_HIP(hipDeviceCanAccessPeer(&can, c->device, pd));
      if (!can) {
        set_error("GPU " + std::to_string(c->device) + " (" + me.bus + ") cannot access GPU " + std::to_string(pd) +
                  " (" + c->peer_bus[r] + ") of " + who + " peer-to-peer: no xGMI/PCIe P2P path");
        return FLEXAR_ERR_UNSUPPORTED;
      }
      uint32_t lt = 0, hops = 0;
      if (hipExtGetLinkTypeAndHopCount(c->device, pd, &lt, &hops) == hipSuccess) {
        c->link_cls[r] = link_class_of_hsa(lt);
        c->link_hops[r] = (int32_t)hops;
      } else {
        (void)hipGetLastError();
        c->link_cls[r] = LINK_OTHER;
      }
    }
  }
  const bool no_ipc = env_u64("FLEXAR_FAULT_NO_IPC", 0) != 0;  // tests: behave as if mapping were impossible
  for (int r = 0; r < c->nranks; ++r) {
    if (r == c->rank) continue;
    const CommHandle& h = hs[r];
    void* p = nullptr;
    hipError_t e = no_ipc ? hipErrorInvalidValue : hipIpcOpenMemHandle(&p, h.stg, hipIpcMemLazyEnablePeerAccess);
    if (e == hipSuccess) {
      c->peer_stg[r] = (char*)p;
      e = hipIpcOpenMemHandle(&p, h.flags, hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) (void)hipIpcCloseMemHandle(c->peer_stg[r]);
    }
    if (e != hipSuccess) {
      (void)hipGetLastError();  // the caller may fall back to the message transport: clear the sticky error
      set_error("mapping the workspace of rank " + std::to_string(r) + " (" + link_name(c->link_cls[r]) + " peer " +
                c->peer_bus[r] + ") failed: hipIpcOpenMemHandle: " + hipGetErrorString(e) +
                " (HSA_ENABLE_IPC_MODE_LEGACY=0 is needed on dmabuf-only drivers)");
      return FLEXAR_ERR_HIP;
    }
    c->peer_flags[r] = (uint64_t*)p;
    c->opened[r] = true;
    {
      CrumbArgs ca;
      ca.type = CRUMB_HOST;
      ca.what = "peer mapped";
      ca.rank = (int16_t)c->rank;
      ca.nranks = (int16_t)c->nranks;
      ca.grid = (uint32_t)r;  // the peer
      ca.bytes = h.ws_bytes;
      ca.label = link_name(c->link_cls[r]);
      crumb(ca);
    }
  }
  // FLEXAR_TEST_PROBE="RANK:class=pcie|xgmi|same|other" or "RANK:links=K" (tests only): that rank reports
  // a different link class for every peer, or a different link count - what probe agreement must catch
  if (const char* tp = getenv("FLEXAR_TEST_PROBE")) {
    int rk = -1;
    char what[16] = {0}, val[16] = {0};
    if (sscanf(tp, "%d:%15[a-z]=%15s", &rk, what, val) == 3 && rk == c->rank) {
      if (!strcmp(what, "links")) {
        c->links_local = atoi(val);
      } else if (!strcmp(what, "class")) {
        const int32_t k = !strcmp(val, "pcie") ? LINK_PCIE : !strcmp(val, "xgmi") ? LINK_XGMI
                          : !strcmp(val, "same") ? LINK_SAME : LINK_OTHER;
        for (int r = 0; r < c->nranks; ++r)
          if (r != c->rank) c->link_cls[r] = k, c->link_hops[r] = 1;
      }
    }
  }
  if (!c->links_local) c->links_local = direct_links(c->link_cls, c->link_hops, c->nranks, c->rank);
  if (!c->links_from_env) c->model.links = c->links_local;
  c->memo_gen++;
  c->connected = true;
  return 0;
}

// Connect-time exact self-test (collective: every rank calls it after connect, in the same order).
// Each protocol family runs three allreduces of an integer pattern whose sum every rank can compute
// locally; the patterns change per call, so a read of a staging line left over from either of the two
// previous calls (the parity halves) is a mismatch. Waits use a short watchdog, so a family whose
// hand-off never becomes visible fails in seconds instead of hanging. Returns the mask of families
// that failed ON THIS RANK; the caller ORs the masks of all ranks and installs the result with
// flexar_comm_set_disabled (a family is usable only if it passed everywhere).
//
// A HIP error on this rank (a failed launch, a failed kernel) fails the family it happened in, with the
// error named in flexar_comm_selftest_note(), as long as the device is still usable; every rank still
// makes every collective call of the family. Only a sticky error (hipDeviceSynchronize fails too: the
// device context is gone) returns FLEXAR_ERR_HIP. After any failure the caller agrees on it and runs the
// collective flexar_comm_resync before the next family: a launch that never ran leaves this rank's
// epochs behind its peers'.
int flexar_comm_selftest(flexar_comm_t c, uint32_t families, uint32_t* failed_out) {
  if (!c || !failed_out) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (!c->connected) { set_error("communicator not connected"); return FLEXAR_ERR_STATE; }
  *failed_out = 0;
  c->selftest_note.clear();
  if (c->nranks == 1) return 0;
  FX_HIP(hipSetDevice(c->device));
  // HIP keeps a failed call's error for the thread until it is read: one left by an earlier, unrelated
  // call (the framework, a teardown) must not be taken for a self-test launch failure (round 3's driver
  // record: "self-test: HIP error" with no name). Name it and drop it.
  if (const hipError_t stale = hipGetLastError(); stale != hipSuccess)
    logf(LOG_WARN, c->rank, "self-test: cleared a HIP error an earlier call left in this thread: %s",
         hipGetErrorString(stale));
  const uint64_t n = 65536 + 77;  // 256 KiB + an odd tail: several workgroups, a scalar tail, LL-sized
  if (!c->st_buf) {
    FX_HIP(hipMalloc(&c->st_buf, 2 * n * sizeof(int)));
    FX_HIP(hipHostMalloc((void**)&c->st_bad, 64, hipHostMallocMapped));
    FX_HIP(hipHostGetDevicePointer((void**)&c->st_bad_dev, c->st_bad, 0));
  }
  hipStream_t st = nullptr;
  FX_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const uint64_t saved_timeout = c->timeout_ticks, saved_gen = c->memo_gen;
  const uint32_t saved_disabled = c->disabled;
  const bool saved_profile = c->profile;
  const uint64_t saved_calls = c->calls, saved_bytes = c->bytes;
  c->disabled = 0;  // the self-test drives each family explicitly
  c->profile = false;  // and stays out of the application's statistics
  c->timeout_ticks = env_u64("FLEXAR_SELFTEST_TIMEOUT_MS", 2000) * 100000ull;
  struct Case { uint32_t fam; const char* spec; };
  const Case cases[] = {{PF_FENCE, "flat+pull"}, {PF_FENCE, "ring"}, {PF_WT, "flat+pull+wt"}, {PF_LL, "ll"},
                        {PF_DMA, "dma"}, {PF_MSG, "flat+rccl"}, {PF_MSG, "ring+rccl"}};
  if (!c->nccl) families &= ~(uint32_t)PF_MSG;
  if (!c->ipc) {  // no peer memory on this communicator: only the message transport exists
    families &= PF_MSG;
    *failed_out |= PF_ALL;
  }
  std::string note;
  auto fail = [&](uint32_t fam, const std::string& why) {
    *failed_out |= fam;
    if (note.size() < 480) note += (note.empty() ? "" : "; ") + why;
  };
  int* in = c->st_buf;
  int* out = c->st_buf + n;
  const int N = c->nranks;
  int rc = 0;
  for (const Case& k : cases) {
    if (!(families & k.fam)) continue;
    if (k.fam == PF_LL && !ll_usable(c, n, 4)) continue;
    c->selftested |= k.fam;
    logf(LOG_INFO, c->rank, "self-test: %s", k.spec);
    crumb_phase("self-test family", k.spec, c->rank, c->nranks);
    for (int call = 0; call < 3 && !rc; ++call) {
      const std::string at = std::string(k.spec) + " call " + std::to_string(call);
      const uint32_t salt = (uint32_t)(call * 131 + k.fam * 17);
      const bool inject = (c->test_hip_fail & k.fam) != 0;  // tests: an invalid block size
      CrumbArgs ca;
      ca.type = CRUMB_LAUNCH;
      ca.rank = (int16_t)c->rank;
      ca.nranks = (int16_t)c->nranks;
      ca.grid = 64;
      ca.bytes = n * sizeof(int);
      ca.label = k.spec;
      ca.what = "selftest_fill";
      crumb(ca);
      hipLaunchKernelGGL(selftest_fill, dim3(64), dim3(inject ? 4096 : 256), 0, st, in, out, n, c->rank, salt);
      const hipError_t le = hipGetLastError();
      if (le != hipSuccess) fail(k.fam, at + ": selftest_fill launch: " + hipGetErrorString(le));
      // the collective call is made whatever happened above: every rank makes every call of the family
      set_error("");
      const int e = flexar_allreduce_ex(c, in, out, n, FLEXAR_INT32, FLEXAR_SUM, st, k.spec, 1.0f);
      if (e) fail(k.fam, at + ": " + (*flexar_last_error() ? flexar_last_error() : "error " + std::to_string(e)));
      __atomic_store_n(c->st_bad, 0u, __ATOMIC_RELEASE);
      ca.what = "selftest_check";
      crumb(ca);
      hipLaunchKernelGGL(selftest_check, dim3(64), dim3(256), 0, st, out, n, N, salt, c->st_bad_dev);
      const hipError_t ce = hipGetLastError();
      if (ce != hipSuccess) fail(k.fam, at + ": selftest_check launch: " + hipGetErrorString(ce));
      const hipError_t se = hipStreamSynchronize(st);
      if (se != hipSuccess) {
        (void)hipGetLastError();
        const hipError_t de = hipDeviceSynchronize();
        (void)hipGetLastError();
        if (de != hipSuccess) {  // sticky: nothing more can run in this process
          set_error("self-test " + at + ": hipStreamSynchronize: " + hipGetErrorString(se) +
                    "; the device is unusable (hipDeviceSynchronize: " + hipGetErrorString(de) + ")");
          rc = FLEXAR_ERR_HIP;
          break;
        }
        fail(k.fam, at + ": hipStreamSynchronize: " + hipGetErrorString(se));
        continue;
      }
      if (le == hipSuccess && ce == hipSuccess && !e) {
        const uint32_t bad = __atomic_load_n(c->st_bad, __ATOMIC_ACQUIRE);
        if (bad) fail(k.fam, at + ": " + std::to_string(bad) + " of " + std::to_string(n) + " sums wrong");
      }
      if (const uint32_t w = __atomic_load_n(c->err_host, __ATOMIC_ACQUIRE)) {
        if (!(*failed_out & k.fam)) fail(k.fam, at + ": device watchdog (word " + std::to_string(w) + ")");
        __atomic_store_n(c->err_host, 0u, __ATOMIC_RELEASE);  // every rank still makes every call
      }
    }
    if (rc) break;
  }
  (void)hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  (void)hipGetLastError();  // a family's failure is reported above, never at the caller's next launch
  c->have_last = false;  // `st` is gone (and synchronised): the next call must not order behind it
  c->timeout_ticks = saved_timeout;
  c->disabled = saved_disabled;
  c->profile = saved_profile;
  c->calls = saved_calls;
  c->bytes = saved_bytes;
  c->memo_gen = saved_gen + 1;
  c->selftest_note = note;
  if (!rc) set_error("");
  logf(*failed_out ? LOG_WARN : LOG_INFO, c->rank, "self-test: ran %s, failed on this rank: %s%s%s",
       family_names(c->selftested).c_str(), family_names(*failed_out).c_str(), note.empty() ? "" : " - ",
       note.c_str());
  return rc;
}

// Why families failed on this rank in the last self-test ("" = none did).
int flexar_comm_selftest_note(flexar_comm_t c, char* buf, size_t buflen) {
  if (!c || !buf || !buflen) return FLEXAR_ERR_INVALID;
  snprintf(buf, buflen, "%s", c->selftest_note.c_str());
  return c->selftest_note.size() < buflen ? 0 : FLEXAR_ERR_NOMEM;
}

// Collective recovery of the peer-memory protocol state (every rank, after an agreement that every
// rank's calls have completed, and followed by one that every rank has reset before any rank issues a
// call): this rank's flags, call epochs, staging (LL / amax granules) and error word return to their
// state after connect. Needed after a call that did not launch on some rank (its epochs fell behind its
// peers'); a plain watchdog timeout only needs flexar_comm_clear_error.
int flexar_comm_resync(flexar_comm_t c) {
  if (!c) return FLEXAR_ERR_INVALID;
  crumb_phase("comm_resync", "memsets of flags, epochs, staging", c->rank, c->nranks);
  FX_HIP(hipSetDevice(c->device));
  FX_HIP(hipDeviceSynchronize());
  FX_HIP(hipMemset(c->flags, 0, kFlagWords * sizeof(uint64_t)));
  FX_HIP(hipMemset(c->epochs, 0, kMaxGridBlocks * sizeof(uint64_t)));
  FX_HIP(hipMemset(c->stg, 0, c->ws_bytes));
  if (c->msg_epochs) FX_HIP(hipMemset(c->msg_epochs, 0, kMaxGridBlocks * sizeof(uint64_t)));
  FX_HIP(hipDeviceSynchronize());
  std::lock_guard<std::mutex> lk(c->mu);
  c->launches = 0;
  c->have_last = false;
  __atomic_store_n(c->err_host, 0u, __ATOMIC_RELEASE);
  return 0;
}

// Cost-model time (us) of `spec` on this communicator's model (links from the connect-time probe).
double flexar_comm_predict_us(flexar_comm_t c, const char* spec, double bytes) {
  if (!c) return -1.0;
  AlgoSpec s;
  std::string err;
  if (!parse_algo(spec ? spec : "auto", c->nranks, &s, &err)) { set_error(err); return -1.0; }
  if (s.kind == AlgoKind::AUTO) s = select_plan(c->model, c->nranks, bytes);
  return c->model.cost_us(s, c->nranks, bytes);
}

int flexar_rccl_available(void) { return rccl().ok ? 1 : 0; }

int flexar_rccl_unique_id(void* out, size_t len) {
  if (!out || len < sizeof(ncclUniqueId)) { set_error("unique id buffer too small (128 bytes)"); return FLEXAR_ERR_INVALID; }
  if (!rccl().ok) { set_error("RCCL not found (librccl.so)"); return FLEXAR_ERR_UNSUPPORTED; }
  ncclUniqueId id;
  int rc = rccl_check(rccl().GetUniqueId(&id), "ncclGetUniqueId");
  if (rc) return rc;
  memcpy(out, &id, sizeof(id));
  return 0;
}

// Collective: every rank passes rank 0's unique id; creates the RCCL communicator of the message
// transport ("+rccl" specs, and every call when the communicator has no IPC mapping).
int flexar_comm_init_msg(flexar_comm_t c, const void* unique_id) {
  if (!c || !unique_id) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (!rccl().ok) { set_error("RCCL not found (librccl.so)"); return FLEXAR_ERR_UNSUPPORTED; }
  if (c->nccl) return 0;
  FX_HIP(hipSetDevice(c->device));
  crumb_phase("comm_init_msg", "ncclCommInitRank of the message transport", c->rank, c->nranks);
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  int rc = rccl_check(rccl().CommInitRank(&c->nccl, c->nranks, id, c->rank), "ncclCommInitRank");
  if (rc) c->nccl = nullptr;
  c->memo_gen++;
  return rc;
}

// After a failed flexar_comm_connect on some rank (no usable IPC mapping): run every call over the
// message transport instead (flexar_comm_init_msg first). Collective in effect.
int flexar_comm_connect_msg_only(flexar_comm_t c) {
  if (!c) return FLEXAR_ERR_INVALID;
  if (!c->nccl) { set_error("message transport not initialised"); return FLEXAR_ERR_STATE; }
  c->ipc = false;
  c->connected = true;
  c->memo_gen++;
  return 0;
}

int flexar_comm_set_model(flexar_comm_t c, double alpha_launch_us, double alpha_sync_us, double link_gbps,
                          double hbm_gbps, int links) {
  if (!c || !(link_gbps > 0) || !(hbm_gbps > 0) || alpha_launch_us < 0 || alpha_sync_us < 0) {
    set_error("cost model: positive bandwidths and non-negative latencies required");
    return FLEXAR_ERR_INVALID;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  c->model.alpha_launch_us = alpha_launch_us;
  c->model.alpha_sync_us = alpha_sync_us;
  c->model.link_gbps = link_gbps;
  c->model.hbm_gbps = hbm_gbps;
  if (links > 0) c->model.links = links;
  c->memo_gen++;
  return 0;
}

int flexar_comm_set_disabled(flexar_comm_t c, uint32_t families) {
  if (!c) return FLEXAR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  c->disabled = families & PF_ALL;
  c->memo_gen++;
  return 0;
}

uint32_t flexar_comm_disabled(flexar_comm_t c) { return c ? c->disabled : 0; }

// JSON: the topology probe's view of every peer and the readiness state.
int flexar_comm_topology(flexar_comm_t c, char* buf, size_t buflen) {
  if (!c || !buf) return FLEXAR_ERR_INVALID;
  std::string j = "{\"rank\": " + std::to_string(c->rank) + ", \"device\": " + std::to_string(c->device) +
                  ", \"links\": " + std::to_string(c->model.links) + ", \"links_local\": " +
                  std::to_string(c->links_local) + ", \"links_agreed\": " + (c->links_agreed ? "true" : "false") +
                  ", \"resident_blocks\": " +
                  std::to_string(c->resident) + ", \"selftested\": \"" + family_names(c->selftested) +
                  "\", \"disabled\": \"" + (c->disabled ? family_names(c->disabled) : std::string()) +
                  "\", \"ipc\": " + (c->ipc ? "true" : "false") + ", \"rccl\": " + (c->nccl ? "true" : "false") +
                  ", \"host_page\": " + (c->hb ? "true" : "false") + ", \"host_page_shared\": " +
                  (c->hb_shared < 0 ? "null" : c->hb_shared ? "true" : "false") +
                  ", \"peers\": [";
  for (int r = 0; r < c->nranks; ++r) {
    char t[256];
    snprintf(t, sizeof(t), "%s{\"rank\": %d, \"bus\": \"%s\", \"device\": %d, \"link\": \"%s\", \"hops\": %d}",
             r ? ", " : "", r, c->peer_bus[r], c->peer_dev[r], r == c->rank ? "self" : link_name(c->link_cls[r]),
             c->link_hops[r]);
    j += t;
  }
  j += "]}";
  snprintf(buf, buflen, "%s", j.c_str());
  return j.size() < buflen ? 0 : FLEXAR_ERR_NOMEM;
}

}  // extern "C"

namespace flexar {

// Exported buffers a teardown could not agree on (a peer never reached it, or a local destroy): a peer
// may still map them, so they stay allocated for the life of the process - their virtual addresses are then
// never handed out again while that mapping lives (a fresh allocation exported at a still-mapped address is
// what ROCm's dmabuf IPC mishandles, see exportable()). Never freed (freeing the oldest past a
// count cap was exactly the case a peer may still map); the parked bytes are counted and a warning names
// them every time they pass another FLEXAR_GRAVE_WARN_BYTES (default 8 GiB).
static std::mutex g_grave_mu;
static std::vector<std::pair<int, void*>> g_grave;  // (device, pointer)
static uint64_t g_grave_bytes = 0, g_grave_warned = 0;

static void grave_keep(int device, void* p, uint64_t bytes, int rank) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_grave_mu);
  g_grave.emplace_back(device, p);
  g_grave_bytes += bytes;
  const uint64_t step = std::max<uint64_t>(1, env_u64("FLEXAR_GRAVE_WARN_BYTES", 8ull << 30));
  if (g_grave_bytes / step > g_grave_warned) {
    g_grave_warned = g_grave_bytes / step;
    logf(LOG_WARN, rank, "destroy: %zu exported buffers (%.2f GiB) parked until the process exits: their peers "
         "never agreed that they were unmapped", g_grave.size(), (double)g_grave_bytes / (1ull << 30));
  }
}

// Teardown. Collective (`agree`, the default): after this rank's own work has drained, the ranks agree
// (host_barrier.hpp) that every rank has finished every call of the communicator, each closes its
// mappings of the peers' workspaces and registrations, and they agree again that every rank has
// unmapped before anything is freed - no rank can then allocate, export or map new memory while a peer
// still holds a mapping of this communicator's. A peer that does not arrive within FLEXAR_TIMEOUT_MS
// (or a local destroy) leaves this rank's exported buffers parked (grave_keep) instead of freed.
// Without the host page (a private /dev/shm per rank, or a host agreement that timed out and dropped it) the
// caller may supply the two agreements itself (`ext`, flexar_comm_destroy_agreed: e.g. a barrier over its
// bootstrap exchange), so the workspace is still freed instead of parked.
static int destroy_impl(flexar_comm* c, bool agree, int (*ext)(void*) = nullptr, void* ext_ctx = nullptr) {
  crumb_phase("comm_destroy", agree ? "collective" : "local", c->rank, c->nranks);
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  const uint64_t timeout_ms = std::max<uint64_t>(1000, c->timeout_ticks / 100000ull);
  int rc = 0;
  bool agreed = false;
  std::string why;
  const bool use_ext = agree && !c->hb && ext != nullptr;
  if (c->hb && agree) {
    int late = -1;
    agreed = c->hb->arrive_and_wait(timeout_ms, &late);
    if (!agreed) why = "rank " + std::to_string(late) + " did not reach the teardown within " +
                       std::to_string(timeout_ms) + " ms";
  } else if (use_ext) {
    agreed = ext(ext_ctx) != 0;
    if (!agreed) why = "the caller's agreement before teardown failed";
  } else if (agree) {
    why = "no teardown agreement (the host page was dropped and the caller gave no agreement of its own)";
  }
  // teardown keeps going past failures; FLEXAR_LOG_LEVEL=info names them
  auto ipc_close = [&](void* p, const char* what, int r) {
    const hipError_t e = hipIpcCloseMemHandle(p);
    if (e != hipSuccess)
      logf(LOG_INFO, c->rank, "destroy: hipIpcCloseMemHandle(%s of rank %d, %p): %s", what, r, p, hipGetErrorString(e));
  };
  for (auto& kv : c->cache) {
    (void)hipFree(kv.second->d_ops);
    (void)hipFree(kv.second->d_chan);
  }
  for (int r = 0; r < c->nranks; ++r)
    if (c->opened[r]) {
      ipc_close(c->peer_stg[r], "workspace", r);
      ipc_close(c->peer_flags[r], "flags", r);
      c->opened[r] = false;
    }
  for (auto& kv : c->ipc_maps) ipc_close(kv.second.first, "registration", -1);
  c->ipc_maps.clear();
  c->regs.clear();
  for (int r = 0; r < kMaxRanks; ++r) {
    if (c->dma_st[r]) (void)hipStreamDestroy(c->dma_st[r]);
    if (c->dma_ag[r]) (void)hipStreamDestroy(c->dma_ag[r]);
    if (c->dma_join[r]) (void)hipEventDestroy(c->dma_join[r]);
    if (c->dma_rs_end[r]) (void)hipEventDestroy(c->dma_rs_end[r]);
    for (int k = 0; k < 2; ++k)
      if (c->dma_ag_done[r][k]) (void)hipEventDestroy(c->dma_ag_done[r][k]);
  }
  if (c->dma_fork) (void)hipEventDestroy(c->dma_fork);
  if (c->order_ev) (void)hipEventDestroy(c->order_ev);
  for (auto& kv : c->msg_cache) {
    for (Op* p : kv.second->d_ops) (void)hipFree(p);
    for (uint32_t* p : kv.second->d_chan) (void)hipFree(p);
  }
  if (c->msg_ws) (void)hipFree(c->msg_ws);
  if (c->msg_epochs) (void)hipFree(c->msg_epochs);
  if (c->nccl && rccl().ok) (void)rccl().CommDestroy(c->nccl);
  if (c->st_buf) (void)hipFree(c->st_buf);
  if (c->cal_dev) (void)hipFree(c->cal_dev);
  if (c->st_bad) (void)hipHostFree(c->st_bad);
  if (agreed && c->hb) {
    int late = -1;
    agreed = c->hb->arrive_and_wait(timeout_ms, &late);  // every rank has unmapped this rank's buffers
    if (!agreed) why = "rank " + std::to_string(late) + " did not finish unmapping within " +
                       std::to_string(timeout_ms) + " ms";
  } else if (agreed && use_ext) {
    agreed = ext(ext_ctx) != 0;
    if (!agreed) why = "the caller's agreement after unmapping failed";
  }
  // peers may map stg / flags only once this rank has exported them, and only through a connect that
  // joined the agreement (hb); without an agreement they stay parked
  const bool exported = c->nranks > 1 && !c->group_member;
  if (agreed || !exported) {
    (void)hipFree(c->stg);
    (void)hipFree(c->flags);
  } else {
    grave_keep(c->device, c->stg, c->ws_bytes, c->rank);
    grave_keep(c->device, c->flags, kFlagWords * sizeof(uint64_t), c->rank);
    if (agree) {  // a collective close that parks memory says so
      set_error("destroy: " + why + "; this rank's workspace (" + std::to_string(c->ws_bytes) +
                " bytes) stays allocated until the process exits");
      logf(LOG_WARN, c->rank, "destroy: %s; keeping this rank's exported workspace allocated", why.c_str());
      rc = c->hb || use_ext ? FLEXAR_ERR_TIMEOUT : FLEXAR_ERR_STATE;
    }
  }
  if (c->hb) c->hb->unlink();  // every rank joined long before (connect): the name is no longer needed
  c->hb.reset();
  (void)hipFree(c->epochs);
  crumb_unregister_comm(c->crumb_slot);  // before its progress words are freed
  (void)hipHostFree(c->err_host);
  delete c;
  // teardown ignores failures (e.g. closing a mapping a peer already released), but HIP keeps the last one
  // as the thread's sticky error, and the caller's framework would report it at its next kernel launch
  (void)hipGetLastError();
  return rc;
}

}  // namespace flexar

extern "C" {

int flexar_comm_destroy(flexar_comm_t c) { return c ? destroy_impl(c, true) : 0; }
int flexar_comm_destroy_agreed(flexar_comm_t c, int (*agree)(void*), void* ctx) {
  return c ? destroy_impl(c, true, agree, ctx) : 0;
}
uint64_t flexar_parked_bytes(void) {
  std::lock_guard<std::mutex> lk(g_grave_mu);
  return g_grave_bytes;
}

// Host-side agreement of this communicator's ranks (collective: every rank, same order): the maximum
// (op 0) or the bitwise OR (op 1) of one 64-bit value over the ranks, through the teardown page
// (host_barrier.hpp) - microseconds, no device call and no bootstrap round trip. FLEXAR_ERR_STATE when the
// communicator has no page (single rank, in-process group), FLEXAR_ERR_TIMEOUT naming a late rank.
int flexar_comm_host_agree(flexar_comm_t c, uint64_t mine, int op, uint64_t* out) {
  if (!c || !out || op < 0 || op > 1) { set_error("bad host agreement arguments"); return FLEXAR_ERR_INVALID; }
  if (!c->hb) { set_error("no host agreement page on this communicator"); return FLEXAR_ERR_STATE; }
  int late = -1;
  const uint64_t tmo = std::max<uint64_t>(1000, c->timeout_ticks / 100000ull);
  if (!c->hb->exchange(mine, out, tmo, &late, op == 1)) {
    set_error("host agreement: rank " + std::to_string(late) + " did not arrive within " + std::to_string(tmo) +
              " ms; the host page is dropped on this rank (its phase counter no longer matches the peers')");
    // a timed-out agreement left this rank's phase advanced: later agreements could pair wrong phases, so the
    // page is gone for good on this rank (its peers time out on their next agreement and drop theirs too)
    c->hb->unlink();
    c->hb.reset();
    c->hb_shared = 0;
    return FLEXAR_ERR_TIMEOUT;
  }
  return 0;
}

// Step 2 of the connect-time page check (step 1, HostBarrier::mark, ran in flexar_comm_connect): after a
// barrier of the caller's bootstrap that every rank passed after connecting, is every rank's identity word
// in this rank's page? *shared = 1 yes, 0 no (then the page is dropped on this rank and a named warning
// says why; the caller agrees on the answer and drops it everywhere with flexar_comm_host_page_drop).
int flexar_comm_host_page_check(flexar_comm_t c, int* shared) {
  if (!c || !shared) return FLEXAR_ERR_INVALID;
  *shared = 0;
  if (!c->hb) return 0;
  int missing = -1;
  if (c->hb->shared(c->hb_token, &missing)) {
    c->hb_shared = 1;
    *shared = 1;
    return 0;
  }
  logf(LOG_WARN, c->rank, "host page not shared: rank %d's mark is missing from %s (a private /dev/shm?): teardown "
       "needs the caller's agreement (flexar_comm_destroy_agreed; otherwise the workspace stays allocated) and "
       "host agreements go to the bootstrap", missing, c->hb->name().c_str());
  c->hb->unlink();
  c->hb.reset();
  c->hb_shared = 0;
  return 0;
}

// Drop the host page on this rank (collective in effect: every rank, when any rank's check failed).
int flexar_comm_host_page_drop(flexar_comm_t c) {
  if (!c) return FLEXAR_ERR_INVALID;
  if (c->hb) {
    c->hb->unlink();
    c->hb.reset();
  }
  c->hb_shared = 0;
  return 0;
}

// Non-collective teardown (garbage collection, a process that is abandoning its peers): no agreement;
// this rank's exported buffers stay allocated for the process's lifetime (bounded, see grave_keep).
int flexar_comm_destroy_local(flexar_comm_t c) { return c ? destroy_impl(c, false) : 0; }

int flexar_comm_rank(flexar_comm_t c) { return c ? c->rank : -1; }
int flexar_comm_size(flexar_comm_t c) { return c ? c->nranks : -1; }

int flexar_comm_set_tune_table(flexar_comm_t c, const char* text) {
  if (!c) return FLEXAR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  TuneTable t;
  if (text && *text) {
    if (!t.load_text(text)) { set_error("tune table: no 'nranks bytes spec' lines"); return FLEXAR_ERR_INVALID; }
    for (auto& n : t.rows)
      for (auto& row : n.second) {
        AlgoSpec s;
        std::string err;
        if (!parse_algo(row.second, c->nranks, &s, &err)) { set_error("tune table: " + err); return FLEXAR_ERR_INVALID; }
      }
  }
  c->tune = t;
  c->have_tune = !t.rows.empty();
  c->memo_gen++;
  return 0;
}

int flexar_comm_set_algo(flexar_comm_t c, const char* spec) {
  if (!c) return FLEXAR_ERR_INVALID;
  std::string err;
  AlgoSpec s;
  if (!parse_algo(spec ? spec : "auto", c->nranks, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  std::lock_guard<std::mutex> lk(c->mu);
  c->spec = s;
  c->memo_gen++;
  return 0;
}

// XFER work split: 0 = per-workgroup slices, else elements per round-robin chunk (a positive multiple of
// kXferChunk). Every rank of a communicator must set the same (like the grid).
int flexar_comm_set_xfer_chunk(flexar_comm_t c, uint64_t elems) {
  if (!c) return FLEXAR_ERR_INVALID;
  if (elems % kXferChunk) {
    set_error("xfer chunk: 0 or a multiple of " + std::to_string(kXferChunk) + " elements");
    return FLEXAR_ERR_INVALID;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  c->xfer_chunk = elems;
  c->memo_gen++;
  return 0;
}

int flexar_comm_set_grid(flexar_comm_t c, int grid_blocks, int block_threads) {
  if (!c) return FLEXAR_ERR_INVALID;
  (void)block_threads;
  std::lock_guard<std::mutex> lk(c->mu);
  c->grid_override = grid_blocks < 0 ? 0 : grid_blocks;
  c->memo_gen++;
  return 0;
}

// After every rank has synchronised (no kernel of this communicator in flight anywhere), forget a
// recorded watchdog timeout: epochs advance once per call on every rank even when a call aborts, and
// flags only ever grow, so the next call starts from a consistent state (the autotuner's recovery).
int flexar_comm_clear_error(flexar_comm_t c) {
  if (!c) return FLEXAR_ERR_INVALID;
  FX_HIP(hipSetDevice(c->device));
  FX_HIP(hipDeviceSynchronize());
  __atomic_store_n(c->err_host, 0u, __ATOMIC_RELEASE);
  return 0;
}

// ---- probe agreement (readiness.hpp probe_agree) -----------------------------------------------------
size_t flexar_probe_blob_size(void) { return sizeof(ProbeBlob); }

int flexar_comm_probe_export(flexar_comm_t c, void* out) {
  if (!c || !out) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  ProbeBlob b;
  memset(&b, 0, sizeof(b));
  b.magic = kProbeMagic;
  b.rank = c->rank;
  b.links = c->links_local > 0 ? c->links_local : 1;
  b.links_fixed = c->links_from_env ? c->model.links : 0;
  b.fingerprint = comm_fingerprint(c);
  b.resident = c->resident;
  for (int r = 0; r < c->nranks && r < 16; ++r) {
    b.cls[r] = (int8_t)(r == c->rank ? LINK_SAME : c->link_cls[r]);
    b.hops[r] = (int8_t)c->link_hops[r];
  }
  memcpy(out, &b, sizeof(b));
  return 0;
}

// Collective in effect: every rank passes every rank's blob (rank-major). Installs the agreed link count;
// a real disagreement fails with a message naming both ranks (and every rank fails the same way).
int flexar_comm_probe_agree(flexar_comm_t c, const void* all) {
  if (!c || !all) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  std::vector<ProbeBlob> v(c->nranks);
  memcpy(v.data(), all, sizeof(ProbeBlob) * c->nranks);
  int links = 1, resident = 0;
  std::string why;
  if (!probe_agree(v.data(), c->nranks, &links, &why, &resident)) {
    set_error(why);
    return FLEXAR_ERR_INVALID;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->links_from_env) c->model.links = links;
  if (resident > 0) c->resident = resident;  // one grid clamp on every rank
  c->links_agreed = true;
  c->memo_gen++;
  return 0;
}

// ---- connect-time calibration (calibration.hpp) ---------------------------------------------------------
// Element-wise MIN over the ranks of n doubles, through this communicator (a verified family: the call
// runs after the self-test). Every rank makes the same calls.
static int agree_min(flexar_comm* c, double* v, int n, hipStream_t st) {
  if (n > kCalAgreeMax || !c->cal_dev) { set_error("calibration: agreement vector"); return FLEXAR_ERR_INVALID; }
  FX_HIP(hipMemcpyAsync(c->cal_dev, v, n * sizeof(double), hipMemcpyHostToDevice, st));
  int rc = flexar_allreduce_ex(c, c->cal_dev, c->cal_dev, (size_t)n, FLEXAR_FLOAT64, FLEXAR_MIN, st, nullptr, 1.0f);
  if (rc) return rc;
  FX_HIP(hipMemcpyAsync(v, c->cal_dev, n * sizeof(double), hipMemcpyDeviceToHost, st));
  FX_HIP(hipStreamSynchronize(st));
  return check_err(c);
}

static std::string json_num(double x) {
  char b[64];
  snprintf(b, sizeof(b), "%.6g", x);
  return b;
}

// Link classes this rank sees, as counts (part of the cache key): x = xGMI one hop, m = xGMI multi-hop,
// s = same device, p = PCIe, u = not visible, o = other.
static std::string link_classes(flexar_comm* c) {
  int x = 0, m = 0, s = 0, p = 0, u = 0, o = 0;
  for (int r = 0; r < c->nranks; ++r) {
    if (r == c->rank) continue;
    switch (c->link_cls[r]) {
      case LINK_XGMI: (c->link_hops[r] <= 1 ? x : m)++; break;
      case LINK_SAME: ++s; break;
      case LINK_PCIE: ++p; break;
      case LINK_UNKNOWN: ++u; break;
      default: ++o;
    }
  }
  char b[96];
  snprintf(b, sizeof(b), "x%dm%ds%dp%du%do%d", x, m, s, p, u, o);
  return b;
}

// Collective (every rank, after connect, probe agreement and the self-test). mode 0 = off, 1 = the cached
// calibration of this node shape if every rank has it, else measure; 2 = measure even if cached. Times the
// calib_points() executor schedules (fp32, skipping families the self-test disabled), takes the max over
// ranks (every rank then fits identical rows to identical theta), fits and installs the model; rank 0
// writes the cache. FLEXAR_MODEL in the environment fixes the model: nothing is measured. Writes a JSON
// report. A failed measurement leaves the model unchanged on every rank (the failure flag is agreed on).
int flexar_comm_calibrate(flexar_comm_t c, int mode, char* json, size_t jlen) {
  if (!c) { set_error("null communicator"); return FLEXAR_ERR_INVALID; }
  if (!c->connected) { set_error("communicator not connected"); return FLEXAR_ERR_STATE; }
  const auto t_start = std::chrono::steady_clock::now();
  auto report = [&](const std::string& j) {
    c->calib_json = j;
    if (json && jlen) snprintf(json, jlen, "%s", j.c_str());
    return j.size() < jlen || !json ? 0 : FLEXAR_ERR_NOMEM;
  };
  const char* env_model = getenv("FLEXAR_MODEL");
  if (c->nranks == 1 || mode == 0) return report("{\"source\": \"off\"}");
  if (env_model && *env_model) return report("{\"source\": \"FLEXAR_MODEL\"}");
  if (!c->ipc) return report("{\"source\": \"off\", \"note\": \"message transport only\"}");
  // From here on every rank makes the same sequence of collective calls whatever fails locally (a rank
  // that skipped one would leave its peers an epoch ahead for good): local failures become "failed" flags
  // carried by the agreements, never early returns.
  FX_HIP(hipSetDevice(c->device));
  std::string arch = "unknown";
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) {
    arch = prop.gcnArchName;
    arch = arch.substr(0, arch.find(':'));
  } else {
    (void)hipGetLastError();
  }
  // the settings fingerprint too (grid cap, block size, chunking, tune table change what a schedule costs)
  char fp[48];
  snprintf(fp, sizeof(fp), ";settings=%016llx", (unsigned long long)comm_fingerprint(c, false));
  const std::string key = calib_key(arch, c->nranks, c->model.links, link_classes(c), c->disabled, flexar_version()) + fp;
  const std::string dir = calib_dir();
  const std::string path = dir.empty() ? std::string() : calib_path(dir, key);
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    st = nullptr;  // the null stream: the communicator orders its calls across streams itself
  }
  const uint64_t saved_timeout = c->timeout_ticks, saved_calls = c->calls, saved_bytes = c->bytes;
  const bool saved_profile = c->profile;
  c->timeout_ticks = env_u64("FLEXAR_SELFTEST_TIMEOUT_MS", 2000) * 100000ull;
  c->profile = false;
  auto finish = [&](int rc) {
    (void)hipStreamSynchronize(st);
    if (st) (void)hipStreamDestroy(st);
    c->have_last = false;
    c->timeout_ticks = saved_timeout;
    c->profile = saved_profile;
    c->calls = saved_calls;
    c->bytes = saved_bytes;
    return rc;
  };
  // 1. the cache: used only if EVERY rank loaded the same constants
  double theta[4] = {0, 0, 0, 0};
  const bool have = mode == 1 && !path.empty() && calib_load(path, key, theta);
  double v[9] = {have ? 1.0 : 0.0, theta[0], theta[1], theta[2], theta[3], -theta[0], -theta[1], -theta[2], -theta[3]};
  int rc = agree_min(c, v, 9, st);
  if (rc) return finish(rc);
  const bool same = v[0] == 1.0 && v[1] == -v[5] && v[2] == -v[6] && v[3] == -v[7] && v[4] == -v[8];
  std::string rows_json = "[]";
  CalibFit fit;
  std::string source;
  if (same) {
    source = "cache";
  } else {
    // 2. measure: every rank runs every point (epochs stay aligned); failures are agreed on below
    const std::vector<CalibPoint> pts = calib_points(c->nranks);
    double maxb = 0;
    for (const auto& p : pts) maxb = std::max(maxb, p.bytes);
    // scratch and timers first, agreed on: a rank without them must not skip calls its peers make
    char* buf = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    double ready = hipMalloc(&buf, 2 * (size_t)maxb) == hipSuccess &&
                   hipMemsetAsync(buf, 0, 2 * (size_t)maxb, st) == hipSuccess && hipEventCreate(&e0) == hipSuccess &&
                   hipEventCreate(&e1) == hipSuccess ? 1.0 : 0.0;
    if (ready == 0.0) (void)hipGetLastError();
    if (const char* tf = getenv("FLEXAR_TEST_CALIB_FAIL"))  // tests only: this rank's scratch "failed"
      if (atoi(tf) == c->rank) ready = 0.0;
    rc = agree_min(c, &ready, 1, st);
    auto release = [&]() {
      if (e0) (void)hipEventDestroy(e0);
      if (e1) (void)hipEventDestroy(e1);
      if (buf) (void)hipFree(buf);
    };
    if (rc || ready == 0.0) {
      release();
      if (rc) return finish(rc);
      finish(0);
      return report("{\"source\": \"failed\", \"key\": \"" + key + "\", \"note\": \"calibration scratch unavailable on some rank\"}");
    }
    std::vector<double> t(pts.size() + 1, 0.0);
    double failed = 0;
    crumb_phase("calibration", "timing the calibration points", c->rank, c->nranks);
    for (size_t i = 0; i < pts.size(); ++i) {
      AlgoSpec s;
      std::string err;
      if (!parse_algo(pts[i].spec, c->nranks, &s, &err) || (c->disabled & proto_family(s))) continue;
      const size_t n = (size_t)(pts[i].bytes / 4);
      const int iters = (int)std::max(5.0, std::min(50.0, 2e8 / pts[i].bytes));
      // every rank makes every call of the point whatever failed before: the first failure is
      // kept, later calls still run (or return at once on a recorded timeout); launch counts that still
      // diverged are repaired by the resync below
      int e = 0;
      auto call = [&]() {
        const int r = flexar_allreduce_ex(c, buf, buf + (size_t)maxb, n, FLEXAR_FLOAT32, FLEXAR_SUM, st,
                                          pts[i].spec.c_str(), 1.0f);
        if (r && !e) e = r;
      };
      for (int k = 0; k < 2; ++k) call();
      if (hipEventRecord(e0, st) != hipSuccess && !e) e = FLEXAR_ERR_HIP;
      for (int k = 0; k < iters; ++k) call();
      if (hipEventRecord(e1, st) != hipSuccess && !e) e = FLEXAR_ERR_HIP;
      if (!e) e = hipStreamSynchronize(st) == hipSuccess ? 0 : FLEXAR_ERR_HIP;
      float ms = 0;
      if (!e) e = hipEventElapsedTime(&ms, e0, e1) == hipSuccess ? 0 : FLEXAR_ERR_HIP;
      if (!e) e = check_err(c);
      if (e) {
        failed = 1;
        (void)hipStreamSynchronize(st);
        (void)hipGetLastError();
        __atomic_store_n(c->err_host, 0u, __ATOMIC_RELEASE);  // every rank still makes every call
        continue;
      }
      t[i] = -(double)ms * 1e3 / iters;  // negated: the MIN agreement below is a max over ranks
    }
    t[pts.size()] = -failed;
    (void)hipStreamSynchronize(st);
    release();
    // A failed call can leave this rank with fewer launches than its peers (a recorded timeout returns
    // before launching), so the device agreement below could pair the wrong epochs. The ranks first agree
    // on the host (host_barrier.hpp); after any failure every rank resets its protocol state and they
    // meet again before the next device call.
    if (c->hb) {
      uint64_t any = 0;
      int late = -1;
      const uint64_t tmo = std::max<uint64_t>(1000, saved_timeout / 100000ull);
      auto drop = [&]() {  // a timed-out agreement: phase counters no longer match (see host_agree)
        c->hb->unlink();
        c->hb.reset();
        c->hb_shared = 0;
      };
      if (!c->hb->exchange_max(failed != 0 ? 1 : 0, &any, tmo, &late)) {
        set_error("calibration: rank " + std::to_string(late) + " did not reach the failure agreement");
        drop();
        return finish(FLEXAR_ERR_TIMEOUT);
      }
      if (any) {
        if ((rc = flexar_comm_resync(c)) != 0) return finish(rc);
        if (!c->hb->arrive_and_wait(tmo, &late)) {
          set_error("calibration: rank " + std::to_string(late) + " did not finish the resync");
          drop();
          return finish(FLEXAR_ERR_TIMEOUT);
        }
      }
    }
    rc = agree_min(c, t.data(), (int)t.size(), st);
    if (rc) return finish(rc);
    std::vector<CalibRow> rows;
    rows_json = "[";
    for (size_t i = 0; i < pts.size(); ++i) {
      if (t[i] == 0.0) continue;
      rows.push_back({pts[i].spec, pts[i].bytes, -t[i]});
      rows_json += std::string(rows.size() > 1 ? ", " : "") + "[\"" + pts[i].spec + "\", " +
                   json_num(pts[i].bytes) + ", " + json_num(-t[i]) + "]";
    }
    rows_json += "]";
    if (-t[pts.size()] != 0.0) {
      logf(LOG_WARN, c->rank, "calibration: a measurement failed on some rank; the model stays unchanged");
      finish(0);
      return report("{\"source\": \"failed\", \"key\": \"" + key + "\", \"rows\": " + rows_json + "}");
    }
    fit = fit_theta(rows, c->model, c->nranks);
    if (!fit.ok) {
      finish(0);
      return report("{\"source\": \"no-fit\", \"key\": \"" + key + "\", \"rows\": " + rows_json + "}");
    }
    for (int j = 0; j < 4; ++j) theta[j] = fit.theta[j];
    source = "measured";
    if (c->rank == 0 && !path.empty() && !calib_store(path, key, theta, rows))
      logf(LOG_INFO, c->rank, "calibration: cannot write the cache %s", path.c_str());
  }
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->model = model_with_theta(c->model, theta);
    c->memo_gen++;
  }
  finish(0);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  logf(LOG_INFO, c->rank, "calibration (%s): alpha_launch %.3g us, alpha_sync %.3g us, link %.4g GB/s, hbm %.4g GB/s",
       source.c_str(), c->model.alpha_launch_us, c->model.alpha_sync_us, c->model.link_gbps, c->model.hbm_gbps);
  std::string j = "{\"source\": \"" + source + "\", \"key\": \"" + key + "\", \"path\": \"" + path +
                  "\", \"alpha_launch_us\": " + json_num(c->model.alpha_launch_us) + ", \"alpha_sync_us\": " +
                  json_num(c->model.alpha_sync_us) + ", \"link_gbps\": " + json_num(c->model.link_gbps) +
                  ", \"hbm_gbps\": " + json_num(c->model.hbm_gbps) + ", \"links\": " + std::to_string(c->model.links) +
                  ", \"rows\": " + rows_json;
  if (source == "measured")
    j += ", \"median_rel_err\": " + json_num(fit.median_rel_err) + ", \"max_rel_err\": " + json_num(fit.max_rel_err);
  j += ", \"ms\": " + json_num(ms) + "}";
  return report(j);
}

// The calibration report of the last flexar_comm_calibrate ("" if none ran).
int flexar_comm_calibration(flexar_comm_t c, char* json, size_t jlen) {
  if (!c || !json) return FLEXAR_ERR_INVALID;
  snprintf(json, jlen, "%s", c->calib_json.c_str());
  return c->calib_json.size() < jlen ? 0 : FLEXAR_ERR_NOMEM;
}

// Back to the environment's / default model (links stay the agreed count): what every rank installs when
// the ranks' calibrations disagree.
int flexar_comm_reset_model(flexar_comm_t c) {
  if (!c) return FLEXAR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  const int links = c->model.links;
  const double cap = c->model.stg_cap;
  c->model = XgmiModel::from_env();
  c->model.stg_cap = cap;
  if (!c->links_from_env) c->model.links = links;
  c->memo_gen++;
  return 0;
}

// Bit pattern hash of the installed model (ranks compare it after calibration).
uint64_t flexar_comm_model_hash(flexar_comm_t c) {
  if (!c) return 0;
  char b[256];
  snprintf(b, sizeof(b), "%a %a %a %a %d %d", c->model.alpha_launch_us, c->model.alpha_sync_us, c->model.link_gbps,
           c->model.hbm_gbps, c->model.links, (int)c->model.partials);
  return fnv1a(b);
}

}  // extern "C"
