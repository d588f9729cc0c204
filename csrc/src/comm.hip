// flexar device communicator: workspace + IPC mapping + plan cache + launch.
//
// Reference counterpart: the public entry MPI_Allreduce_FT and its helpers
// (allreduce_over_mpi/mpi_mod.hpp:216-243 FlexTree_Context, 931-950 the
// grow-only host scratch buffer, 1167-1221 the entry point). MI355X design:
//  * the scratch buffer becomes a per-communicator device workspace, IPC
//    handles exchanged once at connect time; peers write/read it over xGMI;
//  * the per-call geometry/plan is compiled once and cached per
//    (count, dtype, algorithm, scale) — no per-call heap allocation, no
//    per-call getenv (defect D8);
//  * size_t counts (defect D7); unsupported dtype/op return an error code
//    instead of exit(1); a device-side watchdog turns a stuck peer into
//    FLEXAR_ERR_TIMEOUT instead of a hang.
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
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "launch.hpp"
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
};

struct DevProgram {
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
static Roctx& roctx() {
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
static RcclApi& rccl() {
  static RcclApi a;
  return a;
}

// A message plan with its executor segments uploaded.
struct DevMsgPlan {
  MsgPlan plan;
  std::vector<Op*> d_ops;
  std::vector<uint32_t*> d_chan;
};

static uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* e = getenv(name);
  if (!e || !*e) return dflt;
  return strtoull(e, nullptr, 0);
}

}  // namespace flexar

using namespace flexar;

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
  };
  CallMemo memo[16];
  uint64_t memo_gen = 1;
  // readiness (readiness.hpp): protocol families that failed the connect-time self-test, per-peer
  // link classes from the topology probe, residency of the executor kernel
  uint32_t disabled = 0;
  uint32_t selftested = 0;  // families the self-test ran
  int32_t link_cls[kMaxRanks] = {};
  int32_t link_hops[kMaxRanks] = {};
  int32_t peer_dev[kMaxRanks] = {};  // peer's device ordinal in THIS process (-1 = not visible)
  char peer_bus[kMaxRanks][32] = {};
  bool links_from_env = false;  // FLEXAR_MODEL fixed the link count: the probe does not override it
  int resident = 0;             // executor workgroups resident at once on this GPU (occupancy x CUs)
  // message transport (msg_plan.hpp over RCCL): its own staging arena (never the IPC workspace, whose
  // parity halves peers may still read), the RCCL communicator, plans per call shape
  bool ipc = true;              // peer workspaces mapped (false: every call runs the message transport)
  ncclComm_t nccl = nullptr;
  char* msg_ws = nullptr;
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
  int* st_buf = nullptr;        // self-test buffers (device)
  uint32_t* st_bad = nullptr;   // self-test mismatch counter (host-mapped)
  uint32_t* st_bad_dev = nullptr;
};

namespace flexar {

// Serialise this call behind the communicator's previous call when it is issued on another stream.
// Under graph capture the application's graph orders its nodes, and a wait on an event recorded
// outside the capture is not allowed, so nothing is inserted.
static int order_call(flexar_comm* c, hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) { (void)hipGetLastError(); cs = hipStreamCaptureStatusNone; }
  if (cs != hipStreamCaptureStatusNone) c->captured = true;
  if (cs != hipStreamCaptureStatusNone || c->unordered) return 0;
  if (c->have_last && c->last_st != st) {
    if (!c->order_ev) FX_HIP(hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming));
    FX_HIP(hipEventRecord(c->order_ev, c->last_st));
    FX_HIP(hipStreamWaitEvent(st, c->order_ev, 0));
  }
  c->last_st = st;
  c->have_last = true;
  return 0;
}

static int resolve_spec(flexar_comm* c, const char* algo, double bytes, AlgoSpec* out) {
  AlgoSpec s = c->spec;
  if (algo && *algo) {
    std::string err;
    if (!parse_algo(algo, c->nranks, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    if (s.kind == AlgoKind::RING && c->nchannels > 1 && !strchr(algo, ':')) s.channels = c->nchannels;
  }
  if (s.kind == AlgoKind::AUTO) {
    std::string t;
    if (c->have_tune && c->tune.lookup(c->nranks, bytes, &t)) {
      std::string err;
      if (!parse_algo(t, c->nranks, &s, &err)) { set_error("tune table: " + err); return FLEXAR_ERR_INVALID; }
    } else {
      s = select_plan(c->model, c->nranks, bytes);
    }
  }
  if (s.kind == AlgoKind::TREE && s.ag == AgMode::AUTO) s.ag = AgMode::PULL;
  if (!c->ipc) s.msg = true;  // no peer memory: every schedule runs over the message transport
  if (c->disabled) {
    std::string why;
    if (!downgrade_spec(&s, c->nranks, c->disabled, true, &why, c->nccl != nullptr)) {
      set_error(why);
      return FLEXAR_ERR_UNSUPPORTED;
    }
  }
  if (s.msg && !c->nccl) {
    set_error("the message transport (+rccl) is not initialised on this communicator (flexar_comm_init_msg)");
    return FLEXAR_ERR_STATE;
  }
  *out = s;
  return 0;
}

// An executor schedule chosen after resolve_spec (RS/AG/broadcast force their own shape, a captured
// communicator replaces dma): move it onto a verified protocol family, never onto dma.
// Typed staging for an allreduce schedule (AlgoSpec::wire). Multi-hop schedules of 16/8-bit float
// dtypes keep their partial sums in fp32 staging by default (one rounding, like flat) unless the spec
// says "+rw"; fp8 wire modes need flexar_allreduce_fp8 (the amax partials). Other ops / schedules
// run untyped.
static int typed_spec(AlgoSpec* s, int dtype, int op, bool have_amax) {
  const bool sumavg = op == FLEXAR_SUM || op == FLEXAR_AVG;
  const bool narrow = dtype == FLEXAR_BFLOAT16 || dtype == FLEXAR_FLOAT16 || dtype == FLEXAR_FP8_E4M3 ||
                      dtype == FLEXAR_FP8_E5M2;
  const bool multihop = s->kind == AlgoKind::RING || (s->kind == AlgoKind::TREE && s->widths.size() > 1);
  if (s->wire >= 2) {
    if (!have_amax) {
      set_error("fp8 wire compression (" + s->str() + ") needs the amax partials: use flexar_allreduce_fp8");
      return FLEXAR_ERR_INVALID;
    }
    return 0;
  }
  if (s->wire == 1 && !(narrow && sumavg && multihop)) s->wire = 0;  // nothing to widen
  if (s->wire == 0 && !s->round_wire && narrow && sumavg && multihop) s->wire = 1;
  return 0;
}

static int executor_proto(flexar_comm* c, AlgoSpec* s) {
  if (!c->ipc) s->msg = true;
  if (!c->disabled) return 0;
  std::string why;
  if (!downgrade_spec(s, c->nranks, c->disabled, false, &why, c->nccl != nullptr)) {
    set_error(why);
    return FLEXAR_ERR_UNSUPPORTED;
  }
  return 0;
}


// LL is valid for 1/2/4-byte elements up to kLLMaxBytes when the communicator reserved its region.
static bool ll_usable(flexar_comm* c, uint64_t count, uint32_t es) {
  return c->ll_bytes && es <= 4 && (double)count * es <= kLLMaxBytes && c->nranks > 1;
}
static int ll_grid(flexar_comm* c, uint64_t count, uint32_t es) {
  uint64_t words = (count * es + 3) / 4;
  uint64_t g = (words + 2 * kExecThreads - 1) / (2 * kExecThreads);  // ~2 words per lane
  g = std::max<uint64_t>(1, std::min<uint64_t>(g, (uint64_t)c->max_grid));
  return (int)g;
}

// Decide the bit-level barrier-after flags: an XFER needs a workgroup barrier before the next
// XFER of the same SIGNAL/WAIT-free run only if they touch overlapping LOCAL memory.
static void mark_barriers(Program& P, uint32_t rank) {
  (void)rank;
  auto overlap = [&](const Loc& a, uint64_t la, const Loc& b, uint64_t lb) {
    if (a.rank != b.rank || a.buf != b.buf) return false;
    return a.off < b.off + P.extent(b, lb) && b.off < a.off + P.extent(a, la);
  };
  for (uint32_t ch = 0; ch < P.nchan; ++ch) {
    for (uint32_t i = P.chan_start[ch]; i < P.chan_start[ch + 1]; ++i) {
      Op& o = P.ops[i];
      if (o.kind != OP_XFER) continue;
      bool need = false;
      for (uint32_t j = i + 1; j < P.chan_start[ch + 1] && !need; ++j) {
        const Op& q = P.ops[j];
        if (q.kind != OP_XFER) break;
        for (int a = 0; a < o.ndst && !need; ++a) {
          for (int b = 0; b < q.nsrc && !need; ++b) need = overlap(o.dst[a], o.len, q.src[b], q.len);
          for (int b = 0; b < q.ndst && !need; ++b) need = overlap(o.dst[a], o.len, q.dst[b], q.len);
        }
        for (int a = 0; a < o.nsrc && !need; ++a)
          for (int b = 0; b < q.ndst && !need; ++b) need = overlap(o.src[a], o.len, q.dst[b], q.len);
      }
      if (need) o.flags |= kXferBarrierAfter;
    }
  }
}

static int get_program(flexar_comm* c, const AlgoSpec& s, uint64_t count, uint32_t esize, float fscale,
                       DevProgram** out, Coll coll = Coll::ALLREDUCE, uint64_t stride = 0) {
  char key[320];
  uint32_t sb;
  memcpy(&sb, &fscale, 4);
  snprintf(key, sizeof(key), "%d|%s|%llu|%u|%08x|%llu", (int)coll, s.str().c_str(), (unsigned long long)count, esize,
           sb, (unsigned long long)stride);
  auto it = c->cache.find(key);
  if (it != c->cache.end()) { *out = it->second.get(); return 0; }
  std::unique_ptr<DevProgram> dp(new DevProgram);
  std::string err;
  Planner pl(c->nranks, c->rank, count, esize, fscale);
  if (!pl.build_coll(coll, s, stride, &dp->prog, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  uint64_t in_el, out_el;
  io_extent(coll, c->nranks, count, stride, &in_el, &out_el);
  if (!validate_program(dp->prog, c->nranks, c->rank, in_el, out_el, &err)) {
    set_error(err);
    return FLEXAR_ERR_INVALID;
  }
  mark_barriers(dp->prog, c->rank);
  logf(LOG_INFO, c->rank, "plan %s: count=%llu esize=%u ops=%zu channels=%u staging=%llu B", s.str().c_str(),
       (unsigned long long)count, esize, dp->prog.ops.size(), dp->prog.nchan,
       (unsigned long long)dp->prog.stg_bytes());
  if (log_level() >= LOG_DEBUG) logf(LOG_DEBUG, c->rank, "%s", dump_program(dp->prog, c->rank).c_str());
  size_t ob = dp->prog.ops.size() * sizeof(Op), cb = dp->prog.chan_start.size() * sizeof(uint32_t);
  FX_HIP(hipMalloc(&dp->d_ops, ob ? ob : sizeof(Op)));
  FX_HIP(hipMalloc(&dp->d_chan, cb));
  if (ob) FX_HIP(hipMemcpy(dp->d_ops, dp->prog.ops.data(), ob, hipMemcpyHostToDevice));
  FX_HIP(hipMemcpy(dp->d_chan, dp->prog.chan_start.data(), cb, hipMemcpyHostToDevice));
  *out = dp.get();
  c->cache[key] = std::move(dp);
  return 0;
}

static int proto_of(const AlgoSpec& s) { return s.wt ? PM_WT : s.nts ? PM_FENCE_NTS : PM_FENCE; }

// Zero-copy program: the peers' buffers of this call. `in` / `out` must lie inside registrations; every
// rank passes the same offsets into its corresponding registration (the registration contract, like
// NCCL's registered buffers), so rank p's operand is its registered base + the same offset.
static int zc_bind(flexar_comm* c, const Program& P, const void* in, uint64_t in_bytes, const void* out,
                   uint64_t out_bytes, DevCtx* x) {
  const void* ptrs[2] = {in, out};
  const uint64_t sizes[2] = {in_bytes, out_bytes};
  for (int b = 0; b < 2; ++b) {
    if (!(P.zc_bufs & (1u << b))) continue;  // the program never addresses this buffer on a peer
    const char* q = (const char*)ptrs[b];
    const flexar_comm::Reg* g = nullptr;
    for (const auto& r : c->regs)
      if (q >= r.base && q + sizes[b] <= r.base + r.bytes) { g = &r; break; }
    if (!g) {
      set_error(std::string("zero-copy (+zc) needs registered buffers: the ") + (b ? "output" : "input") +
                " is not inside a registration (Communicator.register / flexar_reg_open)");
      return FLEXAR_ERR_INVALID;
    }
    const uint64_t d = (uint64_t)(q - g->base);
    for (int p = 0; p < c->nranks; ++p) x->peer_io[b][p] = p == c->rank ? (char*)q : g->peer[p] + d;
    if (!g->aligned || (d & 15)) x->vec_ok = 0;
  }
  return 0;
}

static int choose_grid(flexar_comm* c, uint64_t bytes, uint32_t nchan) {
  int g = c->grid_override;
  if (g <= 0) {
    uint64_t want = (bytes + c->min_block_bytes - 1) / c->min_block_bytes;
    g = (int)std::min<uint64_t>(want, (uint64_t)c->max_grid);
  }
  if (g < (int)nchan) g = (int)nchan;
  g = (g + nchan - 1) / nchan * nchan;  // whole channels
  const int cap = std::max((int)nchan, std::min(std::max(c->max_grid, c->grid_override), (int)kMaxGridBlocks));
  if (g > cap) g = cap / (int)nchan * (int)nchan;  // round down rather than exceed the cap
  return g;
}

static void fill_ctx(flexar_comm* c, DevProgram* dp, const void* in, void* out, DevCtx* x) {
  memset(x, 0, sizeof(*x));
  if (dp) {
    x->ops = dp->d_ops;
    x->chan_start = dp->d_chan;
    x->nchan = dp->prog.nchan;
  }
  x->ll_off = c->exec_half + kAmaxRegion;
  x->amax_off = c->exec_half;
  x->stg_unit = dp ? dp->prog.stg_unit() : 0;
  x->nranks = c->nranks;
  x->rank = c->rank;
  x->local[BUF_IN] = (char*)in;
  x->local[BUF_OUT] = (char*)out;
  x->local[BUF_STG] = c->stg;
  for (int r = 0; r < c->nranks; ++r) {
    x->peer_stg[r] = c->peer_stg[r];
    x->peer_flags[r] = c->peer_flags[r];
  }
  x->epochs = c->epochs;
  x->stg_half_bytes = c->half_bytes;
  x->err = c->err_dev;
  x->timeout_ticks = c->timeout_ticks;
  x->vec_ok = ((((uintptr_t)in) | ((uintptr_t)out)) & 15) == 0;
  x->fi_kind = c->fi_kind;
  x->fi_slot = c->fi_slot;
  x->fi_ticks = c->fi_ticks;
}

// Both buffers of an allreduce inside registrations (what a zero-copy choice needs).
static bool zc_registered(flexar_comm* c, const void* in, const void* out, uint64_t bytes) {
  auto inside = [&](const void* p) {
    for (const auto& r : c->regs)
      if ((const char*)p >= r.base && (const char*)p + bytes <= r.base + r.bytes) return true;
    return false;
  };
  return inside(in) && inside(out);
}

// ---- message transport (msg_plan.hpp over RCCL) ----------------------------------------------------
static int rccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return 0;
  set_error(std::string(what) + ": " + (rccl().GetErrorString ? rccl().GetErrorString(r) : "RCCL error"));
  return FLEXAR_ERR_RCCL;
}

static int get_msg_plan(flexar_comm* c, const AlgoSpec& s, uint64_t count, uint32_t es, float fs, Coll coll,
                        uint64_t stride, DevMsgPlan** out) {
  char key[320];
  uint32_t sb;
  memcpy(&sb, &fs, 4);
  snprintf(key, sizeof(key), "%d|%s|%llu|%u|%08x|%llu", (int)coll, s.str().c_str(), (unsigned long long)count, es, sb,
           (unsigned long long)stride);
  auto it = c->msg_cache.find(key);
  if (it != c->msg_cache.end()) { *out = it->second.get(); return 0; }
  std::unique_ptr<DevMsgPlan> dp(new DevMsgPlan);
  std::string err;
  if (!build_msg_plan(c->nranks, c->rank, count, es, fs, s, &dp->plan, &err, coll, stride)) {
    set_error(err);
    return FLEXAR_ERR_INVALID;
  }
  uint64_t in_el, out_el;
  io_extent(coll, c->nranks, count, stride, &in_el, &out_el);
  for (auto& st : dp->plan.steps) {
    if (st.kind != MsgStep::EXEC) continue;
    if (!validate_program(st.prog, c->nranks, c->rank, in_el, out_el, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    mark_barriers(st.prog, c->rank);
    Op* d_ops = nullptr;
    uint32_t* d_chan = nullptr;
    FX_HIP(hipMalloc(&d_ops, st.prog.ops.size() * sizeof(Op)));
    FX_HIP(hipMalloc(&d_chan, st.prog.chan_start.size() * sizeof(uint32_t)));
    FX_HIP(hipMemcpy(d_ops, st.prog.ops.data(), st.prog.ops.size() * sizeof(Op), hipMemcpyHostToDevice));
    FX_HIP(hipMemcpy(d_chan, st.prog.chan_start.data(), st.prog.chan_start.size() * sizeof(uint32_t),
                     hipMemcpyHostToDevice));
    dp->d_ops.push_back(d_ops);
    dp->d_chan.push_back(d_chan);
  }
  logf(LOG_INFO, c->rank, "msg plan %s: count=%llu steps=%zu messages=%llu (%llu zero-copy) arena=%llu B",
       s.str().c_str(), (unsigned long long)count, dp->plan.steps.size(), (unsigned long long)dp->plan.msgs,
       (unsigned long long)dp->plan.zero_copy, (unsigned long long)dp->plan.stg_bytes);
  *out = dp.get();
  c->msg_cache[key] = std::move(dp);
  return 0;
}

// One call over the message transport: executor segments (local-only programs) and grouped
// ncclSend / ncclRecv, all on `st`. The arena is the transport's own (parity-free: RCCL orders calls).
static int run_msg(flexar_comm* c, const AlgoSpec& s, Coll coll, const void* in, void* out, uint64_t count, int dtype,
                   int op, float fs, uint64_t stride, hipStream_t st) {
  const uint32_t es = (uint32_t)dtype_size(dtype);
  DevMsgPlan* dp = nullptr;
  int rc = get_msg_plan(c, s, count, es, fs, coll, stride, &dp);
  if (rc) return rc;
  if (dp->plan.stg_bytes > c->msg_ws_bytes) {  // grow (first calls only): nothing of ours may still read it
    FX_HIP(hipDeviceSynchronize());
    if (c->msg_ws) FX_HIP(hipFree(c->msg_ws));
    c->msg_ws = nullptr;
    c->msg_ws_bytes = 0;
    FX_HIP(hipMalloc(&c->msg_ws, dp->plan.stg_bytes + 256));
    c->msg_ws_bytes = dp->plan.stg_bytes;
  }
  const int op_k = coll == Coll::ALLREDUCE || coll == Coll::REDUCE_SCATTER ? op : FLEXAR_SUM;
  auto ptr = [&](uint16_t buf) -> char* {
    return buf == BUF_IN ? (char*)in : (buf == BUF_OUT ? (char*)out : c->msg_ws);
  };
  size_t ex = 0;
  for (const MsgStep& stp : dp->plan.steps) {
    if (stp.kind == MsgStep::EXEC) {
      LaunchArgs la;
      la.kind = LAUNCH_EXEC;
      DevCtx& x = la.ctx;
      memset(&x, 0, sizeof(x));
      x.ops = dp->d_ops[ex];
      x.chan_start = dp->d_chan[ex];
      x.nchan = 1;
      x.rank = c->rank;
      x.nranks = c->nranks;
      x.local[BUF_IN] = (char*)in;
      x.local[BUF_OUT] = (char*)out;
      x.local[BUF_STG] = c->msg_ws;
      for (int r = 0; r < c->nranks; ++r) x.peer_stg[r] = c->msg_ws;  // local-only program
      x.peer_flags[c->rank] = c->flags;
      x.epochs = c->epochs;
      x.stg_half_bytes = 0;
      x.err = c->err_dev;
      x.timeout_ticks = c->timeout_ticks;
      x.vec_ok = ((((uintptr_t)in) | ((uintptr_t)out)) & 15) == 0;
      x.stg_unit = es;
      uint64_t span = 0;
      for (const Op& o : stp.prog.ops) span = std::max<uint64_t>(span, o.len);
      la.grid = choose_grid(c, span * es * 2, 1);
      la.stream = st;
      la.proto = PM_FENCE;
      if ((rc = launch_dtype(dtype, op_k, la))) return rc;
      c->launches++;
      ++ex;
      continue;
    }
    if ((rc = rccl_check(rccl().GroupStart(), "ncclGroupStart"))) return rc;
    for (const MsgXfer& m : stp.sends)
      if ((rc = rccl_check(rccl().Send(ptr(m.buf) + m.off, m.bytes, ncclUint8, (int)m.peer, c->nccl, st), "ncclSend")))
        break;
    for (const MsgXfer& m : stp.recvs) {
      if (rc) break;
      rc = rccl_check(rccl().Recv(ptr(m.buf) + m.off, m.bytes, ncclUint8, (int)m.peer, c->nccl, st), "ncclRecv");
    }
    const int rc2 = rccl_check(rccl().GroupEnd(), "ncclGroupEnd");
    if (rc || rc2) return rc ? rc : rc2;
  }
  return 0;
}

// Split a call into pieces whose staging fits one parity half of the workspace.
static int plan_pieces(flexar_comm* c, const AlgoSpec& s, uint64_t count, uint32_t esize, float fs,
                       uint64_t* piece, Coll coll = Coll::ALLREDUCE, uint64_t stride = 0) {
  DevProgram* dp = nullptr;
  int rc = get_program(c, s, count, esize, fs, &dp, coll, stride);
  if (rc) return rc;
  uint64_t need = dp->prog.stg_bytes();
  const uint64_t bytes = count * esize;
  const bool chunked = c->chunk_bytes && bytes > c->chunk_bytes;
  if (need <= c->exec_half && !chunked) { *piece = count; return 0; }
  uint64_t align = std::max<uint64_t>(1, kStageAlignBytes / esize) * (coll == Coll::ALLREDUCE ? c->nranks : 1);
  uint64_t pieces = std::max<uint64_t>((need + c->exec_half - 1) / c->exec_half,
                                       chunked ? (bytes + c->chunk_bytes - 1) / c->chunk_bytes : 1);
  for (int tries = 0; tries < 64; ++tries, ++pieces) {
    uint64_t p = (count + pieces - 1) / pieces;
    p = (p + align - 1) / align * align;
    if (p == 0) p = align;
    rc = get_program(c, s, p, esize, fs, &dp, coll, stride);
    if (rc) return rc;
    if (dp->prog.stg_bytes() <= c->exec_half) { *piece = p; return 0; }
  }
  set_error("workspace too small for this algorithm");
  return FLEXAR_ERR_NOMEM;
}

// Reduce-scatter / all-gather (count = elements per rank block): split along the block so each
// piece's program sees blocks `stride` = count elements apart in the N*count-sized buffer.
static int run_rs_ag(flexar_comm* c, Coll coll, const void* in, void* out, size_t count, int dtype, int op,
                     hipStream_t st, const char* algo, float scale) {
  const uint32_t es = (uint32_t)dtype_size(dtype);
  float fs = coll == Coll::REDUCE_SCATTER ? scale * (op == FLEXAR_AVG ? 1.0f / (float)c->nranks : 1.0f) : 1.0f;
  AlgoSpec s;
  int rc = resolve_spec(c, algo, (double)count * es * c->nranks, &s);
  if (rc) return rc;
  if (s.kind != AlgoKind::RING) s.kind = AlgoKind::TREE, s.widths = {c->nranks}, s.ag = AgMode::PUSH;
  if ((rc = executor_proto(c, &s))) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  // registered buffers and no named spec: the direct exchange runs zero copy (the buffer the peers address
  // - reduce-scatter: the input, all-gather / all-to-all: the output - must lie inside a registration)
  if (!c->regs.empty() && !s.zc && !s.msg && c->zc_auto && s.kind == AlgoKind::TREE && c->nranks > 1 &&
      !(algo && *algo && strcmp(algo, "auto") != 0) && c->spec.kind == AlgoKind::AUTO &&
      !(c->disabled & proto_family(s))) {
    const uint64_t wide = (uint64_t)c->nranks * count * es;
    const bool rs = coll == Coll::REDUCE_SCATTER;
    const void* p = rs ? in : out;
    for (const auto& r : c->regs)
      if ((const char*)p >= r.base && (const char*)p + wide <= r.base + r.bytes) { s.zc = true; break; }
  }
  if ((rc = order_call(c, st))) return rc;
  if (s.msg) {
    s.wire = 0;
    c->calls++;
    c->bytes += count * es * c->nranks;
    return run_msg(c, s, coll, in, out, count, dtype, coll == Coll::ALL_GATHER ? FLEXAR_SUM : op, fs, count, st);
  }
  uint64_t piece = count;
  if (c->nranks > 1 && (rc = plan_pieces(c, s, count, es, fs, &piece, coll, count))) return rc;
  for (uint64_t off = 0; off < count; off += piece) {
    uint64_t n = std::min<uint64_t>(piece, count - off);
    DevProgram* dp = nullptr;
    if ((rc = get_program(c, s, n, es, fs, &dp, coll, count))) return rc;
    DevCtx x;
    fill_ctx(c, dp, (const char*)in + off * es, (char*)out + off * es, &x);
    if (dp->prog.zc) {  // the N-block side spans (N - 1) rank strides + this piece
      const uint64_t wide = ((uint64_t)(c->nranks - 1) * count + n) * es;
      const uint64_t in_b = coll == Coll::ALL_GATHER ? n * es : wide, out_b = coll == Coll::REDUCE_SCATTER ? n * es : wide;
      if ((rc = zc_bind(c, dp->prog, (const char*)in + off * es, in_b, (char*)out + off * es, out_b, &x))) return rc;
    }
    LaunchArgs la;
    la.kind = LAUNCH_EXEC;
    la.ctx = x;
    la.grid = choose_grid(c, n * es * c->nranks, dp->prog.nchan);
    la.stream = st;
    la.proto = proto_of(s);
    // all-gather moves bytes only: run the SUM instantiation (the op is never applied, K == 1)
    if ((rc = launch_dtype(dtype, coll == Coll::ALL_GATHER ? FLEXAR_SUM : op, la))) return rc;
    c->launches++;
  }
  c->calls++;
  c->bytes += count * es * c->nranks;
  return 0;
}

// Broadcast spec: "oneshot"/"ll" = direct multicast from the root, any other explicit spec = scatter +
// all-gather (its "+wt"/"+nts" protocol modifiers apply); auto: direct up to 256 KiB (one hop wins while
// latency bound), scatter + all-gather above (~2 S / N per link instead of S out of the root).
static int bcast_spec(flexar_comm* c, const char* algo, uint64_t bytes, AlgoSpec* out) {
  AlgoSpec s;
  if (algo && *algo) {
    std::string err;
    if (!parse_algo(algo, c->nranks, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  }
  if (s.kind == AlgoKind::AUTO || s.kind == AlgoKind::DMA) s.kind = bytes <= (256u << 10) ? AlgoKind::ONESHOT : AlgoKind::TREE;
  if (s.kind == AlgoKind::LL) s.kind = AlgoKind::ONESHOT;
  if (s.kind != AlgoKind::ONESHOT) s.kind = AlgoKind::TREE, s.widths = {c->nranks};
  *out = s;
  return executor_proto(c, out);
}

// Broadcast of `count` elements from `root` (root reads `in`; every rank writes `out`), split into
// pieces that fit one staging half. The executor only copies (K = 1), so the SUM instantiation runs.
static int run_bcast(flexar_comm* c, const void* in, void* out, size_t count, int dtype, int root, hipStream_t st,
                     const char* algo) {
  const uint32_t es = (uint32_t)dtype_size(dtype);
  AlgoSpec s;
  int rc = bcast_spec(c, algo, (uint64_t)count * es, &s);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = order_call(c, st))) return rc;
  if (s.msg) {
    c->calls++;
    c->bytes += count * es;
    return run_msg(c, s, Coll::BROADCAST, in, out, count, dtype, FLEXAR_SUM, 1.0f, (uint64_t)root, st);
  }
  uint64_t piece = count;
  if (c->nranks > 1 && (rc = plan_pieces(c, s, count, es, 1.0f, &piece, Coll::BROADCAST, (uint64_t)root))) return rc;
  for (uint64_t off = 0; off < count; off += piece) {
    uint64_t n = std::min<uint64_t>(piece, count - off);
    DevProgram* dp = nullptr;
    if ((rc = get_program(c, s, n, es, 1.0f, &dp, Coll::BROADCAST, (uint64_t)root))) return rc;
    DevCtx x;
    fill_ctx(c, dp, (const char*)in + off * es, (char*)out + off * es, &x);
    if (dp->prog.zc &&
        (rc = zc_bind(c, dp->prog, (const char*)in + off * es, n * es, (char*)out + off * es, n * es, &x)))
      return rc;
    LaunchArgs la;
    la.kind = LAUNCH_EXEC;
    la.ctx = x;
    la.grid = choose_grid(c, n * es, dp->prog.nchan);
    la.stream = st;
    la.proto = proto_of(s);
    if ((rc = launch_dtype(dtype, FLEXAR_SUM, la))) return rc;
    c->launches++;
  }
  c->calls++;
  c->bytes += count * es;
  return 0;
}

// dst (and dst2, if given) = scale * OP(srcs[0..nsrc)) over `count` elements: groups of kMaxSrc
// sources chain through dst (fan-in > 8: dst joins the next group; only the last group scales and
// writes dst2).
static int reduce_chain(char* dst, char* dst2, const char* const* srcs, int nsrc, uint64_t count, int dtype,
                        int op, float fs, hipStream_t st, int proto) {
  const size_t es = dtype_size(dtype);
  int grid = (int)std::min<uint64_t>(1024, std::max<uint64_t>(1, count * es / (64 * 1024)));
  int done = 0;
  while (done < nsrc) {
    SrcTable t;
    memset(&t, 0, sizeof(t));
    int k = 0;
    if (done > 0) t.p[k++] = dst;
    while (k < (int)kMaxSrc && done < nsrc) t.p[k++] = srcs[done++];
    const bool last = done >= nsrc;
    uintptr_t al = (uintptr_t)dst | (last && dst2 ? (uintptr_t)dst2 : 0);
    for (int i = 0; i < k; ++i) al |= (uintptr_t)t.p[i];
    LaunchArgs la;
    la.kind = LAUNCH_REDUCE;
    la.srcs = t;
    la.nsrc = k;
    la.dst = dst;
    la.dst2 = last ? dst2 : nullptr;
    la.n = count;
    la.scale = last ? fs : 1.0f;
    la.vec = (al & 15) == 0 ? 1 : 0;
    la.grid = grid;
    la.stream = st;
    la.proto = proto;
    int rc = launch_dtype(dtype, op, la);
    if (rc) return rc;
  }
  return 0;
}

// ---- copy-engine ("dma") allreduce ------------------------------------------------------------
// The flat two-shot exchange with the bytes moved by copy engines instead of CUs, so an allreduce
// overlapped with compute (DDP backward) takes no CUs beyond a short reduce (SURVEY.md §5.8 (a),
// the reference's MPI_Isend/Irecv per block, mpi_mod.hpp:662-765, as one peer copy per peer). A call is
// split into pieces whose N landing slots + 1 result slot fit one staging parity half; piece k runs
//   RS   on peer p's reduce-scatter stream: copy my block p of piece k into p's landing slot r, then write
//        flag (kDmaSlotRS, r) = e_k into p's flags (stream-ordered after the copy);
//   RED  on the caller's stream: wait for every peer's RS flag e_k, reduce my block (write-through) into
//        OUT and my result slot, write flag (kDmaSlotAG, r) = e_k to every peer;
//   AG   on peer q's all-gather stream: wait for q's AG flag e_k, copy q's result slot into OUT block q.
// Pipelined: the reference serialises send -> recv -> reduce per stage
// (mpi_mod.hpp:988-1029); here the streams of different phases run concurrently, so the SDMA copies of
// piece k+1 overlap the reduce of piece k and the all-gather copies of piece k overlap the reduce-scatter
// copies of piece k+1. Pieces alternate staging halves (parity = epoch & 1); reusing a half is safe
// because piece k+2's RS copy into p waits for my AG copy of piece k from p (event per peer and parity),
// which followed p's AG flag, which p wrote after reducing piece k out of that half - and p reduces piece
// k+2 (overwriting its result slot) only after my RS flag of k+2. The host enqueues RS(k), RED(k),
// AG(k), RS(k+1), ...: every wait depends only on earlier-enqueued work of some rank, so hardware queues
// shared by several streams cannot deadlock.
static int dma_init(flexar_comm* c) {
  if (c->dma_ready) return 0;
  FX_HIP(hipSetDevice(c->device));
  for (int p = 0; p < c->nranks; ++p) {
    if (p == c->rank) continue;
    FX_HIP(hipStreamCreateWithFlags(&c->dma_st[p], hipStreamNonBlocking));
    FX_HIP(hipStreamCreateWithFlags(&c->dma_ag[p], hipStreamNonBlocking));
    FX_HIP(hipEventCreateWithFlags(&c->dma_join[p], hipEventDisableTiming));
    FX_HIP(hipEventCreateWithFlags(&c->dma_rs_end[p], hipEventDisableTiming));
    FX_HIP(hipEventCreateWithFlags(&c->dma_ag_done[p][0], hipEventDisableTiming));
    FX_HIP(hipEventCreateWithFlags(&c->dma_ag_done[p][1], hipEventDisableTiming));
  }
  FX_HIP(hipEventCreateWithFlags(&c->dma_fork, hipEventDisableTiming));
  c->dma_ready = true;
  return 0;
}

// elements per dma piece: N + 1 block slots must fit one parity half (FLEXAR_CHUNK_BYTES caps it too)
static uint64_t dma_piece(flexar_comm* c, uint64_t count, uint32_t es) {
  const uint64_t slot = c->exec_half / (uint64_t)(c->nranks + 1) / kStageAlignBytes * kStageAlignBytes;
  uint64_t per_block = std::max<uint64_t>(1, slot / es);
  if (c->chunk_bytes) per_block = std::max<uint64_t>(1, std::min<uint64_t>(per_block, c->chunk_bytes / es / c->nranks));
  return std::min<uint64_t>(count, per_block * (uint64_t)c->nranks);
}

static int dma_wait(flexar_comm* c, uint32_t slot, const int* srcs, int n, uint64_t e, hipStream_t st) {
  DmaWait w;
  memset(&w, 0, sizeof(w));
  w.flags = c->flags;
  for (int i = 0; i < n; ++i) {
    w.idx[i] = (uint32_t)flag_index(slot, (uint32_t)srcs[i], 0);
    w.src[i] = (uint32_t)srcs[i];
  }
  w.n = (uint32_t)n;
  w.slot = slot;
  w.value = e;
  w.timeout_ticks = c->timeout_ticks;
  w.err = c->err_dev;
  hipLaunchKernelGGL(dma_wait_kernel, dim3(1), dim3(64), 0, st, w);
  FX_HIP(hipGetLastError());
  return 0;
}

// phase: 0 = fork (first piece only), 1 = RS copies of the piece, 2 = reduce, 3 = AG, 4 = join (after the
// last piece). `e` is the piece's epoch.
static int dma_phase(flexar_comm* c, int phase, const char* in, char* out, uint64_t count, int dtype, int op,
                     float fs, hipStream_t st, uint64_t e) {
  const int N = c->nranks, r = c->rank;
  const uint64_t es = dtype_size(dtype);
  const uint64_t B = (count + N - 1) / N;
  const uint64_t Bb = (B * es + kStageAlignBytes - 1) / kStageAlignBytes * kStageAlignBytes;
  const uint64_t par = (e & 1) ? c->half_bytes : 0;
  auto len = [&](int i) -> uint64_t {
    const uint64_t s0 = (uint64_t)i * B;
    return s0 >= count ? 0 : std::min<uint64_t>(B, count - s0);
  };
  if (phase == 0) {  // the streams start after everything the caller enqueued before this call
    FX_HIP(hipEventRecord(c->dma_fork, st));
    for (int p = 0; p < N; ++p) {
      if (p == r) continue;
      FX_HIP(hipStreamWaitEvent(c->dma_st[p], c->dma_fork, 0));
      FX_HIP(hipStreamWaitEvent(c->dma_ag[p], c->dma_fork, 0));
    }
  } else if (phase == 1) {
    for (int j = 1; j < N; ++j) {
      const int p = (r + j) % N;
      hipStream_t s = c->dma_st[p];
      // p's landing slots / result slot of this parity were last used two pieces ago: my AG copy of that
      // piece from p (after p's AG flag, i.e. after p reduced it) must be complete
      FX_HIP(hipStreamWaitEvent(s, c->dma_ag_done[p][e & 1], 0));
      if (len(p))
        FX_HIP(hipMemcpyAsync(c->peer_stg[p] + par + (uint64_t)r * Bb, in + (uint64_t)p * B * es, len(p) * es,
                              hipMemcpyDeviceToDevice, s));
      FX_HIP(hipStreamWriteValue64(s, c->peer_flags[p] + flag_index(kDmaSlotRS, (uint32_t)r, 0), e, 0));
    }
  } else if (phase == 2) {
    int peers[kMaxRanks], np = 0;
    for (int j = 1; j < N; ++j) peers[np++] = (r + j) % N;
    int rc = dma_wait(c, kDmaSlotRS, peers, np, e, st);
    if (rc) return rc;
    if (len(r)) {
      const char* srcs[kMaxRanks];
      int ns = 0;
      srcs[ns++] = in + (uint64_t)r * B * es;
      for (int j = 0; j < np; ++j) srcs[ns++] = c->stg + par + (uint64_t)peers[j] * Bb;
      rc = reduce_chain(out + (uint64_t)r * B * es, c->stg + par + (uint64_t)N * Bb, srcs, ns, len(r), dtype, op, fs,
                        st, PM_WT);
      if (rc) return rc;
    }
    for (int j = 0; j < np; ++j)
      FX_HIP(hipStreamWriteValue64(st, c->peer_flags[peers[j]] + flag_index(kDmaSlotAG, (uint32_t)r, 0), e, 0));
  } else if (phase == 3) {
    for (int j = 1; j < N; ++j) {
      const int q = (r + j) % N;
      hipStream_t s = c->dma_ag[q];
      // q's AG flag: q reduced this piece, which needed my RS flag, which followed my RS copy out of an
      // in-place OUT block q - so the copy below cannot overwrite data my RS copy still reads
      int rc = dma_wait(c, kDmaSlotAG, &q, 1, e, s);
      if (rc) return rc;
      if (len(q))
        FX_HIP(hipMemcpyAsync(out + (uint64_t)q * B * es, c->peer_stg[q] + par + (uint64_t)N * Bb, len(q) * es,
                              hipMemcpyDeviceToDevice, s));
      FX_HIP(hipEventRecord(c->dma_ag_done[q][e & 1], s));
    }
    c->launches = e;
  } else {  // join: the caller's stream continues after every copy of the call; epochs advance to e
    for (int j = 1; j < N; ++j) {
      const int q = (r + j) % N;
      FX_HIP(hipEventRecord(c->dma_join[q], c->dma_ag[q]));
      FX_HIP(hipEventRecord(c->dma_rs_end[q], c->dma_st[q]));
      FX_HIP(hipStreamWaitEvent(st, c->dma_join[q], 0));
      FX_HIP(hipStreamWaitEvent(st, c->dma_rs_end[q], 0));
    }
    hipLaunchKernelGGL(epoch_set_kernel, dim3(1), dim3(256), 0, st, c->epochs, e);
    FX_HIP(hipGetLastError());
  }
  return 0;
}

static int run_dma(flexar_comm* const* cs, int ncomm, const char* const* ins, char* const* outs, uint64_t count,
                   int dtype, int op, float fs, hipStream_t st) {
  const uint32_t es = (uint32_t)dtype_size(dtype);
  for (int i = 0; i < ncomm; ++i) {
    int rc = dma_init(cs[i]);
    if (rc) return rc;
  }
  const uint64_t piece = dma_piece(cs[0], count, es);
  const uint64_t e0 = cs[0]->launches;
  auto each = [&](int phase, uint64_t off, uint64_t n, uint64_t e) {
    // phase by phase across the group: a rank's waits are enqueued after every rank's signals
    for (int i = 0; i < ncomm; ++i) {
      int rc = dma_phase(cs[i], phase, ins[i] + off * es, outs[i] + off * es, n, dtype, op, fs, st, e);
      if (rc) return rc;
    }
    return 0;
  };
  // FLEXAR_DMA_SERIAL=1: join + fork around every piece (the round-1 serial schedule, for A/B measurements)
  static const bool serial = env_u64("FLEXAR_DMA_SERIAL", 0) != 0;
  int rc = each(0, 0, count, e0 + 1);
  uint64_t e = e0;
  for (uint64_t off = 0; off < count && !rc; off += piece) {
    const uint64_t n = std::min<uint64_t>(piece, count - off);
    ++e;
    if (serial && off) rc = each(4, 0, count, e - 1) || each(0, 0, count, e);
    for (int phase = 1; phase <= 3 && !rc; ++phase) rc = each(phase, off, n, e);
  }
  if (!rc) rc = each(4, 0, count, e);
  return rc;
}

// Settings fingerprint exchanged in the handle (readiness.hpp): environment knobs + workspace size +
// the loaded tune table.
static uint64_t comm_fingerprint(flexar_comm* c) {
  std::string extra = "ws=" + std::to_string(c->ws_bytes) + ";";
  for (auto& n : c->tune.rows)
    for (auto& row : n.second) extra += std::to_string(n.first) + " " + std::to_string(row.first) + " " + row.second + ";";
  return env_fingerprint(extra);
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
static int resident_blocks(int device) {
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

static int check_err(flexar_comm* c) {
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

static int validate_call(flexar_comm* c, int dtype, int op, float scale) {
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

static int alloc_workspace(flexar_comm* c, size_t ws) {
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
  FX_HIP(hipDeviceSynchronize());
  return 0;
}

static void init_defaults(flexar_comm* c) {
  c->model = XgmiModel::from_env();
  if (const char* m = getenv("FLEXAR_MODEL")) c->links_from_env = std::count(m, m + strlen(m), ',') >= 4;
  c->have_tune = c->tune.load(getenv("FLEXAR_TUNE_FILE"));
  c->timeout_ticks = env_u64("FLEXAR_TIMEOUT_MS", 20000) * 100000ull;  // 100 MHz s_memrealtime
  c->zc_auto = env_u64("FLEXAR_ZC_AUTO", 1) != 0;
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

// =========================================================================== C API
extern "C" {

int flexar_comm_create(int rank, int nranks, int device, size_t workspace_bytes, flexar_comm_t* out) {
  if (!out || nranks < 1 || nranks > (int)kMaxRanks || rank < 0 || rank >= nranks) {
    set_error("invalid rank/nranks (nranks must be 1..16)");
    return FLEXAR_ERR_INVALID;
  }
  std::unique_ptr<flexar_comm> c(new flexar_comm);
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  init_defaults(c.get());
  size_t ws = workspace_bytes ? workspace_bytes : env_u64("FLEXAR_WORKSPACE_BYTES", 512ull << 20);
  int rc = alloc_workspace(c.get(), ws);
  if (rc) return rc;
  c->resident = resident_blocks(device);
  c->peer_stg[rank] = c->stg;
  c->peer_flags[rank] = c->flags;
  if (nranks == 1) c->connected = true;
  *out = c.release();
  return 0;
}

size_t flexar_handle_size(void) { return sizeof(CommHandle); }

int flexar_comm_export(flexar_comm_t c, void* handle_out) {
  if (!c || !handle_out) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  FX_HIP(hipSetDevice(c->device));
  CommHandle h;
  memset(&h, 0, sizeof(h));
  h.magic = kHandleMagic;
  h.version = FLEXAR_VERSION_MAJOR * 100 + FLEXAR_VERSION_MINOR;
  h.rank = c->rank;
  h.nranks = c->nranks;
  h.ws_bytes = c->ws_bytes;
  FX_HIP(hipIpcGetMemHandle(&h.stg, c->stg));
  FX_HIP(hipIpcGetMemHandle(&h.flags, c->flags));
  h.pid = (int32_t)getpid();
  h.device = c->device;
  gethostname(h.host, sizeof(h.host) - 1);
  if (hipDeviceGetPCIBusId(h.bus, sizeof(h.bus) - 1, c->device) != hipSuccess) {
    (void)hipGetLastError();
    snprintf(h.bus, sizeof(h.bus), "dev%d", c->device);
  }
  h.fingerprint = comm_fingerprint(c);
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
  }
  if (!c->links_from_env) c->model.links = direct_links(c->link_cls, c->link_hops, c->nranks, c->rank);
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
int flexar_comm_selftest(flexar_comm_t c, uint32_t families, uint32_t* failed_out) {
  if (!c || !failed_out) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (!c->connected) { set_error("communicator not connected"); return FLEXAR_ERR_STATE; }
  *failed_out = 0;
  if (c->nranks == 1) return 0;
  FX_HIP(hipSetDevice(c->device));
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
  int* in = c->st_buf;
  int* out = c->st_buf + n;
  const int N = c->nranks;
  int rc = 0;
  for (const Case& k : cases) {
    if (!(families & k.fam)) continue;
    if (k.fam == PF_LL && !ll_usable(c, n, 4)) continue;
    c->selftested |= k.fam;
    logf(LOG_INFO, c->rank, "self-test: %s", k.spec);
    for (int call = 0; call < 3 && !rc; ++call) {
      const uint32_t salt = (uint32_t)(call * 131 + k.fam * 17);
      hipLaunchKernelGGL(selftest_fill, dim3(64), dim3(256), 0, st, in, out, n, c->rank, salt);
      if ((rc = hipGetLastError() != hipSuccess ? FLEXAR_ERR_HIP : 0)) break;
      int e = flexar_allreduce_ex(c, in, out, n, FLEXAR_INT32, FLEXAR_SUM, st, k.spec, 1.0f);
      if (e == FLEXAR_ERR_TIMEOUT || e == FLEXAR_ERR_STATE) {
        *failed_out |= k.fam;  // a previous call of this family timed out
      } else if (e) {
        rc = e;
        break;
      }
      *c->st_bad = 0;
      hipLaunchKernelGGL(selftest_check, dim3(64), dim3(256), 0, st, out, n, N, salt, c->st_bad_dev);
      if (hipStreamSynchronize(st) != hipSuccess) { rc = FLEXAR_ERR_HIP; break; }
      if (__atomic_load_n(c->st_bad, __ATOMIC_ACQUIRE) != 0) *failed_out |= k.fam;
      if (__atomic_load_n(c->err_host, __ATOMIC_ACQUIRE) != 0) {
        *failed_out |= k.fam;
        __atomic_store_n(c->err_host, 0u, __ATOMIC_RELEASE);  // every rank still makes every call
      }
    }
    if (rc) break;
  }
  (void)hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  c->have_last = false;  // `st` is gone (and synchronised): the next call must not order behind it
  c->timeout_ticks = saved_timeout;
  c->disabled = saved_disabled;
  c->profile = saved_profile;
  c->calls = saved_calls;
  c->bytes = saved_bytes;
  c->memo_gen = saved_gen + 1;
  if (rc == FLEXAR_ERR_HIP && std::string(flexar_last_error()).empty()) set_error("self-test: HIP error");
  logf(*failed_out ? LOG_WARN : LOG_INFO, c->rank, "self-test: ran %s, failed on this rank: %s",
       family_names(c->selftested).c_str(), family_names(*failed_out).c_str());
  return rc;
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

// ---- registered buffers (zero-copy "+zc") --------------------------------------------------------
// Registration blob: the IPC handle of the allocation holding the buffer and the buffer's place in it.
struct RegBlob {
  hipIpcMemHandle_t h;
  uint64_t offset;  // buffer start - allocation base
  uint64_t bytes;
  int32_t device, pad;
};
static_assert(sizeof(RegBlob) <= FLEXAR_REG_HANDLE_BYTES, "registration blob size");

size_t flexar_reg_handle_size(void) { return FLEXAR_REG_HANDLE_BYTES; }

static uint64_t buffer_id(const void* p) {
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (uint64_t)id;
}

// Drop registration i: its peer mappings close once no other registration uses them (caller holds mu
// and has synchronised the device).
static void reg_drop(flexar_comm* c, size_t i) {
  for (int p = 0; p < c->nranks; ++p) {
    if (p == c->rank) continue;
    auto it = c->ipc_maps.find(c->regs[i].key[p]);
    if (it == c->ipc_maps.end()) continue;
    if (--it->second.second == 0) {
      (void)hipIpcCloseMemHandle(it->second.first);
      c->ipc_maps.erase(it);
    }
  }
  c->regs.erase(c->regs.begin() + (long)i);
  (void)hipGetLastError();  // an ignored close failure must not surface in the caller's next launch
}

int flexar_reg_export(flexar_comm_t c, const void* ptr, size_t bytes, void* out) {
  if (!c || !ptr || !out || !bytes) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  FX_HIP(hipSetDevice(c->device));
  RegBlob b;
  memset(&b, 0, sizeof(b));
  if (c->nranks > 1 && !c->group_member) {
    void* base = nullptr;
    size_t size = 0;
    FX_HIP(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)));
    if ((const char*)ptr + bytes > (const char*)base + size) {
      set_error("registered range exceeds its allocation");
      return FLEXAR_ERR_INVALID;
    }
    // Importing a peer allocation larger than ~1 GiB through HIP IPC after other imports hangs in
    // hipIpcOpenMemHandle on this platform (ROCm 7, dmabuf IPC; reproduced with hipMalloc'd and torch
    // allocations of 2 GiB+, bench/reg_repro.py), so such allocations are refused up front instead
    // (every rank then keeps the staging schedules). FLEXAR_REG_MAX_ALLOC overrides the cap.
    const uint64_t cap = env_u64("FLEXAR_REG_MAX_ALLOC", 1ull << 30);
    if (size > cap) {
      set_error("registering: the buffer lies in an allocation of " + std::to_string(size) + " bytes, above the " +
                std::to_string(cap) + "-byte cap for IPC-mapped registrations (allocate it on its own)");
      return FLEXAR_ERR_UNSUPPORTED;
    }
    FX_HIP(hipIpcGetMemHandle(&b.h, base));
    b.offset = (uint64_t)((const char*)ptr - (const char*)base);
    logf(LOG_DEBUG, c->rank, "registering: buffer %p (%zu bytes) lies in allocation %p (%zu bytes) at +%llu", ptr,
         bytes, base, size, (unsigned long long)b.offset);
  }
  b.bytes = bytes;
  b.device = c->device;
  memset(out, 0, FLEXAR_REG_HANDLE_BYTES);
  memcpy(out, &b, sizeof(b));
  return 0;
}

// Collective in effect: every rank opens the blobs of all ranks (rank-major, flexar_reg_handle_size()
// bytes each) for its own buffer of the same size.
int flexar_reg_open(flexar_comm_t c, const void* ptr, size_t bytes, const void* all, int* id_out) {
  if (!c || !ptr || !all || !id_out) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (!c->connected && c->nranks > 1) { set_error("communicator not connected"); return FLEXAR_ERR_STATE; }
  if (c->nranks > 1 && !c->ipc) { set_error("zero-copy needs IPC peer access (this communicator runs RCCL messages)"); return FLEXAR_ERR_UNSUPPORTED; }
  if (c->group_member) {
    set_error("in-process groups address every rank's buffers directly: no registration needed");
    return FLEXAR_ERR_INVALID;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  FX_HIP(hipSetDevice(c->device));
  // a new registration replaces an overlapping old one whose allocation is gone (freed, address reused:
  // stale peer mappings) or which it contains (a call outgrew it); every rank registers together, so
  // every rank drops it. Other overlaps (a tensor inside a registered arena) coexist.
  logf(LOG_DEBUG, c->rank, "registering %zu bytes at %p (%zu registrations)", bytes, ptr, c->regs.size());
  bool synced = false;
  for (size_t i = c->regs.size(); i-- > 0;) {
    const flexar_comm::Reg& o = c->regs[i];
    const bool overlap = (const char*)ptr < o.base + o.bytes && o.base < (const char*)ptr + bytes;
    const bool contains = (const char*)ptr <= o.base && o.base + o.bytes <= (const char*)ptr + bytes;
    const bool stale = o.bufid && buffer_id(o.base) != o.bufid;
    if (overlap && (contains || stale)) {
      if (!synced) FX_HIP(hipDeviceSynchronize());
      synced = true;
      reg_drop(c, i);
    }
  }
  flexar_comm::Reg g;
  g.id = c->next_reg++;
  g.bufid = c->nranks > 1 && !c->group_member ? buffer_id(ptr) : 0;
  g.base = (char*)ptr;
  g.bytes = bytes;
  g.aligned = ((uintptr_t)ptr & 15) == 0;
  for (int p = 0; p < kMaxRanks; ++p) g.peer[p] = nullptr;
  std::vector<std::string> opened;
  auto undo = [&]() {
    for (const std::string& k : opened) {
      auto it = c->ipc_maps.find(k);
      if (it != c->ipc_maps.end() && --it->second.second == 0) {
        (void)hipIpcCloseMemHandle(it->second.first);
        c->ipc_maps.erase(it);
      }
    }
    (void)hipGetLastError();  // the failed open (and any close) must not stay the thread's sticky error
  };
  for (int p = 0; p < c->nranks; ++p) {
    RegBlob b;
    memcpy(&b, (const char*)all + (size_t)p * FLEXAR_REG_HANDLE_BYTES, sizeof(b));
    if (b.bytes != bytes) {
      undo();
      set_error("rank " + std::to_string(p) + " registered " + std::to_string(b.bytes) + " bytes, this rank " +
                std::to_string(bytes) + " (corresponding buffers must have the same size)");
      return FLEXAR_ERR_INVALID;
    }
    if (p == c->rank) { g.peer[p] = (char*)ptr; continue; }
    if (b.offset & 15) g.aligned = false;
    const std::string key = std::to_string(p) + ":" + std::string((const char*)&b.h, sizeof(b.h));
    auto it = c->ipc_maps.find(key);
    char* mapped = nullptr;
    if (it != c->ipc_maps.end()) {
      mapped = it->second.first;
      it->second.second++;
    } else {
      void* q = nullptr;
      logf(LOG_DEBUG, c->rank, "registering: opening rank %d's allocation (buffer at +%llu, %zu bytes)", p,
           (unsigned long long)b.offset, bytes);
      hipError_t e = hipIpcOpenMemHandle(&q, b.h, hipIpcMemLazyEnablePeerAccess);
      logf(LOG_DEBUG, c->rank, "registering: rank %d's allocation mapped (%s)", p, hipGetErrorString(e));
      if (e != hipSuccess) {
        undo();
        set_error("registering: mapping rank " + std::to_string(p) + "'s buffer failed: hipIpcOpenMemHandle: " +
                  hipGetErrorString(e));
        return FLEXAR_ERR_HIP;
      }
      mapped = (char*)q;
      c->ipc_maps[key] = {mapped, 1};
    }
    opened.push_back(key);
    g.key[p] = key;
    g.peer[p] = mapped + b.offset;
  }
  c->regs.push_back(g);
  *id_out = g.id;
  logf(LOG_INFO, c->rank, "registered buffer %d: %zu bytes (%zu registrations, %zu peer mappings)", g.id, bytes,
       c->regs.size(), c->ipc_maps.size());
  return 0;
}

// Drop a registration (every rank, after the calls using it completed): its peer mappings are closed
// once no other registration uses them.
int flexar_reg_close(flexar_comm_t c, int id) {
  if (!c) return FLEXAR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  for (size_t i = 0; i < c->regs.size(); ++i) {
    if (c->regs[i].id != id) continue;
    FX_HIP(hipSetDevice(c->device));
    FX_HIP(hipDeviceSynchronize());  // no call of ours still reads through the mappings
    reg_drop(c, i);
    return 0;
  }
  set_error("no registration " + std::to_string(id));
  return FLEXAR_ERR_INVALID;
}

// The registration holding [p, p + bytes): its id, 0 if none, -1 if the allocation behind the registered
// address is not the one registered any more (freed and reused: the peers' mappings are stale).
int flexar_reg_find(flexar_comm_t c, const void* p, size_t bytes) {
  if (!c || !p) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  for (const auto& r : c->regs)
    if ((const char*)p >= r.base && (const char*)p + bytes <= r.base + r.bytes) {
      if (r.bufid && buffer_id(p) != r.bufid) return -1;
      return r.id;
    }
  return 0;
}

int flexar_reg_count(flexar_comm_t c) { return c ? (int)c->regs.size() : -1; }

int flexar_reg_ids(flexar_comm_t c, int* out, int max) {
  if (!c) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  int n = 0;
  for (const auto& r : c->regs)
    if (n < max && out) out[n++] = r.id;
  return (int)c->regs.size();
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
                  ", \"links\": " + std::to_string(c->model.links) + ", \"resident_blocks\": " +
                  std::to_string(c->resident) + ", \"selftested\": \"" + family_names(c->selftested) +
                  "\", \"disabled\": \"" + (c->disabled ? family_names(c->disabled) : std::string()) +
                  "\", \"ipc\": " + (c->ipc ? "true" : "false") + ", \"rccl\": " + (c->nccl ? "true" : "false") +
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

int flexar_comm_destroy(flexar_comm_t c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
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
  if (c->nccl && rccl().ok) (void)rccl().CommDestroy(c->nccl);
  if (c->st_buf) (void)hipFree(c->st_buf);
  if (c->st_bad) (void)hipHostFree(c->st_bad);
  (void)hipFree(c->stg);
  (void)hipFree(c->flags);
  (void)hipFree(c->epochs);
  (void)hipHostFree(c->err_host);
  delete c;
  // teardown ignores failures (e.g. closing a mapping a peer already released), but HIP keeps the last one
  // as the thread's sticky error, and the caller's framework would report it at its next kernel launch
  (void)hipGetLastError();
  return 0;
}

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

int flexar_comm_check(flexar_comm_t c) {
  if (!c) return FLEXAR_ERR_INVALID;
  return check_err(c);
}

int flexar_comm_describe(flexar_comm_t c, size_t count, int dtype, char* buf, size_t buflen) {
  if (!c || !buf) return FLEXAR_ERR_INVALID;
  size_t es = dtype_size(dtype);
  if (!es) { set_error("bad dtype"); return FLEXAR_ERR_INVALID; }
  AlgoSpec s;
  int rc = resolve_spec(c, nullptr, (double)count * es, &s);
  if (rc) return rc;
  if ((rc = typed_spec(&s, dtype, FLEXAR_SUM, false))) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  uint64_t piece = count;
  if (c->nranks > 1 && count) {
    rc = plan_pieces(c, s, count, (uint32_t)es, 1.0f, &piece);
    if (rc) return rc;
  }
  DevProgram* dp = nullptr;
  rc = get_program(c, s, piece ? piece : 1, (uint32_t)es, 1.0f, &dp);
  if (rc) return rc;
  int grid = choose_grid(c, (uint64_t)piece * es, dp->prog.nchan);
  snprintf(buf, buflen, "%s grid=%d pieces=%llu stg_bytes=%llu ops=%zu",
           c->nranks == 1 ? "copy (1 rank)" : s.str().c_str(), grid,
           (unsigned long long)(piece ? (count + piece - 1) / piece : 0),
           (unsigned long long)dp->prog.stg_bytes(), dp->prog.ops.size());
  return 0;
}

int flexar_allreduce_ex(flexar_comm_t c, const void* in, void* out, size_t count, int dtype, int op,
                        void* stream, const char* algo, float scale) {
  int rc = validate_call(c, dtype, op, scale);
  if (rc) return rc;
  if (count == 0) return 0;
  if (!out) { set_error("null recvbuf"); return FLEXAR_ERR_INVALID; }
  if ((rc = check_err(c))) return rc;
  if (!in) in = out;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t es = (uint32_t)dtype_size(dtype);
  float fs = scale * (op == FLEXAR_AVG ? 1.0f / (float)c->nranks : 1.0f);
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = order_call(c, st))) return rc;
  uint32_t fsb;
  memcpy(&fsb, &fs, 4);
  const char* akey = algo ? algo : "";
  flexar_comm::CallMemo& m = c->memo[((uint64_t)count * 0x9E3779B97F4A7C15ull + (uint64_t)dtype * 31u + (uint64_t)op) >> 60];
  bool hit = m.gen == c->memo_gen && m.count == count && m.dtype == dtype && m.op == op && m.fsb == fsb &&
             m.algo == akey;
  AlgoSpec s;
  if (hit) {
    s = m.s;
  } else {
    if ((rc = resolve_spec(c, algo, (double)count * es, &s))) return rc;
    if ((rc = typed_spec(&s, dtype, op, false))) return rc;
    if (s.kind == AlgoKind::LL && !ll_usable(c, count, es)) s.kind = AlgoKind::ONESHOT;
    if (s.kind == AlgoKind::DMA && c->nranks == 1) s.kind = AlgoKind::ONESHOT;  // one rank: the executor's copy
    if ((rc = executor_proto(c, &s))) return rc;  // the LL -> oneshot rewrite above may land on a failed family
  }
  if (s.kind == AlgoKind::DMA && c->captured) {  // not replay-safe (see flexar_comm::captured)
    AlgoSpec f;
    std::string err;
    if (!parse_algo("flat+pull", c->nranks, &f, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    s = f;
    if ((rc = executor_proto(c, &s))) return rc;
  }
  if (s.msg) s.wire = 0;  // the message transport runs the schedule untyped
  // Registered buffers (flexar_reg_*): zero copy or staging for this call (zc_policy.hpp)
  if (!c->regs.empty() || s.zc) {
    ZcFacts f;
    f.nranks = c->nranks;
    f.bytes = (double)count * es;
    f.named = algo && *algo && strcmp(algo, "auto") != 0;
    f.from_auto = !f.named && c->spec.kind == AlgoKind::AUTO;
    f.zc_auto = c->zc_auto;
    f.have_tune = c->have_tune;
    f.disabled = c->disabled;
    f.registered = !s.msg && s.wire == 0 && zc_registered(c, in, out, (uint64_t)count * es);
    const int d = zc_decide(&s, f, c->model);
    if (d > 0) hit = hit && m.s.zc;
    if (d < 0) hit = hit && !m.s.zc;
  }
  auto remember = [&](uint64_t piece, DevProgram* dp, int grid) {
    if (hit) return;
    m.gen = c->memo_gen;
    m.count = count;
    m.dtype = dtype;
    m.op = op;
    m.fsb = fsb;
    m.algo = akey;
    m.s = s;
    m.piece = piece;
    m.dp = dp;
    m.grid = grid;
  };
  if (s.msg) {
    remember(0, nullptr, 0);
    if (roctx().push) roctx().push(("flexar allreduce " + s.str() + " " + std::to_string(count * es) + "B").c_str());
    c->calls++;
    c->bytes += count * es;
    rc = run_msg(c, s, Coll::ALLREDUCE, in, out, count, dtype, op, fs, 0, st);
    if (roctx().pop) roctx().pop();
    return rc;
  }
  if (s.kind == AlgoKind::DMA) {
    remember(0, nullptr, 0);
    if (roctx().push) roctx().push(("flexar allreduce dma " + std::to_string(count * es) + "B").c_str());
    c->calls++;
    c->bytes += count * es;
    const char* ip = (const char*)in;
    char* op_ = (char*)out;
    rc = run_dma(&c, 1, &ip, &op_, count, dtype, op, fs, st);
    if (roctx().pop) roctx().pop();
    return rc;
  }
  if (s.kind == AlgoKind::LL) {
    LaunchArgs la;
    la.kind = LAUNCH_LL;
    fill_ctx(c, nullptr, in, out, &la.ctx);
    la.ctx.count = count;
    la.ctx.scale = fs;
    la.grid = hit ? m.grid : ll_grid(c, count, es);
    la.stream = st;
    if (roctx().push) roctx().push(("flexar allreduce ll " + std::to_string(count * es) + "B").c_str());
    c->calls++;
    c->bytes += count * es;
    rc = launch_dtype(dtype, op, la);
    if (!rc) {
      c->launches++;
      remember(0, nullptr, la.grid);
    }
    if (roctx().pop) roctx().pop();
    return rc;
  }
  uint64_t piece = count;
  if (hit) piece = m.piece;
  else if (c->nranks > 1 && (rc = plan_pieces(c, s, count, es, fs, &piece))) return rc;
  const bool described = roctx().push || c->profile;
  const std::string sdesc = described ? s.str() : std::string();
  if (roctx().push) roctx().push(("flexar allreduce " + sdesc + " " + std::to_string(count * es) + "B").c_str());
  if (piece >= count) {  // one launch: the memoised program and grid
    DevProgram* dp = hit ? m.dp : nullptr;
    if (!dp && (rc = get_program(c, s, count, es, fs, &dp))) return rc;
    LaunchArgs la;
    la.kind = LAUNCH_EXEC;
    fill_ctx(c, dp, in, out, &la.ctx);
    if (dp->prog.zc && (rc = zc_bind(c, dp->prog, in, (uint64_t)count * es, out, (uint64_t)count * es, &la.ctx)))
      return rc;
    la.grid = hit ? m.grid : choose_grid(c, count * es, dp->prog.nchan);
    la.stream = st;
    la.proto = proto_of(s);
    la.wire = dp->prog.wire;
    std::unique_ptr<DeviceTimer> tm(c->profile ? new DeviceTimer : nullptr);
    if (tm) tm->start(st);
    c->calls++;
    c->bytes += count * es;
    rc = launch_dtype(dtype, op, la);
    if (!rc) {
      c->launches++;
      remember(piece, dp, la.grid);
    }
    if (tm) {
      tm->stop(st);
      c->prof_pending.push_back(ProfRec{sdesc, (uint64_t)count * es, std::move(tm)});
    }
    if (roctx().pop) roctx().pop();
    return rc;
  }
  remember(piece, nullptr, 0);
  std::unique_ptr<DeviceTimer> tm(c->profile ? new DeviceTimer : nullptr);
  if (tm) tm->start(st);
  c->calls++;
  c->bytes += count * es;
  for (uint64_t off = 0; off < count; off += piece) {
    uint64_t n = std::min<uint64_t>(piece, count - off);
    DevProgram* dp = nullptr;
    if ((rc = get_program(c, s, n, es, fs, &dp))) return rc;
    DevCtx x;
    fill_ctx(c, dp, (const char*)in + off * es, (char*)out + off * es, &x);
    if (dp->prog.zc &&
        (rc = zc_bind(c, dp->prog, (const char*)in + off * es, n * es, (char*)out + off * es, n * es, &x)))
      break;
    int grid = choose_grid(c, n * es, dp->prog.nchan);
    LaunchArgs la;
    la.kind = LAUNCH_EXEC;
    la.ctx = x;
    la.grid = grid;
    la.stream = st;
    la.proto = proto_of(s);
    la.wire = dp->prog.wire;
    rc = launch_dtype(dtype, op, la);
    if (rc) break;
    c->launches++;
  }
  if (tm) {
    tm->stop(st);
    c->prof_pending.push_back(ProfRec{sdesc, (uint64_t)count * es, std::move(tm)});
  }
  if (roctx().pop) roctx().pop();
  return rc;
}

// JSON statistics: calls/bytes overall and (FLEXAR_PROFILE=1) device time per algorithm.
int flexar_comm_stats(flexar_comm_t c, char* buf, size_t buflen) {
  if (!c || !buf) return FLEXAR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  for (auto& p : c->prof_pending) {
    const double ms = p.t->ms();
    if (ms >= 0) {
      auto& a = c->prof[p.algo];
      a.calls++;
      a.bytes += p.bytes;
      a.ms += ms;
    }
  }
  c->prof_pending.clear();
  std::string j = "{\"calls\": " + std::to_string(c->calls) + ", \"bytes\": " + std::to_string(c->bytes) +
                  ", \"plans_cached\": " + std::to_string(c->cache.size()) + ", \"links\": " +
                  std::to_string(c->model.links) + ", \"resident_blocks\": " + std::to_string(c->resident) +
                  ", \"selftested\": \"" + family_names(c->selftested) + "\", \"disabled\": \"" +
                  (c->disabled ? family_names(c->disabled) : std::string()) + "\", \"profile\": {";
  bool first = true;
  for (auto& kv : c->prof) {
    char t[256];
    snprintf(t, sizeof(t), "%s\"%s\": {\"calls\": %llu, \"bytes\": %llu, \"ms\": %.4f}", first ? "" : ", ",
             kv.first.c_str(), (unsigned long long)kv.second.calls, (unsigned long long)kv.second.bytes, kv.second.ms);
    j += t;
    first = false;
  }
  j += "}}";
  snprintf(buf, buflen, "%s", j.c_str());
  return j.size() < buflen ? 0 : FLEXAR_ERR_NOMEM;
}

int flexar_allreduce(flexar_comm_t c, const void* in, void* out, size_t count, int dtype, int op, void* stream) {
  return flexar_allreduce_ex(c, in, out, count, dtype, op, stream, nullptr, 1.0f);
}

// Compressed allreduce (BASELINE config #5): fp32 / bf16 / fp16 in and out, OCP fp8 on the links. The
// pre-scale s = fp8_max / (N * global amax) is derived inside the executor from every rank's amax
// partials (flexar_amax, one HBM pass) and fused into the first transfer; the post-scale 1/s (and AVG's
// 1/N) into the last: two launches per bucket (amax + this), no separate quantize / dequantize pass.
int flexar_allreduce_fp8(flexar_comm_t c, const void* in, void* out, size_t count, int dtype, int op, void* stream,
                         int wire_dtype, const float* amax_parts, const char* algo) {
  int rc = validate_call(c, dtype, op, 1.0f);
  if (rc) return rc;
  if (count == 0) return 0;
  if (!out || !amax_parts) { set_error("null recvbuf / amax partials"); return FLEXAR_ERR_INVALID; }
  if (dtype != FLEXAR_FLOAT32 && dtype != FLEXAR_BFLOAT16 && dtype != FLEXAR_FLOAT16) {
    set_error("fp8 wire compression takes fp32 / bf16 / fp16 buffers");
    return FLEXAR_ERR_UNSUPPORTED;
  }
  if ((op != FLEXAR_SUM && op != FLEXAR_AVG) || (wire_dtype != FLEXAR_FP8_E4M3 && wire_dtype != FLEXAR_FP8_E5M2)) {
    set_error("fp8 wire compression: SUM/AVG over e4m3 or e5m2");
    return FLEXAR_ERR_UNSUPPORTED;
  }
  if ((rc = check_err(c))) return rc;
  if (!in) in = out;
  if (c->nranks == 1) return flexar_allreduce_ex(c, in, out, count, dtype, op, stream, nullptr, 1.0f);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t es = (uint32_t)dtype_size(dtype);
  const float fs = op == FLEXAR_AVG ? 1.0f / (float)c->nranks : 1.0f;
  AlgoSpec s;
  std::string err;
  if (!parse_algo(algo && *algo ? algo : "flat+pull", c->nranks, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  const bool wt = s.wt;
  s = AlgoSpec();
  s.kind = AlgoKind::TREE;
  s.widths = {c->nranks};
  s.ag = AgMode::PULL;
  s.wt = wt;
  s.wire = wire_dtype == FLEXAR_FP8_E4M3 ? 2 : 3;
  if ((rc = executor_proto(c, &s))) return rc;
  if (s.msg) {
    set_error("fp8 wire compression runs on the IPC executor (the message transport has no typed staging)");
    return FLEXAR_ERR_UNSUPPORTED;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  if ((rc = order_call(c, st))) return rc;
  uint64_t piece = count;
  if ((rc = plan_pieces(c, s, count, es, fs, &piece))) return rc;
  c->calls++;
  c->bytes += count * es;
  for (uint64_t off = 0; off < count; off += piece) {
    const uint64_t n = std::min<uint64_t>(piece, count - off);
    DevProgram* dp = nullptr;
    if ((rc = get_program(c, s, n, es, fs, &dp))) return rc;
    LaunchArgs la;
    la.kind = LAUNCH_EXEC;
    fill_ctx(c, dp, (const char*)in + off * es, (char*)out + off * es, &la.ctx);
    la.ctx.amax_parts = amax_parts;
    la.grid = choose_grid(c, n * es, dp->prog.nchan);
    la.stream = st;
    la.proto = proto_of(s);
    la.wire = dp->prog.wire;
    if ((rc = launch_dtype(dtype, op, la))) return rc;
    c->launches++;
  }
  return 0;
}

int flexar_reduce_scatter(flexar_comm_t c, const void* in, void* out, size_t count, int dtype, int op, void* stream,
                          const char* algo) {
  int rc = validate_call(c, dtype, op, 1.0f);
  if (rc) return rc;
  if (!in || !out) { set_error("reduce_scatter needs distinct send/recv buffers"); return FLEXAR_ERR_INVALID; }
  if ((rc = check_err(c))) return rc;
  if (count == 0) return 0;
  return run_rs_ag(c, Coll::REDUCE_SCATTER, in, out, count, dtype, op, (hipStream_t)stream, algo, 1.0f);
}

int flexar_all_gather(flexar_comm_t c, const void* in, void* out, size_t count, int dtype, void* stream,
                      const char* algo) {
  int rc = validate_call(c, dtype, FLEXAR_SUM, 1.0f);
  if (rc) return rc;
  if (!in || !out) { set_error("all_gather needs send/recv buffers"); return FLEXAR_ERR_INVALID; }
  if ((rc = check_err(c))) return rc;
  if (count == 0) return 0;
  return run_rs_ag(c, Coll::ALL_GATHER, in, out, count, dtype, FLEXAR_SUM, (hipStream_t)stream, algo, 1.0f);
}

int flexar_all_to_all_ex(flexar_comm_t c, const void* in, void* out, size_t count, int dtype, void* stream,
                         const char* algo) {
  int rc = validate_call(c, dtype, FLEXAR_SUM, 1.0f);
  if (rc) return rc;
  if (!in || !out || in == out) { set_error("all_to_all needs distinct send/recv buffers"); return FLEXAR_ERR_INVALID; }
  if ((rc = check_err(c))) return rc;
  if (count == 0) return 0;
  return run_rs_ag(c, Coll::ALL_TO_ALL, in, out, count, dtype, FLEXAR_SUM, (hipStream_t)stream, algo, 1.0f);
}

int flexar_all_to_all(flexar_comm_t c, const void* in, void* out, size_t count, int dtype, void* stream) {
  return flexar_all_to_all_ex(c, in, out, count, dtype, stream, nullptr);
}

int flexar_broadcast(flexar_comm_t c, const void* in, void* out, size_t count, int dtype, int root, void* stream,
                     const char* algo) {
  int rc = validate_call(c, dtype, FLEXAR_SUM, 1.0f);
  if (rc) return rc;
  if (!out) { set_error("broadcast needs a recv buffer"); return FLEXAR_ERR_INVALID; }
  if (root < 0 || root >= c->nranks) { set_error("broadcast root out of range"); return FLEXAR_ERR_INVALID; }
  if ((rc = check_err(c))) return rc;
  if (count == 0) return 0;
  if (!in) in = out;
  return run_bcast(c, in, out, count, dtype, root, (hipStream_t)stream, algo);
}

// ---- in-process group: N ranks on ONE device in one process (tests / calibration) -------------
int flexar_group_create(int nranks, int device, size_t workspace_bytes, flexar_comm_t* comms) {
  if (!comms || nranks < 1 || nranks > (int)kMaxRanks) { set_error("invalid nranks"); return FLEXAR_ERR_INVALID; }
  for (int r = 0; r < nranks; ++r) {
    int rc = flexar_comm_create(r, nranks, device, workspace_bytes, &comms[r]);
    if (rc) return rc;
    comms[r]->group_member = true;
    // every rank's workgroups share one launch and spin on each other: keep the whole grid
    // co-resident (exec_group_kernel: 1 workgroup of 512 threads per CU at its VGPR count)
    comms[r]->max_grid = std::max(1, (int)kGroupMaxBlocks / nranks);
  }
  for (int r = 0; r < nranks; ++r) {
    for (int p = 0; p < nranks; ++p) {
      comms[r]->peer_stg[p] = comms[p]->stg;
      comms[r]->peer_flags[p] = comms[p]->flags;
    }
    comms[r]->connected = true;
  }
  return 0;
}

// The in-process group paths (LocalGroup: tests, calibration) stage their per-rank contexts in one
// device buffer per host thread. A call on another stream must not overwrite it while the previous
// call's kernel still reads it: the copy waits on an event recorded after that kernel's launch.
struct GroupCtxStage {
  DevCtx* d = nullptr;
  hipEvent_t done = nullptr;
  bool used = false;
};
static thread_local GroupCtxStage g_group_ctx;

// In-process group running a zero-copy program: every rank's buffers are plain device pointers.
static void group_zc_bind(std::vector<DevCtx>& h, int nranks, const void* const* ins, void* const* outs,
                          uint64_t off_bytes) {
  for (int r = 0; r < nranks; ++r)
    for (int p = 0; p < nranks; ++p) {
      h[r].peer_io[BUF_IN][p] = (char*)(ins && ins[p] ? ins[p] : outs[p]) + off_bytes;
      h[r].peer_io[BUF_OUT][p] = (char*)outs[p] + off_bytes;
      if ((((uintptr_t)h[r].peer_io[BUF_IN][p]) | ((uintptr_t)h[r].peer_io[BUF_OUT][p])) & 15) h[r].vec_ok = 0;
    }
}

static int stage_group_ctx(const std::vector<DevCtx>& h, int nranks, hipStream_t st, DevCtx** out) {
  GroupCtxStage& g = g_group_ctx;
  if (!g.d) FX_HIP(hipMalloc(&g.d, sizeof(DevCtx) * kMaxRanks));
  if (!g.done) FX_HIP(hipEventCreateWithFlags(&g.done, hipEventDisableTiming));
  if (g.used) FX_HIP(hipStreamWaitEvent(st, g.done, 0));
  FX_HIP(hipMemcpyAsync(g.d, h.data(), sizeof(DevCtx) * nranks, hipMemcpyHostToDevice, st));
  *out = g.d;
  return 0;
}
static int group_ctx_launched(hipStream_t st) {
  FX_HIP(hipEventRecord(g_group_ctx.done, st));
  g_group_ctx.used = true;
  return 0;
}

// One launch runs every rank of the group: ins/outs are nranks device pointers.
static int group_allreduce(flexar_comm_t* comms, int nranks, const void* const* ins, void* const* outs, size_t count,
                           int dtype, int op, void* stream, const char* algo, float scale,
                           const float* const* amax_parts) {
  if (!comms || nranks < 1) return FLEXAR_ERR_INVALID;
  for (int r = 0; r < nranks; ++r) {
    int rc = validate_call(comms[r], dtype, op, scale);
    if (rc) return rc;
    if ((rc = check_err(comms[r]))) return rc;
  }
  if (count == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t es = (uint32_t)dtype_size(dtype);
  float fs = scale * (op == FLEXAR_AVG ? 1.0f / (float)nranks : 1.0f);
  std::vector<AlgoSpec> specs(nranks);
  for (int r = 0; r < nranks; ++r) {
    int rc = resolve_spec(comms[r], algo, (double)count * es, &specs[r]);
    if (rc) return rc;
    if ((rc = typed_spec(&specs[r], dtype, op, amax_parts != nullptr))) return rc;
  }
  DevCtx* d_ctx = nullptr;
  if (specs[0].kind == AlgoKind::LL && !ll_usable(comms[0], count, es))
    for (auto& sp : specs) sp.kind = AlgoKind::ONESHOT;
  if (specs[0].kind == AlgoKind::DMA && nranks > 1) {
    std::vector<const char*> ip(nranks);
    std::vector<char*> op_(nranks);
    for (int r = 0; r < nranks; ++r) {
      ip[r] = ins && ins[r] ? (const char*)ins[r] : (const char*)outs[r];
      op_[r] = (char*)outs[r];
    }
    int rc = run_dma(comms, nranks, ip.data(), op_.data(), count, dtype, op, fs, st);
    if (rc) return rc;
    FX_HIP(hipStreamSynchronize(st));
    return 0;
  }
  if (specs[0].kind == AlgoKind::DMA) specs[0].kind = AlgoKind::ONESHOT;
  if (specs[0].kind == AlgoKind::LL) {
    std::vector<DevCtx> h(nranks);
    for (int r = 0; r < nranks; ++r) {
      const void* in = ins && ins[r] ? ins[r] : outs[r];
      fill_ctx(comms[r], nullptr, in, outs[r], &h[r]);
      h[r].count = count;
      h[r].scale = fs;
    }
    int grid = std::max(1, std::min(ll_grid(comms[0], count, es), (int)kGroupMaxBlocks / nranks));
    if (int e = stage_group_ctx(h, nranks, st, &d_ctx)) return e;
    LaunchArgs la;
    la.kind = LAUNCH_LL_GROUP;
    la.d_ctxs = d_ctx;
    la.nranks = nranks;
    la.grid = grid;
    la.stream = st;
    int rc = launch_dtype(dtype, op, la);
    if (!rc) (void)group_ctx_launched(st);
    if (rc) return rc;
    for (int r = 0; r < nranks; ++r) comms[r]->launches++;
    FX_HIP(hipStreamSynchronize(st));
    return 0;
  }
  uint64_t piece = count;
  if (nranks > 1) {
    int rc = plan_pieces(comms[0], specs[0], count, es, fs, &piece);
    if (rc) return rc;
  }
  for (uint64_t off = 0; off < count; off += piece) {
    uint64_t n = std::min<uint64_t>(piece, count - off);
    std::vector<DevCtx> h(nranks);
    int grid = 0, wire = 0;
    bool zc = false;
    for (int r = 0; r < nranks; ++r) {
      DevProgram* dp = nullptr;
      int rc = get_program(comms[r], specs[r], n, es, fs, &dp);
      if (rc) return rc;
      const char* in = ins && ins[r] ? (const char*)ins[r] : (const char*)outs[r];
      fill_ctx(comms[r], dp, in + off * es, (char*)outs[r] + off * es, &h[r]);
      zc = zc || dp->prog.zc;
      if (amax_parts) h[r].amax_parts = amax_parts[r];
      wire = dp->prog.wire;
      int g = choose_grid(comms[r], n * es, dp->prog.nchan);
      grid = r == 0 ? g : grid;
      if (g != grid) { set_error("group ranks disagree on grid"); return FLEXAR_ERR_STATE; }
    }
    if ((uint64_t)grid * nranks > kGroupMaxBlocks) {
      set_error("group grid too large: ranks x grid must stay <= 256 co-resident workgroups");
      return FLEXAR_ERR_INVALID;
    }
    if (zc) group_zc_bind(h, nranks, ins, outs, off * es);
    if (int e = stage_group_ctx(h, nranks, st, &d_ctx)) return e;
    LaunchArgs la;
    la.kind = LAUNCH_GROUP;
    la.d_ctxs = d_ctx;
    la.nranks = nranks;
    la.grid = grid;
    la.stream = st;
    la.proto = proto_of(specs[0]);
    la.wire = wire;
    int rc = launch_dtype(dtype, op, la);
    if (!rc) (void)group_ctx_launched(st);
    if (rc) return rc;
    for (int r = 0; r < nranks; ++r) comms[r]->launches++;
    FX_HIP(hipStreamSynchronize(st));  // d_ctx is reused by the next piece
  }
  return 0;
}

int flexar_group_allreduce(flexar_comm_t* comms, int nranks, const void* const* ins, void* const* outs, size_t count,
                           int dtype, int op, void* stream, const char* algo, float scale) {
  return group_allreduce(comms, nranks, ins, outs, count, dtype, op, stream, algo, scale, nullptr);
}

// fp8-wire allreduce for an in-process group (tests): amax_parts = nranks device pointers of partials.
int flexar_group_allreduce_fp8(flexar_comm_t* comms, int nranks, const void* const* ins, void* const* outs,
                               size_t count, int dtype, int op, void* stream, int wire_dtype,
                               const float* const* amax_parts) {
  if (!amax_parts) { set_error("null amax partials"); return FLEXAR_ERR_INVALID; }
  if (wire_dtype != FLEXAR_FP8_E4M3 && wire_dtype != FLEXAR_FP8_E5M2) { set_error("wire dtype must be fp8"); return FLEXAR_ERR_INVALID; }
  return group_allreduce(comms, nranks, ins, outs, count, dtype, op, stream,
                         wire_dtype == FLEXAR_FP8_E4M3 ? "flat+pull+e4m3" : "flat+pull+e5m2", 1.0f, amax_parts);
}

// Reduce-scatter / all-gather for an in-process group (tests): one launch, every rank of the group.
int flexar_group_collective(flexar_comm_t* comms, int nranks, int coll, const void* const* ins, void* const* outs,
                            size_t count, int dtype, int op, void* stream, const char* algo) {
  if (!comms || nranks < 1 || (coll != 1 && coll != 2 && coll != 4)) return FLEXAR_ERR_INVALID;
  if (coll == 2 || coll == 4) op = FLEXAR_SUM;
  for (int r = 0; r < nranks; ++r) {
    int rc = validate_call(comms[r], dtype, op, 1.0f);
    if (rc) return rc;
  }
  if (count == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t es = (uint32_t)dtype_size(dtype);
  float fs = coll == 1 && op == FLEXAR_AVG ? 1.0f / (float)nranks : 1.0f;
  DevCtx* d_ctx = nullptr;
  std::vector<DevCtx> h(nranks);
  int grid = 0;
  int proto = PM_FENCE;
  bool zc = false;
  for (int r = 0; r < nranks; ++r) {
    AlgoSpec s;
    int rc = resolve_spec(comms[r], algo, (double)count * es * nranks, &s);
    if (rc) return rc;
    if (s.kind != AlgoKind::RING) s.kind = AlgoKind::TREE, s.widths = {nranks}, s.ag = AgMode::PUSH;
    proto = proto_of(s);
    DevProgram* dp = nullptr;
    if ((rc = get_program(comms[r], s, count, es, fs, &dp, (Coll)coll, count))) return rc;
    if (dp->prog.stg_bytes() > comms[r]->exec_half) { set_error("group collective exceeds workspace"); return FLEXAR_ERR_NOMEM; }
    fill_ctx(comms[r], dp, ins[r], outs[r], &h[r]);
    zc = zc || dp->prog.zc;
    int g = choose_grid(comms[r], count * es * nranks, dp->prog.nchan);
    grid = r == 0 ? g : grid;
  }
  if (zc) group_zc_bind(h, nranks, ins, outs, 0);
  if (int e = stage_group_ctx(h, nranks, st, &d_ctx)) return e;
  LaunchArgs la;
  la.kind = LAUNCH_GROUP;
  la.d_ctxs = d_ctx;
  la.nranks = nranks;
  la.grid = grid;
  la.stream = st;
  la.proto = proto;
  int rc = launch_dtype(dtype, op, la);
  if (!rc) (void)group_ctx_launched(st);
  if (rc) return rc;
  for (int r = 0; r < nranks; ++r) comms[r]->launches++;
  FX_HIP(hipStreamSynchronize(st));
  return 0;
}

// Broadcast for an in-process group (tests): one launch, every rank of the group.
int flexar_group_broadcast(flexar_comm_t* comms, int nranks, int root, const void* const* ins, void* const* outs,
                           size_t count, int dtype, void* stream, const char* algo) {
  if (!comms || nranks < 1 || root < 0 || root >= nranks) { set_error("bad group broadcast arguments"); return FLEXAR_ERR_INVALID; }
  for (int r = 0; r < nranks; ++r) {
    int rc = validate_call(comms[r], dtype, FLEXAR_SUM, 1.0f);
    if (rc) return rc;
  }
  if (count == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t es = (uint32_t)dtype_size(dtype);
  DevCtx* d_ctx = nullptr;
  std::vector<DevCtx> h(nranks);
  int grid = 0, proto = PM_FENCE;
  bool zc = false;
  for (int r = 0; r < nranks; ++r) {
    AlgoSpec s;
    int rc = bcast_spec(comms[r], algo, (uint64_t)count * es, &s);
    if (rc) return rc;
    proto = proto_of(s);
    DevProgram* dp = nullptr;
    if ((rc = get_program(comms[r], s, count, es, 1.0f, &dp, Coll::BROADCAST, (uint64_t)root))) return rc;
    if (dp->prog.stg_bytes() > comms[r]->exec_half) { set_error("group broadcast exceeds workspace"); return FLEXAR_ERR_NOMEM; }
    const void* in = ins && ins[r] ? ins[r] : outs[r];
    fill_ctx(comms[r], dp, in, outs[r], &h[r]);
    zc = zc || dp->prog.zc;
    int g = choose_grid(comms[r], count * es, dp->prog.nchan);
    grid = r == 0 ? g : grid;
  }
  if (zc) group_zc_bind(h, nranks, ins, outs, 0);
  if (int e = stage_group_ctx(h, nranks, st, &d_ctx)) return e;
  LaunchArgs la;
  la.kind = LAUNCH_GROUP;
  la.d_ctxs = d_ctx;
  la.nranks = nranks;
  la.grid = grid;
  la.stream = st;
  la.proto = proto;
  int rc = launch_dtype(dtype, FLEXAR_SUM, la);
  if (!rc) (void)group_ctx_launched(st);
  if (rc) return rc;
  for (int r = 0; r < nranks; ++r) comms[r]->launches++;
  FX_HIP(hipStreamSynchronize(st));
  return 0;
}

// ---- pointer / device helpers (used by the MPI compatibility layer) ---------------------------
int flexar_pointer_is_device(const void* p) {
  if (!p) return 0;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // host pointers unknown to HIP report an error: clear it
    return 0;
  }
  return a.type == hipMemoryTypeDevice ? 1 : 0;
}

int flexar_device_synchronize(void) {
  FX_HIP(hipDeviceSynchronize());
  return 0;
}

int flexar_copy_device_host(void* dst, const void* src, size_t bytes) {
  FX_HIP(hipDeviceSynchronize());  // the device buffer may still be written by queued work
  FX_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
  return 0;
}

void* flexar_device_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
  return p;
}
void flexar_device_free(void* p) { (void)hipFree(p); }

int flexar_kernel_info(int dtype, int op, int kind, int proto, int* blocks_per_cu, int* vgprs) {
  if (kind < 0 || kind > 5 || proto < 0 || proto > 2) { set_error("bad kernel_info arguments"); return FLEXAR_ERR_INVALID; }
  LaunchArgs la;
  la.kind = LAUNCH_QUERY;
  la.query = kind > 2 ? 0 : kind;
  la.wire = kind > 2 ? kind - 2 : 0;  // typed executors: 3 = fp32 partials, 4 = e4m3 wire, 5 = e5m2 wire
  la.proto = proto;
  la.occ_out = blocks_per_cu;
  la.regs_out = vgprs;
  return launch_dtype(dtype, op, la);
}

int flexar_current_device(void) {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 0;
  return d;
}

// ---- standalone reduction kernel --------------------------------------------------------------
int flexar_reduce(void* dst, const void* const* srcs, int nsrc, size_t count, int dtype, int op, float scale,
                  void* stream) {
  if (!dst || !srcs || nsrc < 1 || nsrc > 64) { set_error("bad reduce arguments"); return FLEXAR_ERR_INVALID; }
  if (!op_supported(dtype, op)) { set_error("unsupported dtype/op"); return FLEXAR_ERR_UNSUPPORTED; }
  if (count == 0) return 0;
  float fs = scale * (op == FLEXAR_AVG ? 1.0f / (float)nsrc : 1.0f);
  return reduce_chain((char*)dst, nullptr, (const char* const*)srcs, nsrc, count, dtype, op, fs, (hipStream_t)stream,
                      PM_FENCE);
}

}  // extern "C"
