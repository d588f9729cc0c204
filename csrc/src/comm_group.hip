// flexar in-process groups: N ranks on ONE device in one process, every rank in one launch (tests,
// calibration).
#include "comm_internal.hpp"

extern "C" {

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
      if (!vec_ok_for(((uintptr_t)h[r].peer_io[BUF_IN][p]) | ((uintptr_t)h[r].peer_io[BUF_OUT][p]))) h[r].vec_ok = 0;
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
    int rc = resolve_spec(comms[r], algo, (double)count * es, &specs[r], call_kind(dtype, op));
    if (rc) return rc;
    if ((rc = typed_spec(comms[r], &specs[r], dtype, op, amax_parts != nullptr, (double)count * es))) return rc;
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
    la.epoch = comms[0]->launches + 1;
    la.tag = "in-process group";
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
    int grid = 0, wire = 0, fanin = 0;
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
      fanin = std::max(fanin, (int)dp->prog.max_nsrc);
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
    la.epoch = comms[0]->launches + 1;
    la.tag = "in-process group";
    la.proto = proto_of(specs[0]);
    la.wire = wire;
    la.max_fanin = fanin;
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
  int grid = 0, wire = 0, fanin = 0;
  int proto = PM_FENCE;
  bool zc = false;
  for (int r = 0; r < nranks; ++r) {
    AlgoSpec s;
    int rc = resolve_spec(comms[r], algo, (double)count * es * nranks, &s, call_kind(dtype, op));
    if (rc) return rc;
    if (s.kind != AlgoKind::RING) s.kind = AlgoKind::TREE, s.widths = {nranks}, s.ag = AgMode::PUSH;
    if (s.wire && coll != 1 && !(algo && *algo)) s.wire = 0;  // a default-spec wire: reduce-scatter only
    if (s.wire) {  // the OCP MX wire on the flat reduce-scatter only (as run_rs_ag)
      if (coll != 1 || s.wire < 4) {
        set_error("typed staging on collectives: only the OCP MX wire (+mxe4m3 / +mxe5m2) on the reduce-scatter");
        return FLEXAR_ERR_UNSUPPORTED;
      }
      if ((rc = typed_spec(comms[r], &s, dtype, op, false, (double)count * es * nranks))) return rc;
    }
    proto = proto_of(s);
    DevProgram* dp = nullptr;
    if ((rc = get_program(comms[r], s, count, es, fs, &dp, (Coll)coll, count))) return rc;
    wire = dp->prog.wire;
    fanin = std::max(fanin, (int)dp->prog.max_nsrc);
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
  la.epoch = comms[0]->launches + 1;
  la.tag = "in-process group";
  la.proto = proto;
  la.wire = wire;
  la.max_fanin = fanin;
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
  la.epoch = comms[0]->launches + 1;
  la.tag = "in-process group";
  la.proto = proto;
  int rc = launch_dtype(dtype, FLEXAR_SUM, la);
  if (!rc) (void)group_ctx_launched(st);
  if (rc) return rc;
  for (int r = 0; r < nranks; ++r) comms[r]->launches++;
  FX_HIP(hipStreamSynchronize(st));
  return 0;
}

}  // extern "C"
