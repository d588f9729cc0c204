// flexar message transport: the schedules' transfers as grouped ncclSend / ncclRecv between local executor
// segments (csrc/include/flexar/msg_plan.hpp) instead of peer-memory access over IPC.
#include "comm_internal.hpp"

namespace flexar {

// ---- message transport (msg_plan.hpp over RCCL) ----------------------------------------------------
int rccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return 0;
  set_error(std::string(what) + ": " + (rccl().GetErrorString ? rccl().GetErrorString(r) : "RCCL error"));
  return FLEXAR_ERR_RCCL;
}

int get_msg_plan(flexar_comm* c, const AlgoSpec& s, uint64_t count, uint32_t es, float fs, Coll coll,
                        uint64_t stride, DevMsgPlan** out) {
  char key[320];
  uint32_t sb;
  memcpy(&sb, &fs, 4);
  snprintf(key, sizeof(key), "%d|%s|%llu|%u|%08x|%llu", (int)coll, s.str().c_str(), (unsigned long long)count, es, sb,
           (unsigned long long)stride);
  auto it = c->msg_cache.find(key);
  if (it != c->msg_cache.end()) { *out = it->second.get(); return 0; }
  std::unique_ptr<DevMsgPlan> dp(new DevMsgPlan);
  dp->spec = "msg:" + s.str();
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
int run_msg(flexar_comm* c, const AlgoSpec& s, Coll coll, const void* in, void* out, uint64_t count, int dtype,
                   int op, float fs, uint64_t stride, hipStream_t st) {
  const uint32_t es = (uint32_t)dtype_size(dtype);
  DevMsgPlan* dp = nullptr;
  int rc = get_msg_plan(c, s, count, es, fs, coll, stride, &dp);
  if (rc) return rc;
  if (!c->msg_epochs) {
    FX_HIP(hipMalloc(&c->msg_epochs, kMaxGridBlocks * sizeof(uint64_t)));
    FX_HIP(hipMemset(c->msg_epochs, 0, kMaxGridBlocks * sizeof(uint64_t)));
  }
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
      x.epochs = c->msg_epochs;  // local-only segment: not part of the cross-rank epoch sequence
      x.stg_half_bytes = 0;
      x.err = c->err_dev;
      x.timeout_ticks = c->timeout_ticks;
      x.vec_ok = vec_ok_for(((uintptr_t)in) | ((uintptr_t)out));
      x.stg_unit = es;
      uint64_t span = 0;
      for (const Op& o : stp.prog.ops) span = std::max<uint64_t>(span, o.len);
      la.grid = choose_grid(c, span * es * 2, 1);
      la.stream = st;
      la.proto = PM_FENCE;
      la.tag = dp->spec.c_str();
      la.bytes = span * es;
      if ((rc = launch_dtype(dtype, op_k, la))) return rc;
      ++ex;
      continue;
    }
    {
      CrumbArgs ca;
      ca.type = CRUMB_RCCL;
      ca.what = "ncclSend/ncclRecv group";
      ca.rank = (int16_t)c->rank;
      ca.nranks = (int16_t)c->nranks;
      for (const MsgXfer& m : stp.sends) ca.bytes += m.bytes;
      ca.grid = (uint32_t)(stp.sends.size() * 1000 + stp.recvs.size());  // sends x 1000 + receives
      ca.label = dp->spec.c_str();
      crumb(ca);
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

}  // namespace flexar

