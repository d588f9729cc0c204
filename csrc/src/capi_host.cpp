// Host-only part of the C API: errors, planning utilities, the reference
// cost model, the program dump, the CPU simulator of the device protocol and
// the host reduction. Compiled by the plain host C++ compiler (no HIP).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "flexar/calibration.hpp"
#include "flexar/cost_model.hpp"
#include "flexar/flexar.h"
#include "flexar/host_exec.hpp"
#include "flexar/msg_plan.hpp"
#include "flexar/planner.hpp"
#include "flexar/readiness.hpp"
#include "flexar/zc_policy.hpp"
#include "host_barrier.hpp"
#include "internal.hpp"

namespace flexar {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

static int copy_out(const std::string& s, char* out, size_t outlen) {
  if (!out || outlen == 0) return FLEXAR_ERR_INVALID;
  size_t n = std::min(outlen - 1, s.size());
  memcpy(out, s.data(), n);
  out[n] = 0;
  return s.size() < outlen ? 0 : FLEXAR_ERR_NOMEM;
}

struct RankBarrier {
  std::mutex m;
  std::condition_variable cv;
  int count = 0, gen = 0, n = 0;
  void arrive_and_wait() {
    std::unique_lock<std::mutex> lk(m);
    int g = gen;
    if (++count == n) {
      count = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

struct SimRun {
  template <typename T, typename OP>
  static int run(const std::vector<Program>& progs, int nranks, int grid, int ncalls, int in_place,
                 const void* const* inputs, void* const* outputs, size_t count, float pre = 1.0f) {
    const size_t es = sizeof(T);
    uint64_t stg_bytes = 0;
    uint32_t nslots = 1;
    for (auto& p : progs) {
      stg_bytes = std::max<uint64_t>(stg_bytes, p.stg_bytes());
      nslots = std::max<uint32_t>(nslots, p.nslots);
    }
    uint64_t half = (stg_bytes + 255) / 256 * 256;
    std::vector<std::vector<char>> stg(nranks, std::vector<char>(2 * half + 256, (char)0xA5));  // poison
    size_t nflags = (size_t)nslots * nranks * grid;
    std::vector<std::unique_ptr<std::atomic<uint64_t>[]>> flags(nranks);
    for (int r = 0; r < nranks; ++r) {
      flags[r].reset(new std::atomic<uint64_t>[nflags]);
      for (size_t i = 0; i < nflags; ++i) flags[r][i].store(0);
    }
    std::vector<HostExecCtx> ctx(nranks);
    for (int r = 0; r < nranks; ++r) {
      HostExecCtx& c = ctx[r];
      c.rank = r;
      c.local[BUF_IN] = in_place ? (char*)outputs[r] : (char*)inputs[r];
      c.local[BUF_OUT] = (char*)outputs[r];
      c.local[BUF_STG] = stg[r].data();
      for (int p = 0; p < nranks; ++p) {
        c.peer_stg.push_back(stg[p].data());
        c.peer_flags.push_back(flags[p].get());
        c.peer_io[BUF_IN].push_back(in_place ? (char*)outputs[p] : (char*)inputs[p]);
        c.peer_io[BUF_OUT].push_back((char*)outputs[p]);
      }
      c.ranks_stride = nranks;
      c.blocks_stride = grid;
      c.stg_half_bytes = half;
      c.timeout_s = 30.0;
      c.pre = pre;
      c.post_inv = 1.0f / pre;
    }
    std::vector<RankBarrier> bars(nranks);
    for (auto& b : bars) b.n = grid;
    std::atomic<int> rc{0};
    std::vector<std::thread> th;
    for (int r = 0; r < nranks; ++r)
      for (int b = 0; b < grid; ++b)
        th.emplace_back([&, r, b] {
          for (int e = 1; e <= ncalls; ++e) {
            if (in_place) {  // kernel boundary: rank r re-loads its input before each call
              bars[r].arrive_and_wait();
              if (b == 0) memcpy(outputs[r], inputs[r], count * es);
              bars[r].arrive_and_wait();
            }
            int x = HostExec<T, OP>::run(progs[r], ctx[r], (uint32_t)b, (uint32_t)grid, (uint64_t)e);
            if (x) rc.store(x);
            bars[r].arrive_and_wait();  // all workgroups of rank r finish call e before e + 1 starts
            if (rc.load()) return;
          }
        });
    for (auto& t : th) t.join();
    if (rc.load()) set_error("simulated wait timed out (deadlock in the program?)");
    return rc.load();
  }
};

// Host run of message plans (msg_plan.hpp): one thread per rank; executor segments run on the host
// executor, groups exchange bytes through per-(source, destination) FIFO mailboxes (NCCL matches the
// sends and receives of a rank pair in order, without tags).
struct MsgSimRun {
  template <typename T, typename OP>
  static int run(const std::vector<MsgPlan>& plans, int nranks, int ncalls, const void* const* inputs,
                 void* const* outputs, size_t count) {
    const size_t es = sizeof(T);
    struct Box {
      std::mutex m;
      std::condition_variable cv;
      std::vector<std::vector<char>> q;
      size_t head = 0;
    };
    std::vector<Box> boxes((size_t)nranks * nranks);
    std::atomic<int> rc{0};
    std::vector<std::thread> th;
    for (int r = 0; r < nranks; ++r)
      th.emplace_back([&, r] {
        const MsgPlan& M = plans[r];
        std::vector<char> stg(M.stg_bytes + 256, (char)0xA5);
        HostExecCtx c;
        c.rank = r;
        c.local[BUF_IN] = (char*)inputs[r];
        c.local[BUF_OUT] = (char*)outputs[r];
        c.local[BUF_STG] = stg.data();
        c.peer_stg.assign(nranks, stg.data());
        c.peer_flags.assign(nranks, nullptr);
        c.ranks_stride = nranks;
        c.blocks_stride = 1;
        c.stg_half_bytes = 0;
        auto base = [&](uint16_t b) { return c.local[b]; };
        for (int e = 1; e <= ncalls && !rc.load(); ++e) {
          for (const MsgStep& s : M.steps) {
            if (s.kind == MsgStep::EXEC) {
              if (HostExec<T, OP>::run(s.prog, c, 0, 1, (uint64_t)e)) rc.store(FLEXAR_ERR_TIMEOUT);
              continue;
            }
            for (const MsgXfer& x : s.sends) {
              Box& b = boxes[(size_t)r * nranks + x.peer];
              std::lock_guard<std::mutex> lk(b.m);
              b.q.emplace_back(base(x.buf) + x.off, base(x.buf) + x.off + x.bytes);
              b.cv.notify_all();
            }
            for (const MsgXfer& x : s.recvs) {
              Box& b = boxes[(size_t)x.peer * nranks + r];
              std::unique_lock<std::mutex> lk(b.m);
              if (!b.cv.wait_for(lk, std::chrono::seconds(30), [&] { return b.q.size() > b.head; })) {
                rc.store(FLEXAR_ERR_TIMEOUT);
                return;
              }
              std::vector<char> msg = std::move(b.q[b.head++]);
              if (msg.size() != x.bytes) { rc.store(FLEXAR_ERR_STATE); return; }
              memcpy(base(x.buf) + x.off, msg.data(), msg.size());
            }
          }
        }
        (void)es;
      });
    for (auto& t : th) t.join();
    if (rc.load() == FLEXAR_ERR_STATE) set_error("message size mismatch between a send and its receive");
    else if (rc.load()) set_error("message simulation timed out (unmatched receive)");
    return rc.load();
  }
};

struct HostReduce {
  template <typename T, typename OP>
  static int run(void* dst, const void* const* srcs, int nsrc, size_t count, float scale) {
    std::vector<const T*> s(nsrc);
    for (int i = 0; i < nsrc; ++i) s[i] = (const T*)srcs[i];
    T* d = (T*)dst;
    host_reduce_span<T, OP>(&d, 1, s.data(), nsrc, count, scale);
    return 0;
  }
};

static bool spec_for(const char* spec, int nranks, double bytes, AlgoSpec* s, std::string* err,
                     bool host_only = false) {
  if (!parse_algo(spec ? spec : "auto", nranks, s, err)) return false;
  if (s->kind == AlgoKind::AUTO) *s = select_plan(XgmiModel::from_env(), nranks, bytes);
  if (s->kind == AlgoKind::TREE && s->ag == AgMode::AUTO) s->ag = AgMode::PULL;
  if (s->kind == AlgoKind::LL && host_only) s->kind = AlgoKind::ONESHOT;  // LL is a device-only protocol
  if (s->kind == AlgoKind::DMA && host_only) *s = AlgoSpec(), s->kind = AlgoKind::TREE, s->widths = {nranks},
                                             s->ag = AgMode::PULL;  // same exchange, host-executable
  return true;
}

}  // namespace flexar

using namespace flexar;

extern "C" {

const char* flexar_version(void) {
  static char v[32];
  snprintf(v, sizeof(v), "%d.%d.%d", FLEXAR_VERSION_MAJOR, FLEXAR_VERSION_MINOR, FLEXAR_VERSION_PATCH);
  return v;
}
const char* flexar_last_error(void) { return g_last_error.c_str(); }
size_t flexar_dtype_size(int dtype) { return dtype_size(dtype); }

int flexar_parse_ft_topo(const char* ft_topo, int nranks, char* out, size_t outlen) {
  AlgoSpec s;
  std::string err;
  if (!parse_ft_topo(ft_topo, nranks, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  return copy_out(s.str(), out, outlen);
}

uint64_t flexar_count_factorizations(int n) { return count_factorizations(n); }
// Rank order of ring `channel` of a C-channel ring on n ranks (the planner's ring_order); returns the
// number of channels a ring on n ranks can have (max_ring_channels), or -1 on bad arguments.
int flexar_ring_order(int n, int channel, int C, int* order) {
  if (n < 1 || n > kMaxRanks || channel < 0 || C < 1 || !order) return -1;
  const std::vector<int> o = ring_order(n, channel, C);
  for (int i = 0; i < n; ++i) order[i] = o[i];
  return max_ring_channels(n);
}

int flexar_enumerate_plans(int nranks, char* out, size_t outlen) {
  std::string s;
  for (auto& p : enumerate_plans(nranks)) s += p.str() + "\n";
  return copy_out(s, out, outlen);
}

double flexar_model_cost_us(const char* spec, int nranks, double bytes) {
  AlgoSpec s;
  std::string err;
  if (!spec_for(spec, nranks, bytes, &s, &err)) { set_error(err); return -1.0; }
  return XgmiModel::from_env().cost_us(s, nranks, bytes);
}

// Cost-model feature vector of (spec, nranks, bytes) under `links` concurrent links (<= 0: FLEXAR_MODEL /
// default): cost_us = out[0] alpha_launch + out[1] alpha_sync + out[2] / link_gbps + out[3] / hbm_gbps.
// The spec is priced as written (its typing included: "+f32" fp32 partials, "+rw" per-hop rounding) for
// elements of `esize` bytes.
int flexar_model_features_ex(const char* spec, int nranks, double bytes, int links, int esize, double* out) {
  if (!out || nranks < 1 || esize < 1 || esize > 8) { set_error("bad arguments"); return FLEXAR_ERR_INVALID; }
  AlgoSpec s;
  std::string err;
  if (!spec_for(spec, nranks, bytes, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  XgmiModel m = XgmiModel::from_env();
  if (links > 0) m.links = links;
  if (!m.features(s, nranks, bytes, out, (uint32_t)esize)) {
    set_error("no linear cost features for " + s.str());
    return FLEXAR_ERR_UNSUPPORTED;
  }
  return 0;
}

int flexar_model_features(const char* spec, int nranks, double bytes, int links, double* out) {
  return flexar_model_features_ex(spec, nranks, bytes, links, 4, out);
}

// What rank `rank`'s compiled program of (spec, nranks, count, dtype) costs (cost_model.hpp program_cost):
// out = {handoffs, link_bytes, link_time_bytes, hbm_read, hbm_write}. The spec is built as written:
// "+f32" types the partials of a 16/8-bit dtype, "+rw" or no suffix leaves them in the dtype.
int flexar_program_cost(const char* spec, int rank, int nranks, size_t count, int dtype, int links, double* out) {
  const size_t es = dtype_size(dtype);
  if (!out || !es || nranks < 1 || rank < 0 || rank >= nranks) { set_error("bad arguments"); return FLEXAR_ERR_INVALID; }
  AlgoSpec s;
  std::string err;
  if (!spec_for(spec, nranks, (double)count * es, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  if (s.kind == AlgoKind::LL || s.kind == AlgoKind::DMA) { set_error("no op program for " + s.str()); return FLEXAR_ERR_UNSUPPORTED; }
  Program P;
  Planner pl(nranks, rank, count, (uint32_t)es, 1.0f);
  if (!pl.build(s, &P, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  const ProgramCost c = program_cost(P, (uint32_t)rank, links > 0 ? links : XgmiModel::from_env().links);
  out[0] = c.handoffs;
  out[1] = c.link_bytes;
  out[2] = c.link_time_bytes;
  out[3] = c.hbm_read;
  out[4] = c.hbm_write;
  return 0;
}

// The typed form `spec` runs for a call of dtype / op (cost_model.hpp apply_partials; FLEXAR_PARTIALS and
// FLEXAR_MODEL apply): "+f32" fp32 partials, "+rw" per-hop rounding, or unchanged.
int flexar_apply_partials(const char* spec, int nranks, double bytes, int dtype, int op, char* out, size_t outlen) {
  AlgoSpec s;
  std::string err;
  if (nranks < 1 || !dtype_size(dtype) || !parse_algo(spec ? spec : "", nranks, &s, &err) || s.kind == AlgoKind::AUTO) {
    set_error(err.empty() ? "apply_partials needs a concrete spec" : err);
    return FLEXAR_ERR_INVALID;
  }
  if (s.kind == AlgoKind::TREE && s.ag == AgMode::AUTO) s.ag = AgMode::PULL;
  CallKind k;
  k.esize = (uint32_t)dtype_size(dtype);
  k.narrow_sum = (op == FLEXAR_SUM || op == FLEXAR_AVG) && dtype_is_float(dtype) && k.esize < 4;
  apply_partials(&s, nranks, bytes, k, XgmiModel::from_env());
  return copy_out(s.str(), out, outlen);
}

// The selector's choice for a call of `dtype` / `op` (the typed form it would run included).
int flexar_select_plan_ex(int nranks, double bytes, int dtype, int op, int links, char* out, size_t outlen) {
  if (nranks < 1 || !dtype_size(dtype)) return FLEXAR_ERR_INVALID;
  XgmiModel m = XgmiModel::from_env();
  if (links > 0) m.links = links;
  CallKind k;
  k.esize = (uint32_t)dtype_size(dtype);
  k.narrow_sum = (op == FLEXAR_SUM || op == FLEXAR_AVG) && dtype_is_float(dtype) && k.esize < 4;
  return copy_out(select_plan(m, nranks, bytes, nullptr, k).str(), out, outlen);
}

int flexar_select_plan(int nranks, double bytes, char* out, size_t outlen) {
  if (nranks < 1) return FLEXAR_ERR_INVALID;
  return copy_out(select_plan(XgmiModel::from_env(), nranks, bytes).str(), out, outlen);
}

double flexar_legacy_cost(const char* widths_csv, int nranks, double chunk) {
  std::vector<int> w;
  std::string err;
  if (!parse_int_list(widths_csv ? widths_csv : "", &w, &err) || w.empty()) { set_error(err); return -1.0; }
  return legacy_cost(w, nranks, chunk);
}

int flexar_plan_dump(const char* spec, int rank, int nranks, size_t count, int dtype, char* out, size_t outlen) {
  size_t es = dtype_size(dtype);
  if (!es || rank < 0 || rank >= nranks) { set_error("bad arguments"); return FLEXAR_ERR_INVALID; }
  AlgoSpec s;
  std::string err;
  if (!spec_for(spec, nranks, (double)count * es, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  Program P;
  Planner pl(nranks, rank, count, (uint32_t)es, 1.0f);
  if (!pl.build(s, &P, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  return copy_out(dump_program(P, rank), out, outlen);
}

int flexar_simulate(const char* spec, int nranks, size_t count, int dtype, int op, const void* const* inputs,
                    void* const* outputs, int grid, int ncalls, int in_place, float scale) {
  size_t es = dtype_size(dtype);
  if (!es || nranks < 1 || nranks > 64 || grid < 1 || grid > 64 || ncalls < 1 || !inputs || !outputs) {
    set_error("bad simulate arguments");
    return FLEXAR_ERR_INVALID;
  }
  if (!op_supported(dtype, op)) { set_error("unsupported dtype/op"); return FLEXAR_ERR_UNSUPPORTED; }
  AlgoSpec s;
  std::string err;
  if (!spec_for(spec, nranks, (double)count * es, &s, &err, true)) { set_error(err); return FLEXAR_ERR_INVALID; }
  float fs = scale * (op == FLEXAR_AVG ? 1.0f / (float)nranks : 1.0f);
  std::vector<Program> progs(nranks);
  for (int r = 0; r < nranks; ++r) {
    Planner pl(nranks, r, count, (uint32_t)es, fs);
    if (!pl.build(s, &progs[r], &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    if (!validate_program(progs[r], nranks, r, count, count, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    if (progs[r].nchan > (uint32_t)grid) { set_error("grid must be >= number of channels"); return FLEXAR_ERR_INVALID; }
  }
  if (grid % progs[0].nchan) { set_error("grid must be a multiple of the channel count"); return FLEXAR_ERR_INVALID; }
  return dispatch_dtype_op<SimRun>(dtype, op, progs, nranks, grid, ncalls, in_place, inputs, outputs, count);
}

// Typed programs ("+f32" fp32 partials, "+e4m3"/"+e5m2" fp8 wire) with an explicit fp8 pre-scale
// (the device derives it from the global amax: s = fp8_max / (N * amax)).
int flexar_simulate_typed(const char* spec, int nranks, size_t count, int dtype, int op, const void* const* inputs,
                          void* const* outputs, int grid, int ncalls, float scale, float pre) {
  size_t es = dtype_size(dtype);
  if (!es || nranks < 1 || nranks > 64 || grid < 1 || grid > 64 || ncalls < 1 || !inputs || !outputs || !(pre > 0)) {
    set_error("bad simulate arguments");
    return FLEXAR_ERR_INVALID;
  }
  if (!dtype_is_float(dtype) || (op != FLEXAR_SUM && op != FLEXAR_AVG)) {
    set_error("typed staging needs a float dtype with SUM/AVG");
    return FLEXAR_ERR_UNSUPPORTED;
  }
  AlgoSpec s;
  std::string err;
  if (!spec_for(spec, nranks, (double)count * es, &s, &err, true)) { set_error(err); return FLEXAR_ERR_INVALID; }
  float fs = scale * (op == FLEXAR_AVG ? 1.0f / (float)nranks : 1.0f);
  std::vector<Program> progs(nranks);
  for (int r = 0; r < nranks; ++r) {
    Planner pl(nranks, r, count, (uint32_t)es, fs);
    if (!pl.build(s, &progs[r], &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    if (!validate_program(progs[r], nranks, r, count, count, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  }
  if (grid % progs[0].nchan) { set_error("grid must be a multiple of the channel count"); return FLEXAR_ERR_INVALID; }
  return dispatch_dtype_op<SimRun>(dtype, op, progs, nranks, grid, ncalls, 0, inputs, outputs, count, pre);
}

// Message transport (RCCL send/recv) plans on host memory: inputs/outputs nranks host pointers.
int flexar_simulate_msg(const char* spec, int nranks, size_t count, int dtype, int op, const void* const* inputs,
                        void* const* outputs, int ncalls, float scale) {
  size_t es = dtype_size(dtype);
  if (!es || nranks < 1 || nranks > 64 || ncalls < 1 || !inputs || !outputs) {
    set_error("bad simulate arguments");
    return FLEXAR_ERR_INVALID;
  }
  if (!op_supported(dtype, op)) { set_error("unsupported dtype/op"); return FLEXAR_ERR_UNSUPPORTED; }
  AlgoSpec s;
  std::string err;
  if (!parse_algo(spec ? spec : "auto", nranks, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  if (s.kind == AlgoKind::AUTO) s = select_plan(XgmiModel::from_env(), nranks, (double)count * es);
  float fs = scale * (op == FLEXAR_AVG ? 1.0f / (float)nranks : 1.0f);
  std::vector<MsgPlan> plans(nranks);
  for (int r = 0; r < nranks; ++r) {
    if (!build_msg_plan(nranks, r, count, (uint32_t)es, fs, s, &plans[r], &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    for (auto& st : plans[r].steps)
      if (st.kind == MsgStep::EXEC && !validate_program(st.prog, nranks, r, count, count, &err)) {
        set_error(err);
        return FLEXAR_ERR_INVALID;
      }
  }
  return dispatch_dtype_op<MsgSimRun>(dtype, op, plans, nranks, ncalls, inputs, outputs, count);
}

// Message-plan summary (JSON): per step, the executor segment's op count or the group's sends/receives
// (peer, bytes, zero-copy source buffer) - what the RCCL transport posts for (spec, count, dtype) on `rank`.
int flexar_msg_plan_dump(const char* spec, int rank, int nranks, size_t count, int dtype, char* out, size_t outlen) {
  size_t es = dtype_size(dtype);
  if (!es || rank < 0 || rank >= nranks) { set_error("bad arguments"); return FLEXAR_ERR_INVALID; }
  AlgoSpec s;
  std::string err;
  if (!parse_algo(spec ? spec : "auto", nranks, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  if (s.kind == AlgoKind::AUTO) s = select_plan(XgmiModel::from_env(), nranks, (double)count * es);
  MsgPlan M;
  if (!build_msg_plan(nranks, rank, count, (uint32_t)es, 1.0f, s, &M, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  static const char* bn[] = {"in", "out", "stg"};
  std::string j = "{\"stg_bytes\": " + std::to_string(M.stg_bytes) + ", \"messages\": " + std::to_string(M.msgs) +
                  ", \"message_bytes\": " + std::to_string(M.msg_bytes) + ", \"zero_copy\": " +
                  std::to_string(M.zero_copy) + ", \"steps\": [";
  for (size_t i = 0; i < M.steps.size(); ++i) {
    const MsgStep& st = M.steps[i];
    j += i ? ", " : "";
    if (st.kind == MsgStep::EXEC) {
      j += "{\"exec\": " + std::to_string(st.prog.ops.size()) + "}";
      continue;
    }
    auto lst = [&](const std::vector<MsgXfer>& v) {
      std::string t = "[";
      for (size_t k = 0; k < v.size(); ++k)
        t += std::string(k ? ", " : "") + "[" + std::to_string(v[k].peer) + ", " + std::to_string(v[k].bytes) + ", \"" +
             bn[v[k].buf] + "\"]";
      return t + "]";
    };
    j += "{\"send\": " + lst(st.sends) + ", \"recv\": " + lst(st.recvs) + "}";
  }
  j += "]}";
  return copy_out(j, out, outlen);
}

int flexar_simulate_coll(int coll, const char* spec, int nranks, size_t count, int dtype, int op,
                         const void* const* inputs, void* const* outputs, int grid, int ncalls, float scale) {
  size_t es = dtype_size(dtype);
  if (!es || nranks < 1 || nranks > 64 || grid < 1 || grid > 64 || ncalls < 1 || !inputs || !outputs || coll < 0 ||
      coll > 4 || coll == 3) {
    set_error("bad simulate arguments");
    return FLEXAR_ERR_INVALID;
  }
  if (!op_supported(dtype, op)) { set_error("unsupported dtype/op"); return FLEXAR_ERR_UNSUPPORTED; }
  AlgoSpec s;
  std::string err;
  if (!spec_for(spec, nranks, (double)count * es, &s, &err, true)) { set_error(err); return FLEXAR_ERR_INVALID; }
  float fs = coll == 1 ? scale * (op == FLEXAR_AVG ? 1.0f / (float)nranks : 1.0f) : 1.0f;
  std::vector<Program> progs(nranks);
  for (int r = 0; r < nranks; ++r) {
    Planner pl(nranks, r, count, (uint32_t)es, fs);
    if (!pl.build_coll((Coll)coll, s, count, &progs[r], &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    uint64_t in_el, out_el;
    io_extent((Coll)coll, nranks, count, count, &in_el, &out_el);
    if (!validate_program(progs[r], nranks, r, in_el, out_el, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  }
  if (grid % progs[0].nchan) { set_error("grid must be a multiple of the channel count"); return FLEXAR_ERR_INVALID; }
  return dispatch_dtype_op<SimRun>(dtype, (coll == 2 || coll == 4) ? FLEXAR_SUM : op, progs, nranks, grid, ncalls, 0, inputs,
                                   outputs, count);
}

int flexar_simulate_bcast(const char* spec, int nranks, size_t count, int dtype, int root, const void* const* inputs,
                          void* const* outputs, int grid, int ncalls) {
  size_t es = dtype_size(dtype);
  if (!es || nranks < 1 || nranks > 64 || grid < 1 || grid > 64 || ncalls < 1 || !inputs || !outputs || root < 0 ||
      root >= nranks) {
    set_error("bad simulate arguments");
    return FLEXAR_ERR_INVALID;
  }
  AlgoSpec s;
  std::string err;
  if (!parse_algo(spec ? spec : "auto", nranks, &s, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  if (s.kind == AlgoKind::AUTO) s.kind = count * es <= (256u << 10) ? AlgoKind::ONESHOT : AlgoKind::TREE;
  std::vector<Program> progs(nranks);
  for (int r = 0; r < nranks; ++r) {
    Planner pl(nranks, r, count, (uint32_t)es, 1.0f);
    if (!pl.build_coll(Coll::BROADCAST, s, (uint64_t)root, &progs[r], &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
    if (!validate_program(progs[r], nranks, r, count, count, &err)) { set_error(err); return FLEXAR_ERR_INVALID; }
  }
  return dispatch_dtype_op<SimRun>(dtype, FLEXAR_SUM, progs, nranks, grid, ncalls, 0, inputs, outputs, count);
}

int flexar_downgrade_spec(const char* spec, int nranks, uint32_t disabled, int allow_dma, char* out, size_t outlen) {
  AlgoSpec s;
  std::string err;
  if (nranks < 1 || !parse_algo(spec ? spec : "auto", nranks, &s, &err)) { set_error(err.empty() ? "bad arguments" : err); return FLEXAR_ERR_INVALID; }
  if (s.kind == AlgoKind::AUTO) { set_error("downgrade needs a concrete spec"); return FLEXAR_ERR_INVALID; }
  if (!downgrade_spec(&s, nranks, disabled, allow_dma != 0, &err)) { set_error(err); return FLEXAR_ERR_UNSUPPORTED; }
  return copy_out(s.str(), out, outlen);
}

// Zero-copy policy (zc_policy.hpp) on a resolved spec: the spec a call runs and the decision (1 = switched
// to zero copy, -1 = fell back to staging, 0 = unchanged) in *decision. flags: 1 registered, 2 named,
// 4 from_auto, 8 zc_auto, 16 have_tune. Default cost model (FLEXAR_MODEL applies).
int flexar_zc_decide(const char* spec, int nranks, double bytes, int flags, uint32_t disabled, int* decision,
                     char* out, size_t outlen) {
  AlgoSpec s;
  std::string err;
  if (nranks < 1 || !decision || !parse_algo(spec ? spec : "", nranks, &s, &err) || s.kind == AlgoKind::AUTO) {
    set_error(err.empty() ? "zc_decide needs a concrete spec" : err);
    return FLEXAR_ERR_INVALID;
  }
  if (s.kind == AlgoKind::TREE && s.ag == AgMode::AUTO) s.ag = AgMode::PULL;
  ZcFacts f;
  f.nranks = nranks;
  f.bytes = bytes;
  f.registered = flags & 1;
  f.named = flags & 2;
  f.from_auto = flags & 4;
  f.zc_auto = flags & 8;
  f.have_tune = flags & 16;
  f.disabled = disabled;
  *decision = zc_decide(&s, f, XgmiModel::from_env());
  return copy_out(s.str(), out, outlen);
}

// Probe agreement on rank-major ProbeBlobs (readiness.hpp probe_agree), host-only: the agreed link count
// in *links_out, or FLEXAR_ERR_INVALID with the disagreement in flexar_last_error().
int flexar_probe_agree(const void* blobs, int nranks, int* links_out) {
  if (!blobs || nranks < 1 || nranks > 16) { set_error("bad arguments"); return FLEXAR_ERR_INVALID; }
  std::vector<ProbeBlob> v(nranks);
  memcpy(v.data(), blobs, sizeof(ProbeBlob) * nranks);
  std::string why;
  if (!probe_agree(v.data(), nranks, links_out, &why)) { set_error(why); return FLEXAR_ERR_INVALID; }
  return 0;
}
// Settings fingerprint of this process's environment (readiness.hpp env_fingerprint, no tune table):
// with_calib = 1 is the connect-time form, 0 the calibration cache's.
uint64_t flexar_settings_fingerprint(int with_calib) { return env_fingerprint("", with_calib != 0); }

// The same, also returning the agreed resident-workgroup count (0 = no rank knew its own).
int flexar_probe_agree_resident(const void* blobs, int nranks, int* links_out, int* resident_out) {
  if (!blobs || nranks < 1 || nranks > 16) { set_error("bad arguments"); return FLEXAR_ERR_INVALID; }
  std::vector<ProbeBlob> v(nranks);
  memcpy(v.data(), blobs, sizeof(ProbeBlob) * nranks);
  std::string why;
  if (!probe_agree(v.data(), nranks, links_out, &why, resident_out)) { set_error(why); return FLEXAR_ERR_INVALID; }
  return 0;
}

// ---- calibration helpers (calibration.hpp), host-only: the device measurement is flexar_comm_calibrate ----
static std::vector<CalibRow> calib_rows(int nrows, const char* specs_nl, const double* bytes, const double* us) {
  std::vector<CalibRow> rows;
  std::istringstream ss(specs_nl ? specs_nl : "");
  std::string spec;
  for (int i = 0; i < nrows && std::getline(ss, spec); ++i) rows.push_back({spec, bytes[i], us[i]});
  return rows;
}

// Fit theta to rows (specs newline-separated): out = {alpha_launch_us, alpha_sync_us, link_gbps, hbm_gbps,
// median_rel_err, max_rel_err, rows used}. links <= 0: the default model's.
int flexar_calib_fit(int nrows, const char* specs_nl, const double* bytes, const double* us, int nranks, int links,
                     int esize, double* out) {
  if (nrows < 0 || !out || nranks < 1 || (nrows && (!bytes || !us))) { set_error("bad arguments"); return FLEXAR_ERR_INVALID; }
  XgmiModel m = XgmiModel::from_env();
  if (links > 0) m.links = links;
  const CalibFit f = fit_theta(calib_rows(nrows, specs_nl, bytes, us), m, nranks, (uint32_t)(esize > 0 ? esize : 4));
  if (!f.ok) { set_error("calibration: fewer than 4 usable rows or no non-negative fit"); return FLEXAR_ERR_INVALID; }
  const XgmiModel fm = model_with_theta(m, f.theta);
  out[0] = fm.alpha_launch_us;
  out[1] = fm.alpha_sync_us;
  out[2] = fm.link_gbps;
  out[3] = fm.hbm_gbps;
  out[4] = f.median_rel_err;
  out[5] = f.max_rel_err;
  out[6] = f.rows;
  return 0;
}

int flexar_calib_key(const char* arch, int nranks, int links, const char* classes, uint32_t disabled, char* out,
                     size_t outlen) {
  return copy_out(calib_key(arch ? arch : "", nranks, links, classes ? classes : "", disabled, flexar_version()), out,
                  outlen);
}

int flexar_calib_path(const char* key, char* out, size_t outlen) {
  const std::string d = calib_dir();
  if (d.empty()) { set_error("no calibration cache directory (FLEXAR_CALIB_DIR / HOME)"); return FLEXAR_ERR_UNSUPPORTED; }
  return copy_out(calib_path(d, key ? key : ""), out, outlen);
}

// theta = {alpha_launch_us, alpha_sync_us, 1/link_gbps, 1/hbm_gbps}; 1 = loaded, 0 = miss
int flexar_calib_load(const char* path, const char* key, double* theta) {
  if (!path || !key || !theta) return FLEXAR_ERR_INVALID;
  return calib_load(path, key, theta) ? 1 : 0;
}

int flexar_calib_store(const char* path, const char* key, const double* theta, int nrows, const char* specs_nl,
                       const double* bytes, const double* us) {
  if (!path || !key || !theta) return FLEXAR_ERR_INVALID;
  if (!calib_store(path, key, theta, calib_rows(nrows, specs_nl, bytes, us))) {
    set_error(std::string("calibration cache: cannot write ") + path);
    return FLEXAR_ERR_INVALID;
  }
  return 0;
}

// The measurement set of flexar_comm_calibrate for nranks: "spec bytes" lines.
int flexar_calib_points(int nranks, char* out, size_t outlen) {
  std::string s;
  for (const CalibPoint& p : calib_points(nranks)) s += p.spec + " " + std::to_string((long long)p.bytes) + "\n";
  return copy_out(s, out, outlen);
}

int flexar_direct_links(const int32_t* cls, const int32_t* hops, int nranks, int self) {
  if (!cls || !hops || nranks < 1 || self < 0 || self >= nranks) return -1;
  return direct_links(cls, hops, nranks, self);
}

int flexar_reduce_host(void* dst, const void* const* srcs, int nsrc, size_t count, int dtype, int op, float scale) {
  if (!dst || !srcs || nsrc < 1) { set_error("bad reduce arguments"); return FLEXAR_ERR_INVALID; }
  float fs = scale * (op == FLEXAR_AVG ? 1.0f / (float)nsrc : 1.0f);
  return dispatch_dtype_op<HostReduce>(dtype, op, dst, srcs, nsrc, count, fs);
}


// The teardown agreement (host_barrier.hpp) on its own, for CPU tests: join `name` as `rank` of `nranks`,
// pass `phases` barriers, sleeping `delay_ms` before each. Returns 0, or FLEXAR_ERR_TIMEOUT naming the
// straggler (flexar_last_error). Rank 0 removes the name after the first barrier.
// The connect-time shared-page check on its own (tests): join `name` and write this rank's mark; after the
// caller's own barrier, flexar_host_page_shared tells whether every rank's mark is in this rank's page.
void* flexar_host_page_open(const char* name, int rank, int nranks, uint64_t token) {
  if (!name || nranks < 1 || nranks > (int)kMaxRanks || rank < 0 || rank >= nranks) {
    set_error("bad arguments");
    return nullptr;
  }
  std::unique_ptr<HostBarrier> hb(new HostBarrier);
  std::string err;
  if (!hb->join(name, rank, nranks, &err)) {
    set_error(err);
    return nullptr;
  }
  hb->mark(token);
  return hb.release();
}
int flexar_host_page_shared(void* h, uint64_t token, int* missing) {
  if (!h) return 0;
  return static_cast<HostBarrier*>(h)->shared(token, missing) ? 1 : 0;
}
void flexar_host_page_close(void* h) {
  if (!h) return;
  static_cast<HostBarrier*>(h)->unlink();
  delete static_cast<HostBarrier*>(h);
}

int flexar_host_barrier_run(const char* name, int rank, int nranks, int phases, uint64_t timeout_ms, int delay_ms) {
  if (!name || nranks < 1 || nranks > (int)kMaxRanks || rank < 0 || rank >= nranks) {
    set_error("bad arguments");
    return FLEXAR_ERR_INVALID;
  }
  HostBarrier hb;
  std::string err;
  if (!hb.join(name, rank, nranks, &err)) {
    set_error(err);
    return FLEXAR_ERR_STATE;
  }
  for (int p = 0; p < phases; ++p) {
    if (delay_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms));
    int late = -1;
    uint64_t mx = 0;
    // odd phases also exchange a value: the maximum of rank * 1000 + phase is the last rank's; phases
    // 2 mod 4 OR one bit per rank
    const bool ok = (p & 1) ? hb.exchange_max((uint64_t)rank * 1000 + p, &mx, timeout_ms, &late)
                  : (p % 4 == 2) ? hb.exchange(1ull << rank, &mx, timeout_ms, &late, true)
                                 : hb.arrive_and_wait(timeout_ms, &late);
    if (!ok) {
      hb.unlink();
      set_error("phase " + std::to_string(p) + ": rank " + std::to_string(late) + " did not arrive");
      return FLEXAR_ERR_TIMEOUT;
    }
    if ((p & 1) && mx != (uint64_t)(nranks - 1) * 1000 + p) {
      set_error("phase " + std::to_string(p) + ": exchanged maximum " + std::to_string(mx));
      return FLEXAR_ERR_STATE;
    }
    if (p % 4 == 2 && mx != (nranks == 64 ? ~0ull : (1ull << nranks) - 1)) {
      set_error("phase " + std::to_string(p) + ": exchanged OR " + std::to_string(mx));
      return FLEXAR_ERR_STATE;
    }
    if (p == 0 && rank == 0) hb.unlink();
  }
  return 0;
}

}  // extern "C"
