// Runtime algorithm selector: an alpha-beta-gamma cost model for a fully
// connected xGMI mesh, plus the reference's offline model kept for parity.
//
// Reference: cost_model/CostModel.h:1-119 (+ GetWidth.h, ChooseWidth.h,
// main.cpp) enumerates every ordered factorization of N, scores each with
//   sum_layers latency_control_overhead (2*lo, + s*(w-9)*co if w > 9)
//   + memory_read_write_overhead (steps*s/n*o) + bandwidth ((n-1)/n*s*bo)
// and prints the argmin; a human then exports FT_TOPO. It is not linked into
// the runtime, its bandwidth term is topology independent, and it has defects
// (D10: uninitialised accumulator, hard-coded chunk 100 in the latency term,
// no return for height 0 or > 9). legacy_cost() reproduces the intended model
// with those fixed; XgmiModel is the model actually used at run time. It prices
// the op program the planner compiles for (schedule, N, count, dtype), not a
// per-schedule formula (program_cost below):
//
//   cost_us = alpha_launch + handoffs * alpha_sync
//             + busiest-link bytes / link_bw     (per phase: max(max_peer, total / links))
//             + HBM bytes / hbm_bw               (every operand, at its real element size)
//
// so typed fp32 partials, the fp8 wire, zero copy and multicast all count
// exactly. Parameters are calibrated at connect time (flexar_comm_calibrate:
// measured executor schedules, max over ranks, least squares; cached on disk per
// node shape), by FLEXAR_MODEL="alpha_launch,alpha_sync,link_gbps,hbm_gbps,links",
// and a measured tune table overrides the model entirely (FLEXAR_TUNE_FILE).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "flexar/planner.hpp"
#include "flexar/topology.hpp"

namespace flexar {

constexpr double kLLMaxBytes = 1 << 20;  // LL protocol only for latency-bound sizes

// What a compiled op program costs one rank, read off the program itself (the model
// prices what the planner emits instead of per-schedule formulas and fudge factors):
//  * handoffs: signal -> wait hand-offs on the longest channel (consecutive WAIT ops = one hand-off);
//  * link_bytes: bytes this rank's transfers move across links - remote reads + remote writes, each
//    operand at its real element size (fp32 partials of typed staging, fp8 wire, the call's dtype);
//  * link_time_bytes: the busiest link's bytes, phase by phase (a phase runs from one hand-off to the
//    next; channels progress in lockstep on disjoint links): sum_phase max(max_peer b, sum_peer b / links).
//    Under the schedules' symmetry a peer's accesses to this rank mirror this rank's accesses to it, so
//    the bytes a rank's XFERs name on a peer are what that link carries in each direction;
//  * hbm_read / hbm_write: every operand's bytes, local or remote (a remote access lands in the peer's HBM,
//    and by the same symmetry the peers' accesses to this rank's HBM add up to the same amount).
// Reference: cost_model/CostModel.h:22-79 - a topology-independent bandwidth term (n-1)/n*s*bo plus a
// memory term counting read/write steps per layer; both become these per-program counts.
struct ProgramCost {
  double stg_bytes = 0;  // staging the program needs per parity half (pieces when it exceeds the workspace)
  double handoffs = 0;
  double link_bytes = 0;
  double link_time_bytes = 0;
  double hbm_read = 0;
  double hbm_write = 0;
};

inline ProgramCost program_cost(const Program& P, uint32_t rank, int links,
                                std::vector<std::map<uint32_t, double>>* phases_out = nullptr) {
  ProgramCost c;
  c.stg_bytes = (double)P.stg_bytes();
  const double L = links < 1 ? 1.0 : (double)links;
  auto bytes_of = [&](const Loc& l, uint64_t len) -> double {
    const uint32_t sz = (P.wire && l.buf == BUF_STG && (l.pad & 1)) ? P.wsize : P.esize;
    return (double)len * sz;
  };
  std::vector<std::map<uint32_t, double>> phases;  // phase -> peer -> bytes (all channels)
  for (uint32_t ch = 0; ch + 1 < P.chan_start.size(); ++ch) {
    uint32_t phase = 0;
    bool after_wait = false;
    for (uint32_t i = P.chan_start[ch]; i < P.chan_start[ch + 1]; ++i) {
      const Op& o = P.ops[i];
      if (o.kind == OP_WAIT) {
        if (!after_wait) ++phase;
        after_wait = true;
        continue;
      }
      if (o.kind != OP_XFER) continue;
      after_wait = false;
      if (phases.size() <= phase) phases.resize(phase + 1);
      for (int k = 0; k < o.nsrc; ++k) {
        const double b = bytes_of(o.src[k], o.len);
        c.hbm_read += b;
        if (o.src[k].rank != rank) c.link_bytes += b, phases[phase][o.src[k].rank] += b;
      }
      for (int k = 0; k < o.ndst; ++k) {
        const double b = bytes_of(o.dst[k], o.len);
        c.hbm_write += b;
        if (o.dst[k].rank != rank) c.link_bytes += b, phases[phase][o.dst[k].rank] += b;
      }
    }
    c.handoffs = std::max(c.handoffs, (double)phase);
  }
  for (const auto& ph : phases) {
    double mx = 0, tot = 0;
    for (const auto& kv : ph) mx = std::max(mx, kv.second), tot += kv.second;
    c.link_time_bytes += std::max(mx, tot / L);
  }
  if (phases_out) *phases_out = std::move(phases);
  return c;
}

// Partial sums of multi-hop schedules for 16/8-bit float SUM/AVG (FLEXAR_PARTIALS):
//   fp32:           typed staging keeps every partial in fp32 - one rounding, like flat (<= 1 ulp of the
//                   exact sum, tests/test_gpu_kernels.py::test_group_typed_fp32_partials) - at the price of
//                   fp32 link bytes on every hop but the first (bf16 ring at N = 8: 20/8 S instead of 14/8 S);
//   wire:           partials travel in the call's dtype and are rounded at every hop ("+rw", the reference's
//                   ring semantics, mpi_mod.hpp:1129-1147, and RCCL's): h roundings (ring N - 1, tree one per
//                   stage), error <= h ulps of the partial sums' magnitude;
//   auto (default): the cost model prices both forms of the schedule and takes the per-hop one when it is at
//                   least kAutoRwGain faster AND rounds at most kAutoRwMaxRoundings times (RHD at N = 8: 3;
//                   a ring at N = 8 rounds 7 times and keeps fp32 partials): at most 3 roundings, each
//                   within u = 2^-8 (bf16) of its partial sum.
// Round 4 measured the fp32-partials executor at the untyped executor's HBM rate (5.15 vs 5.25 TB/s, RHD bf16,
// 4 ranks on one GPU, profiles/r4_partials): its extra time is exactly its extra bytes (1.19x for RHD), so the
// default is the policy that drops those bytes where they are worth more than two extra roundings.
enum class Partials { FP32 = 0, WIRE = 1, AUTO = 2 };
constexpr double kAutoRwGain = 0.10;
constexpr int kAutoRwMaxRoundings = 3;

inline Partials partials_from_env() {
  const char* e = getenv("FLEXAR_PARTIALS");
  if (!e || !*e || !strcmp(e, "auto")) return Partials::AUTO;
  if (!strcmp(e, "wire") || !strcmp(e, "rw")) return Partials::WIRE;
  if (!strcmp(e, "fp32")) return Partials::FP32;
  return Partials::AUTO;
}

// The call a schedule is priced for: element size, and whether it is a 16/8-bit float SUM/AVG (the
// calls whose multi-hop schedules carry typed partials).
struct CallKind {
  uint32_t esize = 4;
  bool narrow_sum = false;
  bool wire_ok = false;  // fp32 / bf16 / fp16 SUM or AVG: an fp8 wire can carry it
};

// times a multi-hop schedule rounds its partials when they travel in the call's dtype
inline int hop_roundings(const AlgoSpec& s, int N) {
  if (s.kind == AlgoKind::RING) return N - 1;
  if (s.kind == AlgoKind::TREE) return (int)s.widths.size();
  return 1;
}
inline bool multihop(const AlgoSpec& s) {
  return s.kind == AlgoKind::RING || (s.kind == AlgoKind::TREE && s.widths.size() > 1);
}

struct XgmiModel {
  double alpha_launch_us = 6.0;  // kernel launch + first-touch
  double alpha_sync_us = 4.0;    // one signal->wait hand-off incl. release/acquire (measured ~4-5 us, BASELINE §5.8)
  double link_gbps = 64.0;       // usable per-direction bandwidth of one xGMI link (GB/s)
  double hbm_gbps = 5000.0;      // effective HBM bandwidth of the executor (every operand byte, read + write)
  int links = 7;                 // point-to-point links per GPU (fully connected 8-GPU node)
  double alpha_dma_us = 15.0;    // copy-engine path: stream fork/join + stream-memory wait/write per phase
  double dma_link_gbps = 50.0;   // one SDMA engine's peer-copy rate
  Partials partials = Partials::FP32;
  double stg_cap = 0;            // staging bytes one launch may use (the communicator's parity half; 0 = unbounded)

  static XgmiModel from_env() {
    XgmiModel m;
    const char* e = getenv("FLEXAR_MODEL");
    if (e && *e) {
      double v[5] = {m.alpha_launch_us, m.alpha_sync_us, m.link_gbps, m.hbm_gbps, (double)m.links};
      std::stringstream ss(e);
      std::string t;
      for (int i = 0; i < 5 && std::getline(ss, t, ','); ++i)
        if (!t.empty()) v[i] = atof(t.c_str());
      m.alpha_launch_us = v[0]; m.alpha_sync_us = v[1]; m.link_gbps = v[2]; m.hbm_gbps = v[3]; m.links = (int)v[4];
    }
    m.partials = partials_from_env();
    return m;
  }

  // time (us) to move `bytes` to each of `fan` peers concurrently
  double fanout_us_at(double bytes, int fan, double gbps) const {
    if (fan <= 0 || bytes <= 0) return 0.0;
    double par = fan <= links ? 1.0 : (double)links / fan;  // more peers than links share them
    return bytes / (gbps * 1e3 * par);
  }
  double reduce_us(double bytes_read) const { return bytes_read / (hbm_gbps * 1e3); }

  // The executor schedules' cost is linear in theta = (alpha_launch_us, alpha_sync_us, 1 / link_gbps,
  // 1 / hbm_gbps): cost_us = f . theta with f = (launches, hand-offs, busiest-link bytes / 1e3, HBM bytes
  // / 1e3), read off the compiled programs (program_cost; every rank's for lonely trees, whose ranks
  // differ, component-wise max). features() returns false for the copy-engine path (its own terms) and LL
  // above its cap; LL has no op program (a dedicated kernel) and keeps its closed form. costfit.py fits
  // theta to measured (spec, bytes, us) rows by least squares.
  bool features(const AlgoSpec& s, int N, double S, double f[4], uint32_t esize = 4) const {
    f[0] = 1.0; f[1] = f[2] = f[3] = 0.0;
    if (N <= 1) { f[3] = 2 * S / 1e3; return true; }
    if (s.kind == AlgoKind::DMA || s.kind == AlgoKind::AUTO) return false;
    if (s.kind == AlgoKind::LL) {  // flag-free 8-B {data, epoch} granules: half the hop cost, 2x the bytes
      if (S > kLLMaxBytes) return false;
      f[1] = 0.5; f[2] = std::max(2 * S, 2 * S * (N - 1) / std::max(1, links)) / 1e3; f[3] = 2 * (N + 1) * S / 1e3;
      return true;
    }
    if (N > (int)kMaxRanks || s.msg) return analytic_features(s, N, S, f);
    ProgramCost pc;
    if (!cached_cost(s, N, S, esize, &pc)) return false;
    // a program larger than the workspace runs as pieces: one launch and one hand-off chain each
    const double pieces = stg_cap > 0 && pc.stg_bytes > stg_cap ? std::ceil(pc.stg_bytes / stg_cap) : 1.0;
    f[0] = pieces;
    f[1] = pc.handoffs * pieces;
    f[2] = pc.link_time_bytes / 1e3;
    f[3] = (pc.hbm_read + pc.hbm_write) / 1e3;
    return true;
  }

  double cost_us(const AlgoSpec& s, int N, double S, uint32_t esize = 4) const {
    double f[4];
    if (features(s, N, S, f, esize))
      return f[0] * alpha_launch_us + f[1] * alpha_sync_us + f[2] / link_gbps + f[3] / hbm_gbps;
    if (s.kind == AlgoKind::DMA)  // copy engines: CU-free, but a host-enqueued fork/join and 2 stream-memory hand-offs
      return alpha_launch_us + 2.0 * alpha_dma_us + 2.0 * fanout_us_at(S / N, N - 1, dma_link_gbps) + reduce_us(S);
    return 1e30;
  }

  // Program costs of (spec, N, count, esize) for this model's link count, component-wise max over the
  // ranks that differ (lonely trees: every rank; otherwise the schedules are symmetric and rank 0 stands
  // for all). Memoised: the selector prices every candidate once per call shape.
  bool cached_cost(const AlgoSpec& s, int N, double S, uint32_t esize, ProgramCost* out) const {
    const uint64_t count = std::max<uint64_t>(1, (uint64_t)(S / std::max<uint32_t>(1, esize)));
    char key[160];
    snprintf(key, sizeof(key), "|%d|%llu|%u|%d", N, (unsigned long long)count, esize, links);
    const std::string k = s.str() + key;
    static std::mutex mu;
    static std::unordered_map<std::string, std::pair<bool, ProgramCost>> memo;
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = memo.find(k);
      if (it != memo.end()) { *out = it->second.second; return it->second.first; }
    }
    long prod = 1;
    for (int w : s.widths) prod *= w;
    const bool lonely = s.kind == AlgoKind::TREE && prod != N;
    ProgramCost acc;
    bool ok = true;
    for (int r = 0; r < (lonely ? N : 1) && ok; ++r) {
      Program P;
      std::string err;
      Planner pl((uint32_t)N, (uint32_t)r, count, esize, 1.0f);
      if (!pl.build(s, &P, &err)) { ok = false; break; }
      const ProgramCost c = program_cost(P, (uint32_t)r, links);
      acc.stg_bytes = std::max(acc.stg_bytes, c.stg_bytes);
      acc.handoffs = std::max(acc.handoffs, c.handoffs);
      acc.link_bytes = std::max(acc.link_bytes, c.link_bytes);
      acc.link_time_bytes = std::max(acc.link_time_bytes, c.link_time_bytes);
      acc.hbm_read = std::max(acc.hbm_read, c.hbm_read);
      acc.hbm_write = std::max(acc.hbm_write, c.hbm_write);
    }
    std::lock_guard<std::mutex> lk(mu);
    if (memo.size() > 8192) memo.clear();
    memo[k] = {ok, acc};
    *out = acc;
    return ok;
  }

  // Closed-form features for world sizes beyond the device mesh (flexar_plan's reference sweep to N = 999)
  // and the message transport (whose bytes leave through RCCL, not the executor): the round-2 per-schedule
  // formulas, untyped.
  bool analytic_features(const AlgoSpec& s, int N, double S, double f[4]) const {
    auto share = [&](int fan) { return fan <= links ? 1.0 : (double)links / fan; };
    switch (s.kind) {
      case AlgoKind::ONESHOT:
        f[1] = 1.0; f[2] = S / (1e3 * share(N - 1)); f[3] = 2.0 * N * S / 1e3;
        return true;
      case AlgoKind::RING: {
        const int C = s.channels < 1 ? 1 : s.channels;
        const double blk = S / ((double)C * N);
        f[1] = 2.0 * (N - 1); f[2] = 2.0 * (N - 1) * blk / 1e3; f[3] = 2.0 * (N - 1) * 3 * blk * C / 1e3;
        return true;
      }
      case AlgoKind::TREE: {
        double G = 1;
        for (int w : s.widths) {
          G *= w;
          const double per_peer = S / G;
          f[1] += 2.0;
          f[2] += 2.0 * per_peer / (1e3 * share(w - 1));
          f[3] += 2.0 * (w + 1) * per_peer * (G / w) / 1e3;
        }
        return true;
      }
      default:
        return false;
    }
  }
};

// The typed form of an executor schedule for a call (comm.hip typed_spec, the selector): multi-hop
// schedules of 16/8-bit float SUM/AVG carry fp32 partials (wire 1) or round per hop ("+rw") by the
// partials policy; explicit "+f32" / "+rw" in the spec win; everything else runs untyped.
inline void apply_partials(AlgoSpec* s, int N, double S, const CallKind& k, const XgmiModel& m) {
  if (s->wire >= 2 || s->msg) return;
  const bool mh = multihop(*s);
  if (s->wire == 1) {
    if (!(k.narrow_sum && mh)) s->wire = 0;  // nothing to widen
    return;
  }
  if (s->round_wire || !k.narrow_sum || !mh) return;
  switch (m.partials) {
    case Partials::FP32: s->wire = 1; return;
    case Partials::WIRE: s->round_wire = true; return;
    case Partials::AUTO: {
      AlgoSpec f32 = *s, rw = *s;
      f32.wire = 1;
      rw.round_wire = true;
      const double t32 = m.cost_us(f32, N, S, k.esize), trw = m.cost_us(rw, N, S, k.esize);
      *s = (hop_roundings(*s, N) <= kAutoRwMaxRoundings && trw < (1.0 - kAutoRwGain) * t32) ? rw : f32;
      return;
    }
  }
}

// Measured tune table: lines "nranks bytes spec" (bytes = lower bound of the range the spec wins).
struct TuneTable {
  std::map<int, std::map<double, std::string>> rows;
  bool load(const char* path) {
    if (!path || !*path) return false;
    std::ifstream f(path);
    if (!f) return false;
    return parse(f);
  }
  // the same "nranks bytes spec" lines from memory (Communicator.autotune installs its measurements)
  bool load_text(const char* text) {
    if (!text) return false;
    std::istringstream f(text);
    return parse(f);
  }
  bool parse(std::istream& f) {
    std::string line;
    while (std::getline(f, line)) {
      if (line.empty() || line[0] == '#') continue;
      std::istringstream ss(line);
      int n; double b; std::string spec;
      if (ss >> n >> b >> spec) rows[n][b] = spec;
    }
    return !rows.empty();
  }
  bool lookup(int N, double bytes, std::string* spec) const {
    auto it = rows.find(N);
    if (it == rows.end() || it->second.empty()) return false;
    auto jt = it->second.upper_bound(bytes);
    if (jt == it->second.begin()) { *spec = jt->second; return true; }
    --jt;
    *spec = jt->second;
    return true;
  }
};

inline AlgoSpec select_plan(const XgmiModel& m, int N, double bytes, double* best_cost = nullptr,
                            const CallKind& k = CallKind()) {
  AlgoSpec best;
  best.kind = AlgoKind::TREE;
  best.widths = {N};
  double bc = 1e300;
  for (AlgoSpec s : enumerate_plans(N)) {
    if (s.kind == AlgoKind::TREE) s.ag = AgMode::PULL;  // pull-AG avoids the local copy-out
    apply_partials(&s, N, bytes, k, m);                  // priced in the form the call would run
    double c = m.cost_us(s, N, bytes, k.esize);
    if (c < bc) bc = c, best = s;
  }
  if (best_cost) *best_cost = bc;
  return best;
}

// ---- reference cost model (cost_model/CostModel.h), defects D10 fixed ----------------------------
inline double legacy_latency_control_overhead(double chunk, double width) {
  const double lo = 0.004, co = 0.0002;  // CostModel.h:3-4
  return width > 9 ? 2 * lo + chunk * (width - 9) * co : 2 * lo;
}
inline double legacy_bandwidth_overhead(int n, double chunk) {
  const double bo = 0.0068;  // CostModel.h:24
  return ((double)(n - 1) / n) * chunk * bo;
}
// steps = n + 2*(w0) + 2*(w0*w1) + ... over the first height-1 layers, + 1 (CostModel.h:40-78, any height)
inline double legacy_memory_rw_overhead(const std::vector<int>& w, int n, double chunk) {
  const double o = 0.0004;  // CostModel.h:37
  double steps = n + 1;
  double prod = 1;
  for (size_t i = 0; i + 1 < w.size(); ++i) {
    prod *= w[i];
    steps += 2 * prod;
  }
  return steps * chunk / n * o;
}
inline double legacy_cost(const std::vector<int>& w, int n, double chunk) {
  double c = 0;  // D10: the reference accumulates into an uninitialised double
  for (int x : w) c += legacy_latency_control_overhead(chunk, x);  // D10: reference hard-codes 100 here
  c += legacy_memory_rw_overhead(w, n, chunk);
  c += legacy_bandwidth_overhead(n, chunk);
  return c;
}

}  // namespace flexar
