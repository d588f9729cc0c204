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
// with those fixed; XgmiModel is the model actually used at run time:
//
//   stage cost  = alpha_sync + bytes_per_peer / (link_bw * min(1, links/(w-1)))
//                 + (w * bytes_per_peer) / hbm_bw              (fused reduce)
//   ring        = 2(N-1) steps of S/(C N) bytes on C concurrent links
//   tree (w_s)  = 2 * sum_s stage(w_s, S / G_s)               (RS + AG)
//   oneshot     = one stage pushing S to N-1 peers, fan-in N reduce
// plus alpha_launch. Parameters are calibrated from measurements
// (FLEXAR_MODEL="alpha_launch,alpha_sync,link_gbps,hbm_gbps,links") and a
// measured tune table overrides the model entirely (FLEXAR_TUNE_FILE).
#pragma once

#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "flexar/topology.hpp"

namespace flexar {

constexpr double kLLMaxBytes = 1 << 20;  // LL protocol only for latency-bound sizes

struct XgmiModel {
  double alpha_launch_us = 6.0;  // kernel launch + first-touch
  double alpha_sync_us = 4.0;    // one signal->wait hand-off incl. release/acquire (measured ~4-5 us, BASELINE §5.8)
  double link_gbps = 64.0;       // usable per-direction bandwidth of one xGMI link (GB/s)
  double hbm_gbps = 4000.0;      // effective local HBM bandwidth of the fused reduce
  int links = 7;                 // point-to-point links per GPU (fully connected 8-GPU node)
  double alpha_dma_us = 15.0;    // copy-engine path: stream fork/join + stream-memory wait/write per phase
  double dma_link_gbps = 50.0;   // one SDMA engine's peer-copy rate

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
    return m;
  }

  // time (us) to move `bytes` to each of `fan` peers concurrently
  double fanout_us(double bytes, int fan) const { return fanout_us_at(bytes, fan, link_gbps); }
  double fanout_us_at(double bytes, int fan, double gbps) const {
    if (fan <= 0 || bytes <= 0) return 0.0;
    double par = fan <= links ? 1.0 : (double)links / fan;  // more peers than links share them
    return bytes / (gbps * 1e3 * par);
  }
  double reduce_us(double bytes_read) const { return bytes_read / (hbm_gbps * 1e3); }

  // The executor schedules' cost is linear in theta = (alpha_launch_us, alpha_sync_us, 1 / link_gbps,
  // 1 / hbm_gbps): cost_us = f . theta with f = (launches, hand-offs, link bytes / (1e3 * link share),
  // HBM bytes / 1e3). features() returns f (false for the copy-engine path and out-of-range LL, which
  // have their own terms); costfit.py fits theta to measured (spec, bytes, us) rows by least squares.
  bool features(const AlgoSpec& s, int N, double S, double f[4]) const {
    auto share = [&](int fan) { return fan <= links ? 1.0 : (double)links / fan; };
    f[0] = 1.0; f[1] = f[2] = f[3] = 0.0;
    if (N <= 1) { f[3] = 2 * S / 1e3; return true; }
    switch (s.kind) {
      case AlgoKind::ONESHOT:
        f[1] = 1.0; f[2] = S / (1e3 * share(N - 1)); f[3] = N * S / 1e3;
        return true;
      case AlgoKind::LL:  // flag-free 8-B {data, epoch} granules: half the hop cost, 2x the bytes
        if (S > kLLMaxBytes) return false;
        f[1] = 0.5; f[2] = 2 * S / (1e3 * share(N - 1)); f[3] = 2 * N * S / 1e3;
        return true;
      case AlgoKind::RING: {  // C rings on distinct links; 2 (N - 1) steps of S / (C N) bytes
        const int C = s.channels < 1 ? 1 : s.channels;
        const double blk = S / ((double)C * N);
        f[1] = 2.0 * (N - 1); f[2] = 2.0 * (N - 1) * blk / 1e3; f[3] = 2.0 * (N - 1) * 2 * blk / 1e3;
        return true;
      }
      case AlgoKind::TREE: {
        double G = 1;
        for (int w : s.widths) {
          G *= w;
          const double per_peer = S / G;
          f[1] += 2.0;
          f[2] += 2.0 * per_peer / (1e3 * share(w - 1));
          f[3] += 2.0 * w * per_peer / 1e3;
        }
        if (s.zc) {  // registered buffers (flat only), no staging writes / reads: pull = a third hand-off
          if (s.put) {  // put: the contributions land in the owners' staging and are read back once
            f[3] *= 0.7;
          } else if (s.ag == AgMode::PUSH) {  // and 3/5 of the staging schedule's HBM bytes (profiles/r2_zc);
            f[3] *= 0.4;               // push = each input byte read once, each result byte written once
          } else {
            f[1] += 1.0;
            f[3] *= 0.6;
          }
          return true;
        }
        if (s.ag == AgMode::PUSH || s.ag == AgMode::AUTO) f[3] += S / 1e3;  // local copy-out of pushed blocks
        return true;
      }
      default:
        return false;
    }
  }

  double cost_us(const AlgoSpec& s, int N, double S) const {
    double f[4];
    if (features(s, N, S, f))
      return f[0] * alpha_launch_us + f[1] * alpha_sync_us + f[2] / link_gbps + f[3] / hbm_gbps;
    if (s.kind == AlgoKind::DMA)  // copy engines: CU-free, but a host-enqueued fork/join and 2 stream-memory hand-offs
      return alpha_launch_us + 2.0 * alpha_dma_us + 2.0 * fanout_us_at(S / N, N - 1, dma_link_gbps) + reduce_us(S);
    return 1e30;
  }
};

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

inline AlgoSpec select_plan(const XgmiModel& m, int N, double bytes, double* best_cost = nullptr) {
  AlgoSpec best;
  best.kind = AlgoKind::TREE;
  best.widths = {N};
  double bc = 1e300;
  for (AlgoSpec s : enumerate_plans(N)) {
    if (s.kind == AlgoKind::TREE) s.ag = AgMode::PULL;  // pull-AG avoids the local copy-out
    double c = m.cost_us(s, N, bytes);
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
