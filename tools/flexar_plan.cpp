// flexar_plan — the offline topology tool of the reference, rebuilt on the
// runtime's own planner/selector (so the tool and the library cannot disagree).
//
// Reference: cost_model/main.cpp:1-27 (sweep N = 1..999 -> numofstru.csv),
// CostModel.h (argmin printout), ChooseWidth.h (prime N -> N+1 / N-1 structures),
// PrintTreeStructure.h ("a*b*c" printing), timer.h (stopwatch).
//
//   flexar_plan model N [bytes]      every candidate plan: reference cost (chunk = bytes/1MiB) and
//                                    xGMI model cost (us); marks both argmins
//   flexar_plan choose N             reference ChooseWidth: structures for N (and N +- 1 if N is prime)
//   flexar_plan sweep [NMAX]         reference main.cpp: "#structures,microseconds" per N (CSV to stdout)
//   flexar_plan dump SPEC N RANK [COUNT]   per-rank op program (Operations::print_ops equivalent)
//   flexar_plan select N BYTES       the runtime's choice
//   flexar_plan cost SPEC N BYTES [ESIZE]  what the compiled programs cost (hand-offs, link / HBM bytes)
//                                    and the model's time, per rank
//   flexar_plan links SPEC N BYTES [RANK]  bytes this rank moves to / from each peer in each phase (between
//                                    hand-offs, all channels together): which xGMI links a schedule drives
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "flexar/cost_model.hpp"
#include "flexar/planner.hpp"
#include "flexar/topology.hpp"

using namespace flexar;

static std::string star(const std::vector<int>& w) {
  std::string s;
  for (size_t i = 0; i < w.size(); ++i) s += (i ? "*" : "") + std::to_string(w[i]);
  return s;
}

static int usage() {
  fprintf(stderr,
          "usage: flexar_plan model N [bytes] | choose N | sweep [NMAX] | dump SPEC N RANK [COUNT] | select N BYTES | links SPEC N BYTES [RANK] |"
          " cost SPEC N BYTES [ESIZE]\n");
  return 2;
}

int main(int argc, char** argv) {
  if (argc < 2) return usage();
  std::string cmd = argv[1];
  XgmiModel m = XgmiModel::from_env();
  if (cmd == "model" && argc >= 3) {
    int n = atoi(argv[2]);
    double bytes = argc > 3 ? atof(argv[3]) : 100.0 * (1 << 20);
    double chunk = bytes / (1 << 20);
    printf("%-22s %14s %14s\n", "plan", "legacy_cost", "xgmi_us");
    std::string best_l, best_x;
    double bl = 1e300, bx = 1e300;
    for (auto& s : enumerate_plans(n)) {
      double x = m.cost_us(s, n, bytes);
      double l = s.kind == AlgoKind::TREE ? legacy_cost(s.widths, n, chunk) : -1;
      printf("%-22s %14.4f %14.2f\n", s.str().c_str(), l, x);
      if (l >= 0 && l < bl) bl = l, best_l = star(s.widths);
      if (x < bx) bx = x, best_x = s.str();
    }
    printf("the optimized tree structure for %d total nodes should be (reference model): %s\n", n, best_l.c_str());
    printf("xGMI runtime model choice for %.0f bytes: %s (%.2f us)\n", bytes, best_x.c_str(), bx);
    return 0;
  }
  if (cmd == "choose" && argc >= 3) {
    int n = atoi(argv[2]);
    auto show = [](int k, const char* suffix) {
      for (auto& w : ordered_factorizations(k)) printf("%s%s\n", star(w).c_str(), suffix);
    };
    if (!is_prime(n)) show(n, "");
    show(n + 1, "-1");  // one lonely rank short of the structure (reference PrintTreeStructure_right)
    show(n - 1, "+1");  // one lonely rank beyond it
    return 0;
  }
  if (cmd == "sweep") {
    int nmax = argc > 2 ? atoi(argv[2]) : 999;
    printf("N,structures,microseconds\n");
    for (int n = 1; n <= nmax; ++n) {
      auto t0 = std::chrono::steady_clock::now();
      auto plans = enumerate_plans(n);
      double best = 1e300;
      for (auto& s : plans) best = std::min(best, m.cost_us(s, n, 100.0 * (1 << 20)));
      double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      printf("%d,%zu,%.1f\n", n, plans.size(), us);
    }
    return 0;
  }
  if (cmd == "dump" && argc >= 5) {
    AlgoSpec s;
    std::string err;
    int n = atoi(argv[3]), r = atoi(argv[4]);
    uint64_t count = argc > 5 ? strtoull(argv[5], nullptr, 0) : 1 << 20;
    if (!parse_algo(argv[2], n, &s, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
    if (s.kind == AlgoKind::AUTO) s = select_plan(m, n, count * 4.0);
    Program P;
    Planner pl(n, r, count, 4, 1.0f);
    if (!pl.build(s, &P, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
    fputs(dump_program(P, r).c_str(), stdout);
    return 0;
  }
  if (cmd == "cost" && argc >= 5) {
    AlgoSpec s;
    std::string err;
    const int n = atoi(argv[3]);
    const double bytes = atof(argv[4]);
    const uint32_t es = argc > 5 ? (uint32_t)atoi(argv[5]) : 4;
    if (!parse_algo(argv[2], n, &s, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
    if (s.kind == AlgoKind::AUTO) s = select_plan(m, n, bytes);
    if (s.kind == AlgoKind::TREE && s.ag == AgMode::AUTO) s.ag = AgMode::PULL;
    printf("%s on %d ranks, %.0f bytes of %u-byte elements, %d links: %.2f us\n", s.str().c_str(), n, bytes, es, m.links,
           m.cost_us(s, n, bytes, es));
    if (s.kind == AlgoKind::LL || s.kind == AlgoKind::DMA) return 0;
    printf("%-6s %10s %16s %18s %16s %16s\n", "rank", "handoffs", "link_bytes", "busiest_link_bytes", "hbm_read",
           "hbm_write");
    for (int r = 0; r < n; ++r) {
      Program P;
      Planner pl(n, r, (uint64_t)(bytes / es), es, 1.0f);
      if (!pl.build(s, &P, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
      const ProgramCost c = program_cost(P, (uint32_t)r, m.links);
      printf("%-6d %10.0f %16.0f %18.0f %16.0f %16.0f\n", r, c.handoffs, c.link_bytes, c.link_time_bytes, c.hbm_read,
             c.hbm_write);
    }
    return 0;
  }
  if (cmd == "links" && argc >= 5) {
    AlgoSpec s;
    std::string err;
    const int n = atoi(argv[3]);
    const double bytes = atof(argv[4]);
    const uint32_t r = argc > 5 ? (uint32_t)atoi(argv[5]) : 0;
    if (!parse_algo(argv[2], n, &s, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
    if (s.kind == AlgoKind::AUTO) s = select_plan(m, n, bytes);
    if (s.kind == AlgoKind::TREE && s.ag == AgMode::AUTO) s.ag = AgMode::PULL;
    if (s.kind == AlgoKind::LL || s.kind == AlgoKind::DMA || (int)r >= n) return usage();
    Program P;
    Planner pl(n, r, (uint64_t)(bytes / 4), 4, 1.0f);
    if (!pl.build(s, &P, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
    std::vector<std::map<uint32_t, double>> ph;
    const ProgramCost c = program_cost(P, r, m.links, &ph);
    printf("%s on %d ranks, rank %u, %.0f bytes (fp32): %zu phases, busiest-link bytes %.0f\n", s.str().c_str(), n, r,
           bytes, ph.size(), c.link_time_bytes);
    printf("%-6s %6s", "phase", "links");
    for (int p = 0; p < n; ++p)
      if ((uint32_t)p != r) printf(" %12s", ("peer " + std::to_string(p)).c_str());
    printf("\n");
    for (size_t i = 0; i < ph.size(); ++i) {
      printf("%-6zu %6zu", i, ph[i].size());
      for (int p = 0; p < n; ++p) {
        if ((uint32_t)p == r) continue;
        auto it = ph[i].find((uint32_t)p);
        printf(" %12.0f", it == ph[i].end() ? 0.0 : it->second);
      }
      printf("\n");
    }
    return 0;
  }
  if (cmd == "select" && argc >= 4) {
    printf("%s\n", select_plan(m, atoi(argv[2]), atof(argv[3])).str().c_str());
    return 0;
  }
  return usage();
}
