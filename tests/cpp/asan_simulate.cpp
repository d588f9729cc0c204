// Host-code sanitizer driver: the planner, the host executor and the simulator of
// the device protocol built with -fsanitize=address,undefined and run over many algorithms, sizes,
// dtypes and world sizes. The reference's ASan run found a heap-buffer-overflow in its reduce
// (defect D2); this keeps flexar's host code clean. Exit 0 = clean and correct.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "flexar/flexar.h"
#include "flexar/topology.hpp"

int main() {
  int fails = 0, runs = 0;
  std::mt19937 rng(7);
  for (int n : {2, 3, 4, 5, 6, 7, 8, 12}) {
    std::vector<std::pair<std::string, int>> specs = {{"flat", 1}, {"ring", 1}, {"ring:2", 2}, {"oneshot", 1},
                                                      {"flat+push", 1}, {"flat+nofuse", 1}};
    for (auto& p : flexar::enumerate_plans(n))  // trees, multi-channel ones included ("tree:2,2,2:7")
      if (p.kind == flexar::AlgoKind::TREE)
        specs.push_back({p.str() + "+push", p.channels}), specs.push_back({p.str() + "+pull", p.channels});
    for (auto& sc : specs) {
      const std::string& spec = sc.first;
      for (size_t count : {1ul, 7ul, 1000ul, 4099ul}) {
        std::vector<std::vector<float>> in(n, std::vector<float>(count)), out(n, std::vector<float>(count));
        std::vector<double> ref(count, 0.0);
        for (int r = 0; r < n; ++r)
          for (size_t i = 0; i < count; ++i) {
            in[r][i] = (float)(rng() % 1000) / 100.0f;
            ref[i] += in[r][i];
          }
        std::vector<const void*> ip(n);
        std::vector<void*> op(n);
        for (int r = 0; r < n; ++r) ip[r] = in[r].data(), op[r] = out[r].data();
        int grid = sc.second > 1 ? 2 * sc.second : 3;  // whole channels
        int rc = flexar_simulate(spec.c_str(), n, count, FLEXAR_FLOAT32, FLEXAR_SUM, ip.data(), op.data(), grid, 2, 0,
                                 1.0f);
        ++runs;
        bool ok = rc == 0;
        for (int r = 0; r < n && ok; ++r)
          for (size_t i = 0; i < count; ++i)
            if (std::fabs(out[r][i] - ref[i]) > 1e-3) { ok = false; break; }
        if (!ok) {
          ++fails;
          fprintf(stderr, "FAIL n=%d spec=%s count=%zu rc=%d %s\n", n, spec.c_str(), count, rc, flexar_last_error());
        }
      }
    }
  }
  // host reduction: every dtype/op combination at fan-in 1..12
  for (int dt = 0; dt < FLEXAR_NUM_DTYPES; ++dt)
    for (int opx = 0; opx < FLEXAR_NUM_OPS; ++opx)
      for (int k : {1, 3, 12}) {
        size_t es = flexar_dtype_size(dt), count = 333;
        std::vector<std::vector<unsigned char>> src(k, std::vector<unsigned char>(count * es, 1));
        std::vector<unsigned char> dst(count * es);
        std::vector<const void*> sp(k);
        for (int i = 0; i < k; ++i) sp[i] = src[i].data();
        int rc = flexar_reduce_host(dst.data(), sp.data(), k, count, dt, opx, 1.0f);
        (void)rc;  // unsupported combinations return an error code; the point is memory safety
        ++runs;
      }
  printf("asan_simulate: %d runs, %d failures\n", runs, fails);
  return fails ? 1 : 0;
}
