// Negative control for the ThreadSanitizer run of the host executor (tests/test_sanitizers.py): the same
// SimRun threads (one per workgroup of every rank, ordered only by the programs' SIGNAL / WAIT flags) over
// one channelled schedule, unmodified or with the WAITs of one channel of rank 0 turned into no-ops. The
// unmodified run must be clean; the mutated one must be reported as a data race, which shows the clean
// verdict on every planner program means the flags order every reader after its writer.
//   tsan_negative         -> exit 0, prints "ok"
//   tsan_negative drop    -> ThreadSanitizer reports a race (exit code from TSAN_OPTIONS)
#include "../../csrc/src/capi_host.cpp"

int main(int argc, char** argv) {
  using namespace flexar;
  const bool drop = argc > 1 && std::string(argv[1]) == "drop";
  const int n = 4, grid = 6;
  const size_t count = 4099;
  AlgoSpec s;
  std::string err;
  if (!parse_algo("rhd:3+pull", n, &s, &err)) { fprintf(stderr, "%s\n", err.c_str()); return 2; }
  std::vector<Program> progs(n);
  for (int r = 0; r < n; ++r) {
    Planner pl(n, r, count, sizeof(float), 1.0f);
    if (!pl.build(s, &progs[r], &err)) { fprintf(stderr, "%s\n", err.c_str()); return 2; }
  }
  int dropped = 0;
  if (drop)  // channel 1 of rank 0 no longer waits for its peers' data
    for (uint32_t i = progs[0].chan_start[1]; i < progs[0].chan_start[2]; ++i)
      if (progs[0].ops[i].kind == OP_WAIT) progs[0].ops[i].kind = OP_NOP, ++dropped;
  std::vector<std::vector<float>> in(n, std::vector<float>(count)), out(n, std::vector<float>(count));
  std::vector<const void*> ip(n);
  std::vector<void*> op(n);
  for (int r = 0; r < n; ++r) {
    for (size_t i = 0; i < count; ++i) in[r][i] = (float)((r * 31 + i) % 97);
    ip[r] = in[r].data(), op[r] = out[r].data();
  }
  int rc = SimRun::run<float, OpSum>(progs, n, grid, 2, 0, ip.data(), op.data(), count);
  printf("%s rc=%d dropped=%d\n", rc == 0 ? "ok" : "fail", rc, dropped);
  return rc == 0 ? 0 : 1;
}
