// Host unit test of flexar::validate_program: every planner program is accepted, and each kind of
// corruption a planner bug could produce is rejected before it can reach the GPU.
#include <cstdio>
#include <string>

#include "flexar/planner.hpp"

using namespace flexar;

static int failures = 0;
#define EXPECT(cond, what)                                   \
  do {                                                       \
    if (!(cond)) {                                           \
      std::printf("FAIL: %s (line %d)\n", what, __LINE__);   \
      ++failures;                                            \
    }                                                        \
  } while (0)

static Program plan(const char* spec, uint32_t N, uint32_t r, uint64_t count, Coll coll = Coll::ALLREDUCE,
                    uint64_t stride = 0) {
  AlgoSpec s;
  std::string err;
  if (!parse_algo(spec, N, &s, &err)) std::printf("parse %s: %s\n", spec, err.c_str());
  if (s.kind == AlgoKind::TREE && s.ag == AgMode::AUTO) s.ag = AgMode::PULL;
  Program P;
  Planner pl(N, r, count, 4, 1.0f);
  if (!pl.build_coll(coll, s, coll == Coll::BROADCAST ? 0 : (stride ? stride : count), &P, &err))
    std::printf("build %s: %s\n", spec, err.c_str());
  return P;
}

static bool ok(const Program& P, uint32_t N, uint32_t r, uint64_t in, uint64_t out) {
  std::string err;
  return validate_program(P, N, r, in, out, &err);
}

static int first_xfer(const Program& P) {
  for (size_t i = 0; i < P.ops.size(); ++i)
    if (P.ops[i].kind == OP_XFER) return (int)i;
  return -1;
}
static int first_sync(const Program& P) {
  for (size_t i = 0; i < P.ops.size(); ++i)
    if (P.ops[i].kind == OP_SIGNAL || P.ops[i].kind == OP_WAIT) return (int)i;
  return -1;
}

int main() {
  const char* specs[] = {"flat", "flat+push", "ring", "ring:2", "ring:4", "rhd", "tree:2,4", "tree:4,2+push",
                         "oneshot", "ll", "tree:2,2,2+wt"};
  int checked = 0;
  for (uint32_t N : {2u, 4u, 8u}) {
    for (const char* sp : specs) {
      if (std::string(sp).rfind("tree:2,4", 0) == 0 && N != 8) continue;
      if (std::string(sp).rfind("tree:4,2", 0) == 0 && N != 8) continue;
      if (std::string(sp).rfind("tree:2,2,2", 0) == 0 && N != 8) continue;
      if (std::string(sp) == "ring:4" && N < 8) continue;
      for (uint64_t count : {1ull, 7ull, 1000ull, 1ull << 20}) {
        for (uint32_t r = 0; r < N; ++r) {
          Program P = plan(sp, N, r, count);
          EXPECT(ok(P, N, r, count, count), (std::string("valid ") + sp).c_str());
          ++checked;
        }
      }
    }
    for (Coll c : {Coll::REDUCE_SCATTER, Coll::ALL_GATHER, Coll::ALL_TO_ALL, Coll::BROADCAST}) {
      const uint64_t m = 1000, stride = 1024;  // a piece of a wider call: blocks `stride` apart
      for (uint32_t r = 0; r < N; ++r) {
        Program P = plan("flat", N, r, m, c, stride);
        uint64_t in, out;
        io_extent(c, N, m, c == Coll::BROADCAST ? 0 : stride, &in, &out);
        EXPECT(ok(P, N, r, in, out), "valid collective");
        ++checked;
      }
    }
  }

  // corruptions
  const uint32_t N = 4, r = 1;
  const uint64_t count = 4096;
  Program base = plan("flat", N, r, count);
  EXPECT(ok(base, N, r, count, count), "base");
  int x = first_xfer(base), y = first_sync(base);
  EXPECT(x >= 0 && y >= 0, "base has XFER and SIGNAL/WAIT ops");
  {
    Program P = base;  // caller buffer too small for the program
    EXPECT(!ok(P, N, r, count - 1, count), "IN extent");
    EXPECT(!ok(P, N, r, count, count - 1), "OUT extent");
  }
  {
    Program P = base;
    P.ops[x].src[0].off = P.stg_elems + count;  // past everything
    P.ops[x].src[0].buf = BUF_STG;
    EXPECT(!ok(P, N, r, count, count), "staging offset");
  }
  {
    Program P = base;
    P.ops[x].dst[0].rank = N;  // no such rank
    EXPECT(!ok(P, N, r, count, count), "rank out of range");
  }
  {
    Program P = base;
    P.ops[x].src[0].buf = BUF_IN;
    P.ops[x].src[0].rank = (r + 1) % N;  // a caller buffer on a peer
    P.ops[x].src[0].off = 0;
    EXPECT(!ok(P, N, r, count, count), "IN addressed on a peer");
  }
  {
    Program P = base;
    P.ops[x].nsrc = 0;
    EXPECT(!ok(P, N, r, count, count), "no sources");
    P = base;
    P.ops[x].ndst = kMaxDst + 1;
    EXPECT(!ok(P, N, r, count, count), "too many destinations");
  }
  {
    Program P = base;
    P.ops[y].slot = kProgSlots;  // the dma path's slots
    EXPECT(!ok(P, N, r, count, count), "flag slot");
    P = base;
    P.ops[y].peers[0] = (uint16_t)r;  // signalling itself
    EXPECT(!ok(P, N, r, count, count), "self peer");
    P = base;
    P.ops[y].npeers = kMaxPeersPerOp + 1;
    EXPECT(!ok(P, N, r, count, count), "peer count");
  }
  {
    Program P = base;
    P.chan_start.back() += 1;
    EXPECT(!ok(P, N, r, count, count), "channel table end");
    P = base;
    P.ops[x].kind = 9;
    EXPECT(!ok(P, N, r, count, count), "op kind");
  }
  {
    // fp8 / MX wires: every planner program validates, and an op with a third destination is rejected (the
    // executor instantiates those transfers for 2 destinations only: device_exec.hpp xfer_mx_k / xfer_mxb_k)
    for (const char* sp : {"flat+mxe4m3", "flat+e4m3", "flat+mxe5m2"})
      for (uint32_t n : {2u, 4u, 8u})
        for (uint32_t rr = 0; rr < n; ++rr) {
          Program P = plan(sp, n, rr, 1u << 16);
          EXPECT(ok(P, n, rr, 1u << 16, 1u << 16), (std::string("valid ") + sp).c_str());
          ++checked;
        }
    Program P = plan("flat+mxe4m3", N, r, count);
    int red = -1;
    for (size_t i = 0; i < P.ops.size(); ++i)
      if (P.ops[i].kind == OP_XFER && P.ops[i].nsrc >= 2 && P.ops[i].ndst == 2) red = (int)i;
    EXPECT(red >= 0, "MX reduction with 2 destinations");
    if (red >= 0) {
      Op& o = P.ops[red];
      o.dst[2] = o.dst[1];  // a third (wire) destination, masks kept consistent
      o.ndst = 3;
      o.pad16[1] |= (uint16_t)(((o.pad16[1] >> 1) & 1u) << 2);
      EXPECT(!ok(P, N, r, count, count), "MX op with 3 destinations");
    }
  }
  std::printf("%d programs validated, %d failures\n", checked, failures);
  return failures ? 1 : 0;
}
