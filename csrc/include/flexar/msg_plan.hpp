// Message transport plan: the op program of one rank rewritten as local executor segments and grouped
// point-to-point messages, for a transport that moves bytes with send/recv instead of peer memory access
// (RCCL ncclSend / ncclRecv on device buffers: comm.hip msg path; host simulator: flexar_simulate_msg).
//
// Reference counterpart: handle_send / handle_recv post one MPI_Isend / MPI_Irecv per (peer, block)
// (allreduce_over_mpi/mpi_mod.hpp:662-765) and every stage waits on them. Here the SAME schedule the
// device executor runs over IPC (planner.hpp) is translated once per (spec, count, dtype):
//  * every XFER destination on a peer becomes a local outbox region; the regions a rank sends one peer
//    between two SIGNALs form ONE message (the reference's per-block sends, coalesced per peer and stage);
//  * a WAIT receives the matching message from each peer: its layout is what the peer's program writes
//    into this rank under that flag slot (replayed from the peer's program), and copy XFERs scatter it to
//    the staging locations the next reduction reads;
//  * consecutive SIGNALs / WAITs form one group (ncclGroupStart/End: every rank posts a stage's sends and
//    receives together, so no ordering of ranks can deadlock), the XFERs between groups one executor
//    launch (a local-only program: one channel, no flags);
//  * zero copy: a single-region message produced by a pure copy is sent straight from its source, and a
//    single-region incoming message lands straight in its staging location.
// Push-form programs only (a pull reads peer memory): trees run with the push all-gather.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "flexar/planner.hpp"

namespace flexar {

struct MsgXfer {
  uint32_t peer = 0;
  uint16_t buf = BUF_STG;  // BUF_IN / BUF_OUT / BUF_STG (the transport's own staging arena)
  uint64_t off = 0;        // byte offset inside buf
  uint64_t bytes = 0;
};

struct MsgStep {
  enum Kind { EXEC = 0, GROUP = 1 } kind = EXEC;
  Program prog;                          // EXEC: local-only XFER program, one channel
  std::vector<MsgXfer> sends, recvs;     // GROUP
};

struct MsgPlan {
  std::vector<MsgStep> steps;
  uint64_t stg_bytes = 0;   // staging arena bytes (program staging + message buffers)
  uint64_t msgs = 0, msg_bytes = 0, zero_copy = 0;  // statistics: messages, bytes sent, zero-copy messages
};

// The regions (staging offsets in units, element lengths) `src`'s program writes into `dst` between two
// SIGNALs, per SIGNAL occurrence (with its flag slot), in program order (channels flattened in order).
// Shared by this transport and the MPI point-to-point engine (mpi_mod.hpp build_p2p): both coalesce the
// same regions into one message per (peer, SIGNAL).
struct MsgRegions {
  uint32_t slot;
  std::vector<std::pair<uint64_t, uint64_t>> regions;  // (staging offset, elements)
};
inline std::vector<MsgRegions> msg_regions(const Program& Q, uint32_t src, uint32_t dst) {
  std::vector<MsgRegions> out;
  std::vector<std::pair<uint64_t, uint64_t>> pend;
  for (const Op& o : Q.ops) {
    if (o.kind == OP_XFER) {
      for (int d = 0; d < o.ndst; ++d)
        if (o.dst[d].rank == dst && dst != src) pend.push_back({o.dst[d].off, o.len});
    } else if (o.kind == OP_SIGNAL) {
      for (int k = 0; k < o.npeers; ++k)
        if (o.peers[k] == dst) {
          out.push_back({o.slot, pend});
          pend.clear();
        }
    }
  }
  return out;
}

inline bool build_msg_plan(uint32_t N, uint32_t r, uint64_t count, uint32_t esize, float scale, AlgoSpec spec,
                           MsgPlan* M, std::string* err, Coll coll = Coll::ALLREDUCE, uint64_t stride = 0) {
  *M = MsgPlan();
  if (spec.kind == AlgoKind::LL) spec.kind = AlgoKind::ONESHOT;
  if (spec.kind == AlgoKind::DMA) spec = AlgoSpec(), spec.kind = AlgoKind::TREE, spec.widths = {(int)N};
  if (spec.kind == AlgoKind::TREE) spec.ag = AgMode::PUSH;  // no peer reads
  spec.wire = 0;
  spec.msg = false;
  spec.zc = false;  // messages carry the bytes: no peer buffer is read
  spec.put = spec.bidir = false;
  std::vector<Program> progs(N);
  for (uint32_t p = 0; p < N; ++p) {
    Planner pl(N, p, count, esize, scale);
    if (!pl.build_coll(coll, spec, stride, &progs[p], err)) return false;
  }
  const Program& P = progs[r];
  const uint64_t es = esize;
  // flattened op order (channel 0 ops, then channel 1, ...): identical on every rank
  std::vector<Op> ops = P.ops;
  for (const Op& o : ops)
    if (o.kind == OP_XFER)
      for (int k = 0; k < o.nsrc; ++k)
        if (o.src[k].rank != r) {
          if (err) *err = "message transport needs a push-form schedule (" + spec.str() + " reads peer memory)";
          return false;
        }
  // incoming message layouts per peer (one entry per SIGNAL of that peer towards r)
  std::vector<std::vector<MsgRegions>> incoming(N);
  std::vector<size_t> next_in(N, 0);
  for (uint32_t p = 0; p < N; ++p)
    if (p != r) incoming[p] = msg_regions(progs[p], p, r);

  uint64_t arena = (P.stg_elems * es + 255) / 256 * 256;  // message buffers after the program's staging
  auto arena_alloc = [&](uint64_t bytes) {
    const uint64_t o = arena;
    arena += (bytes + 255) / 256 * 256;
    return o;
  };
  // pass 1: outgoing messages - per peer, the (op index, dst index) regions since its last SIGNAL
  struct Reg { size_t op; uint32_t peer; uint64_t off; uint64_t bytes; };  // dst identified by (peer, offset)
  std::vector<std::vector<Reg>> pend(N);
  std::map<size_t, std::vector<std::vector<Reg>>> closed;  // SIGNAL op index -> per listed peer regions
  for (size_t i = 0; i < ops.size(); ++i) {
    const Op& o = ops[i];
    if (o.kind == OP_XFER) {
      for (int d = 0; d < o.ndst; ++d)
        if (o.dst[d].rank != r) pend[o.dst[d].rank].push_back({i, o.dst[d].rank, o.dst[d].off, o.len * es});
    } else if (o.kind == OP_SIGNAL) {
      auto& v = closed[i];
      for (int k = 0; k < o.npeers; ++k) {
        v.push_back(pend[o.peers[k]]);
        pend[o.peers[k]].clear();
      }
    }
  }
  // pass 2: decide zero-copy sends, lay out the outbox, patch destinations
  std::vector<bool> drop(ops.size(), false);
  auto find_dst = [&](Op& w, uint32_t peer, uint64_t off) {
    for (int d = 0; d < w.ndst; ++d)
      if (w.dst[d].rank == peer && w.dst[d].off == off) return d;
    return -1;
  };
  std::map<std::pair<size_t, int>, MsgXfer> send_of;  // (SIGNAL op, peer slot k) -> message
  auto writes_overlap = [&](size_t from, size_t to, const Loc& src, uint64_t len) {
    // any op in (from, to) writing the source buffer range (IN and OUT may alias: same user buffer)
    for (size_t j = from + 1; j < to; ++j) {
      const Op& q = ops[j];
      if (q.kind != OP_XFER) continue;
      for (int d = 0; d < q.ndst; ++d) {
        const Loc& w = q.dst[d];
        if (w.rank != r) continue;
        const bool same = w.buf == src.buf || (w.buf != BUF_STG && src.buf != BUF_STG);
        if (same && w.off < src.off + len && src.off < w.off + q.len) return true;
      }
    }
    return false;
  };
  for (auto& kv : closed) {
    const Op& sig = ops[kv.first];
    for (size_t k = 0; k < kv.second.size(); ++k) {
      const auto& regs = kv.second[k];
      MsgXfer m;
      m.peer = sig.peers[k];
      uint64_t total = 0;
      for (const Reg& g : regs) total += g.bytes;
      m.bytes = total;
      bool zc = false;
      // zero copy: every destination of an XFER receives the same value, so a message whose regions are
      // contiguous at the receiver is sent straight from a local copy of the same bytes - the ops' local
      // destinations (e.g. OUT of a reduction) or the sources of pure copies - when those are contiguous
      // too (the digit-reversed tree layout makes every (stage, peer) payload one span, planner.hpp
      // build_tree) and nothing overwrites them before the message goes out
      bool dst_contig = true;
      for (size_t i = 1; i < regs.size() && dst_contig; ++i)
        dst_contig = regs[i - 1].off + regs[i - 1].bytes / es == regs[i].off;
      const Loc* from = nullptr;
      if (dst_contig && !regs.empty()) {
        // candidate source of region i: local destination d (d >= 0) or the copy source (d = -1)
        auto cand = [&](size_t i, int d) -> const Loc* {
          const Op& o = ops[regs[i].op];
          if (d >= 0) return o.dst[d].rank == r ? &o.dst[d] : nullptr;
          return o.nsrc == 1 && o.scale == 1.0f && o.src[0].rank == r ? &o.src[0] : nullptr;
        };
        const Op& o0 = ops[regs[0].op];
        for (int d0 = 0; d0 <= o0.ndst && !from; ++d0) {
          const int sel = d0 < o0.ndst ? d0 : -1;  // local destinations first, then the copy source
          const Loc* first = cand(0, sel);
          if (!first || writes_overlap(regs[0].op, kv.first, *first, ops[regs[0].op].len)) continue;
          uint64_t next = first->off + ops[regs[0].op].len;
          bool ok = true;
          for (size_t i = 1; i < regs.size() && ok; ++i) {
            const Op& o = ops[regs[i].op];
            const Loc* hit = nullptr;
            for (int d = (sel >= 0 ? 0 : -1); d < (sel >= 0 ? o.ndst : 0) && !hit; ++d) {
              const Loc* c = cand(i, d);
              if (c && c->buf == first->buf && c->off == next) hit = c;
            }
            ok = hit && !writes_overlap(regs[i].op, kv.first, *hit, o.len);
            next += o.len;
          }
          if (ok) from = first;
        }
      }
      if (from) {
        m.buf = from->buf;
        m.off = from->off * es;
        zc = true;
        ++M->zero_copy;
        for (const Reg& g : regs) {  // remove the peer destinations (drop an op if nothing else is left)
          Op& w = ops[g.op];
          const int d0 = find_dst(w, g.peer, g.off);
          if (d0 < 0) { if (err) *err = "internal: message region lost"; return false; }
          for (int d = d0; d + 1 < w.ndst; ++d) w.dst[d] = w.dst[d + 1];
          --w.ndst;
          if (w.ndst == 0) drop[g.op] = true;
        }
      }
      if (!zc) {
        m.buf = BUF_STG;
        m.off = arena_alloc(total);
        uint64_t at = m.off;
        for (const Reg& g : regs) {
          // the remote destination becomes the local outbox region (offset in elements of the dtype)
          Op& w = ops[g.op];
          const int d = find_dst(w, g.peer, g.off);
          if (d < 0) { if (err) *err = "internal: message region lost"; return false; }
          w.dst[d].rank = (uint16_t)r;
          w.dst[d].off = at / es;
          at += g.bytes;
        }
      }
      M->msgs++;
      M->msg_bytes += total;
      send_of[{kv.first, k}] = m;
    }
  }
  // pass 3: emit steps
  Program cur;
  auto flush_exec = [&]() {
    if (cur.ops.empty()) return;
    MsgStep s;
    s.kind = MsgStep::EXEC;
    s.prog = cur;
    s.prog.count = count;
    s.prog.esize = esize;
    s.prog.nchan = 1;
    s.prog.chan_start = {0, (uint32_t)cur.ops.size()};
    s.prog.desc = "msg-local";
    M->steps.push_back(s);
    cur.ops.clear();
  };
  std::vector<Op> scatter;  // copies out of inbox regions, prepended to the next executor segment
  for (size_t i = 0; i < ops.size(); ++i) {
    const Op& o = ops[i];
    if (o.kind == OP_XFER) {
      if (drop[i]) continue;
      for (const Op& sc : scatter) cur.ops.push_back(sc);
      scatter.clear();
      cur.ops.push_back(o);
      continue;
    }
    // SIGNAL / WAIT: one group per maximal run of sync ops (scatters of its receives run after it)
    if (M->steps.empty() || M->steps.back().kind != MsgStep::GROUP || !cur.ops.empty()) {
      flush_exec();
      MsgStep g;
      g.kind = MsgStep::GROUP;
      M->steps.push_back(g);
    }
    MsgStep& G = M->steps.back();
    if (o.kind == OP_SIGNAL) {
      for (int k = 0; k < o.npeers; ++k) G.sends.push_back(send_of[{i, (size_t)k}]);
    } else if (o.kind == OP_WAIT) {
      for (int k = 0; k < o.npeers; ++k) {
        const uint32_t p = o.peers[k];
        if (next_in[p] >= incoming[p].size()) {
          if (err) *err = "internal: message plan has more WAITs than the peer's SIGNALs";
          return false;
        }
        const auto& regs = incoming[p][next_in[p]++].regions;
        MsgXfer m;
        m.peer = p;
        bool contig = true;
        for (size_t j = 0; j < regs.size(); ++j) {
          m.bytes += regs[j].second * es;
          if (j) contig = contig && regs[j - 1].first + regs[j - 1].second == regs[j].first;
        }
        if (!regs.empty() && contig) {  // one span of staging: lands in place
          m.buf = BUF_STG;
          m.off = regs[0].first * es;
        } else {
          m.buf = BUF_STG;
          m.off = arena_alloc(m.bytes);
          uint64_t at = m.off;
          for (auto& g : regs) {  // inbox region -> its staging location
            Op c;
            memset(&c, 0, sizeof(c));
            c.kind = OP_XFER;
            c.scale = 1.0f;
            c.nsrc = c.ndst = 1;
            c.len = g.second;
            c.src[0].buf = BUF_STG;
            c.src[0].rank = (uint16_t)r;
            c.src[0].off = at / es;
            c.dst[0].buf = BUF_STG;
            c.dst[0].rank = (uint16_t)r;
            c.dst[0].off = g.first;
            scatter.push_back(c);
            at += g.second * es;
          }
        }
        G.recvs.push_back(m);
      }
    }
  }
  for (const Op& sc : scatter) cur.ops.push_back(sc);
  flush_exec();
  // every executor segment sees the whole arena as its staging
  M->stg_bytes = arena;
  for (auto& s : M->steps)
    if (s.kind == MsgStep::EXEC) s.prog.stg_elems = arena / es;
  return true;
}

}  // namespace flexar
