// Host-side planner: compiles an AlgoSpec into the per-rank op program
// (program.hpp) that the gfx950 executor kernel, the host simulator and the
// host shared-memory engine all run unchanged.
//
// Schedules (same mathematics as the reference, different mechanics):
//  * TREE (FlexTree mixed radix; flat = {N}; RHD = {2,..,2}):
//      reference Send_Ops/Recv_Ops (mpi_mod.hpp:147-214) + tree_allreduce
//      (mpi_mod.hpp:952-1111). Stage s, g = prod(w_<s), G = g*w_s: rank r's
//      group = ranks differing only in mixed-radix digit s; RS sends member p the
//      blocks k == p (mod G) and reduces the blocks k == r (mod G) with fan-in w_s;
//      AG replays the stages in reverse.
//      New: staging slot per (stage, sender digit, block) so a payload lands at
//      an explicit offset (no tag matching, no global barrier); optional fusion
//      writes a stage's reduce output straight into the next stage's receiver
//      and multicasts all-gather blocks to every later-stage member at once.
//  * RING: reference ring_allreduce (mpi_mod.hpp:1113-1163): N-1 RS steps with
//      block (v - i) mod N, then N-1 AG steps. New: reduce-and-forward fusion
//      (the reduced partial is written directly into the right neighbour's
//      staging) and C arc-disjoint channels so C xGMI links run concurrently.
//  * ONESHOT: new (small messages): multicast the whole buffer to every peer,
//      one wait, fan-in-N reduce.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <sstream>
#include <string>
#include <vector>

#include "flexar/program.hpp"
#include "flexar/topology.hpp"

namespace flexar {

struct Program {
  std::vector<Op> ops;
  std::vector<uint32_t> chan_start;  // nchan + 1 entries into ops
  uint32_t nchan = 1;
  uint64_t stg_elems = 0;            // staging units needed per parity (units of `unit` bytes)
  uint32_t nslots = 0;
  uint64_t count = 0;
  uint32_t esize = 0;
  // Typed operands (AlgoSpec::wire): 0 = every operand has the call's dtype. Otherwise a STG operand
  // whose Loc.pad bit 0 is set holds the wire type (wsize bytes: fp32 partials for wire 1, fp8 for
  // wire 2/3), STG offsets count `unit` = min(esize, wsize) bytes, and every XFER carries its source /
  // destination wire-type masks in pad16[0] / pad16[1] (bit k = operand k).
  int wire = 0;
  uint32_t wsize = 0;
  uint32_t unit = 0;
  // MX wire (wire 4 / 5): the e8m0 scale of the 32-element block of a wire operand at staging byte o lives
  // at byte mx_shadow + o / 32 of the same rank's staging half (offset units; 0 = no shadow)
  uint64_t mx_shadow = 0;
  uint32_t max_nsrc = 0;  // the widest XFER fan-in (typed launches pick a kernel instantiation by it)
  // zero-copy program (AlgoSpec::zc): IN / OUT operands of other ranks address their registered buffers;
  // zc_bufs = which of them the program addresses on a peer (bit BUF_IN, bit BUF_OUT)
  bool zc = false;
  uint32_t zc_bufs = 0;
  std::string desc;
  uint32_t stg_unit() const { return unit ? unit : esize; }
  uint64_t stg_bytes() const { return stg_elems * stg_unit(); }
  // extent (in offset units) of `len` elements at location l
  uint64_t extent(const Loc& l, uint64_t len) const {
    if (!wire || l.buf != BUF_STG) return len;
    return len * ((l.pad & 1) ? wsize : esize) / unit;
  }
};

enum class Coll { ALLREDUCE = 0, REDUCE_SCATTER = 1, ALL_GATHER = 2, BROADCAST = 3, ALL_TO_ALL = 4 };

class Planner {
 public:
  Planner(uint32_t nranks, uint32_t rank, uint64_t count, uint32_t esize, float final_scale)
      : N(nranks), r(rank), count(count), esize(esize), scale(final_scale) {
    align = kStageAlignBytes / esize;
    if (align == 0) align = 1;
  }

  bool build(const AlgoSpec& spec, Program* P, std::string* err) {
    prog = P;
    *P = Program();
    P->count = count;
    P->esize = esize;
    P->chan_start.push_back(0);
    stg = 0;
    if (!set_wire(spec, err)) return false;
    if (N == 1) {  // reference: memcpy unless in place (mpi_mod.hpp:1181-1188)
      if (count) xfer(count, {loc(BUF_IN, r, 0)}, {loc(BUF_OUT, r, 0)}, scale);
      finish_channel();
      P->desc = "copy";
    } else if ((spec.zc || spec.bidir) && spec.channels > 1) {
      if (err) *err = "channels (:C) apply to the staging trees and rings, not to " + spec.str();
      return false;
    } else if (spec.zc) {
      if (wire || spec.msg || !(spec.kind == AlgoKind::TREE && spec.widths.size() == 1 && spec.widths[0] == (int)N)) {
        if (err) *err = "zero-copy (+zc) runs the flat schedule over IPC-registered buffers (no wire type, no +rccl)";
        return false;
      }
      if (spec.put) build_flat_zc_put();
      else build_flat_zc(spec.ag == AgMode::PUSH);
      P->zc = true;
      P->desc = spec.str();
    } else if (spec.bidir) {
      if (wire || spec.msg || !(spec.kind == AlgoKind::TREE && spec.widths.size() == 1 && spec.widths[0] == (int)N)) {
        if (err) *err = "+bidir is the flat schedule over IPC staging (no wire type, no +rccl)";
        return false;
      }
      build_flat_bidir();
      P->desc = spec.str();
    } else if (wire >= 2 && !(spec.kind == AlgoKind::TREE && spec.widths.size() == 1 && spec.widths[0] == (int)N)) {
      if (err) *err = "fp8 wire compression needs the flat schedule (one quantisation per contribution)";
      return false;
    } else if (wire >= 2 && N > kMaxSrc) {
      if (err) *err = "fp8 wire compression supports up to 8 ranks (one reduction of every contribution)";
      return false;
    } else if (spec.kind == AlgoKind::RING) {
      int C = std::max(1, std::min(spec.channels, max_ring_channels(N)));
      if (2ull * (N - 1) * C > kProgSlots) { if (err) *err = "too many ring channels"; return false; }
      build_ring(C);
      P->desc = spec.str();
    } else if (spec.kind == AlgoKind::TREE) {
      long prod = 1;
      for (int w : spec.widths) prod *= w;
      // product == N: plain tree. N/2 <= product < N: the N - product "lonely" ranks fold into
      // partners first (the reference's intended-but-dead lonely-node path, mpi_mod.hpp:1075-1099).
      if (spec.widths.empty() || prod > (long)N || 2 * prod < (long)N) {
        if (err) *err = "tree widths must multiply to N (or to at least N/2 with lonely ranks)";
        return false;
      }
      if (2 * spec.widths.size() + 2 > kProgSlots) { if (err) *err = "too many stages"; return false; }
      for (int w : spec.widths)
        if (w < 2) { if (err) *err = "tree width < 2"; return false; }
      // typed staging: fp32 partials need the fused forms (no partial sum passes through OUT); fp8 wire
      // pulls (one quantised copy of each result instead of a re-quantised multicast)
      const bool pull = spec.ag == AgMode::PULL || wire >= 2, fuse = spec.fuse || wire == 1;
      if (spec.channels > 1) {
        if (prod != (long)N) {
          if (err) *err = "tree channels (tree:...:C, rhd:C) need widths whose product is the world size";
          return false;
        }
        build_tree_channels(spec.widths, std::min(spec.channels, max_tree_channels((int)spec.widths.size())), pull,
                            fuse);
      } else {
        build_tree_lonely(spec.widths, (uint32_t)prod, pull, fuse);
      }
      if (r >= (uint32_t)prod) {
        // A lonely rank allocates only its fold slots, the tree ranks much more. Every rank sizes its
        // pieces (and the MPI engine its shared window) from its own stg_elems, so all ranks must report
        // the same figure: take the tree's (rank 0 is always a tree rank and a partner).
        Program Q;
        Planner twin(N, 0, count, esize, scale);
        if (!twin.build(spec, &Q, err)) return false;
        stg = std::max(stg, Q.stg_elems);
      }
      P->desc = spec.str();
    } else if (wire && spec.kind != AlgoKind::TREE) {
      if (err) *err = "typed staging (" + spec.str() + ") applies to ring / tree / flat schedules only";
      return false;
    } else if (spec.kind == AlgoKind::ONESHOT) {
      build_oneshot();
      P->desc = spec.str();
    } else if (spec.kind == AlgoKind::DMA) {
      // the copy-engine engine runs the flat two-shot exchange (RS push, AG pull) with SDMA copies and
      // stream-ordered flag writes (comm.hip run_dma); this program is its host-executable equivalent
      build_tree_lonely({(int)N}, N, true, true);
      P->desc = spec.str();
    } else if (spec.kind == AlgoKind::LL) {
      // executed by the dedicated LL kernel (no op program): only the staging size is planned
      stg = (uint64_t)N * ((count * esize + 3) / 4) * 8 / esize + align;
      finish_channel();
      P->desc = spec.str();
    } else {
      if (err) *err = "planner needs a concrete algorithm (not auto)";
      return false;
    }
    if (wire >= 4 && N > 1) {  // MX scale shadow: one byte per 32 staging bytes, after the payload
      P->mx_shadow = round_up(stg);
      stg = P->mx_shadow + round_up((stg + kMxBlock - 1) / kMxBlock);
    }
    P->stg_elems = stg;
    P->nchan = (uint32_t)P->chan_start.size() - 1;
    finish_types(*P);
    mark_runs(*P, r);
    return true;
  }

  // Reduce-scatter / all-gather programs. `count` = elements per rank-block (m); `stride` = elements
  // between consecutive rank-blocks of the N*m side (IN for reduce-scatter, OUT for all-gather), so a
  // call can be split into pieces along m. Ring for "ring*", otherwise the direct (flat) exchange.
  // Broadcast: `stride` is the root rank; "oneshot" = direct multicast, otherwise scatter + all-gather.
  bool build_coll(Coll coll, const AlgoSpec& spec, uint64_t stride, Program* P, std::string* err) {
    if (coll == Coll::ALLREDUCE) return build(spec, P, err);
    if (coll == Coll::BROADCAST) {
      if (stride >= N) { if (err) *err = "broadcast root out of range"; return false; }
      prog = P;
      *P = Program();
      P->count = count;
      P->esize = esize;
      P->chan_start.push_back(0);
      stg = 0;
      if (N == 1) {
        if (count) xfer(count, {loc(BUF_IN, r, 0)}, {loc(BUF_OUT, r, 0)}, 1.0f);
        finish_channel();
        P->desc = "copy";
      } else if (spec.zc) {
        build_bcast_zc((uint32_t)stride);
        P->zc = true;
        P->desc = "bcast-zc";
      } else if (spec.kind == AlgoKind::ONESHOT || spec.kind == AlgoKind::LL) {
        build_bcast_direct((uint32_t)stride);
        P->desc = "bcast-direct";
      } else {
        build_bcast_scatter_ag((uint32_t)stride);
        P->desc = "bcast-scatter-ag";
      }
      P->stg_elems = stg;
      P->nchan = (uint32_t)P->chan_start.size() - 1;
      mark_runs(*P, r);
      return true;
    }
    prog = P;
    *P = Program();
    P->count = count;
    P->esize = esize;
    P->chan_start.push_back(0);
    stg = 0;
    // the MX wire (wire 4 / 5) on the flat reduce-scatter (FSDP / ZeRO gradient shards): quantising pushes,
    // the owner's reduction of its own value + N-1 wire contributions into OUT in the dtype
    if (spec.wire) {
      if (spec.wire < 4 || coll != Coll::REDUCE_SCATTER || spec.kind == AlgoKind::RING || spec.zc || spec.msg) {
        if (err) *err = "typed staging on collectives: only the OCP MX wire on the flat reduce-scatter";
        return false;
      }
      if (N > kMaxSrc) { if (err) *err = "MX wire reduce-scatter supports up to 8 ranks"; return false; }
      if (!set_wire(spec, err)) return false;
    }
    const bool ring = spec.kind == AlgoKind::RING && N > 2;
    if (spec.zc && (spec.kind == AlgoKind::RING || spec.msg)) {
      if (err) *err = "zero-copy (+zc) collectives run the direct exchange over IPC-registered buffers";
      return false;
    }
    if (N == 1) {
      if (count) xfer(count, {loc(BUF_IN, r, 0)}, {loc(BUF_OUT, r, 0)}, coll == Coll::REDUCE_SCATTER ? scale : 1.0f);
      finish_channel();
      P->desc = "copy";
    } else if (spec.zc) {
      build_coll_zc(coll, stride);
      P->zc = true;
      P->desc = coll == Coll::ALL_TO_ALL ? "a2a-zc" : coll == Coll::REDUCE_SCATTER ? "rs-zc" : "ag-zc";
    } else if (coll == Coll::ALL_TO_ALL) {
      build_flat_a2a(stride);
      P->desc = "flat-a2a";
    } else if (coll == Coll::REDUCE_SCATTER) {
      ring ? build_ring_rs(stride) : build_flat_rs(stride);
      P->desc = ring ? "ring-rs" : wire ? "flat-rs" + spec.str().substr(spec.str().rfind('+')) : "flat-rs";
    } else {
      ring ? build_ring_ag(stride) : build_flat_ag(stride);
      P->desc = ring ? "ring-ag" : "flat-ag";
    }
    if (wire >= 4 && N > 1) {  // MX scale shadow (see build)
      P->mx_shadow = round_up(stg);
      stg = P->mx_shadow + round_up((stg + kMxBlock - 1) / kMxBlock);
    }
    P->stg_elems = stg;
    P->nchan = (uint32_t)P->chan_start.size() - 1;
    finish_types(*P);
    mark_runs(*P, r);
    return true;
  }

  // Rotatable runs: maximal sequences of consecutive XFERs that each touch a remote rank and are
  // pairwise independent in local memory (no overlap between one op's local destinations and
  // another's local sources/destinations). Executed in a per-workgroup rotated order.
  static void mark_runs(Program& P, uint32_t rank) {
    P.zc_bufs = 0;
    for (const Op& o : P.ops)
      if (o.kind == OP_XFER) {
        for (int k = 0; k < o.nsrc; ++k)
          if (o.src[k].buf != BUF_STG && o.src[k].rank != rank) P.zc_bufs |= 1u << o.src[k].buf;
        for (int k = 0; k < o.ndst; ++k)
          if (o.dst[k].buf != BUF_STG && o.dst[k].rank != rank) P.zc_bufs |= 1u << o.dst[k].buf;
      }
    auto remote = [&](const Op& o) {
      for (int k = 0; k < o.nsrc; ++k) if (o.src[k].rank != rank) return true;
      for (int k = 0; k < o.ndst; ++k) if (o.dst[k].rank != rank) return true;
      return false;
    };
    // any rank: a run may not read what another op of the run writes, locally or in a peer's staging
    auto ovl = [&](const Loc& a, uint64_t la, const Loc& b, uint64_t lb) {
      return a.rank == b.rank && a.buf == b.buf && a.off < b.off + P.extent(b, lb) && b.off < a.off + P.extent(a, la);
    };
    auto indep = [&](const Op& a, const Op& b) {
      for (int i = 0; i < a.ndst; ++i) {
        for (int j = 0; j < b.nsrc; ++j) if (ovl(a.dst[i], a.len, b.src[j], b.len)) return false;
        for (int j = 0; j < b.ndst; ++j) if (ovl(a.dst[i], a.len, b.dst[j], b.len)) return false;
      }
      for (int i = 0; i < b.ndst; ++i)
        for (int j = 0; j < a.nsrc; ++j) if (ovl(b.dst[i], b.len, a.src[j], a.len)) return false;
      return true;
    };
    for (uint32_t c = 0; c < P.nchan; ++c) {
      uint32_t i = P.chan_start[c], end = P.chan_start[c + 1];
      while (i < end) {
        uint32_t j = i;
        while (j < end && P.ops[j].kind == OP_XFER && remote(P.ops[j]) && j - i < 0xffff) {
          bool ok = true;
          for (uint32_t k = i; k < j && ok; ++k) ok = indep(P.ops[k], P.ops[j]);
          if (!ok) break;
          ++j;
        }
        if (j - i > 1) P.ops[i].run = (uint16_t)(j - i);
        i = (j > i) ? j : i + 1;
      }
    }
  }

 private:
  uint32_t N, r;
  uint64_t count;
  uint32_t esize;
  float scale;
  uint64_t align;
  uint64_t stg = 0;
  Program* prog = nullptr;
  int wire = 0;        // AlgoSpec::wire of the program being built
  uint32_t wsize = 0;  // bytes of a wire-typed element
  uint32_t unit = 0;   // bytes per staging offset unit

  // Typed staging setup (see Program::wire). Offsets of STG operands count `unit` bytes, IN/OUT
  // operands stay in elements of the call's dtype.
  bool set_wire(const AlgoSpec& spec, std::string* err) {
    wire = spec.wire;
    if (wire < 0 || wire > 5) { if (err) *err = "bad wire type"; return false; }
    if (wire == 1 && esize >= 4) wire = 0;  // fp32 (or wider) partials already: nothing to widen
    wsize = wire == 1 ? 4u : (wire >= 2 ? 1u : esize);
    if (wire >= 2 && esize < 2) { if (err) *err = "fp8 wire compression needs a 16/32-bit float input"; return false; }
    unit = wire ? std::min(esize, wsize) : esize;
    align = std::max<uint64_t>(1, kStageAlignBytes / unit);
    prog->wire = wire;
    prog->wsize = wire ? wsize : 0;
    prog->unit = wire ? unit : 0;
    return true;
  }

  static Loc loc(uint16_t buf, uint32_t rank, uint64_t off) {
    Loc l;
    l.buf = buf;
    l.rank = (uint16_t)rank;
    l.pad = 0;
    l.off = off;
    return l;
  }
  // a staging location holding the wire type (fp32 partial sums in wire mode 1)
  static Loc wloc(uint32_t rank, uint64_t off) {
    Loc l = loc(BUF_STG, rank, off);
    l.pad = 1;
    return l;
  }
  uint64_t round_up(uint64_t x) const { return (x + align - 1) / align * align; }
  // staging for `elems` elements of the program's default staging type (in units): the call's dtype,
  // or fp8 in wire modes 2/3 where every staging operand carries the wire type
  uint64_t alloc(uint64_t elems) {
    uint64_t o = stg;
    stg += round_up(wire == 1 ? elems * esize / unit : elems);
    return o;
  }
  uint64_t talloc(uint64_t elems) {  // staging for `elems` elements of the call's dtype, any mode
    uint64_t o = stg;
    stg += round_up(wire ? elems * esize / unit : elems);
    return o;
  }
  uint64_t walloc(uint64_t elems) {  // staging for `elems` wire-typed elements (in units)
    uint64_t o = stg;
    stg += round_up(wire ? elems * wsize / unit : elems);
    return o;
  }
  // element span -> offset units, for a typed slot
  uint64_t wunits(uint64_t elems) const { return wire ? elems * wsize / unit : elems; }
  uint64_t tunits(uint64_t elems) const { return wire ? elems * esize / unit : elems; }

  // Final typing pass: fp8 wire = every staging operand carries the wire type; per-XFER masks.
  void finish_types(Program& P) const {
    for (const Op& o : P.ops)
      if (o.kind == OP_XFER) P.max_nsrc = std::max<uint32_t>(P.max_nsrc, o.nsrc);
    if (!wire) return;
    for (Op& o : P.ops) {
      if (o.kind != OP_XFER) continue;
      uint16_t sm = 0, dm = 0;
      for (int k = 0; k < o.nsrc; ++k) {
        if (wire >= 2 && o.src[k].buf == BUF_STG && !(o.src[k].pad & 2)) o.src[k].pad = 1;
        if (o.src[k].pad & 1) sm |= (uint16_t)(1u << k);
      }
      for (int k = 0; k < o.ndst; ++k) {
        if (wire >= 2 && o.dst[k].buf == BUF_STG && !(o.dst[k].pad & 2)) o.dst[k].pad = 1;
        if (o.dst[k].pad & 1) dm |= (uint16_t)(1u << k);
      }
      o.pad16[0] = sm;
      o.pad16[1] = dm;
    }
  }
  void finish_channel() { prog->chan_start.push_back((uint32_t)prog->ops.size()); }

  void push(const Op& o) { prog->ops.push_back(o); }

  static Op blank(uint16_t kind) {
    Op o;
    memset(&o, 0, sizeof(o));
    o.kind = kind;
    o.scale = 1.0f;
    return o;
  }

  void sync_op(uint16_t kind, const std::vector<uint32_t>& peers, uint32_t slot) {
    if (slot + 1 > prog->nslots) prog->nslots = slot + 1;
    for (size_t i = 0; i < peers.size(); i += kMaxPeersPerOp) {
      Op o = blank(kind);
      o.slot = slot;
      size_t n = std::min<size_t>(kMaxPeersPerOp, peers.size() - i);
      o.npeers = (uint16_t)n;
      for (size_t j = 0; j < n; ++j) o.peers[j] = (uint16_t)peers[i + j];
      if (n) push(o);
    }
  }
  void signal(const std::vector<uint32_t>& peers, uint32_t slot) { sync_op(OP_SIGNAL, peers, slot); }
  void wait(const std::vector<uint32_t>& peers, uint32_t slot) { sync_op(OP_WAIT, peers, slot); }

  // dsts = scale * OP(srcs). Splits fan-in > kMaxSrc through a local temp and
  // fan-out > kMaxDst into follow-up copies from the first (local) destination.
  void xfer(uint64_t len, std::vector<Loc> srcs, std::vector<Loc> dsts, float sc) {
    if (len == 0 || srcs.empty() || dsts.empty()) return;
    if (srcs.size() > kMaxSrc) {
      // partial-sum temp: fp32 in wire mode 1, the call's dtype otherwise (never fp8: pad bit 1 keeps
      // finish_types from retyping it)
      Loc tmp = wire == 1 ? wloc(r, walloc(len)) : loc(BUF_STG, r, talloc(len));
      if (wire >= 2) tmp.pad = 2;
      std::vector<Loc> first(srcs.begin(), srcs.begin() + kMaxSrc);
      emit_xfer(len, first, {tmp}, 1.0f);
      size_t i = kMaxSrc;
      while (srcs.size() - i > kMaxSrc - 1) {
        std::vector<Loc> nxt{tmp};
        nxt.insert(nxt.end(), srcs.begin() + i, srcs.begin() + i + (kMaxSrc - 1));
        emit_xfer(len, nxt, {tmp}, 1.0f);
        i += kMaxSrc - 1;
      }
      std::vector<Loc> last{tmp};
      last.insert(last.end(), srcs.begin() + i, srcs.end());
      srcs = last;
    }
    if (dsts.size() > kMaxDst) {
      if (srcs.size() == 1 && sc == 1.0f) {  // pure copy: every chunk of destinations reads the source
        for (size_t i = 0; i < dsts.size(); i += kMaxDst) {
          std::vector<Loc> part(dsts.begin() + i, dsts.begin() + std::min(dsts.size(), i + kMaxDst));
          emit_xfer(len, srcs, part, 1.0f);
        }
        return;
      }
      // reduction: materialise once in a LOCAL location, then fan out from it (never read back
      // through a peer's staging)
      std::stable_partition(dsts.begin(), dsts.end(), [&](const Loc& l) { return l.rank == r; });
      if (dsts[0].rank != r) dsts.insert(dsts.begin(), loc(BUF_STG, r, alloc(len)));
      std::vector<Loc> head(dsts.begin(), dsts.begin() + kMaxDst);
      emit_xfer(len, srcs, head, sc);
      Loc from = head[0];
      for (size_t i = kMaxDst; i < dsts.size(); i += kMaxDst) {
        std::vector<Loc> more(dsts.begin() + i, dsts.begin() + std::min(dsts.size(), i + kMaxDst));
        emit_xfer(len, {from}, more, 1.0f);
      }
      return;
    }
    emit_xfer(len, srcs, dsts, sc);
  }
  void emit_xfer(uint64_t len, const std::vector<Loc>& srcs, const std::vector<Loc>& dsts, float sc) {
    Op o = blank(OP_XFER);
    o.len = len;
    o.scale = sc;
    o.nsrc = (uint8_t)srcs.size();
    o.ndst = (uint8_t)dsts.size();
    for (size_t i = 0; i < srcs.size(); ++i) o.src[i] = srcs[i];
    for (size_t i = 0; i < dsts.size(); ++i) o.dst[i] = dsts[i];
    push(o);
  }

  // ------------------------------------------------------------------ ring
  void build_ring(int C) {
    // Partition the buffer into C aligned channel ranges.
    uint64_t per = round_up((count + C - 1) / C);
    uint32_t slots_per = 2 * (N - 1);
    for (int c = 0; c < C; ++c) {
      uint64_t c_off = std::min<uint64_t>(count, (uint64_t)c * per);
      uint64_t c_cnt = std::min<uint64_t>(count - c_off, per);
      std::vector<int> ord = ring_order(N, c, C);
      uint32_t v = 0;
      for (uint32_t p = 0; p < N; ++p)
        if ((uint32_t)ord[p] == r) v = p;
      uint32_t right = ord[(v + 1) % N], left = ord[(v + N - 1) % N];
      uint64_t split = round_up((c_cnt + N - 1) / N);
      auto boff = [&](uint32_t k) { return c_off + (uint64_t)k * split; };
      auto blen = [&](uint32_t k) -> uint64_t {
        uint64_t s = (uint64_t)k * split;
        return s >= c_cnt ? 0 : std::min(split, c_cnt - s);
      };
      // Every rank computes the same staging layout (same sequence of allocs). Wire mode 1: the RS slots
      // that receive partial sums (i >= 1) hold fp32; slot 0 (a raw input) and the AG slots the dtype.
      const bool acc = wire == 1;
      uint64_t base = alloc((uint64_t)N * split);            // rs slot 0 + N - 1 AG slots
      uint64_t wbase = acc ? walloc((uint64_t)(N - 2) * split) : 0;  // rs slots 1 .. N - 2
      if (!acc) base = (alloc((uint64_t)(N - 2) * split), base);     // same extent as before: 2 (N - 1) slots
      auto rs_loc = [&](uint32_t rank, uint32_t i) {
        if (acc && i >= 1) return wloc(rank, wbase + (uint64_t)(i - 1) * wunits(split));
        return loc(BUF_STG, rank, i == 0 ? base : base + (uint64_t)(N + i - 1) * split);
      };
      auto ag_off = [&](uint32_t i) { return base + (uint64_t)(1 + i) * split; };
      uint32_t slot0 = c * slots_per;
      auto mod = [&](long x) { return (uint32_t)(((x % (long)N) + N) % N); };

      uint32_t b0 = v;
      xfer(blen(b0), {loc(BUF_IN, r, boff(b0))}, {rs_loc(right, 0)}, 1.0f);
      signal({right}, slot0 + 0);
      for (uint32_t i = 0; i + 1 < N; ++i) {
        wait({left}, slot0 + i);
        uint32_t b = mod((long)v - 1 - (long)i);
        std::vector<Loc> srcs{loc(BUF_IN, r, boff(b)), rs_loc(r, i)};
        if (i + 2 < N) {
          xfer(blen(b), srcs, {rs_loc(right, i + 1)}, 1.0f);
        } else {  // owned block (v + 1): final value -> OUT and start the all-gather
          xfer(blen(b), srcs, {loc(BUF_OUT, r, boff(b)), loc(BUF_STG, right, ag_off(0))}, scale);
        }
        signal({right}, slot0 + i + 1);
      }
      for (uint32_t i = 0; i + 1 < N; ++i) {
        wait({left}, slot0 + (N - 1) + i);
        uint32_t b = mod((long)v - (long)i);
        if (i + 2 < N) {
          xfer(blen(b), {loc(BUF_STG, r, ag_off(i))}, {loc(BUF_OUT, r, boff(b)), loc(BUF_STG, right, ag_off(i + 1))},
               1.0f);
          signal({right}, slot0 + N + i);
        } else {
          xfer(blen(b), {loc(BUF_STG, r, ag_off(i))}, {loc(BUF_OUT, r, boff(b))}, 1.0f);
        }
      }
      finish_channel();
    }
  }

  // ------------------------------------------------------------------ tree
  struct Stage {
    uint32_t w, g, G, base, myj;
    std::vector<uint32_t> members;  // index j -> rank
    std::vector<uint32_t> others() const {
      std::vector<uint32_t> o;
      for (uint32_t jj = 1; jj < w; ++jj) o.push_back(members[(myj + jj) % w]);  // rotated: spreads links
      return o;
    }
  };

  // Lonely folding around the tree: rank P + i (i < L = N - P) pushes its input to partner i,
  // partner i pre-reduces it into OUT, runs the tree from OUT, then pushes the result back.
  void build_tree_lonely(const std::vector<int>& widths, uint32_t P, bool pull, bool fuse) {
    const uint32_t L = N - P, S = (uint32_t)widths.size();
    // every span below uses the tree's block geometry, so each grid block touches exactly the
    // slices it later reads/writes in the tree (no cross-workgroup dependency)
    const uint64_t split = round_up((count + P - 1) / P);
    auto blen = [&](uint32_t k) -> uint64_t {
      uint64_t s0 = (uint64_t)k * split;
      return s0 >= count ? 0 : std::min(split, count - s0);
    };
    uint64_t lone_in = 0, lone_out = 0;
    if (L) {
      lone_in = alloc((uint64_t)P * split);
      lone_out = alloc((uint64_t)P * split);
    }
    const uint32_t s_in = 2 * S, s_out = 2 * S + 1;
    if (r >= P) {  // lonely rank: ship input, wait for the result
      uint32_t partner = r - P;
      for (uint32_t k = 0; k < P; ++k)
        xfer(blen(k), {loc(BUF_IN, r, k * split)}, {loc(BUF_STG, partner, lone_in + k * split)}, 1.0f);
      signal({partner}, s_in);
      wait({partner}, s_out);
      for (uint32_t k = 0; k < P; ++k)
        xfer(blen(k), {loc(BUF_STG, r, lone_out + k * split)}, {loc(BUF_OUT, r, k * split)}, 1.0f);
      finish_channel();
      return;
    }
    uint16_t first = BUF_IN;
    if (r < L) {  // partner: fold the lonely rank's input in first
      wait({r + P}, s_in);
      for (uint32_t k = 0; k < P; ++k)
        xfer(blen(k), {loc(BUF_IN, r, k * split), loc(BUF_STG, r, lone_in + k * split)}, {loc(BUF_OUT, r, k * split)},
             1.0f);
      first = BUF_OUT;
    }
    build_tree(widths, P, first, pull, fuse);
    if (r < L) {
      for (uint32_t k = 0; k < P; ++k)
        xfer(blen(k), {loc(BUF_OUT, r, k * split)}, {loc(BUF_STG, r + P, lone_out + k * split)}, 1.0f);
      signal({r + P}, s_out);
    }
    finish_channel();
  }

  // Link-balanced multi-channel tree ("rhd:C", "tree:a,b:C"): channel c runs the tree on its own aligned
  // slice of the buffer, in logical ranks relabelled by tree_channel_labels (topology.hpp), with its own
  // staging and its own flag slots. Same blocks, same fan-ins, same hand-off count as the one-channel tree;
  // in every stage the C channels' groups cover the xGMI links evenly instead of loading w_s - 1 of them.
  void build_tree_channels(const std::vector<int>& widths, int C, bool pull, bool fuse) {
    const uint32_t S = (uint32_t)widths.size();
    const auto& labels = tree_channel_labels((int)N, widths, C);
    const uint64_t per = round_up((count + C - 1) / C);
    for (int c = 0; c < C; ++c) {
      const uint64_t c_off = std::min<uint64_t>(count, (uint64_t)c * per);
      const uint64_t c_cnt = std::min<uint64_t>(count - c_off, per);
      build_tree(widths, N, BUF_IN, pull, fuse, &labels[c], c_off, c_cnt, (uint32_t)c * 2 * S);
      finish_channel();
    }
  }

  // One tree over ranks [0, N) (N = the tree ranks' count when lonely ranks fold in). `phys` relabels it:
  // the schedule is built in logical ranks and logical rank l is physical rank (*phys)[l] (null = identity).
  // [c_off, c_off + c_cnt) is the slice of the buffer it reduces, slot0 its first flag slot.
  void build_tree(const std::vector<int>& widths, const uint32_t N, uint16_t first, bool pull, bool fuse,
                  const std::vector<uint32_t>* phys = nullptr, uint64_t c_off = 0, uint64_t c_cnt = ~0ull,
                  uint32_t slot0 = 0) {
    const uint32_t S = (uint32_t)widths.size();
    const uint64_t cnt = c_cnt == ~0ull ? count : c_cnt;
    uint64_t split = round_up((cnt + N - 1) / N);
    std::vector<uint32_t> lab(N), lg(std::max<uint32_t>(N, this->N));
    for (uint32_t l = 0; l < N; ++l) lab[l] = phys ? (*phys)[l] : l;
    for (uint32_t l = 0; l < N; ++l) lg[lab[l]] = l;
    const uint32_t lr = lg[r];  // this rank's logical rank
    std::vector<Stage> st(S);
    uint32_t g = 1;
    for (uint32_t s = 0; s < S; ++s) {
      Stage& x = st[s];
      x.w = widths[s];
      x.g = g;
      x.G = g * x.w;
      x.base = lr / x.G * x.G + lr % g;
      x.myj = (lr / g) % x.w;
      for (uint32_t j = 0; j < x.w; ++j) x.members.push_back(lab[x.base + j * g]);  // physical ranks
      g = x.G;
    }
    auto digit = [&](uint32_t l, uint32_t s) { return (l / st[s].g) % st[s].w; };  // of a logical index
    // Digit-reversed block placement: block k, with mixed-radix digits d_s = digit(k, s),
    // lives at physical block pos(k) = sum_s d_s * N / G_s (the stage-0 digit most significant). The blocks
    // a stage-s member sends one peer (k == p mod G_s: digits 0..s fixed) are then ONE contiguous span of
    // the buffer, and the slot index pos(k) mod (N / G_s) keeps their staging slots contiguous in the same
    // order: one region per (stage, peer) message (msg_plan.hpp sends it in place, zero copy). Flat (one
    // stage) is the identity. Ops stay one per block: the executor slices every op over the workgroups, so
    // all ops touching a block must share its span for each workgroup to read only what it wrote.
    std::vector<uint32_t> pos(N, 0);
    for (uint32_t k = 0; k < N; ++k)
      for (uint32_t s = 0; s < S; ++s) pos[k] += digit(k, s) * (N / st[s].G);
    auto rel = [&](uint32_t k) { return (uint64_t)pos[k] * split; };  // offset of block k in the slice
    auto boff = [&](uint32_t k) { return c_off + rel(k); };
    auto blen = [&](uint32_t k) -> uint64_t {
      uint64_t s = rel(k);
      return s >= cnt ? 0 : std::min(split, cnt - s);
    };
    auto sidx = [&](uint32_t s, uint32_t k) { return (uint64_t)(pos[k] % (N / st[s].G)); };
    // blocks of (physical) member p at stage s: k == logical(p) (mod G_s), in buffer order
    auto blocks_of = [&](uint32_t p, uint32_t s) {
      std::vector<uint32_t> b;
      for (uint32_t k = lg[p] % st[s].G; k < N; k += st[s].G) b.push_back(k);
      std::sort(b.begin(), b.end(), [&](uint32_t a, uint32_t c) { return pos[a] < pos[c]; });
      return b;
    };
    // Staging layout (identical on every rank): rs[s], ag[s] (push) or pub (pull). Wire mode 1: the RS
    // slots of stages s >= 1 receive partial sums and hold fp32 (slot stride in units scales with it);
    // a rank's own partial for stage s + 1 goes to its own (otherwise unused) slot of that stage.
    const bool acc = wire == 1;
    auto slot_units = [&](uint32_t s) { return acc && s > 0 ? wunits(split) : split; };
    std::vector<uint64_t> rs_base(S), ag_base(S);
    for (uint32_t s = 0; s < S; ++s)
      rs_base[s] = acc && s > 0 ? walloc((uint64_t)st[s].w * (N / st[s].G) * split)
                                : alloc((uint64_t)st[s].w * (N / st[s].G) * split);
    uint64_t pub_base = 0;
    if (pull) pub_base = alloc((uint64_t)N * split);
    else
      for (uint32_t s = 0; s < S; ++s) ag_base[s] = alloc((uint64_t)st[s].w * (N / st[s].G) * split);
    auto rs_off = [&](uint32_t s, uint32_t j, uint32_t k) {
      return rs_base[s] + ((uint64_t)j * (N / st[s].G) + sidx(s, k)) * slot_units(s);
    };
    auto rs_loc = [&](uint32_t s, uint32_t rank, uint32_t j, uint32_t k) {
      return acc && s > 0 ? wloc(rank, rs_off(s, j, k)) : loc(BUF_STG, rank, rs_off(s, j, k));
    };
    // this rank's running value of block k entering stage s
    auto own_at = [&](uint32_t s, uint32_t k, uint16_t first_buf) {
      if (s == 0) return loc(first_buf, r, boff(k));
      return acc ? rs_loc(s, r, st[s].myj, k) : loc(BUF_OUT, r, boff(k));
    };
    auto ag_off = [&](uint32_t s, uint32_t j, uint32_t k) {
      return ag_base[s] + ((uint64_t)j * (N / st[s].G) + sidx(s, k)) * split;
    };
    auto pub_off = [&](uint32_t k) { return pub_base + rel(k); };
    // (physical) rank in stage-s group of `r` that owns block k after stage s
    auto owner_at = [&](uint32_t k, uint32_t s) { return lab[st[s].base + digit(k, s) * st[s].g]; };

    // ---------------- reduce-scatter
    for (uint32_t s = 0; s < S; ++s) {
      const Stage& x = st[s];
      bool sends_fused = fuse && s > 0;  // previous stage already wrote our sends into the receivers
      if (!sends_fused) {
        for (uint32_t p : x.others())
          for (uint32_t k : blocks_of(p, s)) xfer(blen(k), {own_at(s, k, first)}, {rs_loc(s, p, x.myj, k)}, 1.0f);
      }
      signal(x.others(), slot0 + s);
      wait(x.others(), slot0 + s);
      bool last = (s + 1 == S);
      for (uint32_t k : blocks_of(r, s)) {
        std::vector<Loc> srcs{own_at(s, k, first)};
        for (uint32_t jj = 1; jj < x.w; ++jj) {
          uint32_t j = (x.myj + jj) % x.w;
          srcs.push_back(rs_loc(s, r, j, k));
        }
        std::vector<Loc> dsts;
        if (!last) {
          uint32_t p = owner_at(k, s + 1);
          if (fuse && p != r) dsts.push_back(rs_loc(s + 1, p, st[s + 1].myj, k));
          else if (acc) dsts.push_back(rs_loc(s + 1, r, st[s + 1].myj, k));
          else dsts.push_back(loc(BUF_OUT, r, boff(k)));
          xfer(blen(k), srcs, dsts, 1.0f);
        } else {
          dsts.push_back(loc(BUF_OUT, r, boff(k)));
          if (pull) {
            dsts.push_back(loc(BUF_STG, r, pub_off(k)));
          } else if (fuse) {  // multicast the final block to every member of every AG stage
            for (uint32_t t = 0; t < S; ++t)
              for (uint32_t p : st[t].others()) dsts.push_back(loc(BUF_STG, p, ag_off(t, st[t].myj, k)));
          }
          xfer(blen(k), srcs, dsts, scale);
        }
      }
    }
    // ---------------- all-gather (stages in reverse)
    for (int si = (int)S - 1; si >= 0; --si) {
      uint32_t s = (uint32_t)si;
      const Stage& x = st[s];
      uint32_t slot = slot0 + S + s;
      if (pull) {
        signal(x.others(), slot);  // my pub holds blocks_of(r, s)
        wait(x.others(), slot);
        for (uint32_t p : x.others())
          for (uint32_t k : blocks_of(p, s)) {
            std::vector<Loc> dsts{loc(BUF_OUT, r, boff(k))};
            if (s > 0) dsts.push_back(loc(BUF_STG, r, pub_off(k)));
            xfer(blen(k), {loc(BUF_STG, p, pub_off(k))}, dsts, 1.0f);
          }
      } else {
        if (!fuse) {
          for (uint32_t k : blocks_of(r, s)) {
            std::vector<Loc> dsts;
            for (uint32_t p : x.others()) dsts.push_back(loc(BUF_STG, p, ag_off(s, x.myj, k)));
            xfer(blen(k), {loc(BUF_OUT, r, boff(k))}, dsts, 1.0f);
          }
        }
        signal(x.others(), slot);
        wait(x.others(), slot);
        for (uint32_t p : x.others()) {
          uint32_t j = digit(lg[p], s);
          for (uint32_t k : blocks_of(p, s)) {
            std::vector<Loc> dsts{loc(BUF_OUT, r, boff(k))};
            if (fuse)  // forward to every member of every lower AG stage right away
              for (uint32_t t = 0; t < s; ++t)
                for (uint32_t q : st[t].others()) dsts.push_back(loc(BUF_STG, q, ag_off(t, st[t].myj, k)));
            xfer(blen(k), {loc(BUF_STG, r, ag_off(s, j, k))}, dsts, 1.0f);
          }
        }
      }
    }
  }

  // Zero-copy flat allreduce over registered buffers ("+zc"): no staging and no copies into it. Rank k
  // reduces block k straight from every rank's IN (remote loads over xGMI; rank order, so every owner
  // sums in the same order). The reference's flat exchange (mpi_mod.hpp:952-1111 with one stage of width
  // N) moves the same bytes through send/recv buffers; here HBM sees each byte far fewer times.
  //  pull (default): the owner writes its own OUT, then every rank copies the other blocks from their
  //    owners' OUT. Three hand-offs, per workgroup like every flag: slot 0 "my IN is final" (every rank
  //    has entered the call), slot 1 "my block is reduced" (and I have read your IN), slot 2 "I have read
  //    your OUT" - the last keeps a rank in the call until no peer can still read its buffers, so its
  //    caller may overwrite them as soon as the call completes on its stream.
  //  push ("+zc+push"): the owner writes the reduced block into its own OUT and every peer's OUT (remote
  //    stores) - each input byte is read once and each result byte written once per rank. Two hand-offs:
  //    slot 0 as above, slot 1 "I have read your IN and written your block".
  // In place (IN == OUT) is safe in both: block k of a rank's IN is read only by its owner k, which
  // writes that rank's block k (push) or lets it be overwritten (pull, after slot 1) only afterwards.
  void build_flat_zc(bool push) {
    const uint64_t split = round_up((count + N - 1) / N);
    auto boff = [&](uint32_t k) { return (uint64_t)k * split; };
    auto blen = [&](uint32_t k) -> uint64_t {
      const uint64_t s = boff(k);
      return s >= count ? 0 : std::min(split, count - s);
    };
    auto peers = rotated_peers();
    signal(peers, 0);
    wait(peers, 0);
    std::vector<Loc> srcs;
    for (uint32_t p = 0; p < N; ++p) srcs.push_back(loc(BUF_IN, p, boff(r)));
    std::vector<Loc> dsts{loc(BUF_OUT, r, boff(r))};
    if (push)
      for (uint32_t p : peers) dsts.push_back(loc(BUF_OUT, p, boff(r)));
    xfer(blen(r), srcs, dsts, scale);
    signal(peers, 1);
    wait(peers, 1);
    if (!push) {
      for (uint32_t p : peers) xfer(blen(p), {loc(BUF_OUT, p, boff(p))}, {loc(BUF_OUT, r, boff(p))}, 1.0f);
      signal(peers, 2);
      wait(peers, 2);
    }
    finish_channel();
  }

  // Direction-balanced flat over staging ("flat+bidir"): the staging twin of "+zc+push". The staging flat
  // schedules move the reduce-scatter and the all-gather in SEPARATE phases, each in one link direction
  // (RS push = outgoing, then AG pull = incoming, or both outgoing), so one direction idles at a time.
  // Here one XFER does both: every rank first copies its IN blocks p != r into its own staging (local
  // HBM, ~S of 8 TB/s), then owner r pulls block r from every peer's copy (incoming) and writes the reduced
  // block into its OUT and every peer's landing slot r (outgoing) - both directions of all N - 1 links
  // busy at once - and finally copies the landed blocks into OUT (local). Two hand-offs: slot 0 "my IN
  // copy is published", slot 1 "your landing slot r holds my block" (and I have read your copy). In place
  // is safe: peers read the copy, never IN, and this rank writes OUT block p != r only from the landing
  // slots after slot 1. Rank-order sum: the same bits as "+zc".
  void build_flat_bidir() {
    const uint64_t split = round_up((count + N - 1) / N);
    auto boff = [&](uint32_t k) { return (uint64_t)k * split; };
    auto blen = [&](uint32_t k) -> uint64_t {
      const uint64_t s = boff(k);
      return s >= count ? 0 : std::min(split, count - s);
    };
    const uint64_t pub = alloc((uint64_t)N * split);   // my IN copy, block p at p * split
    const uint64_t land = alloc((uint64_t)N * split);  // owner j's reduced block j at j * split
    auto peers = rotated_peers();
    for (uint32_t p : peers) xfer(blen(p), {loc(BUF_IN, r, boff(p))}, {loc(BUF_STG, r, pub + boff(p))}, 1.0f);
    signal(peers, 0);
    wait(peers, 0);
    std::vector<Loc> srcs;
    for (uint32_t j = 0; j < N; ++j) srcs.push_back(j == r ? loc(BUF_IN, r, boff(r)) : loc(BUF_STG, j, pub + boff(r)));
    std::vector<Loc> dsts{loc(BUF_OUT, r, boff(r))};
    for (uint32_t p : peers) dsts.push_back(loc(BUF_STG, p, land + boff(r)));
    xfer(blen(r), srcs, dsts, scale);
    signal(peers, 1);
    wait(peers, 1);
    for (uint32_t p : peers) xfer(blen(p), {loc(BUF_STG, r, land + boff(p))}, {loc(BUF_OUT, r, boff(p))}, 1.0f);
    finish_channel();
  }

  // Zero-copy put form ("+zc+put"): only remote WRITES cross the links (no remote load waits on a round
  // trip). Every rank writes its IN block p into slot r of owner p's staging (the reduce-scatter, like the
  // staging flat push), then each owner sums its block in rank order - its own IN and the N - 1 landed slots
  // - straight into its own OUT and every peer's registered OUT (the all-gather). Two hand-offs: slot 0 "my
  // contributions are in your staging and I have entered the call" (so my OUT may be written), slot 1 "I
  // have written your block" (no rank leaves the call before its OUT is complete). Only OUT is addressed on
  // peers. In place is safe: a rank's IN block p is read by that rank (the push to p) before its slot-0
  // signal, and p writes that block of its OUT only after waiting for that signal - per workgroup, over the
  // same slice. Same rank-order sum as "+zc", so all forms give identical bits.
  void build_flat_zc_put() {
    const uint64_t split = round_up((count + N - 1) / N);
    auto boff = [&](uint32_t k) { return (uint64_t)k * split; };
    auto blen = [&](uint32_t k) -> uint64_t {
      const uint64_t s = boff(k);
      return s >= count ? 0 : std::min(split, count - s);
    };
    const uint64_t land = alloc((uint64_t)N * split);  // slot j: rank j's contribution to my block
    auto slot = [&](uint32_t j) { return land + (uint64_t)j * split; };
    auto peers = rotated_peers();
    for (uint32_t p : peers) xfer(blen(p), {loc(BUF_IN, r, boff(p))}, {loc(BUF_STG, p, slot(r))}, 1.0f);
    signal(peers, 0);
    wait(peers, 0);
    std::vector<Loc> srcs;
    for (uint32_t j = 0; j < N; ++j) srcs.push_back(j == r ? loc(BUF_IN, r, boff(r)) : loc(BUF_STG, r, slot(j)));
    std::vector<Loc> dsts{loc(BUF_OUT, r, boff(r))};
    for (uint32_t p : peers) dsts.push_back(loc(BUF_OUT, p, boff(r)));
    xfer(blen(r), srcs, dsts, scale);
    signal(peers, 1);
    wait(peers, 1);
    finish_channel();
  }

  // Zero-copy reduce-scatter / all-gather / all-to-all over registered buffers: the direct exchange with
  // the peers' IN / OUT as operands, no staging. Slot 0 "I have entered the call" (my IN is final, my OUT
  // may be written), slot 1 "I have finished with your buffers" (no rank leaves while a peer still
  // reads or writes its buffers).
  //  reduce-scatter: pull - rank r sums block r of every rank's IN (rank order) into its OUT;
  //  all-gather: push - rank r writes its IN into block r of every rank's OUT;
  //  all-to-all: push - rank r writes block p of its IN into block r of rank p's OUT.
  void build_coll_zc(Coll coll, uint64_t stride) {
    const uint64_t m = count;
    auto peers = rotated_peers();
    signal(peers, 0);
    wait(peers, 0);
    if (coll == Coll::REDUCE_SCATTER) {
      std::vector<Loc> srcs;
      for (uint32_t p = 0; p < N; ++p) srcs.push_back(loc(BUF_IN, p, (uint64_t)r * stride));
      xfer(m, srcs, {loc(BUF_OUT, r, 0)}, scale);
    } else if (coll == Coll::ALL_GATHER) {
      std::vector<Loc> dsts{loc(BUF_OUT, r, (uint64_t)r * stride)};
      for (uint32_t p : peers) dsts.push_back(loc(BUF_OUT, p, (uint64_t)r * stride));
      xfer(m, {loc(BUF_IN, r, 0)}, dsts, 1.0f);
    } else {
      for (uint32_t p : peers) xfer(m, {loc(BUF_IN, r, (uint64_t)p * stride)}, {loc(BUF_OUT, p, (uint64_t)r * stride)}, 1.0f);
      xfer(m, {loc(BUF_IN, r, (uint64_t)r * stride)}, {loc(BUF_OUT, r, (uint64_t)r * stride)}, 1.0f);
    }
    signal(peers, 1);
    wait(peers, 1);
    finish_channel();
  }
  // Zero-copy broadcast: the root writes its IN into every rank's OUT once every rank has entered the
  // call, then tells them it is done.
  void build_bcast_zc(uint32_t root) {
    std::vector<uint32_t> others;
    for (uint32_t p = 0; p < N; ++p)
      if (p != root) others.push_back(p);
    if (r == root) {
      wait(others, 0);
      std::vector<Loc> dsts{loc(BUF_OUT, r, 0)};
      for (uint32_t p : others) dsts.push_back(loc(BUF_OUT, p, 0));
      xfer(count, {loc(BUF_IN, r, 0)}, dsts, 1.0f);
      signal(others, 1);
    } else {
      signal({root}, 0);
      wait({root}, 1);
    }
    finish_channel();
  }

  // ------------------------------------------------------------------ reduce-scatter / all-gather
  std::vector<uint32_t> rotated_peers() const {
    std::vector<uint32_t> v;
    for (uint32_t jj = 1; jj < N; ++jj) v.push_back((r + jj) % N);
    return v;
  }
  void build_flat_rs(uint64_t stride) {
    const uint64_t m = count, m_al = round_up(m);
    uint64_t base = alloc((uint64_t)N * m_al);
    auto peers = rotated_peers();
    for (uint32_t p : peers) xfer(m, {loc(BUF_IN, r, (uint64_t)p * stride)}, {loc(BUF_STG, p, base + r * m_al)}, 1.0f);
    signal(peers, 0);
    wait(peers, 0);
    std::vector<Loc> srcs;  // rank order: identical summation order for every block owner
    for (uint32_t p = 0; p < N; ++p)
      srcs.push_back(p == r ? loc(BUF_IN, r, (uint64_t)r * stride) : loc(BUF_STG, r, base + p * m_al));
    if (wire) std::rotate(srcs.begin(), srcs.begin() + r, srcs.begin() + r + 1);  // typed: own value first
    xfer(m, srcs, {loc(BUF_OUT, r, 0)}, scale);
    finish_channel();
  }
  void build_flat_ag(uint64_t stride) {
    const uint64_t m = count, m_al = round_up(m);
    uint64_t base = alloc((uint64_t)N * m_al);
    auto peers = rotated_peers();
    std::vector<Loc> dsts{loc(BUF_OUT, r, (uint64_t)r * stride)};
    for (uint32_t p : peers) dsts.push_back(loc(BUF_STG, p, base + r * m_al));
    xfer(m, {loc(BUF_IN, r, 0)}, dsts, 1.0f);
    signal(peers, 0);
    wait(peers, 0);
    for (uint32_t p : peers) xfer(m, {loc(BUF_STG, r, base + p * m_al)}, {loc(BUF_OUT, r, (uint64_t)p * stride)}, 1.0f);
    finish_channel();
  }
  // All-to-all (expert parallelism): block p of IN goes to rank p, block q of OUT comes from rank q.
  // One direct exchange over all N-1 links (rotated run), then the landed blocks are copied out.
  void build_flat_a2a(uint64_t stride) {
    const uint64_t m = count, m_al = round_up(m);
    uint64_t base = alloc((uint64_t)N * m_al);
    auto peers = rotated_peers();
    for (uint32_t p : peers) xfer(m, {loc(BUF_IN, r, (uint64_t)p * stride)}, {loc(BUF_STG, p, base + r * m_al)}, 1.0f);
    xfer(m, {loc(BUF_IN, r, (uint64_t)r * stride)}, {loc(BUF_OUT, r, (uint64_t)r * stride)}, 1.0f);
    signal(peers, 0);
    wait(peers, 0);
    for (uint32_t p : peers) xfer(m, {loc(BUF_STG, r, base + p * m_al)}, {loc(BUF_OUT, r, (uint64_t)p * stride)}, 1.0f);
    finish_channel();
  }
  // Ring reduce-scatter: the rank at ring position v ends up owning ITS block (data of rank ord[v]).
  void build_ring_rs(uint64_t stride) {
    const uint64_t m = count, m_al = round_up(m);
    std::vector<int> ord = ring_order(N, 0);
    uint32_t v = 0;
    for (uint32_t q = 0; q < N; ++q)
      if ((uint32_t)ord[q] == r) v = q;
    const uint32_t right = ord[(v + 1) % N], left = ord[(v + N - 1) % N];
    auto mod = [&](long x) { return (uint32_t)(((x % (long)N) + N) % N); };
    auto boff = [&](uint32_t j) { return (uint64_t)ord[mod((long)j - 1)] * stride; };  // block j <-> rank ord[j-1]
    uint64_t base = alloc((uint64_t)(N - 1) * m_al);
    xfer(m, {loc(BUF_IN, r, boff(v))}, {loc(BUF_STG, right, base)}, 1.0f);
    signal({right}, 0);
    for (uint32_t i = 0; i + 1 < N; ++i) {
      wait({left}, i);
      uint32_t b = mod((long)v - 1 - (long)i);
      std::vector<Loc> srcs{loc(BUF_IN, r, boff(b)), loc(BUF_STG, r, base + i * m_al)};
      if (i + 2 < N) {
        xfer(m, srcs, {loc(BUF_STG, right, base + (i + 1) * m_al)}, 1.0f);
        signal({right}, i + 1);
      } else {
        xfer(m, srcs, {loc(BUF_OUT, r, 0)}, scale);  // b == v + 1  <->  rank ord[v] == r
      }
    }
    finish_channel();
  }
  void build_ring_ag(uint64_t stride) {
    const uint64_t m = count, m_al = round_up(m);
    std::vector<int> ord = ring_order(N, 0);
    uint32_t v = 0;
    for (uint32_t q = 0; q < N; ++q)
      if ((uint32_t)ord[q] == r) v = q;
    const uint32_t right = ord[(v + 1) % N], left = ord[(v + N - 1) % N];
    auto mod = [&](long x) { return (uint32_t)(((x % (long)N) + N) % N); };
    uint64_t base = alloc((uint64_t)(N - 1) * m_al);
    xfer(m, {loc(BUF_IN, r, 0)}, {loc(BUF_OUT, r, (uint64_t)r * stride), loc(BUF_STG, right, base)}, 1.0f);
    signal({right}, 0);
    for (uint32_t i = 0; i + 1 < N; ++i) {
      wait({left}, i);
      uint32_t owner = (uint32_t)ord[mod((long)v - 1 - (long)i)];  // the block that reached us at step i
      std::vector<Loc> dsts{loc(BUF_OUT, r, (uint64_t)owner * stride)};
      if (i + 2 < N) dsts.push_back(loc(BUF_STG, right, base + (i + 1) * m_al));
      xfer(m, {loc(BUF_STG, r, base + i * m_al)}, dsts, 1.0f);
      if (i + 2 < N) signal({right}, i + 1);
    }
    finish_channel();
  }

  // ------------------------------------------------------------------ broadcast
  // Every non-root rank acknowledges (slot 2) once it has consumed its staging, and the root waits for
  // all acks before its call ends: without this back edge a root that never waits could run two calls
  // ahead and overwrite a staging half a peer is still reading.
  std::vector<uint32_t> others_of(uint32_t root) const {
    std::vector<uint32_t> v;
    for (uint32_t jj = 1; jj < N; ++jj)
      if ((r + jj) % N != root) v.push_back((r + jj) % N);
    return v;
  }
  // Small buffers: one hop. The root multicasts the whole buffer into every peer's staging.
  void build_bcast_direct(uint32_t root) {
    const uint64_t base = alloc(count);
    if (r == root) {
      std::vector<Loc> dsts{loc(BUF_OUT, r, 0)};
      for (uint32_t p : rotated_peers()) dsts.push_back(loc(BUF_STG, p, base));
      xfer(count, {loc(BUF_IN, r, 0)}, dsts, 1.0f);
      signal(rotated_peers(), 0);
      wait(rotated_peers(), 2);
    } else {
      wait({root}, 0);
      xfer(count, {loc(BUF_STG, r, base)}, {loc(BUF_OUT, r, 0)}, 1.0f);
      signal({root}, 2);
    }
    finish_channel();
  }
  // Large buffers: the root scatters block p to rank p (and multicasts its own block), then the
  // non-root ranks all-gather their blocks. Every link carries ~2 S / N instead of S out of the root.
  void build_bcast_scatter_ag(uint32_t root) {
    const uint64_t split = round_up((count + N - 1) / N);
    auto blen = [&](uint32_t k) -> uint64_t {
      uint64_t s0 = (uint64_t)k * split;
      return s0 >= count ? 0 : std::min(split, count - s0);
    };
    auto boff = [&](uint32_t k) { return (uint64_t)k * split; };
    const uint64_t base = alloc((uint64_t)N * split);  // slot k holds block k
    if (r == root) {
      auto peers = rotated_peers();
      for (uint32_t p : peers) xfer(blen(p), {loc(BUF_IN, r, boff(p))}, {loc(BUF_STG, p, base + boff(p))}, 1.0f);
      std::vector<Loc> mine{loc(BUF_OUT, r, boff(r))};
      for (uint32_t p : peers) mine.push_back(loc(BUF_STG, p, base + boff(r)));
      xfer(blen(r), {loc(BUF_IN, r, boff(r))}, mine, 1.0f);
      for (uint32_t p : peers) xfer(blen(p), {loc(BUF_IN, r, boff(p))}, {loc(BUF_OUT, r, boff(p))}, 1.0f);
      signal(peers, 0);
      wait(peers, 2);
    } else {
      auto others = others_of(root);
      wait({root}, 0);
      std::vector<Loc> fwd{loc(BUF_OUT, r, boff(r))};
      for (uint32_t q : others) fwd.push_back(loc(BUF_STG, q, base + boff(r)));
      xfer(blen(r), {loc(BUF_STG, r, base + boff(r))}, fwd, 1.0f);
      xfer(blen(root), {loc(BUF_STG, r, base + boff(root))}, {loc(BUF_OUT, r, boff(root))}, 1.0f);
      if (!others.empty()) {
        signal(others, 1);
        wait(others, 1);
        for (uint32_t q : others) xfer(blen(q), {loc(BUF_STG, r, base + boff(q))}, {loc(BUF_OUT, r, boff(q))}, 1.0f);
      }
      signal({root}, 2);
    }
    finish_channel();
  }

  // ------------------------------------------------------------------ oneshot
  void build_oneshot() {
    uint64_t cnt_al = round_up(count);
    uint64_t base = alloc((uint64_t)N * cnt_al);
    std::vector<uint32_t> peers;
    for (uint32_t jj = 1; jj < N; ++jj) peers.push_back((r + jj) % N);
    std::vector<Loc> dsts;
    for (uint32_t p : peers) dsts.push_back(loc(BUF_STG, p, base + (uint64_t)r * cnt_al));
    xfer(count, {loc(BUF_IN, r, 0)}, dsts, 1.0f);
    signal(peers, 0);
    wait(peers, 0);
    // every rank reduces the full buffer: sum in rank order so all ranks get bit-identical results
    std::vector<Loc> srcs;
    for (uint32_t p = 0; p < N; ++p)
      srcs.push_back(p == r ? loc(BUF_IN, r, 0) : loc(BUF_STG, r, base + (uint64_t)p * cnt_al));
    xfer(count, srcs, {loc(BUF_OUT, r, 0)}, scale);
    finish_channel();
  }
};

// Element extents of the caller's IN / OUT buffers that a (coll, count, stride) program may touch.
inline void io_extent(Coll coll, uint32_t N, uint64_t count, uint64_t stride, uint64_t* in, uint64_t* out) {
  const uint64_t wide = N > 1 ? (uint64_t)(N - 1) * stride + count : count;
  switch (coll) {
    case Coll::REDUCE_SCATTER: *in = wide; *out = count; break;
    case Coll::ALL_GATHER: *in = count; *out = wide; break;
    case Coll::ALL_TO_ALL: *in = wide; *out = wide; break;
    default: *in = count; *out = count; break;  // allreduce, broadcast (stride = root)
  }
}

// The typed XFER forms the device executor runs (device_exec.hpp xfer_mx_k): sources all dtype (SP_T),
// own dtype + peers wire (SP_TW) or all wire (SP_W); fp8 wire: K = 1 pushes / all-gathers and K >= 2
// reductions, fp32 partials: K >= 2 (SP_TW only as the ring's K = 2 step). Masks must match the operands.
inline bool typed_pattern_ok(const Program& P, const Op& o) {
  uint32_t sm = 0, dm = 0;
  for (int k = 0; k < o.nsrc; ++k) sm |= (o.src[k].pad & 1u) << k;
  for (int k = 0; k < o.ndst; ++k) dm |= (o.dst[k].pad & 1u) << k;
  if (sm != o.pad16[0] || dm != o.pad16[1]) return false;
  const uint32_t all_s = (1u << o.nsrc) - 1, all_d = (1u << o.ndst) - 1;
  const bool fp8 = P.wire >= 2;
  const int K = o.nsrc;
  // MX wire: a wire-to-wire copy would have to carry the block scales too (the flat schedule has none)
  if (P.wire >= 4 && sm == all_s && dm) return false;
  // MX ops write at most 2 destinations (a reduction: own output + the published wire block; fp8 wires always
  // pull): the executor instantiates that form only (device_exec.hpp xfer_mxb_k)
  if (P.wire >= 2 && o.ndst > 2) return false;  // the same for the global-scale fp8 wire (device_exec.hpp xfer_mx_k)
  // wire type throughout: fp32 partials of any fan-in; an fp8 wire only copies (its kernels carry no fp8 sum)
  if (sm == all_s && dm == all_d) return fp8 ? K == 1 : true;
  if (!fp8 && sm == 0 && dm == 0) return true;  // dtype throughout
  if (sm == 0) return fp8 ? K == 1 : K >= 2;
  if (sm == (all_s & ~1u)) return K >= 2 && (fp8 || K == 2);
  if (sm == all_s) return fp8 ? K == 1 : K >= 2;
  return false;
}

// Host-side bounds check of a compiled program before it is uploaded or launched: every XFER operand
// stays inside its buffer (IN/OUT: this rank's, within the call's extent; STG: any rank's, within the
// program's staging), fan-in/fan-out and peer lists within the kernel's fixed arrays, flag slots within
// the program range, channel table well formed. The executor trusts the program (no per-access
// checks in the hot loop), so a planner bug must stop here instead of faulting the GPU.
inline bool validate_program(const Program& P, uint32_t N, uint32_t rank, uint64_t in_elems, uint64_t out_elems,
                             std::string* err) {
  auto fail = [&](const std::string& m) {
    if (err) *err = "internal: invalid program '" + P.desc + "': " + m;
    return false;
  };
  if (P.chan_start.size() != (size_t)P.nchan + 1 || P.chan_start.front() != 0 || P.chan_start.back() != P.ops.size())
    return fail("channel table");
  for (size_t c = 0; c + 1 < P.chan_start.size(); ++c)
    if (P.chan_start[c] > P.chan_start[c + 1]) return fail("channel table not monotonic");
  auto loc_ok = [&](const Loc& l, uint64_t len) {
    if (l.rank >= N || l.buf >= BUF_COUNT) return false;
    if (l.pad > 2 || (l.pad && (!P.wire || l.buf != BUF_STG))) return false;
    if (l.buf == BUF_STG) return l.off + P.extent(l, len) <= P.stg_elems;
    if (l.rank != rank && !P.zc) return false;  // a caller buffer is addressed on a peer only when registered
    return l.off + len <= (l.buf == BUF_IN ? in_elems : out_elems);
  };
  for (size_t i = 0; i < P.ops.size(); ++i) {
    const Op& o = P.ops[i];
    const std::string at = "op " + std::to_string(i);
    if (o.kind == OP_XFER) {
      if (o.nsrc < 1 || o.nsrc > kMaxSrc || o.ndst < 1 || o.ndst > kMaxDst) return fail(at + ": operand count");
      if (P.wire && !typed_pattern_ok(P, o)) return fail(at + ": typed operand pattern the executor does not run");
      for (int k = 0; k < o.nsrc; ++k)
        if (!loc_ok(o.src[k], o.len)) return fail(at + ": source " + std::to_string(k) + " out of bounds");
      for (int k = 0; k < o.ndst; ++k)
        if (!loc_ok(o.dst[k], o.len)) return fail(at + ": destination " + std::to_string(k) + " out of bounds");
      if (o.run > 1 && i + o.run > P.ops.size()) return fail(at + ": run past the end");
    } else if (o.kind == OP_SIGNAL || o.kind == OP_WAIT) {
      if (o.npeers > kMaxPeersPerOp) return fail(at + ": peer count");
      if (o.slot >= kProgSlots) return fail(at + ": flag slot");
      for (int k = 0; k < o.npeers; ++k)
        if (o.peers[k] >= N || o.peers[k] == rank) return fail(at + ": peer");
    } else if (o.kind != OP_NOP) {
      return fail(at + ": kind");
    }
  }
  return true;
}

// Human-readable program dump (the reference's Operations::print_ops, mpi_mod.hpp:107-144).
inline std::string dump_program(const Program& P, uint32_t rank) {
  static const char* bn[] = {"IN", "OUT", "STG"};
  std::ostringstream ss;
  ss << "rank " << rank << " program '" << P.desc << "': " << P.ops.size() << " ops, " << P.nchan
     << " channel(s), staging " << P.stg_elems << " elems/parity, " << P.nslots << " flag slots";
  static const char* wn[] = {"", "fp32", "e4m3", "e5m2", "mx e4m3", "mx e5m2"};
  if (P.wire) ss << ", wire type " << wn[P.wire] << " ('~'), unit " << P.unit << " B";
  if (P.mx_shadow) ss << ", block scales at " << P.mx_shadow;
  ss << "\n";
  for (uint32_t c = 0; c < P.nchan; ++c) {
    ss << "channel " << c << ":\n";
    for (uint32_t i = P.chan_start[c]; i < P.chan_start[c + 1]; ++i) {
      const Op& o = P.ops[i];
      if (o.kind == OP_XFER) {
        ss << "  XFER len=" << o.len << (o.scale != 1.0f ? " scale" : "") << " [";
        // a wire-typed staging operand is marked with '~'
        for (int k = 0; k < o.nsrc; ++k)
          ss << (k ? " + " : "") << bn[o.src[k].buf] << ((o.src[k].pad & 1) ? "~" : "") << "@" << o.src[k].rank << ":"
             << o.src[k].off;
        ss << "] -> [";
        for (int k = 0; k < o.ndst; ++k)
          ss << (k ? ", " : "") << bn[o.dst[k].buf] << ((o.dst[k].pad & 1) ? "~" : "") << "@" << o.dst[k].rank << ":"
             << o.dst[k].off;
        ss << "]\n";
      } else {
        ss << (o.kind == OP_SIGNAL ? "  SIGNAL" : "  WAIT  ") << " slot=" << o.slot << " peers=";
        for (int k = 0; k < o.npeers; ++k) ss << (k ? "," : "") << o.peers[k];
        ss << "\n";
      }
    }
  }
  return ss.str();
}

}  // namespace flexar
