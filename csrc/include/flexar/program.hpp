// The "op program": the compiled, per-rank schedule of one allreduce call.
//
// The reference builds its schedule every call as Send_Ops/Recv_Ops lists of
// (peer, block-list) edges (allreduce_over_mpi/mpi_mod.hpp:44-214) and then
// interprets them with MPI_Isend/Irecv/Waitall/Barrier + a CPU reduce
// (mpi_mod.hpp:662-878, 952-1163). Here a host planner compiles the same
// mathematical schedule ONCE per (comm, count, dtype, algorithm) into a flat
// list of three op kinds that one GPU kernel executes end to end:
//
//   XFER   dst[0..ndst) = scale * OP(src[0..nsrc))   over one block span.
//          A src/dst may live in a PEER's IPC-mapped staging buffer, so one
//          XFER is a fused "load remote + reduce + store local/remote".
//   SIGNAL release my prior stores, then bump my flag in each listed peer.
//   WAIT   acquire: poll my local flags until each listed peer has signalled.
//
// Every grid block executes the whole program on its own slice of every
// span (slice_range), with per-block flags and per-block epochs, so there is
// no grid-wide barrier and no global MPI_Barrier equivalent (defect D9).
#pragma once

#include <stdint.h>

#include "flexar/types.hpp"

namespace flexar {

enum : uint32_t {
  kMaxRanks = 16,        // intra-node xGMI mesh (8) with headroom; host/MPI path has its own limit
  kMaxSrc = 8,           // fan-in per XFER; the planner chains wider reductions
  kMaxDst = 8,           // multicast fan-out per XFER (one-shot pushes to 7 peers)
  kMaxPeersPerOp = 8,    // peers per SIGNAL/WAIT
  kMaxSlots = 128,       // flag slots per rank: op programs use [0, kProgSlots), the copy-engine
                         // (dma) allreduce the last two
  kMaxGridBlocks = 1024, // grid blocks per launch (per-block flags/epochs)
  kStageAlignBytes = 256 // staging regions / block boundaries alignment
};

enum OpKind : uint16_t { OP_NOP = 0, OP_XFER = 1, OP_SIGNAL = 2, OP_WAIT = 3 };
enum BufKind : uint16_t { BUF_IN = 0, BUF_OUT = 1, BUF_STG = 2, BUF_COUNT = 3 };

// A location: buffer kind + owning rank + element offset. Only BUF_STG may be
// owned by a remote rank (it is the IPC-registered workspace); IN/OUT are the
// caller's own (unregistered) tensors.
struct Loc {
  uint16_t buf;
  uint16_t rank;
  uint32_t pad;
  uint64_t off;
};

struct Op {
  uint16_t kind;
  uint8_t nsrc;
  uint8_t ndst;
  uint32_t slot;           // SIGNAL/WAIT flag slot
  uint64_t len;            // XFER element count (span length; 0 = empty tail block)
  float scale;             // XFER fused post-scale (1 = none)
  uint16_t npeers;         // SIGNAL/WAIT
  uint16_t flags;          // XFER: kXferApplyOp (nsrc>1 implies reduction)
  uint16_t peers[kMaxPeersPerOp];
  uint16_t run;            // >1 on the first op of a run of mutually independent XFERs: each
                           // workgroup starts the run at a different op (lb % run), so at any
                           // moment a rank's workgroups target different peers = all links busy
  uint16_t pad16[3];
  Loc src[kMaxSrc];
  Loc dst[kMaxDst];
};

// Deterministic split of a span across the grid blocks of one channel.
// Boundaries are multiples of `quantum` elements (slice_quantum), so the vector
// path stays aligned on every block. Identical on every rank => sender block b
// writes exactly the slice receiver block b reads.
FX_HD FX_INLINE void slice_range(uint64_t len, uint32_t lb, uint32_t nb, uint32_t quantum, uint64_t* lo,
                                 uint64_t* hi) {
  uint64_t per = (len + nb - 1) / nb;
  per = (per + quantum - 1) / quantum * quantum;
  uint64_t l = (uint64_t)lb * per;
  if (l > len) l = len;
  uint64_t h = l + per;
  if (h > len) h = len;
  *lo = l;
  *hi = h;
}

// Slice boundaries in whole FLEXAR_SLICE_ALIGN-byte runs of the narrowest operand (`unit` bytes per element),
// and never finer than `min_quantum` elements (16 B of vector access, an MX block). Op offsets are already
// kStageAlignBytes-aligned (the planner's round_up), so every workgroup's slice then starts on a cache-line
// boundary: with 16-B boundaries three slices in four started mid-line, and each 1 KiB wave access touched 17
// 64-B lines instead of 16 (profiles/r6_channels/req_split: +8 % TCP->TCC read requests on the 3-channel split).
#ifndef FLEXAR_SLICE_ALIGN
#define FLEXAR_SLICE_ALIGN 256
#endif
FX_HD FX_INLINE constexpr uint32_t slice_quantum(uint32_t unit, uint32_t min_quantum) {
  return (uint32_t)FLEXAR_SLICE_ALIGN / unit > min_quantum ? (uint32_t)FLEXAR_SLICE_ALIGN / unit : min_quantum;
}

constexpr uint32_t kProgSlots = kMaxSlots - 2;
constexpr uint32_t kDmaSlotRS = kMaxSlots - 2, kDmaSlotAG = kMaxSlots - 1;

// Flag word index: flags[slot][src_rank][grid_block]
FX_HD FX_INLINE uint64_t flag_index(uint32_t slot, uint32_t src_rank, uint32_t gblock) {
  return ((uint64_t)slot * kMaxRanks + src_rank) * kMaxGridBlocks + gblock;
}
constexpr uint64_t kFlagWords = (uint64_t)kMaxSlots * kMaxRanks * kMaxGridBlocks;

}  // namespace flexar
