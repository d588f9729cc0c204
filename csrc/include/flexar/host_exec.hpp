// Host executor of op programs: the same XFER/SIGNAL/WAIT semantics as the
// gfx950 kernel, on host memory with std::atomic flags. Two users:
//   * flexar_simulate(): runs every (rank, grid block) of a program in its own
//     thread — validates every algorithm / topology / tail geometry on CPU.
//   * the MPI shared-memory engine in mpi_mod.hpp (CPU plumbing path, the
//     reference's own domain: host buffers reduced across MPI ranks).
//
// Replaces the reference's handle_send/handle_recv/handle_reduce executors
// (allreduce_over_mpi/mpi_mod.hpp:662-878) and its OpenMP reduce_sum /
// reduce_band kernels (mpi_mod.hpp:245-660) — the fan-in is unbounded here
// (defect D3: fan-in > 20 silently produced garbage) and no per-call heap
// allocation happens in the hot path (defect D8).
#pragma once

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "flexar/planner.hpp"
#include "flexar/program.hpp"
#include "flexar/types.hpp"

namespace flexar {

struct HostExecCtx {
  uint32_t rank = 0;
  float pre = 1.0f, post_inv = 1.0f;  // typed programs, fp8 wire: pre-scale s and 1/s
  char* local[BUF_COUNT] = {nullptr, nullptr, nullptr};  // IN, OUT, STG of this rank
  std::vector<char*> peer_stg;                          // per rank (self = local STG)
  std::vector<char*> peer_io[2];                        // zero-copy programs: every rank's IN / OUT
  std::vector<std::atomic<uint64_t>*> peer_flags;       // per rank flag arrays
  uint32_t ranks_stride = 0, blocks_stride = 0;         // flag layout strides
  uint64_t stg_half_bytes = 0;                          // parity offset
  double timeout_s = 60.0;
};

inline uint64_t host_flag_index(const HostExecCtx& c, uint32_t slot, uint32_t src, uint32_t gblock) {
  return ((uint64_t)slot * c.ranks_stride + src) * c.blocks_stride + gblock;
}

// Chunked accumulate: fp32 (or native) accumulator buffer, one pass per source
// => the inner loops are simple streams the compiler vectorises.
template <typename T, typename OP>
inline void host_reduce_span(T* const* dsts, int ndst, const T* const* srcs, int nsrc, uint64_t n, float scale) {
  using A = typename Elem<T>::acc;
  constexpr uint64_t CH = 2048;
  A acc[CH];
  const bool do_scale = Elem<T>::is_float && scale != 1.0f;
  for (uint64_t base = 0; base < n; base += CH) {
    uint64_t m = n - base < CH ? n - base : CH;
    const T* s0 = srcs[0] + base;
    for (uint64_t i = 0; i < m; ++i) acc[i] = Elem<T>::load(s0[i]);
    for (int k = 1; k < nsrc; ++k) {
      const T* sk = srcs[k] + base;
      for (uint64_t i = 0; i < m; ++i) acc[i] = OP::apply(acc[i], Elem<T>::load(sk[i]));
    }
    if (do_scale)
      for (uint64_t i = 0; i < m; ++i) acc[i] = (A)(acc[i] * (A)scale);
    for (int d = 0; d < ndst; ++d) {
      T* dd = dsts[d] + base;
      for (uint64_t i = 0; i < m; ++i) dd[i] = Elem<T>::store(acc[i]);
    }
  }
}

// Wire-typed elements (Program::wire): 1 = fp32, 2 = OCP e4m3, 3 = OCP e5m2 (saturating).
inline float wire_load(int wire, const char* p, uint64_t i) {
  if (wire == 1) { float f; memcpy(&f, p + 4 * i, 4); return f; }
  return wire == 2 ? e4m3_to_f32((uint8_t)p[i]) : e5m2_to_f32((uint8_t)p[i]);
}
inline void wire_store(int wire, char* p, uint64_t i, float v) {
  if (wire == 1) { memcpy(p + 4 * i, &v, 4); return; }
  p[i] = (char)(wire == 2 ? f32_to_e4m3(v) : f32_to_e5m2(v));
}
inline float wire_round(int wire, float v) {
  if (wire == 1) return v;
  return wire == 2 ? e4m3_to_f32(f32_to_e4m3(v)) : e5m2_to_f32(f32_to_e5m2(v));
}

// One typed XFER on host memory (the device kernel's xfer_mx semantics, element by element):
//   source of the wire type: its value; source of the dtype: its value, or in fp8 wire modes the value
//   quantised with the pre-scale (x * s -> fp8 -> float), so every contribution is rounded the same way;
//   y = scale * sum; with an fp8 destination y is rounded to fp8 first, so dtype destinations (x 1/s)
//   and the fp8 copies the peers receive hold the same value.
template <typename T>
inline void host_xfer_typed(int wire, const Op& o, char* const* src, char* const* dst, uint64_t n, float pre,
                            float post_inv) {
  const uint16_t sm = o.pad16[0], dm = o.pad16[1];
  for (uint64_t i = 0; i < n; ++i) {
    float acc = 0.0f;
    for (int k = 0; k < o.nsrc; ++k) {
      float v;
      if (sm & (1u << k)) v = wire_load(wire, src[k], i);
      else {
        v = (float)Elem<T>::load(reinterpret_cast<const T*>(src[k])[i]);
        if (wire >= 2) v = wire_round(wire, v * pre);
      }
      acc = k ? acc + v : v;
    }
    float y = acc * o.scale;
    if (wire >= 2 && dm) y = wire_round(wire, y);
    for (int k = 0; k < o.ndst; ++k) {
      if (dm & (1u << k)) wire_store(wire, dst[k], i, y);
      else reinterpret_cast<T*>(dst[k])[i] = Elem<T>::store((typename Elem<T>::acc)(wire >= 2 ? y * post_inv : y));
    }
  }
}

// MX wire (Program::wire 4 = e4m3, 5 = e5m2): one typed XFER in OCP MX form over a slice that starts on a
// block boundary, block by block - the device's xfer_mxb, bit for bit (docs/DESIGN.md §9.2):
//   quantising push (K = 1, dtype source): y = x * scale; the block's scale 2^X from max |y|
//     (mx_scale_byte); q = rne(y / 2^X); wire destinations get q and the scale byte, dtype ones q * 2^X;
//   dequantising all-gather (K = 1, wire source): y = q * 2^X * scale into dtype destinations;
//   reduction (K >= 2, own dtype value first): the own value rounded through MX with its own block scale,
//     each peer's q * 2^X, summed in source order, times scale; with a wire destination the sum is
//     quantised again (its own block scale) and every destination gets that value.
inline uint32_t mx_mag_bits(float v) { return f2u(v) & 0x7fffffffu; }
inline uint8_t mx_q(bool e4, float v) { return e4 ? f32_to_e4m3(v) : f32_to_e5m2(v); }
inline float mx_dq(bool e4, uint8_t q) { return e4 ? e4m3_to_f32(q) : e5m2_to_f32(q); }

template <typename T>
inline void host_xfer_mxb(int wire, const Op& o, char* const* src, const uint8_t* const* ssc, char* const* dst,
                          uint8_t* const* dsc, uint64_t n) {
  const bool e4 = wire == 4;
  const uint16_t sm = o.pad16[0], dm = o.pad16[1];
  const int K = o.nsrc;
  auto ld = [&](int k, uint64_t i) { return (float)Elem<T>::load(reinterpret_cast<const T*>(src[k])[i]); };
  for (uint64_t b0 = 0; b0 < n; b0 += kMxBlock) {
    const uint64_t m = n - b0 < kMxBlock ? n - b0 : kMxBlock, blk = b0 / kMxBlock;
    float y[kMxBlock];
    uint8_t q[kMxBlock];
    uint32_t xr = 0;
    if (K == 1 && !(sm & 1u)) {
      uint32_t am = 0;
      for (uint64_t i = 0; i < m; ++i) {
        y[i] = ld(0, b0 + i) * o.scale;
        am = std::max(am, mx_mag_bits(y[i]));
      }
      xr = mx_scale_byte(am, e4);
    } else if (K == 1) {
      const float sc = mx_scale_value(ssc[0][blk]);
      for (uint64_t i = 0; i < m; ++i) y[i] = mx_dq(e4, (uint8_t)src[0][b0 + i]) * sc * o.scale;
    } else {
      for (int k = 0; k < K; ++k) {
        float v[kMxBlock];
        if (sm & (1u << k)) {
          const float sc = mx_scale_value(ssc[k][blk]);
          for (uint64_t i = 0; i < m; ++i) v[i] = mx_dq(e4, (uint8_t)src[k][b0 + i]) * sc;
        } else {
          uint32_t am = 0;
          for (uint64_t i = 0; i < m; ++i) {
            v[i] = ld(k, b0 + i);
            am = std::max(am, mx_mag_bits(v[i]));
          }
          const float sc = mx_scale_value(mx_scale_byte(am, e4));
          for (uint64_t i = 0; i < m; ++i) v[i] = mx_dq(e4, mx_q(e4, v[i] / sc)) * sc;
        }
        for (uint64_t i = 0; i < m; ++i) y[i] = k ? y[i] + v[i] : v[i];
      }
      uint32_t am = 0;
      for (uint64_t i = 0; i < m; ++i) {
        y[i] *= o.scale;
        am = std::max(am, mx_mag_bits(y[i]));
      }
      if (dm) xr = mx_scale_byte(am, e4);
    }
    if (xr) {
      const float sc = mx_scale_value(xr);
      for (uint64_t i = 0; i < m; ++i) {
        q[i] = mx_q(e4, y[i] / sc);
        y[i] = mx_dq(e4, q[i]) * sc;
      }
    }
    for (int d = 0; d < o.ndst; ++d) {
      if (dm & (1u << d)) {
        memcpy(dst[d] + b0, q, m);
        dsc[d][blk] = (uint8_t)xr;
      } else {
        for (uint64_t i = 0; i < m; ++i)
          reinterpret_cast<T*>(dst[d])[b0 + i] = Elem<T>::store((typename Elem<T>::acc)y[i]);
      }
    }
  }
}

template <typename T, typename OP>
struct HostExec {
  // Returns 0, or FLEXAR_ERR_TIMEOUT if a WAIT exceeded the timeout.
  static int run(const Program& P, const HostExecCtx& c, uint32_t gblock, uint32_t grid, uint64_t epoch) {
    const uint32_t nchan = P.nchan;
    const uint32_t ch = gblock % nchan, lb = gblock / nchan;
    const uint32_t nb = (grid - ch + nchan - 1) / nchan;
    const uint32_t unit = P.stg_unit();
    // slice boundaries as on the device (slice_quantum): whole 256-B runs of the narrowest operand type
    const uint32_t ub = P.wire ? unit : (uint32_t)sizeof(T);
    const uint32_t quantum = P.wire >= 4 ? slice_quantum(1, kMxBlock) : slice_quantum(ub, ub >= 16 ? 1 : 16 / ub);
    const uint64_t par = (epoch & 1) ? c.stg_half_bytes : 0;
    auto addr = [&](const Loc& l) -> char* {
      if (l.buf == BUF_STG) return c.peer_stg[l.rank] + par + l.off * unit;
      if (l.rank != c.rank) return c.peer_io[l.buf][l.rank] + l.off * sizeof(T);  // registered peer buffer
      return c.local[l.buf] + l.off * sizeof(T);
    };
    auto esz = [&](const Loc& l) -> uint64_t { return (l.pad & 1) ? P.wsize : sizeof(T); };
    for (uint32_t i = P.chan_start[ch]; i < P.chan_start[ch + 1]; ++i) {
      const Op& o0 = P.ops[i];
      if (o0.kind == OP_XFER) {
        const uint32_t n = o0.run > 1 ? o0.run : 1;  // rotated run, as on the device
        for (uint32_t k = 0; k < n; ++k) {
          const Op& o = P.ops[i + (n > 1 ? (k + lb) % n : 0)];
          uint64_t lo, hi;
          slice_range(o.len, lb, nb, quantum, &lo, &hi);
          if (hi <= lo) continue;
          if (P.wire && (o.pad16[0] || o.pad16[1] || P.wire >= 2)) {
            char* sp[kMaxSrc];
            char* dp[kMaxDst];
            for (int q = 0; q < o.nsrc; ++q) sp[q] = addr(o.src[q]) + lo * esz(o.src[q]);
            for (int q = 0; q < o.ndst; ++q) dp[q] = addr(o.dst[q]) + lo * esz(o.dst[q]);
            if (P.wire >= 4) {  // block scales: the shadow byte of each wire operand's first block
              auto sc = [&](const Loc& l) -> uint8_t* {
                return (l.pad & 1) ? (uint8_t*)c.peer_stg[l.rank] + par + P.mx_shadow * unit + (l.off * unit + lo) / kMxBlock
                                   : nullptr;
              };
              const uint8_t* ss[kMaxSrc];
              uint8_t* ds[kMaxDst];
              for (int q = 0; q < o.nsrc; ++q) ss[q] = sc(o.src[q]);
              for (int q = 0; q < o.ndst; ++q) ds[q] = sc(o.dst[q]);
              host_xfer_mxb<T>(P.wire, o, sp, ss, dp, ds, hi - lo);
              continue;
            }
            host_xfer_typed<T>(P.wire, o, sp, dp, hi - lo, c.pre, c.post_inv);
            continue;
          }
          const T* srcs[kMaxSrc];
          T* dsts[kMaxDst];
          for (int q = 0; q < o.nsrc; ++q) srcs[q] = (const T*)addr(o.src[q]) + lo;
          for (int q = 0; q < o.ndst; ++q) dsts[q] = (T*)addr(o.dst[q]) + lo;
          host_reduce_span<T, OP>(dsts, o.ndst, srcs, o.nsrc, hi - lo, o.scale);
        }
        i += n - 1;
        continue;
      }
      const Op& o = o0;
      if (o.kind == OP_SIGNAL) {
        std::atomic_thread_fence(std::memory_order_release);
        for (int k = 0; k < o.npeers; ++k)
          c.peer_flags[o.peers[k]][host_flag_index(c, o.slot, c.rank, gblock)].store(epoch, std::memory_order_release);
      } else if (o.kind == OP_WAIT) {
        for (int k = 0; k < o.npeers; ++k) {
          std::atomic<uint64_t>& f = c.peer_flags[c.rank][host_flag_index(c, o.slot, o.peers[k], gblock)];
          auto t0 = std::chrono::steady_clock::now();
          unsigned spins = 0;
          while (f.load(std::memory_order_acquire) < epoch) {
            if (++spins > 64) {
              std::this_thread::yield();
              if ((spins & 1023) == 0 &&
                  std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > c.timeout_s)
                return FLEXAR_ERR_TIMEOUT;
            }
          }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
      }
    }
    return 0;
  }
};

}  // namespace flexar
