// gfx950 executor kernel for op programs (program.hpp) and the standalone
// reduction kernel.
//
// One launch runs a whole allreduce: every workgroup walks the rank's op
// program over ITS slice of every span. XFER fuses remote loads (xGMI reads
// of a peer's IPC-mapped staging), the reduction (fp32 accumulate for
// bf16/fp16/fp8) and local + remote stores (xGMI writes) into one pass with
// 16-byte-per-lane vector memory operations. SIGNAL/WAIT are per-workgroup
// system-scope release/acquire hand-offs on 64-bit epoch flags, so there is
// no grid barrier and no host round trip between stages.
//
// Replaces reference hot loops #1-#3 (mpi_mod.hpp:988-1060, 1129-1159):
// MPI_Isend/Irecv per block, MPI_Waitall, MPI_Barrier per stage and the
// 14-thread OpenMP reduce_sum (mpi_mod.hpp:245-452).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "flexar/program.hpp"
#include "flexar/types.hpp"

namespace flexar {

constexpr int kExecThreads = 512;  // 8 waves of 64

enum : uint16_t { kXferBarrierAfter = 1 };

struct DevCtx {
  const Op* ops;
  const uint32_t* chan_start;
  uint32_t nchan;
  uint32_t rank;
  char* local[BUF_COUNT];          // IN, OUT, STG (this rank)
  char* peer_stg[kMaxRanks];       // IPC-mapped staging of every rank (self = local)
  uint64_t* peer_flags[kMaxRanks]; // IPC-mapped flag arrays of every rank (self = local)
  char* peer_io[2][kMaxRanks];     // zero-copy programs: every rank's registered IN / OUT for this call
  uint64_t* epochs;                // [kMaxGridBlocks] per-workgroup call counter (local)
  uint64_t stg_half_bytes;         // parity offset (calls alternate staging halves)
  uint32_t* err;                   // device pointer of a host-mapped error word
  uint64_t timeout_ticks;          // s_memrealtime ticks (100 MHz)
  uint32_t vec_ok;                 // IN/OUT may take 16-B vector accesses (any alignment unless
                                   // FLEXAR_SCALAR_MISALIGNED=1, then only 16-B aligned bases)
  // fault injection (tests only, FLEXAR_FAULT_INJECT): 1 = delay SIGNAL(slot) by fi_ticks, 2 = drop it
  uint32_t fi_kind;
  uint32_t fi_slot;
  uint64_t fi_ticks;
  // LL protocol (ll_body): no op program
  uint64_t ll_off;  // byte offset of the LL granule region inside each staging parity half
  uint32_t nranks;
  uint64_t count;  // elements
  float scale;
  // typed programs (Program::wire, planner.hpp): STG offsets count stg_unit bytes; fp8 wire modes
  // derive the pre-scale from this rank's amax partials and the peers' amax granules
  uint32_t stg_unit;
  const float* amax_parts;  // FLEXAR_AMAX_PARTIALS per-workgroup max |x| of this rank's input
  uint64_t amax_off;        // byte offset of the amax granule slots in each staging parity half
  uint64_t mx_shadow;       // MX wire: byte offset of the block-scale shadow in each staging parity half
  // fault attribution (crumbs.hpp): host-mapped {started, finished} epoch words of this communicator;
  // workgroup 0 stores the epoch it starts and finishes (one system-scope store each; null = not recorded)
  uint64_t* progress;
  // XFER work split (exec_body): 0 = every workgroup takes one contiguous slice of each span; otherwise spans of
  // at least 4 x grid x ichunk elements go in ichunk-element chunks dealt round-robin to the workgroups (the
  // whole grid then works in one narrow window of every operand, as reduce_interleaved); ichunk is a multiple
  // of every slicing quantum and typed super-group (kXferChunk)
  uint64_t ichunk;
};
constexpr uint64_t kXferChunk = 8192;  // elements: 32 KiB of fp32; a multiple of 512 x G for every typed layout
constexpr uint32_t kAmaxParts = 256;    // == FLEXAR_AMAX_PARTIALS
constexpr uint64_t kAmaxRegion = 256;   // bytes reserved per parity half for the amax granules

// 16-byte vector memory ops (global_load/store_dwordx4). Payload bytes are touched once, so loads use
// the streaming (nontemporal) policy by default: measured on MI355X (bench/kernel_bench.py, profiles/)
// 6.0-6.5 TB/s vs 5.0-5.2 TB/s with the default policy for fan-in 1..8 reductions and copies.
// FLEXAR_PLAIN_LOADS restores the default policy; FLEXAR_NT_STORES makes stores streaming too.
#if !defined(FLEXAR_PLAIN_LOADS) && !defined(FLEXAR_NT_LOADS)
#define FLEXAR_NT_LOADS 1
#endif
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Payload pointers are always global memory (HBM, local or IPC-mapped): address-space-1 accesses
// compile to global_load/store (one counter, no flat aperture check) instead of flat_*.
// The payload vector type claims no alignment: a caller's tensor view may start at any element offset
// (a +4 B fp32 view, a +2 B bf16 view). amdhsa code objects run with unaligned access mode, so the
// compiler still emits ONE global_load/store_dwordx4 per 16 B (checked in the ISA) and the memory
// pipeline splits only the accesses that cross a cache line - instead of the whole span dropping to
// 4-byte scalar code (round 3). FLEXAR_SCALAR_MISALIGNED=1 restores the old policy.
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) u32x4u g_u32x4;
__device__ FX_INLINE uint4 ld16(const char* p) {
#if defined(FLEXAR_NT_LOADS)
  u32x4u v = __builtin_nontemporal_load((const g_u32x4*)(p));
#else
  u32x4u v = *(const g_u32x4*)(p);
#endif
  return uint4{v.x, v.y, v.z, v.w};
}
template <bool NTS = false>
__device__ FX_INLINE void st16(char* p, uint4 x) {
  u32x4u v = {x.x, x.y, x.z, x.w};
#if defined(FLEXAR_NT_STORES)
  __builtin_nontemporal_store(v, (g_u32x4*)(p));
#else
  if constexpr (NTS) __builtin_nontemporal_store(v, (g_u32x4*)(p));  // "+nts": streaming stores
  else *(g_u32x4*)(p) = v;
#endif
}

// Executor protocol modes (template parameter PM of the executor):
//   PM_FENCE      plain stores; SIGNAL = system release (buffer_wbl2 sc0 sc1), WAIT = system acquire
//                 (buffer_inv sc0 sc1)
//   PM_FENCE_NTS  the same with streaming (nontemporal) stores ("+nts")
//   PM_WT         write-through ("+wt"): every payload load/store is system-coherent (sc0 sc1), so a
//                 drained store (vmcnt(0)) is already visible to every agent and the hand-off needs no
//                 L2 write-back or invalidate — SIGNAL is vmcnt(0) + barrier + flag store, WAIT is poll +
//                 barrier. This is the LL protocol's visibility rule (sc0 sc1 granules) applied to bulk
//                 data, and MI355X_MICROARCH.md's "sc1 stores + drained flag + sc1 loads" hand-off at
//                 system scope.
enum : int { PM_FENCE = 0, PM_FENCE_NTS = 1, PM_WT = 2 };
constexpr int kAuxSys = 1 | 16;  // buffer cache-policy bits: sc0 | sc1 (system coherence)
constexpr uint32_t kRsrcWord3 = 0x00020000u;  // gfx9 raw buffer descriptor word 3 (dword data format)
constexpr uint64_t kWtChunkBytes = 1ull << 30;  // buffer offsets are 32-bit: spans go in <= 1 GiB pieces

// Operands are workgroup-uniform; readfirstlane states it so the descriptor lives in SGPRs (otherwise
// the compiler wraps every buffer access in a waterfall loop).
__device__ FX_INLINE __amdgpu_buffer_rsrc_t rsrc_of(const char* p, uint64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                     ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
  const int nrec = __builtin_amdgcn_readfirstlane((int)(uint32_t)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0, nrec, (int)kRsrcWord3);
}
__device__ FX_INLINE uint4 ld16_sys(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSys);
  return uint4{v.x, v.y, v.z, v.w};
}
__device__ FX_INLINE void st16_sys(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 x) {
  u32x4 v = {x.x, x.y, x.z, x.w};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSys);
}

// Sub-chunks of a lane-interleaved typed group (xfer_mx): 4, 8 or 16 bytes moved between a buffer and
// component j of a lane's packed group. The buffer descriptor and the sub-chunk's offset are uniform
// (SGPRs); the lane's offset is ONE VGPR shared by every sub-chunk and source, so no per-access 64-bit
// address is kept live. Component indices are compile-time after unrolling, so the group stays in
// registers. Cache policy: plain (aux 0) or non-temporal (aux 2, "nt") like the global forms.
__device__ FX_INLINE void set_word(uint4& u, int c, uint32_t x) {
  if (c == 0) u.x = x;
  else if (c == 1) u.y = x;
  else if (c == 2) u.z = x;
  else u.w = x;
}
__device__ FX_INLINE uint32_t get_word(const uint4& u, int c) { return c == 0 ? u.x : c == 1 ? u.y : c == 2 ? u.z : u.w; }
#if defined(FLEXAR_NT_LOADS)
constexpr int kAuxLd = 2;
#else
constexpr int kAuxLd = 0;
#endif
typedef int i32x2 __attribute__((ext_vector_type(2)));
template <int SB, int N>
__device__ FX_INLINE void ld_sub(uint4 (&r)[N], int j, __amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
  static_assert(SB == 4 || SB == 8 || SB == 16, "4, 8 or 16 bytes");
  if constexpr (SB == 16) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, kAuxLd);
    r[j] = uint4{v.x, v.y, v.z, v.w};
  } else if constexpr (SB == 8) {
    const i32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, kAuxLd);
    set_word(r[(2 * j) / 4], (2 * j) % 4, (uint32_t)v.x);
    set_word(r[(2 * j + 1) / 4], (2 * j + 1) % 4, (uint32_t)v.y);
  } else {
    set_word(r[j / 4], j % 4, (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, kAuxLd));
  }
}
template <int SB, bool NTS, int N>
__device__ FX_INLINE void st_sub(__amdgpu_buffer_rsrc_t rd, uint32_t voff, uint32_t soff, const uint4 (&r)[N], int j) {
  static_assert(SB == 4 || SB == 8 || SB == 16, "4, 8 or 16 bytes");
  constexpr int aux = NTS ? 2 : 0;
  if constexpr (SB == 16) {
    const u32x4 v = {r[j].x, r[j].y, r[j].z, r[j].w};
    __builtin_amdgcn_raw_buffer_store_b128(v, rd, voff, soff, aux);
  } else if constexpr (SB == 8) {
    const i32x2 v = {(int)get_word(r[(2 * j) / 4], (2 * j) % 4), (int)get_word(r[(2 * j + 1) / 4], (2 * j + 1) % 4)};
    __builtin_amdgcn_raw_buffer_store_b64(v, rd, voff, soff, aux);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32((int)get_word(r[j / 4], j % 4), rd, voff, soff, aux);
  }
}
template <int B> struct UintOf;
template <> struct UintOf<1> { using type = uint8_t; };
template <> struct UintOf<2> { using type = uint16_t; };
template <> struct UintOf<4> { using type = uint32_t; };
template <> struct UintOf<8> { using type = uint64_t; };
// scalar element access; PM_WT: system-coherent (global_load/store_* sc0 sc1)
template <int PM, typename T>
__device__ FX_INLINE T ld_elem(const char* base, uint64_t i) {
  if constexpr (PM == PM_WT) {
    using U = typename UintOf<sizeof(T)>::type;
    U u = __hip_atomic_load(reinterpret_cast<U*>(const_cast<char*>(base)) + i, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_SYSTEM);
    T t;
    __builtin_memcpy(&t, &u, sizeof(T));
    return t;
  } else {
    return reinterpret_cast<const T*>(base)[i];
  }
}
template <int PM, typename T>
__device__ FX_INLINE void st_elem(char* base, uint64_t i, T t) {
  if constexpr (PM == PM_WT) {
    using U = typename UintOf<sizeof(T)>::type;
    U u;
    __builtin_memcpy(&u, &t, sizeof(T));
    __hip_atomic_store(reinterpret_cast<U*>(base) + i, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    reinterpret_cast<T*>(base)[i] = t;
  }
}

template <typename S> struct IsFp8;
template <typename S> __device__ FX_INLINE void fp8_word_decode(uint32_t w, float* x);
template <typename S> __device__ FX_INLINE uint32_t fp8_word_encode(const float* x);

// 4 fp8 values from fp32 with the element store's semantics (f32_to_e4m3 / _e5m2: NaN -> 0x7f, saturate to the
// largest finite, RNE) at the packed converter's rate: clamp, pack with 2 converts, then put 0x7f in the bytes
// whose input was a NaN (the clamp maps a NaN to a bound). Branch-free.
template <typename T>
__device__ FX_INLINE uint32_t fp8_store4(const float (&a)[4]) {
  constexpr float M = IsFp8<T>::e4m3 ? 448.0f : 57344.0f;
  float c[4];
  uint32_t nan = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = __builtin_fminf(__builtin_fmaxf(a[j], -M), M);
    nan |= a[j] != a[j] ? 0xffu << (8 * j) : 0u;
  }
  return (fp8_word_encode<T>(c) & ~nan) | (0x7f7f7f7fu & nan);
}

// PACK = false keeps fp8 on the per-element converts. The executor's transfers (xfer_k) use it: packed, the fp8
// flat executor measured 2 % slower (364 against 356 us, 4 ranks x 100 MiB, profiles/r5_fp8_packed/verify), and
// the write-through kernels would lose their second workgroup per CU. The grid-interleaved standalone reduction
// packs (reduce_interleaved).
template <typename T, typename OP, int K, bool PACK = true>
__device__ FX_INLINE uint4 combine16(const uint4 (&x)[K], float scale, bool sc) {
  if (K == 1 && !sc) return x[0];  // pure move: no decode/encode round trip (fp8/bf16 copies at HBM rate)
  if constexpr (IsFp8<T>::value && PACK) {
    // fp8, one 4-byte word at a time (few live registers): packed decode (2 converts per 4 elements instead of
    // 4), fp32 accumulate in source order, post-scale, packed saturating encode (fp8_store4). Bit-identical to
    // the per-element path below.
    const float f = sc ? scale : 1.0f;
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float acc[4], t[4];
      fp8_word_decode<T>((&x[0].x)[i], acc);
#pragma unroll
      for (int k = 1; k < K; ++k) {
        fp8_word_decode<T>((&x[k].x)[i], t);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = OP::apply(acc[j], t[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = acc[j] * f;
      w[i] = fp8_store4<T>(acc);
    }
    uint4 r;
    __builtin_memcpy(&r, w, 16);
    return r;
  }
  using A = typename Elem<T>::acc;
  constexpr int E = 16 / sizeof(T);
  T v[E];
  A acc[E];
  __builtin_memcpy(v, &x[0], 16);
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = Elem<T>::load(v[e]);
#pragma unroll
  for (int k = 1; k < K; ++k) {
    __builtin_memcpy(v, &x[k], 16);
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = OP::apply(acc[e], Elem<T>::load(v[e]));
  }
  // The post-scale multiplies unconditionally (x * 1 is exact): a runtime `if (sc)` here is if-converted
  // by the compiler into a multiply AND a select per element (v_pk_mul + v_cndmask), the select being pure
  // overhead in the common unscaled case. Integer types never scale (sc is false at compile time).
  if constexpr (Elem<T>::is_float) {
    const A f = sc ? (A)scale : (A)1;
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = (A)(acc[e] * f);
  }
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = Elem<T>::store(acc[e]);
  uint4 r;
  __builtin_memcpy(&r, v, 16);
  return r;
}

// dst[0..nd) = OP(src[0..K)) over n elements; this workgroup's threads only.
template <typename T, typename OP, int K, int PM>
__device__ FX_INLINE void xfer_k(const char* const (&s)[kMaxSrc], char* const (&d)[kMaxDst], int nd, uint64_t n,
                                 float scale, bool vec) {
  using A = typename Elem<T>::acc;
  constexpr int E = 16 / sizeof(T);
// Groups in flight per lane for fan-in 5-8 transfers: 2 since round 5 (16 loads of 16 B per lane at fan-in 8).
// Standalone reduction at fan-in 8 +1-3 % (profiles/r5_reduce/grid_unroll), executor schedules at 2-8 ranks in
// one launch unchanged within noise (profiles/r5_reduce/executor_unroll), no occupancy change (fence executor
// 145 -> 164 VGPRs, still 3 waves per SIMD); more remote loads in flight on the 8-GPU node's xGMI latency.
#ifndef FLEXAR_UNROLL_WIDE
#define FLEXAR_UNROLL_WIDE 2
#endif
  // 8-bit PROD / MAX / MIN (16 lanes of byte arithmetic per vector) spill at the unroll above in the write-through
  // and group kernels; FLEXAR_BYTE_OP_U1=1 is the A/B build with one group per lane for them (docs/ROUND6.md)
#ifndef FLEXAR_BYTE_OP_U1
#define FLEXAR_BYTE_OP_U1 0
#endif
  constexpr bool BYTE_OP = FLEXAR_BYTE_OP_U1 && sizeof(T) == 1 &&
                           (std::is_same<OP, OpProd>::value || std::is_same<OP, OpMax>::value || std::is_same<OP, OpMin>::value);
  constexpr int U = BYTE_OP ? 1 : (K <= 2) ? 4 : ((K <= 4) ? 2 : FLEXAR_UNROLL_WIDE);  // 16-B loads in flight per lane
  constexpr bool WT = PM == PM_WT;
  constexpr bool NTS = PM == PM_FENCE_NTS;
  const bool sc = Elem<T>::is_float && scale != 1.0f;
  const uint64_t nt = blockDim.x;
  const uint64_t nv = vec ? n / E : 0;
  // PM_WT: one raw buffer descriptor per operand (bounded by the span: n * sizeof(T) < 4 GiB)
  __amdgpu_buffer_rsrc_t rs[K], rd[kMaxDst];
  if constexpr (WT) {
#pragma unroll
    for (int k = 0; k < K; ++k) rs[k] = rsrc_of(s[k], n * sizeof(T));
#pragma unroll
    for (int dd = 0; dd < kMaxDst; ++dd)
      if (dd < nd) rd[dd] = rsrc_of(d[dd], n * sizeof(T));
  }
  auto ld = [&](int k, uint64_t v) -> uint4 {
    if constexpr (WT) return ld16_sys(rs[k], (uint32_t)(v * 16));
    else return ld16(s[k] + v * 16);
  };
  auto st = [&](int dd, uint64_t v, uint4 y) {
    if constexpr (WT) st16_sys(rd[dd], (uint32_t)(v * 16), y);
    else st16<NTS>(d[dd] + v * 16, y);
  };
  uint64_t v = threadIdx.x;
  for (; v + (U - 1) * nt < nv; v += U * nt) {
    uint4 x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < K; ++k) x[u][k] = ld(k, v + u * nt);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint4 y = combine16<T, OP, K, false>(x[u], scale, sc);
#pragma unroll
      for (int dd = 0; dd < kMaxDst; ++dd)
        if (dd < nd) st(dd, v + u * nt, y);
    }
  }
  for (; v < nv; v += nt) {
    uint4 x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = ld(k, v);
    uint4 y = combine16<T, OP, K, false>(x, scale, sc);
#pragma unroll
    for (int dd = 0; dd < kMaxDst; ++dd)
      if (dd < nd) st(dd, v, y);
  }
  // scalar tail (or whole span when a base address is not 16-B aligned)
  for (uint64_t i = nv * E + threadIdx.x; i < n; i += nt) {
    if (K == 1 && !sc) {
      const T y = ld_elem<PM, T>(s[0], i);
#pragma unroll
      for (int dd = 0; dd < kMaxDst; ++dd)
        if (dd < nd) st_elem<PM, T>(d[dd], i, y);
      continue;
    }
    A acc = Elem<T>::load(ld_elem<PM, T>(s[0], i));
#pragma unroll
    for (int k = 1; k < K; ++k) acc = OP::apply(acc, Elem<T>::load(ld_elem<PM, T>(s[k], i)));
    if (sc) acc = (A)(acc * (A)scale);
    T y = Elem<T>::store(acc);
#pragma unroll
    for (int dd = 0; dd < kMaxDst; ++dd)
      if (dd < nd) st_elem<PM, T>(d[dd], i, y);
  }
}

// KM caps the fan-in compiled in. The fp8-wire kernels use the untyped path for wire-to-wire copies only (K 1:
// typed_pattern_ok admits no other all-wire op for them); compiling K 2-8 in as well had put the bf16 fp8-wire
// fence kernel at 216 VGPRs (2 waves per SIMD) against 148 without them. Returns false for K > KM.
template <typename T, typename OP, int PM, int KM = kMaxSrc>
__device__ FX_INLINE bool xfer_dispatch(int K, const char* const (&s)[kMaxSrc], char* const (&d)[kMaxDst], int nd,
                                        uint64_t n, float scale, bool vec) {
  switch (K) {
    case 1: xfer_k<T, OP, 1, PM>(s, d, nd, n, scale, vec); return true;
    case 2: if constexpr (KM >= 2) { xfer_k<T, OP, 2, PM>(s, d, nd, n, scale, vec); return true; } return false;
    case 3: if constexpr (KM >= 3) { xfer_k<T, OP, 3, PM>(s, d, nd, n, scale, vec); return true; } return false;
    case 4: if constexpr (KM >= 4) { xfer_k<T, OP, 4, PM>(s, d, nd, n, scale, vec); return true; } return false;
    case 5: if constexpr (KM >= 5) { xfer_k<T, OP, 5, PM>(s, d, nd, n, scale, vec); return true; } return false;
    case 6: if constexpr (KM >= 6) { xfer_k<T, OP, 6, PM>(s, d, nd, n, scale, vec); return true; } return false;
    case 7: if constexpr (KM >= 7) { xfer_k<T, OP, 7, PM>(s, d, nd, n, scale, vec); return true; } return false;
    default: if constexpr (KM >= 8) { xfer_k<T, OP, 8, PM>(s, d, nd, n, scale, vec); return true; } return false;
  }
}

__device__ FX_INLINE uint64_t ld_flag(uint64_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ FX_INLINE void st_flag(uint64_t* f, uint64_t v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Caller-buffer operand: this rank's IN / OUT, or a peer's registered one (zero-copy programs only; the
// planner addresses peer IN / OUT nowhere else, planner.hpp validate_program)
__device__ FX_INLINE char* io_base(const DevCtx& c, const Loc& l) {
  return l.rank == c.rank ? c.local[l.buf] : c.peer_io[l.buf][l.rank];
}

template <typename T, typename OP, int PM>
__device__ FX_INLINE void xfer_op_range(const DevCtx& c, const Op* o, uint64_t lo, uint64_t hi, uint64_t par) {
  if (hi <= lo) return;
  const int ns = o->nsrc, nd = o->ndst;
  const char* s[kMaxSrc];
  char* d[kMaxDst];
  bool vec = true;
#pragma unroll
  for (int k = 0; k < kMaxSrc; ++k) {
    s[k] = nullptr;
    if (k < ns) {
      const Loc l = o->src[k];
      char* base = (l.buf == BUF_STG) ? c.peer_stg[l.rank] + par : io_base(c, l);
      s[k] = base + (l.off + lo) * sizeof(T);
      vec &= (l.buf == BUF_STG) || c.vec_ok;
    }
  }
#pragma unroll
  for (int k = 0; k < kMaxDst; ++k) {
    d[k] = nullptr;
    if (k < nd) {
      const Loc l = o->dst[k];
      char* base = (l.buf == BUF_STG) ? c.peer_stg[l.rank] + par : io_base(c, l);
      d[k] = base + (l.off + lo) * sizeof(T);
      vec &= (l.buf == BUF_STG) || c.vec_ok;
    }
  }
  if constexpr (PM == PM_WT) {
    const uint64_t step = kWtChunkBytes / sizeof(T);  // 32-bit buffer offsets
    for (uint64_t p = 0; p < hi - lo; p += step) {
      const char* s2[kMaxSrc];
      char* d2[kMaxDst];
#pragma unroll
      for (int k = 0; k < kMaxSrc; ++k) s2[k] = k < ns ? s[k] + p * sizeof(T) : nullptr;
#pragma unroll
      for (int k = 0; k < kMaxDst; ++k) d2[k] = k < nd ? d[k] + p * sizeof(T) : nullptr;
      xfer_dispatch<T, OP, PM>(ns, s2, d2, nd, (hi - lo - p) < step ? (hi - lo - p) : step, o->scale, vec);
    }
  } else {
    xfer_dispatch<T, OP, PM>(ns, s, d, nd, hi - lo, o->scale, vec);
  }
}

// ---------------------------------------------------------------------------------------------
// Typed XFER (Program::wire): operands of two storage types in one fused pass. Each lane handles G
// elements per step, G = 16 bytes of the narrower type, so every operand moves in whole 16-B vectors
// (VT / VW of them for a dtype / wire-typed operand) and all of a step's loads are issued before the
// first is consumed (the operand type is workgroup-uniform: the per-operand branches are scalar).
//   wire-typed source: its value;  dtype source: its value, or with an fp8 wire the value quantised with
//   the pre-scale (x * s -> fp8 -> f32) so every contribution is rounded once and identically;
//   y = scale * sum (fp32);  with an fp8 destination y is rounded to fp8 first, so the dtype destination
//   (y / s) and the fp8 copies the peers receive carry the same value on every rank.
template <typename W>
__device__ FX_INLINE float wround(float x) {
  return (float)Elem<W>::load(Elem<W>::store((typename Elem<W>::acc)x));
}
template <typename S> struct IsFp8 { static constexpr bool value = false; static constexpr bool e4m3 = false; };
template <> struct IsFp8<fp8e4m3_t> { static constexpr bool value = true; static constexpr bool e4m3 = true; };
template <> struct IsFp8<fp8e5m2_t> { static constexpr bool value = true; static constexpr bool e4m3 = false; };

// fp8 words through the packed gfx950 converters: v_cvt_pk_f32_fp8 / _bf8 turn two bytes of a word into
// two floats, v_cvt_pk_fp8_f32 / _bf8_f32 two floats into two bytes (RNE) — 2 instructions per 4 elements.
// No saturation: only for values the fp8 wire's pre-scale keeps in range (|x| <= fp8 max by construction).
template <typename S>
__device__ FX_INLINE void fp8_word_decode(uint32_t w, float* x) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 lo, hi;
  if constexpr (IsFp8<S>::e4m3) {
    lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false);
    hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
  } else {
    lo = __builtin_amdgcn_cvt_pk_f32_bf8((int)w, false);
    hi = __builtin_amdgcn_cvt_pk_f32_bf8((int)w, true);
  }
  x[0] = lo.x; x[1] = lo.y; x[2] = hi.x; x[3] = hi.y;
}
template <typename S>
__device__ FX_INLINE uint32_t fp8_word_encode(const float* x) {
  int w;
  if constexpr (IsFp8<S>::e4m3) {
    w = __builtin_amdgcn_cvt_pk_fp8_f32(x[0], x[1], 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(x[2], x[3], w, true);
  } else {
    w = __builtin_amdgcn_cvt_pk_bf8_f32(x[0], x[1], 0, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(x[2], x[3], w, true);
  }
  return (uint32_t)w;
}

// gfx950 scaled fp8 conversions (v_cvt_scalef32_pk_*): quantise a pair of f32 / bf16 / f16 values to fp8,
// or dequantise an fp8 pair back, with a scale in ONE instruction. Measured on the device
// (tools/probes/scaled_cvt_probe.hip, profiles/r4_scaled_cvt): q = rne(x / 2^floor(log2 scale)) and
// x = q * 2^floor(log2 scale) - only the scale's exponent counts (OCP MX e8m0 semantics) - and an overflow
// is NaN, as with the unscaled packed converts. The fp8 wire's pre-scale is a power of two (fp8_scale), so
// these give bit for bit what decode -> x * s -> encode gave, with 1 instruction per 2 elements instead of
// 3-5 (bf16: no f32 decode at all; the pair IS the instruction's packed operand).
typedef short fx_s2 __attribute__((ext_vector_type(2)));
typedef __bf16 fx_bf2 __attribute__((ext_vector_type(2)));
typedef _Float16 fx_h2 __attribute__((ext_vector_type(2)));
typedef float fx_f2 __attribute__((ext_vector_type(2)));
template <> struct IsFp8<mxe4m3_t> { static constexpr bool value = true; static constexpr bool e4m3 = true; };
template <> struct IsFp8<mxe5m2_t> { static constexpr bool value = true; static constexpr bool e4m3 = false; };
template <typename S> struct IsMx { static constexpr bool value = false; };
template <> struct IsMx<mxe4m3_t> { static constexpr bool value = true; };
template <> struct IsMx<mxe5m2_t> { static constexpr bool value = true; };
template <typename T> struct HasScaledCvt { static constexpr bool value = false; };
template <> struct HasScaledCvt<float> { static constexpr bool value = true; };
template <> struct HasScaledCvt<bf16_t> { static constexpr bool value = true; };
template <> struct HasScaledCvt<f16_t> { static constexpr bool value = true; };

// G values of T (packed in raw) -> G fp8 values (packed in out): q = rne(x / inv), inv a power of two;
// inv[r] applies to the run of RL elements r (RL = G: one scale for the group; MX blocks: one per run)
template <typename T, typename W, int G, int RL = G>
__device__ FX_INLINE void sq_group(const uint4* raw, const float* inv, uint4* out) {
  static_assert(RL % 4 == 0 && G % RL == 0, "runs of whole 4-element words");
  constexpr bool E4 = IsFp8<W>::e4m3;
  uint32_t w[G / 4];
  if constexpr (std::is_same<T, float>::value) {
    float f[G];
    __builtin_memcpy(f, raw, sizeof(f));
#pragma unroll
    for (int i = 0; i < G / 4; ++i) {
      fx_s2 r = {0, 0};
      if constexpr (E4) {
        r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, f[4 * i], f[4 * i + 1], inv[4 * i / RL], false);
        r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, f[4 * i + 2], f[4 * i + 3], inv[4 * i / RL], true);
      } else {
        r = __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(r, f[4 * i], f[4 * i + 1], inv[4 * i / RL], false);
        r = __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(r, f[4 * i + 2], f[4 * i + 3], inv[4 * i / RL], true);
      }
      __builtin_memcpy(&w[i], &r, 4);
    }
  } else {
    uint32_t p[G / 2];
    __builtin_memcpy(p, raw, sizeof(p));
#pragma unroll
    for (int i = 0; i < G / 4; ++i) {
      fx_s2 r = {0, 0};
      if constexpr (std::is_same<T, bf16_t>::value) {
        fx_bf2 a, b;
        __builtin_memcpy(&a, &p[2 * i], 4);
        __builtin_memcpy(&b, &p[2 * i + 1], 4);
        if constexpr (E4) {
          r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, a, inv[4 * i / RL], false);
          r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, b, inv[4 * i / RL], true);
        } else {
          r = __builtin_amdgcn_cvt_scalef32_pk_bf8_bf16(r, a, inv[4 * i / RL], false);
          r = __builtin_amdgcn_cvt_scalef32_pk_bf8_bf16(r, b, inv[4 * i / RL], true);
        }
      } else {
        fx_h2 a, b;
        __builtin_memcpy(&a, &p[2 * i], 4);
        __builtin_memcpy(&b, &p[2 * i + 1], 4);
        if constexpr (E4) {
          r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(r, a, inv[4 * i / RL], false);
          r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(r, b, inv[4 * i / RL], true);
        } else {
          r = __builtin_amdgcn_cvt_scalef32_pk_bf8_f16(r, a, inv[4 * i / RL], false);
          r = __builtin_amdgcn_cvt_scalef32_pk_bf8_f16(r, b, inv[4 * i / RL], true);
        }
      }
      __builtin_memcpy(&w[i], &r, 4);
    }
  }
  __builtin_memcpy(out, w, sizeof(w));
}

// G fp8 values (packed in raw) -> G values of T (packed in out): x = q * scale, scale a power of two
// (scale[r] for the run of RL elements r)
template <typename T, typename W, int G, int RL = G>
__device__ FX_INLINE void dq_group(const uint4* raw, const float* scale, uint4* out) {
  constexpr bool E4 = IsFp8<W>::e4m3;
  uint32_t w[G / 4];
  __builtin_memcpy(w, raw, sizeof(w));
  if constexpr (std::is_same<T, float>::value) {
    float f[G];
#pragma unroll
    for (int i = 0; i < G / 4; ++i) {
      fx_f2 lo, hi;
      if constexpr (E4) {
        lo = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(w[i], scale[4 * i / RL], false);
        hi = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(w[i], scale[4 * i / RL], true);
      } else {
        lo = __builtin_amdgcn_cvt_scalef32_pk_f32_bf8(w[i], scale[4 * i / RL], false);
        hi = __builtin_amdgcn_cvt_scalef32_pk_f32_bf8(w[i], scale[4 * i / RL], true);
      }
      f[4 * i] = lo.x; f[4 * i + 1] = lo.y; f[4 * i + 2] = hi.x; f[4 * i + 3] = hi.y;
    }
    __builtin_memcpy(out, f, sizeof(f));
  } else {
    uint32_t p[G / 2];
#pragma unroll
    for (int i = 0; i < G / 4; ++i) {
      if constexpr (std::is_same<T, bf16_t>::value) {
        fx_bf2 lo, hi;
        if constexpr (E4) {
          lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[i], scale[4 * i / RL], false);
          hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[i], scale[4 * i / RL], true);
        } else {
          lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(w[i], scale[4 * i / RL], false);
          hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(w[i], scale[4 * i / RL], true);
        }
        __builtin_memcpy(&p[2 * i], &lo, 4);
        __builtin_memcpy(&p[2 * i + 1], &hi, 4);
      } else {
        fx_h2 lo, hi;
        if constexpr (E4) {
          lo = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w[i], scale[4 * i / RL], false);
          hi = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w[i], scale[4 * i / RL], true);
        } else {
          lo = __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(w[i], scale[4 * i / RL], false);
          hi = __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(w[i], scale[4 * i / RL], true);
        }
        __builtin_memcpy(&p[2 * i], &lo, 4);
        __builtin_memcpy(&p[2 * i + 1], &hi, 4);
      }
    }
    __builtin_memcpy(out, p, sizeof(p));
  }
}

template <typename S, int G>
__device__ FX_INLINE void decode_g(const uint4* raw, float (&x)[G]) {
  if constexpr (IsFp8<S>::value && G % 4 == 0) {
    uint32_t w[G / 4];
    __builtin_memcpy(w, raw, G);
#pragma unroll
    for (int i = 0; i < G / 4; ++i) fp8_word_decode<S>(w[i], x + 4 * i);
  } else {
    S v[G];
    __builtin_memcpy(v, raw, sizeof(S) * G);
#pragma unroll
    for (int e = 0; e < G; ++e) x[e] = (float)Elem<S>::load(v[e]);
  }
}
// SAT = false: packed fp8 encode without saturation (fp8 wire values, in range by construction)
template <typename S, int G, bool SAT = true>
__device__ FX_INLINE void encode_g(const float (&x)[G], uint4* raw) {
  if constexpr (!SAT && IsFp8<S>::value && G % 4 == 0) {
    uint32_t w[G / 4];
#pragma unroll
    for (int i = 0; i < G / 4; ++i) w[i] = fp8_word_encode<S>(x + 4 * i);
    __builtin_memcpy(raw, w, G);
  } else {
    S v[G];
#pragma unroll
    for (int e = 0; e < G; ++e) v[e] = Elem<S>::store((typename Elem<S>::acc)x[e]);
    __builtin_memcpy(raw, v, sizeof(S) * G);
  }
}
// x <- fp8(x) for G values in range (packed encode + decode)
template <typename S, int G>
__device__ FX_INLINE void fp8_round_g(float (&x)[G]) {
#pragma unroll
  for (int i = 0; i < G / 4; ++i) fp8_word_decode<S>(fp8_word_encode<S>(x + 4 * i), x + 4 * i);
}

// Source patterns of a typed XFER (bit k of the source mask = operand k has the wire type). The
// planner only emits three (validate_typed_patterns): SP_T every source has the dtype (tree stage 0
// into fp32 partials, fp8 quantising push), SP_TW the first source (the rank's own value) has the dtype
// and the rest the wire type (ring step, fp8 reduction), SP_W every source has the wire type (final
// stage out of fp32 partials, fp8 all-gather). The pattern is a template parameter, so every operand's
// vector count is known at compile time and UU groups per lane are in flight per step (the same
// ~4-8 outstanding 16-B loads per lane as the untyped path).
enum : int { SP_T = 0, SP_TW = 1, SP_W = 2 };

// Per-lane batch of the typed executors (xfer_mx / xfer_mxb): UU super-groups' loads are issued before the
// first conversion - 4 when a group needs at most FLEXAR_TYPED_UU4_MAXV 16-B vectors per lane, 2 up to
// FLEXAR_TYPED_UU2_MAXV, else 1. Build-time knobs for A/B builds (bytes in flight).
#ifndef FLEXAR_TYPED_UU4_MAXV
#define FLEXAR_TYPED_UU4_MAXV 2
#endif
#ifndef FLEXAR_TYPED_UU2_MAXV
#define FLEXAR_TYPED_UU2_MAXV 4
#endif
constexpr int typed_uu(int v) { return v <= FLEXAR_TYPED_UU4_MAXV ? 4 : (v <= FLEXAR_TYPED_UU2_MAXV ? 2 : 1); }
// Software pipelining of the typed lane-interleaved loop (xfer_mx): on when a batch holds at most
// FLEXAR_TYPED_PIPE_MAXV 16-B vectors per lane (two batches are live; 0 = off). Build-time A/B knob.
#ifndef FLEXAR_TYPED_PIPE_MAXV
#define FLEXAR_TYPED_PIPE_MAXV 0
#endif
constexpr bool typed_pipe(int v) { return v <= FLEXAR_TYPED_PIPE_MAXV; }

template <typename T, typename W, int K, int SP, int PM, int ND = kMaxDst>
__device__ FX_INLINE void xfer_mx(const char* const (&s)[kMaxSrc], char* const (&d)[kMaxDst], int nd, uint32_t dm,
                                  uint64_t n, float scale, float pre, float post_inv, bool vec) {
  constexpr int U = sizeof(T) < sizeof(W) ? (int)sizeof(T) : (int)sizeof(W);
  constexpr int G = 16 / U;
  constexpr int VT = (int)sizeof(T) * G / 16, VW = (int)sizeof(W) * G / 16;
  constexpr int VM = VT > VW ? VT : VW;
  constexpr int V = SP == SP_T ? K * VT : (SP == SP_TW ? VT + (K - 1) * VW : K * VW);
  constexpr int UU = typed_uu(V);
  constexpr bool FP8 = sizeof(W) == 1;
  constexpr bool WT = PM == PM_WT;
  constexpr bool NTS = PM == PM_FENCE_NTS;
  auto isw = [](int k) constexpr -> bool { return SP == SP_W || (SP == SP_TW && k > 0); };
  const uint64_t nt = blockDim.x;
  const uint64_t ng = vec ? n / G : 0;
  __amdgpu_buffer_rsrc_t rs[K], rd[ND];
  if constexpr (WT) {
#pragma unroll
    for (int k = 0; k < K; ++k) rs[k] = rsrc_of(s[k], n * (isw(k) ? sizeof(W) : sizeof(T)));
#pragma unroll
    for (int dd = 0; dd < ND; ++dd)
      if (dd < nd) rd[dd] = rsrc_of(d[dd], n * ((dm >> dd) & 1 ? sizeof(W) : sizeof(T)));
  }
  auto ld = [&](int k, uint64_t byte) -> uint4 {
    if constexpr (WT) return ld16_sys(rs[k], (uint32_t)byte);
    else return ld16(s[k] + byte);
  };
  auto st = [&](int dd, uint64_t byte, uint4 y) {
    if constexpr (WT) st16_sys(rd[dd], (uint32_t)byte, y);
    else st16<NTS>(d[dd] + byte, y);
  };
  auto load_group = [&](uint64_t g, uint4 (&raw)[K][VM]) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t at = g * G * (isw(k) ? sizeof(W) : sizeof(T));
#pragma unroll
      for (int j = 0; j < (isw(k) ? VW : VT); ++j) raw[k][j] = ld(k, at + 16 * j);
    }
  };
  // fp8 wire: a single dtype source quantised straight into fp8 destinations (the push) needs one
  // rounding, done by the store's encode; any dtype destination needs the rounded value itself
  const bool direct = FP8 && K == 1 && SP == SP_T && dm == (1u << nd) - 1 && scale == 1.0f;
  const bool round_y = FP8 && dm && !direct;
  // gfx950 scaled converts (sq_group / dq_group): the quantising push (dtype -> fp8 everywhere) and the
  // dequantising all-gather (fp8 -> dtype everywhere) become one conversion per element pair, with no f32
  // round trip; `post_inv` = 1 / pre is the power of two both directions take
  constexpr bool SCV = FP8 && HasScaledCvt<T>::value;
  const bool fast_push = SCV && K == 1 && SP == SP_T && direct;
  const bool fast_ag = SCV && K == 1 && SP == SP_W && dm == 0 && scale == 1.0f;
  auto compute_group = [&](const uint4 (&raw)[K][VM], float (&acc)[G]) {
    if (fast_push || fast_ag) return;  // encode_dst converts straight from `raw`
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float x[G];
      if (isw(k)) {
        decode_g<W, G>(raw[k], x);
      } else if constexpr (SCV) {
        // every own contribution is the value the peers receive: fp8(x * pre), in one scaled convert
        uint4 q[VW > 0 ? VW : 1];
        sq_group<T, W, G>(raw[k], &post_inv, q);
        decode_g<W, G>(q, x);
      } else {
        decode_g<T, G>(raw[k], x);
        if constexpr (FP8) {
#pragma unroll
          for (int e = 0; e < G; ++e) x[e] *= pre;
          if (!direct) fp8_round_g<W, G>(x);
        }
      }
#pragma unroll
      for (int e = 0; e < G; ++e) acc[e] = k ? acc[e] + x[e] : x[e];
    }
#pragma unroll
    for (int e = 0; e < G; ++e) acc[e] *= scale;  // unconditional (x * 1 is exact): no per-element select
    if constexpr (FP8) {
      if (round_y) fp8_round_g<W, G>(acc);
    }
  };
  // destination dd's G values, packed in its element type
  auto encode_dst = [&](int dd, const uint4 (&raw)[K][VM], const float (&acc)[G], uint4 (&y)[VM]) {
    if constexpr (SCV && K == 1) {
      if (fast_push) return sq_group<T, W, G>(raw[0], &post_inv, y);
      if (fast_ag) return dq_group<T, W, G>(raw[0], &post_inv, y);
    }
    if ((dm >> dd) & 1) {
      encode_g<W, G, !FP8>(acc, y);  // fp8 wire values are in range: packed encode, no clamp
    } else {
      float t[G];
#pragma unroll
      for (int e = 0; e < G; ++e) t[e] = FP8 ? acc[e] * post_inv : acc[e];
      encode_g<T, G>(t, y);
    }
  };
  auto finish_group = [&](uint64_t g, const uint4 (&raw)[K][VM]) {
    float acc[G];
    compute_group(raw, acc);
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
      if (dd >= nd) continue;
      uint4 y[VM];
      encode_dst(dd, raw, acc, y);
      if ((dm >> dd) & 1) {
#pragma unroll
        for (int j = 0; j < VW; ++j) st(dd, g * G * sizeof(W) + 16 * j, y[j]);
      } else {
#pragma unroll
        for (int j = 0; j < VT; ++j) st(dd, g * G * sizeof(T) + 16 * j, y[j]);
      }
    }
  };
  uint64_t v = threadIdx.x;
  // Lane-interleaved super-groups (fence protocols, operands of two widths): a lane's G elements are VM
  // sub-chunks of SE elements, sub-chunk j of lane l at element sg * nt * G + (j * nt + l) * SE. Every
  // memory instruction (one j, one operand) then covers nt * SE contiguous elements across the wave -
  // 16 B per lane of the wider type, 4 or 8 B of the narrower - instead of lanes G elements apart (64 B
  // per lane for fp32 next to an fp8 wire: every instruction strided). Round 3: the fp32 -> e4m3 wire
  // executor ran at 3.5 TB/s of HBM traffic against 5.8 TB/s for the untyped flat (bench/
  // typed_exec_probe.py). Same arithmetic per element, other lanes: the results are bit-identical.
  if constexpr (!WT && VM > 1) {
    constexpr int SE = G / VM;
    const uint64_t span = nt * (uint64_t)G;
    const uint64_t nsg = vec ? n / span : 0;
    constexpr int SBT = SE * (int)sizeof(T), SBW = SE * (int)sizeof(W);
    const uint32_t lt = threadIdx.x * SBT, lw = threadIdx.x * SBW;  // the lane's offset, per element size
    uint64_t sg = 0;
    // one iteration over UI super-groups; full super-groups beyond the last multiple of UU take the same
    // lane-interleaved layout one at a time (a slice of a few super-groups - DDP buckets, small pieces -
    // would otherwise fall to the contiguous layout's lane-strided instructions)
    // `lim` elements from super-group sg: UI * span, or fewer for the last, partial super-group, whose lanes
    // past `lim` load zeros and drop their stores (the buffer descriptors' range check; lim is a multiple of
    // G, so every sub-chunk access is wholly inside or outside)
    // descriptors over UI super-groups from sg0 (<= UI * 16 KiB * 4 B: 32-bit offsets); the loads and the
    // compute + stores are separate halves, so the pipelined loop below can issue one batch's loads before
    // the previous batch's stores
    auto load_it = [&](auto ucnt, uint64_t sg0, uint64_t lim, uint4 (&raw)[decltype(ucnt)::value][K][VM]) {
      constexpr int UI = decltype(ucnt)::value;
      __amdgpu_buffer_rsrc_t bs[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint64_t es = isw(k) ? sizeof(W) : sizeof(T);
        bs[k] = rsrc_of(s[k] + sg0 * span * es, lim * es);
      }
#pragma unroll
      for (int u = 0; u < UI; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
          for (int j = 0; j < VM; ++j) {
            const uint32_t e0 = (uint32_t)(u * span + j * nt * SE);  // uniform
            if (isw(k)) ld_sub<SBW>(raw[u][k], j, bs[k], lw, e0 * (uint32_t)sizeof(W));
            else ld_sub<SBT>(raw[u][k], j, bs[k], lt, e0 * (uint32_t)sizeof(T));
          }
    };
    auto finish_it = [&](auto ucnt, uint64_t sg0, uint64_t lim, const uint4 (&raw)[decltype(ucnt)::value][K][VM]) {
      constexpr int UI = decltype(ucnt)::value;
      __amdgpu_buffer_rsrc_t bd[ND];
#pragma unroll
      for (int dd = 0; dd < ND; ++dd) {
        if (dd >= nd) continue;
        const uint64_t es = (dm >> dd) & 1 ? sizeof(W) : sizeof(T);
        bd[dd] = rsrc_of(d[dd] + sg0 * span * es, lim * es);
      }
#pragma unroll
      for (int u = 0; u < UI; ++u) {
        float acc[G];
        compute_group(raw[u], acc);
#pragma unroll
        for (int dd = 0; dd < ND; ++dd) {
          if (dd >= nd) continue;
          uint4 y[VM];
          encode_dst(dd, raw[u], acc, y);
          const bool wide = (dm >> dd) & 1;
#pragma unroll
          for (int j = 0; j < VM; ++j) {
            const uint32_t e0 = (uint32_t)(u * span + j * nt * SE);
            if (wide) st_sub<SBW, NTS>(bd[dd], lw, e0 * (uint32_t)sizeof(W), y, j);
            else st_sub<SBT, NTS>(bd[dd], lt, e0 * (uint32_t)sizeof(T), y, j);
          }
        }
      }
    };
    auto iter = [&](auto ucnt, uint64_t lim) {
      uint4 raw[decltype(ucnt)::value][K][VM];
      load_it(ucnt, sg, lim, raw);
      finish_it(ucnt, sg, lim, raw);
    };
    using UUc = std::integral_constant<int, UU>;
    if constexpr (typed_pipe(UU * K * VM)) {
      // two batches in flight: batch i+1's loads are issued before batch i's converts and stores. On gfx9
      // one counter (vmcnt) tracks loads and stores in issue order, so in the plain loop each batch's loads
      // also wait out the previous batch's store acknowledgements; here they are older than those stores.
      const uint64_t nmain = nsg - nsg % UU;
      if (nmain) {
        uint4 ra[UU][K][VM], rb[UU][K][VM];
        const uint64_t lim = (uint64_t)UU * span;
        load_it(UUc{}, 0, lim, ra);
        for (;;) {
          const bool more = sg + UU < nmain;
          if (more) load_it(UUc{}, sg + UU, lim, rb);
          finish_it(UUc{}, sg, lim, ra);
          sg += UU;
          if (!more) break;
          const bool more2 = sg + UU < nmain;
          if (more2) load_it(UUc{}, sg + UU, lim, ra);
          finish_it(UUc{}, sg, lim, rb);
          sg += UU;
          if (!more2) break;
        }
      }
    } else {
      for (; sg + UU <= nsg; sg += UU) iter(UUc{}, (uint64_t)UU * span);
    }
    if constexpr (UU > 1)
      for (; sg < nsg; ++sg) iter(std::integral_constant<int, 1>{}, span);
    if (sg * span < ng * G) iter(std::integral_constant<int, 1>{}, ng * G - sg * span);
    v = ng;  // every whole group done; the scalar tail takes the last < G elements
  }
  // the contiguous layout: write-through executors (their coherent loads take whole-group descriptors)
  if constexpr (WT || VM == 1) {
  for (; v + (UU - 1) * nt < ng; v += UU * nt) {
    uint4 raw[UU][K][VM];
#pragma unroll
    for (int u = 0; u < UU; ++u) load_group(v + u * nt, raw[u]);
#pragma unroll
    for (int u = 0; u < UU; ++u) finish_group(v + u * nt, raw[u]);
  }
  for (; v < ng; v += nt) {
    uint4 raw[K][VM];
    load_group(v, raw);
    finish_group(v, raw);
  }
  }
  // scalar tail: the last < G elements (or the whole span when FLEXAR_SCALAR_MISALIGNED=1 and a caller buffer is
  // not 16-B aligned)
  for (uint64_t i = ng * G + threadIdx.x; i < n; i += nt) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float x;
      if (isw(k)) {
        x = (float)Elem<W>::load(ld_elem<PM, W>(s[k], i));
      } else {
        x = (float)Elem<T>::load(ld_elem<PM, T>(s[k], i));
        if constexpr (FP8) x = wround<W>(x * pre);
      }
      acc = k ? acc + x : x;
    }
    acc *= scale;
    if (FP8 && dm) acc = wround<W>(acc);
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
      if (dd >= nd) continue;
      if ((dm >> dd) & 1) st_elem<PM, W>(d[dd], i, Elem<W>::store((typename Elem<W>::acc)acc));
      else st_elem<PM, T>(d[dd], i, Elem<T>::store((typename Elem<T>::acc)(FP8 ? acc * post_inv : acc)));
    }
  }
}

// ---- MX wire: OCP MX block-scaled fp8 (AlgoSpec::wire 4 / 5) ------------------------------------------
// The flat schedule of the fp8 wire with a scale per 32-element block instead of one per call: no amax
// pass and no amax agreement before the launch, and each block's scale follows its own magnitude (a
// block of small gradients next to large ones keeps fp8's relative precision instead of flushing to zero).
// The block scales of a staging operand live in the same rank's staging half at mx_shadow + byte / 32
// (planner.hpp Program::mx_shadow). Semantics, element for element what host_exec.hpp host_xfer_mxb
// computes (docs/DESIGN.md §9.2):
//   quantising push (K = 1, SP_T): 2^X from the block's max |x * scale|, q = rne(x * scale / 2^X) (one
//     scaled convert per element pair), q and the e8m0 byte to every wire destination;
//   dequantising all-gather (K = 1, SP_W): q * 2^X * scale into dtype destinations;
//   reduction (K >= 2, SP_TW): the own value rounded through MX with its own block scale, each peer's
//     q * 2^X, summed in fp32 in source order, times scale, re-quantised with the sum's block scale for the
//     wire destinations, and that value (q * 2^X) into the dtype ones.
// A block's 32 elements sit in consecutive lanes of one wave (8 lanes x 4 for fp32 inputs, 4 x 8 for
// 16-bit ones, 2 x 16 in the contiguous layout), so its maximum is a few cross-lane swaps.

// per run of RL elements of a packed group of 16 values of T: the f32 bits of the largest magnitude (an
// unsigned maximum of the sign-cleared bits, as mx_scale_byte expects)
typedef unsigned short fx_u16x2 __attribute__((ext_vector_type(2)));
template <typename T, int RL>
__device__ FX_INLINE void mx_run_amax(const uint4* raw, uint32_t (&m)[16 / RL]) {
  constexpr int R = 16 / RL;
  if constexpr (std::is_same<T, float>::value) {
    uint32_t w[16];
    __builtin_memcpy(w, raw, sizeof(w));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      uint32_t a = 0;
#pragma unroll
      for (int e = r * RL; e < (r + 1) * RL; ++e) a = max(a, w[e] & 0x7fffffffu);
      m[r] = a;
    }
  } else {
    uint32_t w[8];
    __builtin_memcpy(w, raw, sizeof(w));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      fx_u16x2 a = {0, 0};
#pragma unroll
      for (int i = r * RL / 2; i < (r + 1) * RL / 2; ++i)
        a = __builtin_elementwise_max(a, __builtin_bit_cast(fx_u16x2, w[i] & 0x7fff7fffu));  // v_pk_max_u16
      const uint16_t h = a.x > a.y ? a.x : a.y;
      if constexpr (std::is_same<T, bf16_t>::value) m[r] = (uint32_t)h << 16;
      else m[r] = __float_as_uint((float)__builtin_bit_cast(_Float16, h));
    }
  }
}
template <int RL>
__device__ FX_INLINE void mx_run_amax_f(const float (&x)[16], uint32_t (&m)[16 / RL]) {
#pragma unroll
  for (int r = 0; r < 16 / RL; ++r) {
    uint32_t a = 0;
#pragma unroll
    for (int e = r * RL; e < (r + 1) * RL; ++e) a = max(a, __float_as_uint(x[e]) & 0x7fffffffu);
    m[r] = a;
  }
}
// maximum over the LPB consecutive lanes that hold one block (LPB a power of two dividing 64)
template <int LPB>
__device__ FX_INLINE uint32_t mx_block_max(uint32_t m) {
#pragma unroll
  for (int o = 1; o < LPB; o <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  return m;
}

// The reduction's three steps (SP_TW), also run in operand batches by xfer_mxb for fan-ins above 4:
// acc = the own value rounded through MX with its own block scale (what a peer would receive) ...
template <typename T, typename W, int RL>
__device__ FX_INLINE void mx_own(const uint4 (&raw)[(int)sizeof(T)], float (&acc)[16]) {
  constexpr int R = 16 / RL, LPB = (int)kMxBlock / RL;
  uint32_t m[R];
  mx_run_amax<T, RL>(raw, m);
  float s0[R];
#pragma unroll
  for (int r = 0; r < R; ++r) s0[r] = mx_scale_value(mx_scale_byte(mx_block_max<LPB>(m[r]), IsFp8<W>::e4m3));
  uint4 q, t[4];
  sq_group<T, W, 16, RL>(raw, s0, &q);
  dq_group<float, W, 16, RL>(&q, s0, t);
  __builtin_memcpy(acc, t, sizeof(acc));
}
// ... plus each peer's q * 2^X ...
template <typename W, int RL>
__device__ FX_INLINE void mx_wire_add(const uint4& raw, const uint32_t (&sb)[16 / RL], float (&acc)[16]) {
  float sk[16 / RL];
#pragma unroll
  for (int r = 0; r < 16 / RL; ++r) sk[r] = mx_scale_value(sb[r]);
  uint4 t[4];
  dq_group<float, W, 16, RL>(&raw, sk, t);
  float x[16];
  __builtin_memcpy(x, t, sizeof(x));
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] += x[e];
}
// ... then times scale and, with a wire destination, re-quantised with the sum's own block scales.
template <typename T, typename W, int RL>
__device__ FX_INLINE void mx_finish(float (&acc)[16], float scale, int nd, uint32_t dm, uint4& yq,
                                    uint32_t (&xb)[16 / RL], uint4 (&yt)[(int)sizeof(T)]) {
  constexpr int R = 16 / RL, LPB = (int)kMxBlock / RL;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] *= scale;
  if (dm) {
    uint32_t m[R];
    float sc[R];
    mx_run_amax_f<RL>(acc, m);
#pragma unroll
    for (int r = 0; r < R; ++r) xb[r] = mx_scale_byte(mx_block_max<LPB>(m[r]), IsFp8<W>::e4m3), sc[r] = mx_scale_value(xb[r]);
    uint4 t[4];
    __builtin_memcpy(t, acc, sizeof(acc));
    sq_group<float, W, 16, RL>(t, sc, &yq);
    if (dm != (1u << nd) - 1) dq_group<T, W, 16, RL>(&yq, sc, yt);
  } else {
    encode_g<T, 16>(acc, yt);
  }
}

// One lane's group of 16 elements in runs of RL (sb[k][r] = the scale byte of wire source k's block for
// run r, loaded with the payload): the fp8 result `yq` with its block scale bytes `xb` (wire
// destinations) and / or the dtype result `yt` (dtype destinations).
template <typename T, typename W, int K, int SP, int RL>
__device__ FX_INLINE void mx_group(const uint4 (&raw)[K][(int)sizeof(T)], const uint32_t (&sb)[K][16 / RL], float scale,
                                   int nd, uint32_t dm, uint4& yq, uint32_t (&xb)[16 / RL], uint4 (&yt)[(int)sizeof(T)]) {
  constexpr int R = 16 / RL, LPB = (int)kMxBlock / RL;
  constexpr bool E4 = IsFp8<W>::e4m3;
  const uint32_t all_d = (1u << nd) - 1;
  float sc[R];
  if constexpr (SP == SP_T) {
    uint32_t m[R];
    if (scale == 1.0f) {
      mx_run_amax<T, RL>(raw[0], m);
#pragma unroll
      for (int r = 0; r < R; ++r) xb[r] = mx_scale_byte(mx_block_max<LPB>(m[r]), E4), sc[r] = mx_scale_value(xb[r]);
      sq_group<T, W, 16, RL>(raw[0], sc, &yq);
    } else {
      float y[16];
      decode_g<T, 16>(raw[0], y);
#pragma unroll
      for (int e = 0; e < 16; ++e) y[e] *= scale;
      mx_run_amax_f<RL>(y, m);
#pragma unroll
      for (int r = 0; r < R; ++r) xb[r] = mx_scale_byte(mx_block_max<LPB>(m[r]), E4), sc[r] = mx_scale_value(xb[r]);
      uint4 t[4];
      __builtin_memcpy(t, y, sizeof(y));
      sq_group<float, W, 16, RL>(t, sc, &yq);
    }
    if (dm != all_d) dq_group<T, W, 16, RL>(&yq, sc, yt);
  } else if constexpr (SP == SP_W) {
#pragma unroll
    for (int r = 0; r < R; ++r) sc[r] = mx_scale_value(sb[0][r]);
    if (scale == 1.0f) {
      dq_group<T, W, 16, RL>(&raw[0][0], sc, yt);
    } else {
      uint4 t[4];
      dq_group<float, W, 16, RL>(&raw[0][0], sc, t);
      float y[16];
      __builtin_memcpy(y, t, sizeof(y));
#pragma unroll
      for (int e = 0; e < 16; ++e) y[e] *= scale;
      encode_g<T, 16>(y, yt);
    }
  } else {
    float acc[16];
    mx_own<T, W, RL>(raw[0], acc);
#pragma unroll
    for (int k = 1; k < K; ++k) mx_wire_add<W, RL>(raw[k][0], sb[k], acc);
    mx_finish<T, W, RL>(acc, scale, nd, dm, yq, xb, yt);
  }
}

// One element of an MX operation by itself (the tail of a slice: fewer than 32 elements, or the whole
// slice when a caller buffer takes no vector access): each thread recomputes its block's scale from the
// block's elements, so it needs no other lane.
template <typename T, typename W, int K, int SP, int PM>
__device__ FX_INLINE void mx_elem(const char* const (&s)[kMaxSrc], const uint8_t* const (&ss)[kMaxSrc],
                                  char* const (&d)[kMaxDst], uint8_t* const (&sd)[kMaxDst], int nd, uint32_t dm,
                                  uint64_t n, float scale, uint64_t i) {
  constexpr bool E4 = IsFp8<W>::e4m3;
  const uint64_t b = i / kMxBlock, b0 = b * kMxBlock, b1 = b0 + kMxBlock < n ? b0 + kMxBlock : n;
  auto own = [&](int k, uint64_t j) { return (float)Elem<T>::load(ld_elem<PM, T>(s[k], j)); };
  auto wire = [&](int k, uint64_t j) {
    return (float)Elem<W>::load(W{ld_elem<PM, uint8_t>(s[k], j)}) *
           mx_scale_value(ld_elem<PM, uint8_t>(reinterpret_cast<const char*>(ss[k]), b));
  };
  float y;
  uint32_t xr = 0;
  if constexpr (SP == SP_T) {
    uint32_t am = 0;
    for (uint64_t j = b0; j < b1; ++j) am = max(am, __float_as_uint(own(0, j) * scale) & 0x7fffffffu);
    xr = mx_scale_byte(am, E4);
    y = own(0, i) * scale;
  } else if constexpr (SP == SP_W) {
    y = wire(0, i) * scale;
  } else {
    uint32_t am0 = 0;
    for (uint64_t j = b0; j < b1; ++j) am0 = max(am0, __float_as_uint(own(0, j)) & 0x7fffffffu);
    const float s0 = mx_scale_value(mx_scale_byte(am0, E4));
    auto sum = [&](uint64_t j) {
      float a = (float)Elem<W>::load(Elem<W>::store(own(0, j) / s0)) * s0;
#pragma unroll
      for (int k = 1; k < K; ++k) a += wire(k, j);
      return a * scale;
    };
    y = sum(i);
    if (dm) {
      uint32_t am = 0;
      for (uint64_t j = b0; j < b1; ++j) am = max(am, __float_as_uint(sum(j)) & 0x7fffffffu);
      xr = mx_scale_byte(am, E4);
    }
  }
  uint8_t q = 0;
  if (xr) {
    const float sc = mx_scale_value(xr);
    q = Elem<W>::store(y / sc).bits;
    y = (float)Elem<W>::load(W{q}) * sc;
  }
#pragma unroll
  for (int dd = 0; dd < kMaxDst; ++dd) {
    if (dd >= nd) continue;
    if ((dm >> dd) & 1) {
      st_elem<PM, uint8_t>(d[dd], i, q);
      if (i == b0) st_elem<PM, uint8_t>(reinterpret_cast<char*>(sd[dd]), b, (uint8_t)xr);
    } else {
      st_elem<PM, T>(d[dd], i, Elem<T>::store((typename Elem<T>::acc)y));
    }
  }
}

// The MX executor over one slice (starting on a block boundary): full super-groups in the lane-interleaved
// layout of xfer_mx (every memory instruction contiguous across the workgroup; the scale bytes through
// buffer descriptors built once, at one per-lane offset shared by every operand), then whole blocks in the
// contiguous layout (16 elements per lane, a block per lane pair), then the last partial block element-wise.
template <typename T, typename W, int K, int SP, int PM, int ND = kMaxDst>
__device__ FX_INLINE void xfer_mxb(const char* const (&s)[kMaxSrc], const uint8_t* const (&ss)[kMaxSrc],
                                   char* const (&d)[kMaxDst], uint8_t* const (&sd)[kMaxDst], int nd, uint32_t dm,
                                   uint64_t n, float scale, bool vec) {
  constexpr int G = 16;
  constexpr int VT = (int)sizeof(T);  // 16-B vectors per group of T (W: one)
  constexpr int V = SP == SP_T ? VT : (SP == SP_TW ? VT + (K - 1) : K);
  constexpr int UU = typed_uu(V);
  constexpr bool WT = PM == PM_WT;
  constexpr bool NTS = PM == PM_FENCE_NTS;
  auto isw = [](int k) constexpr -> bool { return SP == SP_W || (SP == SP_TW && k > 0); };
  const uint64_t nt = blockDim.x;
  uint64_t v = threadIdx.x;  // next contiguous group of this lane
  if constexpr (!WT) {
    constexpr int VM = VT, SE = G / VM, RL = SE;  // lane l's run j: elements (j * nt + l) * SE .. + SE
    constexpr int LPB = (int)kMxBlock / SE;
    const uint64_t span = nt * (uint64_t)G;
    const uint64_t nsg = vec ? n / span : 0;
    constexpr int SBT = SE * (int)sizeof(T), SBW = SE;
    const uint32_t lt = threadIdx.x * SBT, lw = threadIdx.x * SBW;
    const uint32_t lb = threadIdx.x / LPB;  // the lane's block within a run's row of nt * SE elements
    const bool lead = (threadIdx.x % LPB) == 0;
    // the scale shadows cover the whole blocks only: the last partial block is the scalar tail's (mx_elem),
    // so a lane of the partial super-group never writes its scale
    const uint64_t nfull = n / kMxBlock;
    __amdgpu_buffer_rsrc_t rss[K], rsd[ND];
#pragma unroll
    for (int k = 0; k < K; ++k) rss[k] = rsrc_of(isw(k) ? (const char*)ss[k] : nullptr, isw(k) ? nfull : 0);
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) rsd[dd] = rsrc_of((const char*)sd[dd], sd[dd] ? nfull : 0);
    uint64_t sg = 0;
    // one iteration over UI super-groups; full super-groups beyond the last multiple of UU take the same
    // lane-interleaved layout one at a time (a slice of a few super-groups - DDP buckets, small pieces -
    // would otherwise fall to the contiguous layout's lane-strided instructions)
    // `lim` elements from super-group sg (fewer for the last, partial one: see xfer_mx)
    auto iter = [&](auto ucnt, uint64_t lim) {
      constexpr int UI = decltype(ucnt)::value;
      __amdgpu_buffer_rsrc_t bs[K], bd[ND];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint64_t es = isw(k) ? 1 : sizeof(T);
        bs[k] = rsrc_of(s[k] + sg * span * es, lim * es);
      }
#pragma unroll
      for (int dd = 0; dd < ND; ++dd) {
        if (dd >= nd) continue;
        const uint64_t es = (dm >> dd) & 1 ? 1 : sizeof(T);
        bd[dd] = rsrc_of(d[dd] + sg * span * es, lim * es);
      }
      // block of (u, j) = sboff(u, j) (uniform) + lb (per lane)
      auto sboff = [&](int u, int j) -> uint32_t { return (uint32_t)(((sg + u) * span + j * nt * SE) / kMxBlock); };
      uint4 raw[UI][K][VM];
      uint32_t sb[UI][K][VM];
#pragma unroll
      for (int u = 0; u < UI; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
          for (int j = 0; j < VM; ++j) {
            const uint32_t e0 = (uint32_t)(u * span + j * nt * SE);  // uniform
            if (isw(k)) {
              ld_sub<SBW>(raw[u][k], j, bs[k], lw, e0);
              sb[u][k][j] = __builtin_amdgcn_raw_buffer_load_b8(rss[k], lb, sboff(u, j), kAuxLd);
            } else {
              ld_sub<SBT>(raw[u][k], j, bs[k], lt, e0 * (uint32_t)sizeof(T));
              sb[u][k][j] = 0;
            }
          }
#pragma unroll
      for (int u = 0; u < UI; ++u) {
        uint4 yq, yt[VM];
        uint32_t xb[VM];
        mx_group<T, W, K, SP, RL>(raw[u], sb[u], scale, nd, dm, yq, xb, yt);
#pragma unroll
        for (int dd = 0; dd < ND; ++dd) {
          if (dd >= nd) continue;
          const bool wide = (dm >> dd) & 1;
#pragma unroll
          for (int j = 0; j < VM; ++j) {
            const uint32_t e0 = (uint32_t)(u * span + j * nt * SE);
            if (wide) {
              const uint4 q1[1] = {yq};
              st_sub<SBW, NTS>(bd[dd], lw, e0, q1, j);
              if (lead) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)xb[j], rsd[dd], lb, sboff(u, j), NTS ? 2 : 0);
            } else {
              st_sub<SBT, NTS>(bd[dd], lt, e0 * (uint32_t)sizeof(T), yt, j);
            }
          }
        }
      }
    };
    const uint64_t nwhole = vec ? (n / kMxBlock) * kMxBlock : 0;
    for (; sg + UU <= nsg; sg += UU) iter(std::integral_constant<int, UU>{}, (uint64_t)UU * span);
    if constexpr (UU > 1)
      for (; sg < nsg; ++sg) iter(std::integral_constant<int, 1>{}, span);
    if (sg * span < nwhole) iter(std::integral_constant<int, 1>{}, nwhole - sg * span);
    v = (n / kMxBlock) * 2;  // every whole block done
  }
  // whole blocks, contiguous layout (write-through executors): group g = elements 16 g .. 16 g + 15,
  // block g / 2 (lanes g, g ^ 1)
  const uint64_t ng = vec ? (n / kMxBlock) * 2 : 0;
  auto ld = [&](int k, uint64_t byte) -> uint4 {
    if constexpr (WT) return ld16_sys(rsrc_of(s[k], isw(k) ? n : n * sizeof(T)), (uint32_t)byte);
    else return ld16(s[k] + byte);
  };
  auto st = [&](int dd, uint64_t byte, uint4 y) {
    if constexpr (WT) st16_sys(rsrc_of(d[dd], (dm >> dd) & 1 ? n : n * sizeof(T)), (uint32_t)byte, y);
    else st16<NTS>(d[dd] + byte, y);
  };
  if constexpr (WT)
  for (; v < ng; v += nt) {
    uint4 raw[K][VT];
    uint32_t sb[K][1];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (isw(k)) {
        raw[k][0] = ld(k, v * G);
        sb[k][0] = ld_elem<PM, uint8_t>(reinterpret_cast<const char*>(ss[k]), v / 2);
      } else {
        sb[k][0] = 0;
#pragma unroll
        for (int j = 0; j < VT; ++j) raw[k][j] = ld(k, v * G * sizeof(T) + 16 * j);
      }
    }
    uint4 yq, yt[VT];
    uint32_t xb[1];
    mx_group<T, W, K, SP, G>(raw, sb, scale, nd, dm, yq, xb, yt);
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
      if (dd >= nd) continue;
      if ((dm >> dd) & 1) {
        st(dd, v * G, yq);
        if ((v & 1) == 0) st_elem<PM, uint8_t>(reinterpret_cast<char*>(sd[dd]), v / 2, (uint8_t)xb[0]);
      } else {
#pragma unroll
        for (int j = 0; j < VT; ++j) st(dd, v * G * sizeof(T) + 16 * j, yt[j]);
      }
    }
  }
  for (uint64_t i = ng * G + threadIdx.x; i < n; i += nt) mx_elem<T, W, K, SP, PM>(s, ss, d, sd, nd, dm, n, scale, i);
}

// fp8 / MX wire transfers instantiate for at most 2 destinations (xfer_mx_k, xfer_mxb_k); 0 = the A/B build with the
// general (kMaxDst) form
#ifndef FLEXAR_MX_ND2
#define FLEXAR_MX_ND2 1
#endif
// The (K, pattern) combinations the planner emits (validate_typed_patterns): fp8 wire = quantising push
// (K 1, SP_T), reduction (K >= 2, SP_TW), dequantising all-gather (K 1, SP_W); fp32 partials = tree
// stage 0 (SP_T), ring step (K 2, SP_TW), final stage / temp chains (SP_W). Anything else is reported
// as a protocol error instead of being computed wrongly.
template <typename T, typename W, int K, int PM>
__device__ FX_INLINE bool xfer_mx_k(int sp, const char* const (&s)[kMaxSrc], char* const (&d)[kMaxDst], int nd,
                                    uint32_t dm, uint64_t n, float scale, float pre, float post_inv, bool vec) {
  constexpr bool FP8 = sizeof(W) == 1;
  // fp8 wires write at most 2 destinations (they always pull: planner.hpp typed_pattern_ok), the same register
  // saving as the MX wire's (xfer_mxb_k); fp32 partials keep the general form (push all-gathers multicast)
  constexpr int ND = FP8 && FLEXAR_MX_ND2 ? 2 : kMaxDst;
  if (nd > ND) return false;
  if (sp == SP_T && (FP8 ? K == 1 : K >= 2)) {
    if constexpr (FP8 ? K == 1 : K >= 2) xfer_mx<T, W, K, SP_T, PM, ND>(s, d, nd, dm, n, scale, pre, post_inv, vec);
    return true;
  }
  if (sp == SP_TW && K >= 2 && (FP8 || K == 2)) {
    if constexpr (K >= 2 && (FP8 || K == 2)) xfer_mx<T, W, K, SP_TW, PM, ND>(s, d, nd, dm, n, scale, pre, post_inv, vec);
    return true;
  }
  if (sp == SP_W && (FP8 ? K == 1 : K >= 2)) {
    if constexpr (FP8 ? K == 1 : K >= 2) xfer_mx<T, W, K, SP_W, PM, ND>(s, d, nd, dm, n, scale, pre, post_inv, vec);
    return true;
  }
  return false;
}

// MX wire patterns (validate: typed_pattern_ok): quantising push (K 1, SP_T), reduction (K >= 2, SP_TW),
// dequantising all-gather (K 1, SP_W, dtype destinations only).
template <typename T, typename W, int K, int PM>
__device__ FX_INLINE bool xfer_mxb_k(int sp, const char* const (&s)[kMaxSrc], const uint8_t* const (&ss)[kMaxSrc],
                                     char* const (&d)[kMaxDst], uint8_t* const (&sd)[kMaxDst], int nd, uint32_t dm,
                                     uint64_t n, float scale, bool vec) {
  // MX ops write at most 2 destinations (planner.hpp typed_pattern_ok; fp8 wires always pull): an instantiation for
  // 2 keeps 6 destination pointers, 6 scale pointers and their buffer descriptors out of the registers. The general
  // one (up to kMaxDst) set the fan-in-8 kernel's allocation to 256 VGPRs plus scratch spills (profiles/r6_mx_nd/).
  // FLEXAR_MX_ND2=0: the A/B build with the general instantiation.
  constexpr int ND = FLEXAR_MX_ND2 ? 2 : kMaxDst;
  if (nd > ND) return false;
  if constexpr (K == 1) {
    if (sp == SP_T) { xfer_mxb<T, W, 1, SP_T, PM, ND>(s, ss, d, sd, nd, dm, n, scale, vec); return true; }
    if (sp == SP_W && dm == 0) { xfer_mxb<T, W, 1, SP_W, PM, ND>(s, ss, d, sd, nd, dm, n, scale, vec); return true; }
    return false;
  } else {
    if (sp == SP_TW) { xfer_mxb<T, W, K, SP_TW, PM, ND>(s, ss, d, sd, nd, dm, n, scale, vec); return true; }
    return false;
  }
}

// Typed op: operand addresses (STG offsets in units, element slice [lo, hi) in each operand's own
// type), then the all-dtype / all-wire fast paths or the mixed one.
// KMAX: the widest fan-in this instantiation runs (fp8 wire kernels come in KMAX 4 and 8: the K 5..8 cases
// raise the whole kernel's register allocation - 256 VGPRs and scratch spills - which cost the 4-rank MX
// executor 25 % (profiles/r4_mx/README.md); programs with fan-in <= 4 launch the narrow instantiation).
template <typename T, typename W, int PM, int KMAX = kMaxSrc>
__device__ FX_INLINE void xfer_op_typed_range(const DevCtx& c, const Op* o, uint64_t lo, uint64_t hi, uint64_t par,
                                              float pre, float post_inv) {
  if (hi <= lo) return;
  constexpr bool FP8 = sizeof(W) == 1;
  const int ns = o->nsrc, nd = o->ndst;
  const uint32_t sm = o->pad16[0], dm = o->pad16[1];
  const char* s[kMaxSrc];
  char* d[kMaxDst];
  bool vec = true;
#pragma unroll
  for (int k = 0; k < kMaxSrc; ++k) {
    s[k] = nullptr;
    if (k < ns) {
      const Loc l = o->src[k];
      const uint64_t es = (sm >> k) & 1 ? sizeof(W) : sizeof(T);
      s[k] = (l.buf == BUF_STG) ? c.peer_stg[l.rank] + par + l.off * c.stg_unit + lo * es
                                : c.local[l.buf] + (l.off + lo) * sizeof(T);
      vec &= (l.buf == BUF_STG) || c.vec_ok;
    }
  }
#pragma unroll
  for (int k = 0; k < kMaxDst; ++k) {
    d[k] = nullptr;
    if (k < nd) {
      const Loc l = o->dst[k];
      const uint64_t es = (dm >> k) & 1 ? sizeof(W) : sizeof(T);
      d[k] = (l.buf == BUF_STG) ? c.peer_stg[l.rank] + par + l.off * c.stg_unit + lo * es
                                : c.local[l.buf] + (l.off + lo) * sizeof(T);
      vec &= (l.buf == BUF_STG) || c.vec_ok;
    }
  }
  const uint64_t n = hi - lo;
  const uint32_t all_s = (1u << ns) - 1, all_d = (1u << nd) - 1;
  const int sp = sm == 0 ? SP_T : (sm == (all_s & ~1u) ? SP_TW : (sm == all_s ? SP_W : -1));
  bool ok = false;
  if constexpr (IsMx<W>::value) {
    // block scales: the shadow byte of each wire operand's first block (the slice starts on a block)
    const uint8_t* ss[kMaxSrc];
    uint8_t* sd[kMaxDst];
#pragma unroll
    for (int k = 0; k < kMaxSrc; ++k) {
      const Loc l = o->src[k];
      ss[k] = (k < ns && ((sm >> k) & 1))
                  ? (const uint8_t*)c.peer_stg[l.rank] + par + c.mx_shadow + (l.off * c.stg_unit + lo) / kMxBlock
                  : nullptr;
    }
#pragma unroll
    for (int k = 0; k < kMaxDst; ++k) {
      const Loc l = o->dst[k];
      sd[k] = (k < nd && ((dm >> k) & 1))
                  ? (uint8_t*)c.peer_stg[l.rank] + par + c.mx_shadow + (l.off * c.stg_unit + lo) / kMxBlock
                  : nullptr;
    }
    switch (ns) {
      case 1: ok = xfer_mxb_k<T, W, 1, PM>(sp, s, ss, d, sd, nd, dm, n, o->scale, vec); break;
      case 2: ok = xfer_mxb_k<T, W, 2, PM>(sp, s, ss, d, sd, nd, dm, n, o->scale, vec); break;
      case 3: ok = xfer_mxb_k<T, W, 3, PM>(sp, s, ss, d, sd, nd, dm, n, o->scale, vec); break;
      case 4: ok = xfer_mxb_k<T, W, 4, PM>(sp, s, ss, d, sd, nd, dm, n, o->scale, vec); break;
      case 5: if constexpr (KMAX >= 5) ok = xfer_mxb_k<T, W, 5, PM>(sp, s, ss, d, sd, nd, dm, n, o->scale, vec); break;
      case 6: if constexpr (KMAX >= 6) ok = xfer_mxb_k<T, W, 6, PM>(sp, s, ss, d, sd, nd, dm, n, o->scale, vec); break;
      case 7: if constexpr (KMAX >= 7) ok = xfer_mxb_k<T, W, 7, PM>(sp, s, ss, d, sd, nd, dm, n, o->scale, vec); break;
      default: if constexpr (KMAX >= 8) ok = xfer_mxb_k<T, W, 8, PM>(sp, s, ss, d, sd, nd, dm, n, o->scale, vec); break;
    }
    (void)pre;
    (void)post_inv;
  } else {
    if (sm == all_s && dm == all_d) {  // wire type throughout (fp32 partial -> fp32 partial, fp8 copy)
      ok = xfer_dispatch<W, OpSum, PM, FP8 ? 1 : KMAX>(ns, s, d, nd, n, o->scale, vec);
    } else if (!FP8 && sm == 0 && dm == 0) {  // dtype throughout (raw inputs, all-gather copies)
      ok = xfer_dispatch<T, OpSum, PM, KMAX>(ns, s, d, nd, n, o->scale, vec);
    } else switch (ns) {
      case 1: ok = xfer_mx_k<T, W, 1, PM>(sp, s, d, nd, dm, n, o->scale, pre, post_inv, vec); break;
      case 2: ok = xfer_mx_k<T, W, 2, PM>(sp, s, d, nd, dm, n, o->scale, pre, post_inv, vec); break;
      case 3: ok = xfer_mx_k<T, W, 3, PM>(sp, s, d, nd, dm, n, o->scale, pre, post_inv, vec); break;
      case 4: ok = xfer_mx_k<T, W, 4, PM>(sp, s, d, nd, dm, n, o->scale, pre, post_inv, vec); break;
      case 5: if constexpr (KMAX >= 5) ok = xfer_mx_k<T, W, 5, PM>(sp, s, d, nd, dm, n, o->scale, pre, post_inv, vec); break;
      case 6: if constexpr (KMAX >= 6) ok = xfer_mx_k<T, W, 6, PM>(sp, s, d, nd, dm, n, o->scale, pre, post_inv, vec); break;
      case 7: if constexpr (KMAX >= 7) ok = xfer_mx_k<T, W, 7, PM>(sp, s, d, nd, dm, n, o->scale, pre, post_inv, vec); break;
      default: if constexpr (KMAX >= 8) ok = xfer_mx_k<T, W, 8, PM>(sp, s, d, nd, dm, n, o->scale, pre, post_inv, vec); break;
    }
  }
  if (!ok && threadIdx.x == 0)  // unreachable for validated programs: fail loudly, never compute wrongly
    __hip_atomic_store(c.err, (uint32_t)(0x40000000u | (0xfdu << 8)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// fp8 wire prologue: every workgroup derives the call's pre-scale s = fp8_max / (N * global amax).
// Workgroup 0 publishes this rank's amax (max over its partials) to every rank as an {epoch, value}
// granule (the LL protocol's data-tagged hand-off: no flag, no fence); every workgroup gathers all N
// granules and takes the max, so all ranks use the same s. Returns false on a watchdog timeout.
template <typename W>
__device__ FX_INLINE bool fp8_scale(const DevCtx& c, uint32_t b, uint64_t epoch, uint64_t par, float* s_out) {
  const uint32_t lane = threadIdx.x;
  float m = 0.0f;
  for (uint32_t i = lane; i < kAmaxParts; i += 64) m = __builtin_fmaxf(m, c.amax_parts[i]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = __builtin_fmaxf(m, __shfl_xor(m, off, 64));
  const uint64_t tag = epoch & 0xffffffffull;
  if (b == 0 && lane < c.nranks)
    st_flag(reinterpret_cast<uint64_t*>(c.peer_stg[lane] + par + c.amax_off) + c.rank, (tag << 32) | f2u(m));
  float g = 0.0f;
  bool ok = true;
  if (lane < c.nranks) {
    uint64_t* slot = reinterpret_cast<uint64_t*>(c.peer_stg[c.rank] + par + c.amax_off) + lane;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t v;
    while (((v = ld_flag(slot)) >> 32) != tag) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > c.timeout_ticks) {
        __hip_atomic_store(c.err, (uint32_t)(0x80000000u | (0xfeu << 8) | lane), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        ok = false;
        break;
      }
    }
    g = u2f((uint32_t)v);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) g = __builtin_fmaxf(g, __shfl_xor(g, off, 64));
  // s = fp8_max / (N * amax * (1 + h)), h = the fp8 type's largest relative rounding step (2^-4 e4m3,
  // 2^-3 e5m2): each quantised contribution is at most fp8_max / N * (1 + h) / (1 + h), so the N-term sum
  // (and every rounding of it) stays within fp8_max and the packed converters need no saturation
  const float wmax = (float)Elem<W>::load(Elem<W>::store(1e30f));  // saturating encode: the type's max
  const float head = IsFp8<W>::e4m3 ? 1.0625f : 1.125f;
  float sc = (g > 0.0f && g < 3.0e38f) ? wmax / ((float)c.nranks * g * head) : 1.0f;
  // a power of two (round down: the sum still cannot saturate): x * s and x / (1 / s) are then exact, which
  // is what lets the scaled converts (e8m0 semantics, sq_group / dq_group) replace decode -> scale -> encode
  // bit for bit; fp8 keeps its relative precision, at most one binade of range goes unused
  sc = fminf(fmaxf(sc, 0x1p-120f), 0x1p+120f);
  *s_out = __uint_as_float(__float_as_uint(sc) & 0x7f800000u);
  return __all(ok) != 0;
}

template <typename T, typename OP, int PM, typename W = void, int KMAX = kMaxSrc>
__device__ FX_INLINE void exec_body(const DevCtx& c, const uint32_t b, const uint32_t grid) {
  __shared__ int s_abort;
  __shared__ float s_pre;
  const uint32_t tid = threadIdx.x;
  const uint32_t nchan = c.nchan;
  // channel c = workgroups b == c (mod nchan); contiguous workgroups per channel measured the same bytes and
  // time (profiles/r6_channels/)
  const uint32_t ch = b % nchan, lb = b / nchan;
  const uint32_t nb = (grid - ch + nchan - 1) / nchan;
  constexpr bool TYPED = !std::is_void<W>::value;
  using WT_ = typename std::conditional<TYPED, W, T>::type;
  constexpr uint32_t U = sizeof(T) < sizeof(WT_) ? sizeof(T) : sizeof(WT_);
  const uint32_t quantum = IsMx<WT_>::value ? slice_quantum(1, kMxBlock)
                           : TYPED         ? slice_quantum(U, 16 / U)
                                           : slice_quantum(sizeof(T), sizeof(T) >= 16 ? 1u : (uint32_t)(16 / sizeof(T)));
  const uint64_t epoch = c.epochs[b] + 1;
  const uint64_t par = (epoch & 1) ? c.stg_half_bytes : 0;
  if (tid == 0) s_abort = 0;
  if (b == 0 && tid == 0 && c.progress) __hip_atomic_store(c.progress, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  float pre = 1.0f;
  if constexpr (TYPED && sizeof(WT_) == 1 && !IsMx<WT_>::value) {
    if (tid < 64) {
      float sc;
      const bool ok = fp8_scale<WT_>(c, b, epoch, par, &sc);
      if (tid == 0) {
        s_pre = sc;
        if (!ok) s_abort = 1;
      }
    }
    __syncthreads();
    pre = s_pre;
  } else {
    __syncthreads();
  }
  const float post_inv = 1.0f / pre;
  (void)post_inv;

  const uint32_t i0 = c.chan_start[ch], i1 = c.chan_start[ch + 1];
  for (uint32_t i = s_abort ? i1 : i0; i < i1;) {
    const Op* o = c.ops + i;
    const uint16_t kind = o->kind;
    if (kind == OP_XFER) {
      // a run of independent XFERs starts at a per-workgroup offset: the workgroups of one rank
      // spread over all peers (xGMI links) instead of marching through them in lockstep
      const uint32_t n = o->run > 1 ? o->run : 1;
      bool bar = false;
      for (uint32_t k = 0; k < n; ++k) {
        const Op* q = c.ops + i + (n > 1 ? (k + lb) % n : 0);
        // the work split is a function of (len, grid) only, so the workgroup b of every rank that hands a span
        // on and the one that takes it over cover the same elements
        // one call site for both splits (slices: one pass over [lo, end); chunks: every nb-th chunk): with two,
        // the compiler outlined the whole transfer into a called function (stack frame, captured state through
        // flat pointers) and the slices ran up to 5 % slower
        const uint64_t len = q->len;
        uint64_t lo, end, step, chunk;
        if (c.ichunk && len >= 4ull * nb * c.ichunk) {
          lo = (uint64_t)lb * c.ichunk;
          end = len;
          chunk = c.ichunk;
          step = (uint64_t)nb * c.ichunk;
        } else {
          slice_range(len, lb, nb, quantum, &lo, &end);
          chunk = step = end - lo;  // a single pass (also when empty)
        }
        do {
          const uint64_t hi = lo + chunk < end ? lo + chunk : end;
          if constexpr (TYPED) xfer_op_typed_range<T, WT_, PM, KMAX>(c, q, lo, hi, par, pre, post_inv);
          else xfer_op_range<T, OP, PM>(c, q, lo, hi, par);
          lo += step;
        } while (lo < end);
        bar |= (q->flags & kXferBarrierAfter) != 0;
      }
      if (bar) __syncthreads();
      i += n;
      continue;
    } else if (kind == OP_SIGNAL) {
      // every storing wave drains, the workgroup meets, one wave releases at system scope
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (c.fi_kind && o->slot == c.fi_slot) {
        if (c.fi_kind == 2) { ++i; continue; }  // dropped signal: peers must time out, not hang
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < c.fi_ticks) __builtin_amdgcn_s_sleep(8);
      }
      if (tid < 64) {
        if constexpr (PM != PM_WT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // WT: stores already drained
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the flag must not overtake the write-back
        if (tid < o->npeers) st_flag(c.peer_flags[o->peers[tid]] + flag_index(o->slot, c.rank, b), epoch);
      }
    } else if (kind == OP_WAIT) {
      if (tid < 64) {
        if (tid < o->npeers) {
          uint64_t* f = c.peer_flags[c.rank] + flag_index(o->slot, o->peers[tid], b);
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          uint64_t v;
          while ((v = ld_flag(f)) < epoch) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > c.timeout_ticks) {
              __hip_atomic_store(c.err, (uint32_t)(0x80000000u | (o->slot << 8) | o->peers[tid]), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
              s_abort = 1;
              break;
            }
          }
          // Protocol invariant (docs/DESIGN.md §2): a peer can be at most one call ahead, because its
          // call e+2 needs this rank's contribution to e+1. A flag beyond epoch+1 means two calls of one
          // communicator overlapped (broken stream ordering) and staging may have been overwritten:
          // report it instead of returning a silently wrong sum.
          if (v > epoch + 1)
            __hip_atomic_store(c.err, (uint32_t)(0x40000000u | (o->slot << 8) | o->peers[tid]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if constexpr (PM != PM_WT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // WT: loads are sc0 sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if (s_abort) break;
    }
    ++i;
  }
  __syncthreads();
  // Advance the epoch of EVERY epoch slot congruent to b (mod grid): after the call all
  // kMaxGridBlocks slots hold the same value, so the next call — whatever its grid size — sees one
  // uniform epoch and therefore one staging parity across all its workgroups (a lagging peer still in
  // call k reads parity(k) while an eager rank in call k+1 writes parity(k+1)). No slot is read in
  // this call by another workgroup: workgroup b2 reads only slot b2 < grid, and b2 == b (mod grid)
  // implies b2 == b.
  // All lanes share the stores: one lane alone serialises up to 1024 stores at small grids.
  for (uint32_t j = b + tid * grid; j < kMaxGridBlocks; j += blockDim.x * grid) c.epochs[j] = epoch;
  if (b == 0 && tid == 0 && c.progress) __hip_atomic_store(c.progress + 1, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------------------------
// LL ("low latency") one-shot for latency-bound sizes: every 4-byte payload word travels as an
// 8-byte {word, epoch} granule written with ONE system-scope store into every peer's staging and
// read back with system-scope (cache-bypassing) loads. The data carries its own readiness, so there
// is no SIGNAL/WAIT, no L2 write-back (release) and no L2 invalidate (acquire) on the critical path
// (MI355X_MICROARCH.md "handoff-1to1": data-tagged granules are the cheapest hand-off). Every rank
// reduces the words of all ranks in rank order, so all ranks get bit-identical results.
// Element types of 1, 2 or 4 bytes (a word holds 4 / sizeof(T) elements).
__device__ FX_INLINE uint32_t ld_word(const char* base, uint64_t w, uint64_t nbytes) {
  const uint64_t o = w * 4;
  if (o + 4 <= nbytes) return *reinterpret_cast<const uint32_t*>(base + o);
  uint32_t v = 0;
  for (uint64_t k = o; k < nbytes; ++k) v |= (uint32_t)(uint8_t)base[k] << (8 * (k - o));
  return v;
}
__device__ FX_INLINE void st_word(char* base, uint64_t w, uint64_t nbytes, uint32_t v) {
  const uint64_t o = w * 4;
  if (o + 4 <= nbytes) {
    *reinterpret_cast<uint32_t*>(base + o) = v;
    return;
  }
  for (uint64_t k = o; k < nbytes; ++k) base[k] = (char)((v >> (8 * (k - o))) & 0xff);
}

template <typename T, typename OP>
__device__ FX_INLINE void ll_body(const DevCtx& c, const uint32_t b, const uint32_t grid) {
  using A = typename Elem<T>::acc;
  constexpr int E = 4 / sizeof(T);
  __shared__ int s_abort;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) s_abort = 0;
  __syncthreads();
  const uint64_t epoch = c.epochs[b] + 1;
  if (b == 0 && tid == 0 && c.progress) __hip_atomic_store(c.progress, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t par = ((epoch & 1) ? c.stg_half_bytes : 0) + c.ll_off;  // LL-only region: stale bytes
  const uint64_t nbytes = c.count * sizeof(T), W = (nbytes + 3) / 4;        // there are older granules
  const uint32_t N = c.nranks, r = c.rank;
  uint64_t lo, hi;
  slice_range(W, b, grid, 1, &lo, &hi);
  const char* in = c.local[BUF_IN];
  char* out = c.local[BUF_OUT];
  // phase 1: publish my words to every peer
  for (uint64_t w = lo + tid; w < hi; w += blockDim.x) {
    const uint64_t g = (epoch << 32) | ld_word(in, w, nbytes);
    for (uint32_t p = 0; p < N; ++p)
      if (p != r) st_flag(reinterpret_cast<uint64_t*>(c.peer_stg[p] + par) + (uint64_t)r * W + w, g);
  }
  // phase 2: gather every rank's word (own from registers' source), reduce in rank order
  const uint64_t* mine = reinterpret_cast<const uint64_t*>(c.peer_stg[r] + par);
  const bool sc = Elem<T>::is_float && c.scale != 1.0f;
  for (uint64_t w = lo + tid; w < hi; w += blockDim.x) {
    A acc[E];
    for (uint32_t p = 0; p < N; ++p) {
      uint32_t v;
      if (p == r) {
        v = ld_word(in, w, nbytes);
      } else {
        uint64_t g = ld_flag(const_cast<uint64_t*>(mine + (uint64_t)p * W + w));
        if ((g >> 32) != (epoch & 0xffffffffu)) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          do {
            __builtin_amdgcn_s_sleep(1);
            g = ld_flag(const_cast<uint64_t*>(mine + (uint64_t)p * W + w));
            if (__builtin_amdgcn_s_memrealtime() - t0 > c.timeout_ticks) {
              __hip_atomic_store(c.err, (uint32_t)(0x80000000u | (0xffu << 8) | p), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
              s_abort = 1;
              break;
            }
          } while ((g >> 32) != (epoch & 0xffffffffu));
        }
        v = (uint32_t)g;
      }
      T e[E];
      __builtin_memcpy(e, &v, 4);
#pragma unroll
      for (int k = 0; k < E; ++k) acc[k] = p == 0 ? Elem<T>::load(e[k]) : OP::apply(acc[k], Elem<T>::load(e[k]));
    }
    T e[E];
#pragma unroll
    for (int k = 0; k < E; ++k) e[k] = Elem<T>::store(sc ? (A)(acc[k] * (A)c.scale) : acc[k]);
    uint32_t v;
    __builtin_memcpy(&v, e, 4);
    st_word(out, w, nbytes, v);
    if (s_abort) break;
  }
  __syncthreads();
  // All lanes share the stores: one lane alone serialises up to 1024 stores at small grids.
  for (uint32_t j = b + tid * grid; j < kMaxGridBlocks; j += blockDim.x * grid) c.epochs[j] = epoch;
  if (b == 0 && tid == 0 && c.progress) __hip_atomic_store(c.progress + 1, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Production launches take the context by value (no device copy per launch), but exec_body indexes it with
// run-time values (peer_stg[l.rank], local[l.buf], chan_start[ch]): on a by-value parameter the compiler then
// copies the whole DevCtx to scratch (36 B / lane of private memory in the untyped executor). Read it in
// place through the kernarg segment instead (the only explicit argument, at offset 0): scratch 0.
__device__ FX_INLINE const DevCtx& kernarg_ctx() {
  return *(const DevCtx*)__builtin_amdgcn_kernarg_segment_ptr();  // C cast: constant -> generic address space
}

template <typename T, typename OP>
__global__ void __launch_bounds__(kExecThreads) ll_kernel(DevCtx c) {
  (void)c;
  if constexpr (sizeof(T) <= 4) ll_body<T, OP>(kernarg_ctx(), blockIdx.x, gridDim.x);
}
template <typename T, typename OP>
__global__ void __launch_bounds__(kExecThreads) ll_group_kernel(const DevCtx* ctxs, uint32_t grid_per_rank) {
  if constexpr (sizeof(T) <= 4) ll_body<T, OP>(ctxs[blockIdx.x / grid_per_rank], blockIdx.x % grid_per_rank, grid_per_rank);
}

// Production launch: one rank per process, context by value.
template <typename T, typename OP, int PM>
__global__ void __launch_bounds__(kExecThreads) exec_kernel(DevCtx c) {
  (void)c;
  exec_body<T, OP, PM>(kernarg_ctx(), blockIdx.x, gridDim.x);
}

// Typed programs (Program::wire: fp32 partials or an fp8 wire), SUM/AVG only.
// FLEXAR_TYPED_OCC3: the global-scale fp8 kernels of the narrow class (KMAX 4) ask the register allocator for 3
// waves per SIMD (at most 168 VGPRs). The single-rank kernel fits without it (bf16 167, fp32 155); the in-process
// group kernel needs 179 / 172 otherwise, and with it keeps a few prologue values in scratch.
#ifndef FLEXAR_TYPED_OCC3
#define FLEXAR_TYPED_OCC3 0
#endif
// FLEXAR_TYPED_THREADS (build knob): workgroup size of the typed kernels. At 512 threads (8 waves,
// 2 per SIMD) a second workgroup shares a CU only at <= 128 VGPRs, and the typed kernels use 155-230; at 256 (4 waves,
// 1 per SIMD) two fit at <= 256 VGPRs and three at <= 168. The launch multiplies the grid by the workgroups per CU
// it targets (typed_grid_mul: 3 for the narrow fan-in class, 2 otherwise; flags and epochs are per workgroup,
// kMaxGridBlocks caps it, co-residency holds by the same factor); every rank runs the same build.
#ifndef FLEXAR_TYPED_THREADS
#define FLEXAR_TYPED_THREADS 512
#endif
constexpr int kTypedThreads = FLEXAR_TYPED_THREADS;
static_assert(kTypedThreads == 256 || kTypedThreads == 512, "FLEXAR_TYPED_THREADS: 256 or 512");
template <int KMAX>
constexpr int typed_grid_mul() {
  return kTypedThreads == 256 ? (KMAX <= 4 ? 3 : 2) : 1;
}
template <typename W, int KMAX>
constexpr int typed_min_waves() {
  // 256-thread workgroups: three per CU for the narrow fan-in class (<= 168 VGPRs), two otherwise (<= 256)
  if (kTypedThreads == 256) return KMAX <= 4 ? 3 : 2;
  return FLEXAR_TYPED_OCC3 && KMAX <= 4 && sizeof(W) == 1 && !IsMx<W>::value ? 3 : 1;
}
// 512-thread typed executors stay one workgroup per CU, as every executor was sized and measured: a kernel that
// comes in at <= 128 VGPRs (bf16 over the MX wire, fan-in <= 4, after the 2-destination change) would otherwise
// fit two per CU, and the grid then packs onto half the CUs - measured 33 % slower with 4 processes sharing the
// GPU (profiles/r6_mx_nd/). Claiming v128 keeps the allocation above 128.
__device__ FX_INLINE void one_workgroup_per_cu() {
  if constexpr (kTypedThreads == 512) asm volatile("" ::: "v128");
}
template <typename T, typename W, int PM, int KMAX = kMaxSrc>
__global__ void __launch_bounds__(kTypedThreads) __attribute__((amdgpu_waves_per_eu(typed_min_waves<W, KMAX>())))
exec_mx_kernel(DevCtx c) {
  (void)c;
  one_workgroup_per_cu();
  exec_body<T, OpSum, PM, W, KMAX>(kernarg_ctx(), blockIdx.x, gridDim.x);
}
template <typename T, typename W, int PM, int KMAX = kMaxSrc>
__global__ void __launch_bounds__(kTypedThreads) __attribute__((amdgpu_waves_per_eu(typed_min_waves<W, KMAX>())))
exec_mx_group_kernel(const DevCtx* ctxs, uint32_t grid_per_rank) {
  one_workgroup_per_cu();
  const uint32_t r = blockIdx.x / grid_per_rank;
  exec_body<T, OpSum, PM, W, KMAX>(ctxs[r], blockIdx.x % grid_per_rank, grid_per_rank);
}

// In-process group launch: nranks ranks share one grid (rank = blockIdx / grid_per_rank) —
// every rank's workgroups are co-resident by construction, so the full multi-rank protocol
// runs on a single GPU in a single process (tests, calibration).
template <typename T, typename OP, int PM>
__global__ void __launch_bounds__(kExecThreads) exec_group_kernel(const DevCtx* ctxs, uint32_t grid_per_rank) {
  const uint32_t r = blockIdx.x / grid_per_rank;
  exec_body<T, OP, PM>(ctxs[r], blockIdx.x % grid_per_rank, grid_per_rank);
}

// Standalone reduction: dst[0] = scale * OP(src[0..K)), grid-sliced.
struct SrcTable {
  const char* p[kMaxSrc];
};

// Grid-interleaved form of the standalone reduction (reduce_kernel, vec bit 1): step i of workgroup b covers the
// U x nt 16-B vectors at (i * grid + b) * U * nt of EVERY source, so at any moment the whole grid reads one
// narrow window of each of the K sources (DRAM pages stay open for every workgroup) instead of K x grid
// far-apart streams - the slice form's per-workgroup contiguous spans. Results are identical (the same
// combine16 per element; only which workgroup computes an element changes).
template <typename T, typename OP, int K>
__device__ FX_INLINE void reduce_interleaved(const char* const (&s)[kMaxSrc], char* d0, char* d1, uint64_t n,
                                             float scale) {
  constexpr int E = 16 / sizeof(T);
  constexpr int U = (K <= 2) ? 4 : ((K <= 4) ? 2 : FLEXAR_UNROLL_WIDE);
  const bool sc = Elem<T>::is_float && scale != 1.0f;
  const uint64_t nt = blockDim.x, nv = n / E, step = (uint64_t)U * nt;
  for (uint64_t base = (uint64_t)blockIdx.x * step; base < nv; base += (uint64_t)gridDim.x * step) {
    uint4 x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t v = base + u * nt + threadIdx.x;
#pragma unroll
      for (int k = 0; k < K; ++k) x[u][k] = v < nv ? ld16(s[k] + v * 16) : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t v = base + u * nt + threadIdx.x;
      if (v >= nv) continue;
      const uint4 y = combine16<T, OP, K>(x[u], scale, sc);
      st16(d0 + v * 16, y);
      if (d1) st16(d1 + v * 16, y);
    }
  }
  // the last < E elements, by workgroup 0
  if (blockIdx.x == 0)
    for (uint64_t i = nv * E + threadIdx.x; i < n; i += nt) {
      typename Elem<T>::acc acc = Elem<T>::load(ld_elem<PM_FENCE, T>(s[0], i));
#pragma unroll
      for (int k = 1; k < K; ++k) acc = OP::apply(acc, Elem<T>::load(ld_elem<PM_FENCE, T>(s[k], i)));
      if (sc) acc = (typename Elem<T>::acc)(acc * (typename Elem<T>::acc)scale);
      const T y = Elem<T>::store(acc);
      st_elem<PM_FENCE, T>(d0, i, y);
      if (d1) st_elem<PM_FENCE, T>(d1, i, y);
    }
}

// PM_WT (copy-engine allreduce): sources written by peers' DMA are read system-coherently and the
// result is written through, so a stream-ordered flag write after this kernel publishes it.
// vec bit 0: 16-B vector accesses allowed; bit 1 (fence protocol only): the grid-interleaved form.
// The fp8 fence-protocol reduction asks for 4 waves per SIMD: two 512-thread workgroups per CU, at most 128
// VGPRs (fp32 / bf16 fit that by themselves). The packed fp8 arithmetic would take 131 and keeps 20 B in
// scratch with it. Measured (profiles/r5_fp8_packed): fp8 at fan-in 2 / 4 / 8 runs at 5.98 / 6.06 / 5.71 TB/s,
// against 5.30 / 5.78 / 5.69 with per-element converts and 5.26 / 5.50 / 5.63 packed without it.
// FLEXAR_REDUCE_OCC4=0 is the A/B build without it. Integer types and the write-through form (copy-engine path)
// keep the default: held to 128 VGPRs they spill.
#ifndef FLEXAR_REDUCE_OCC4
#define FLEXAR_REDUCE_OCC4 1
#endif
template <typename T, typename OP, int PM>
__global__ void __launch_bounds__(kExecThreads)
__attribute__((amdgpu_waves_per_eu(FLEXAR_REDUCE_OCC4 && PM != PM_WT && IsFp8<T>::value ? 4 : 1))) reduce_kernel(SrcTable srcs, int nsrc, char* dst, char* dst2,
                                                              uint64_t n, float scale, int vec) {
  if constexpr (PM != PM_WT && sizeof(T) < 16) {
    if ((vec & 3) == 3) {
      const char* s[kMaxSrc];
#pragma unroll
      for (int k = 0; k < kMaxSrc; ++k) s[k] = k < nsrc ? srcs.p[k] : nullptr;
      switch (nsrc) {
        case 1: reduce_interleaved<T, OP, 1>(s, dst, dst2, n, scale); break;
        case 2: reduce_interleaved<T, OP, 2>(s, dst, dst2, n, scale); break;
        case 3: reduce_interleaved<T, OP, 3>(s, dst, dst2, n, scale); break;
        case 4: reduce_interleaved<T, OP, 4>(s, dst, dst2, n, scale); break;
        case 5: reduce_interleaved<T, OP, 5>(s, dst, dst2, n, scale); break;
        case 6: reduce_interleaved<T, OP, 6>(s, dst, dst2, n, scale); break;
        case 7: reduce_interleaved<T, OP, 7>(s, dst, dst2, n, scale); break;
        default: reduce_interleaved<T, OP, 8>(s, dst, dst2, n, scale); break;
      }
      return;
    }
  }
  vec &= 1;
  const uint32_t quantum = slice_quantum(sizeof(T), sizeof(T) >= 16 ? 1u : (uint32_t)(16 / sizeof(T)));
  uint64_t lo, hi;
  slice_range(n, blockIdx.x, gridDim.x, quantum, &lo, &hi);
  const uint64_t step = PM == PM_WT ? kWtChunkBytes / sizeof(T) : ~0ull;  // 32-bit buffer offsets
  for (uint64_t m; lo < hi; lo += m) {
    m = (hi - lo) < step ? (hi - lo) : step;
    const char* s[kMaxSrc];
    char* d[kMaxDst];
#pragma unroll
    for (int k = 0; k < kMaxSrc; ++k) s[k] = k < nsrc ? srcs.p[k] + lo * sizeof(T) : nullptr;
#pragma unroll
    for (int k = 0; k < kMaxDst; ++k) d[k] = nullptr;
    d[0] = dst + lo * sizeof(T);
    if (dst2) d[1] = dst2 + lo * sizeof(T);
    xfer_dispatch<T, OP, PM>(nsrc, s, d, dst2 ? 2 : 1, m, scale, vec != 0);
  }
}

// Copy-engine allreduce: one wave polls up to kMaxRanks flags (system scope) until they reach `value`
// and then lets the stream proceed (the next copy / reduce is stream-ordered behind this kernel).
// Same watchdog as the executor's WAIT.
struct DmaWait {
  const uint64_t* flags;
  uint32_t idx[kMaxRanks];
  uint32_t src[kMaxRanks];
  uint32_t n;
  uint32_t slot;
  uint64_t value;
  uint64_t timeout_ticks;
  uint32_t* err;
};
static __global__ void dma_wait_kernel(DmaWait w) {
  const uint32_t t = threadIdx.x;
  if (t >= w.n) return;
  uint64_t* f = const_cast<uint64_t*>(w.flags) + w.idx[t];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_flag(f) < w.value) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > w.timeout_ticks) {
      __hip_atomic_store(w.err, (uint32_t)(0x80000000u | (w.slot << 8) | w.src[t]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

// Copy-engine allreduce bookkeeping: the call consumed one epoch of the staging protocol.
static __global__ void epoch_set_kernel(uint64_t* epochs, uint64_t e) {
  for (uint32_t j = threadIdx.x; j < kMaxGridBlocks; j += blockDim.x) epochs[j] = e;
}

}  // namespace flexar
