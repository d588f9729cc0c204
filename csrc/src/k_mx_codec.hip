// OCP MX fp8 message codec for the hierarchical communicator's cross-node step
// (allreduce_over_mpi_amd/parallel/hierarchical.py _cross_all_reduce_mx):
//   pack         msg = [q_0 .. q_{n-1} | X_0 .. X_{ceil(n/32)-1}]: one e8m0 byte X per 32-element block
//                (the smallest exponent with amax <= fp8_max * 2^X, types.hpp mx_scale_byte) and the fp8 values
//                q = rne(x / 2^X) - the layout the cross-node all-gather carries, in one HBM pass;
//   unpack_sum   out[i] = post * sum over messages k, in order, of q_k[i] * 2^X_k - the dequantise-and-sum of
//                every node's message in one pass, fp32 accumulation, AVG's 1 / world fused (post).
// Both are bit-identical to ops.quant.mx_quantize / mx_dequantize + the node-order sum (the torch reference
// and CPU fallback). Round 5: 16 elements per lane - a block is a lane pair, one 16-B
// fp8 store per lane, 16-B loads per message - instead of one byte per lane (3.1 / 2.0 TB/s before).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "flexar/flexar.h"
#include "flexar/types.hpp"
#include "crumbs.hpp"
#include "internal.hpp"

namespace flexar {

constexpr int kMxcThreads = 256;

static int mxc_grid(uint64_t items) {
  const uint64_t g = (items + kMxcThreads - 1) / kMxcThreads;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));  // >= 64 workgroups per XCD for large n
}

// 16-B accesses at any byte offset (the all-gathered message rows are mx_message_bytes(n) apart, not a
// multiple of 16): amdhsa code objects run in unaligned mode, one global_load/store_dwordx4 each
typedef unsigned int mxc_u4 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) mxc_u4 mxc_g4;
__device__ __forceinline__ uint4 mxc_ld16(const void* p) {
  const mxc_u4 v = __builtin_nontemporal_load((const mxc_g4*)p);
  return uint4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void mxc_st16(void* p, uint4 x) {
  const mxc_u4 v = {x.x, x.y, x.z, x.w};
  *(mxc_g4*)p = v;
}
typedef short mxc_s2 __attribute__((ext_vector_type(2)));
typedef __bf16 mxc_bf2 __attribute__((ext_vector_type(2)));
typedef _Float16 mxc_h2 __attribute__((ext_vector_type(2)));
typedef float mxc_f2 __attribute__((ext_vector_type(2)));

// f32 bits of element e of a lane's 16 packed T values (the amax runs on sign-cleared f32 bits)
template <typename T>
__device__ __forceinline__ uint32_t mxc_f32_bits(const uint32_t* w, int e) {
  if constexpr (sizeof(T) == 4) return w[e];
  else if constexpr (__is_same(T, bf16_t)) return ((w[e / 2] >> (16 * (e & 1))) & 0xffffu) << 16;
  else return __float_as_uint(f16_to_f32((uint16_t)((w[e / 2] >> (16 * (e & 1))) & 0xffffu)));
}

// Pack. A wave takes chunks of 64 x 16 elements (32 blocks); 16-B sub-chunk j of lane l holds elements
// 64 E j + E l .. + E (E = 16 / sizeof(T): 4 fp32, 8 bf16 / fp16), so every load instruction covers 1 KiB
// contiguous across the wave, and so does every fp8 store (E bytes per lane). A 32-element block is
// 32 / E consecutive lanes of one sub-chunk: its amax takes log2(32 / E) xor-shuffles. q = rne(x / 2^X)
// through gfx950's scaled converts (v_cvt_scalef32_pk_fp8_*: only the scale's exponent counts, as in the MX
// executor), the values mx_quantize gives. Whole blocks only (`nwhole` elements, a multiple of 32: a block is
// wholly inside or outside); the last partial block is mx_pack_tail's.
template <typename T, typename W>
__global__ void __launch_bounds__(kMxcThreads) mx_pack16_kernel(const T* __restrict__ x, uint8_t* __restrict__ msg,
                                                                uint64_t n, uint64_t nwhole) {
  constexpr bool E4 = __is_same(W, mxe4m3_t);
  constexpr int E = 16 / (int)sizeof(T);  // elements per 16-B sub-chunk
  constexpr int J = (int)sizeof(T);       // sub-chunks per lane per chunk (64 x 16 elements)
  constexpr int LPB = kMxBlock / E;       // lanes per block
  constexpr uint64_t kChunk = 64 * 16;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (kMxcThreads / 64) + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * (kMxcThreads / 64);
  for (uint64_t base = wave * kChunk; base < nwhole; base += nwaves * kChunk) {
    uint4 raw[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t e0 = base + (uint64_t)(64 * j + lane) * E;
      raw[j] = e0 < nwhole ? mxc_ld16((const char*)x + e0 * sizeof(T)) : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t e0 = base + (uint64_t)(64 * j + lane) * E;
      const uint32_t w[4] = {raw[j].x, raw[j].y, raw[j].z, raw[j].w};
      uint32_t am = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) am = max(am, mxc_f32_bits<T>(w, e) & 0x7fffffffu);
#pragma unroll
      for (int o = LPB / 2; o > 0; o >>= 1) am = max(am, (uint32_t)__shfl_xor((int)am, o));
      const uint32_t xr = mx_scale_byte(am, E4);
      const float sc = mx_scale_value(xr);
      uint32_t q[E / 4];
#pragma unroll
      for (int i = 0; i < E / 4; ++i) {
        mxc_s2 r = {0, 0};
        if constexpr (sizeof(T) == 4) {
          const float* f = reinterpret_cast<const float*>(w);
          if constexpr (E4) {
            r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, f[4 * i], f[4 * i + 1], sc, false);
            r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, f[4 * i + 2], f[4 * i + 3], sc, true);
          } else {
            r = __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(r, f[4 * i], f[4 * i + 1], sc, false);
            r = __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(r, f[4 * i + 2], f[4 * i + 3], sc, true);
          }
        } else if constexpr (__is_same(T, bf16_t)) {
          mxc_bf2 a, b;
          __builtin_memcpy(&a, &w[2 * i], 4);
          __builtin_memcpy(&b, &w[2 * i + 1], 4);
          if constexpr (E4) {
            r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, a, sc, false);
            r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, b, sc, true);
          } else {
            r = __builtin_amdgcn_cvt_scalef32_pk_bf8_bf16(r, a, sc, false);
            r = __builtin_amdgcn_cvt_scalef32_pk_bf8_bf16(r, b, sc, true);
          }
        } else {
          mxc_h2 a, b;
          __builtin_memcpy(&a, &w[2 * i], 4);
          __builtin_memcpy(&b, &w[2 * i + 1], 4);
          if constexpr (E4) {
            r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(r, a, sc, false);
            r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(r, b, sc, true);
          } else {
            r = __builtin_amdgcn_cvt_scalef32_pk_bf8_f16(r, a, sc, false);
            r = __builtin_amdgcn_cvt_scalef32_pk_bf8_f16(r, b, sc, true);
          }
        }
        __builtin_memcpy(&q[i], &r, 4);
      }
      // NaN inputs: the scaled converts write the NaN byte with the sign set whatever the input's sign; the element
      // store (and ops.quant.mx_quantize) keep the sign: 0x7f | sign. Only blocks holding a NaN take this branch.
      if (am > 0x7f800000u) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const uint32_t b = mxc_f32_bits<T>(w, e);
          if ((b & 0x7fffffffu) > 0x7f800000u) {
            const uint32_t sh = 8 * (e & 3);
            q[e / 4] = (q[e / 4] & ~(0xffu << sh)) | ((0x7fu | ((b >> 24) & 0x80u)) << sh);
          }
        }
      }
      if (e0 < nwhole) {
        if constexpr (E == 4) {
          *(uint32_t*)(msg + e0) = q[0];  // 4 B per lane, 256 B contiguous across the wave
        } else {
          typedef unsigned int u2a1 __attribute__((ext_vector_type(2), aligned(1)));
          *(u2a1*)(msg + e0) = u2a1{q[0], q[1]};  // 8 B per lane, 512 B contiguous across the wave
        }
        if (lane % LPB == 0) msg[n + e0 / kMxBlock] = (uint8_t)xr;
      }
    }
  }
}

// The last partial block (n % 32 elements): lanes 0..31 of one wave, one element each.
template <typename T, typename W>
__global__ void __launch_bounds__(64) mx_pack_tail_kernel(const T* __restrict__ x, uint8_t* __restrict__ msg,
                                                          uint64_t n, uint64_t i0) {
  constexpr bool E4 = __is_same(W, mxe4m3_t);
  if (threadIdx.x >= kMxBlock) return;
  const uint64_t i = i0 + threadIdx.x;
  const float v = i < n ? (float)Elem<T>::load(x[i]) : 0.0f;
  uint32_t am = __float_as_uint(v) & 0x7fffffffu;
#pragma unroll
  for (int o = kMxBlock / 2; o > 0; o >>= 1) am = max(am, (uint32_t)__shfl_xor((int)am, o));
  const uint32_t xr = mx_scale_byte(am, E4);
  if (i < n) {
    // non-finite values as ops.quant.mx_quantize (torch's fp8 casts) and the whole-block converts give them:
    // NaN -> 0x7f | sign, Inf -> the type's Inf (e5m2 0x7c) or NaN (e4m3 has no Inf) | sign; the element store
    // would saturate Inf to the largest finite value
    const uint32_t b = __float_as_uint(v), sg = (b >> 24) & 0x80u;
    if ((b & 0x7fffffffu) > 0x7f800000u) msg[i] = (uint8_t)(0x7fu | sg);
    else if ((b & 0x7fffffffu) == 0x7f800000u) msg[i] = (uint8_t)((E4 ? 0x7fu : 0x7cu) | sg);
    else msg[i] = Elem<W>::store(v / mx_scale_value(xr)).bits;
  }
  if (threadIdx.x == 0) msg[n + i0 / kMxBlock] = (uint8_t)xr;
}

// Unpack-sum, 16 elements per lane: per message one 16-B load of fp8 values and the block's scale byte,
// loads of up to 4 messages in flight before the sums; x = q * 2^X by the scaled converts (exact), summed
// in message order in fp32; `post` (AVG's 1 / world, fused) multiplies the sum; four 16-B stores.
template <typename W>
__global__ void __launch_bounds__(kMxcThreads) mx_unpack_sum16_kernel(const uint8_t* __restrict__ msgs,
                                                                      uint64_t msg_stride, int nmsg, uint64_t n,
                                                                      uint64_t ngrp, float post,
                                                                      float* __restrict__ out) {
  constexpr bool E4 = __is_same(W, mxe4m3_t);
  const uint64_t stride = (uint64_t)gridDim.x * kMxcThreads;
  for (uint64_t g = (uint64_t)blockIdx.x * kMxcThreads + threadIdx.x; g < ngrp; g += stride) {
    float acc[16];
    for (int k0 = 0; k0 < nmsg; k0 += 4) {
      uint4 q[4];
      uint32_t xr[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u < nmsg) {
          const uint8_t* m = msgs + (uint64_t)(k0 + u) * msg_stride;
          q[u] = mxc_ld16(m + g * 16);
          xr[u] = m[n + g / 2];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u >= nmsg) break;
        const float sc = mx_scale_value(xr[u]);
        const uint32_t wq[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          mxc_f2 lo, hi;
          if constexpr (E4) {
            lo = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(wq[i], sc, false);
            hi = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(wq[i], sc, true);
          } else {
            lo = __builtin_amdgcn_cvt_scalef32_pk_f32_bf8(wq[i], sc, false);
            hi = __builtin_amdgcn_cvt_scalef32_pk_f32_bf8(wq[i], sc, true);
          }
          const float v[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[4 * i + e] = (k0 + u) ? acc[4 * i + e] + v[e] : v[e];
        }
      }
    }
    float* o = out + g * 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = acc[4 * j] * post, b = acc[4 * j + 1] * post, c = acc[4 * j + 2] * post, d = acc[4 * j + 3] * post;
      mxc_st16(o + 4 * j, uint4{__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d)});
    }
  }
}

// The last n % 16 elements, one per lane.
template <typename W>
__global__ void __launch_bounds__(64) mx_unpack_tail_kernel(const uint8_t* __restrict__ msgs, uint64_t msg_stride,
                                                            int nmsg, uint64_t n, uint64_t i0, float post,
                                                            float* __restrict__ out) {
  const uint64_t i = i0 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* m = msgs;
  float acc = (float)Elem<W>::load(W{m[i]}) * mx_scale_value(m[n + i / kMxBlock]);
  for (int k = 1; k < nmsg; ++k) {
    m += msg_stride;
    acc += (float)Elem<W>::load(W{m[i]}) * mx_scale_value(m[n + i / kMxBlock]);
  }
  out[i] = acc * post;
}

}  // namespace flexar

using namespace flexar;

#define FXM_CHECK_LAUNCH()                                                         \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess) {                                                        \
      set_error(std::string("mx codec launch: ") + hipGetErrorString(e_));         \
      return FLEXAR_ERR_HIP;                                                       \
    }                                                                              \
  } while (0)

template <typename T, typename W>
static void mx_pack_launch(const void* x, void* msg, uint64_t n, hipStream_t s) {
  const uint64_t nwhole = (n / kMxBlock) * kMxBlock;  // elements in whole blocks
  if (nwhole) {
    const int g = mxc_grid((nwhole + 15) / 16);  // one 16-element item per lane
    CrumbArgs ca;
    ca.type = CRUMB_LAUNCH;
    ca.what = "mx_pack16_kernel";
    ca.bytes = n * sizeof(T);
    ca.grid = (uint32_t)g;
    crumb(ca);
    hipLaunchKernelGGL((mx_pack16_kernel<T, W>), g, kMxcThreads, 0, s, (const T*)x, (uint8_t*)msg, n, nwhole);
  }
  if (n % kMxBlock)
    hipLaunchKernelGGL((mx_pack_tail_kernel<T, W>), 1, 64, 0, s, (const T*)x, (uint8_t*)msg, n,
                       (uint64_t)(n / kMxBlock) * kMxBlock);
}

template <typename W>
static int mx_pack_t(const void* x, int dtype, void* msg, uint64_t n, hipStream_t s) {
  switch (dtype) {
    case FLEXAR_FLOAT32: mx_pack_launch<float, W>(x, msg, n, s); break;
    case FLEXAR_BFLOAT16: mx_pack_launch<bf16_t, W>(x, msg, n, s); break;
    case FLEXAR_FLOAT16: mx_pack_launch<f16_t, W>(x, msg, n, s); break;
    default: set_error("mx pack: dtype must be float32, bfloat16 or float16"); return FLEXAR_ERR_UNSUPPORTED;
  }
  FXM_CHECK_LAUNCH();
  return 0;
}

template <typename W>
static void mx_unpack_launch(const void* msgs, size_t msg_stride, int nmsg, uint64_t n, float post, float* out,
                             hipStream_t s) {
  const uint64_t ngrp = n / 16;
  if (ngrp) {
    CrumbArgs ca;
    ca.type = CRUMB_LAUNCH;
    ca.what = "mx_unpack_sum16_kernel";
    ca.bytes = n * (uint64_t)nmsg;
    ca.grid = (uint32_t)mxc_grid(ngrp);
    crumb(ca);
    hipLaunchKernelGGL((mx_unpack_sum16_kernel<W>), mxc_grid(ngrp), kMxcThreads, 0, s, (const uint8_t*)msgs,
                       (uint64_t)msg_stride, nmsg, n, ngrp, post, out);
  }
  if (n % 16)
    hipLaunchKernelGGL((mx_unpack_tail_kernel<W>), 1, 64, 0, s, (const uint8_t*)msgs, (uint64_t)msg_stride, nmsg, n,
                       ngrp * 16, post, out);
}

extern "C" {

// msg: n + ceil(n/32) bytes (fp8 values, then the block scale bytes). wire: 4 = e4m3, 5 = e5m2.
int flexar_mx_pack(const void* x, int dtype, void* msg, size_t n, int wire, void* stream) {
  if (!x || !msg) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (wire != 4 && wire != 5) { set_error("mx pack: wire must be 4 (e4m3) or 5 (e5m2)"); return FLEXAR_ERR_INVALID; }
  if (n == 0) return 0;
  return wire == 4 ? mx_pack_t<mxe4m3_t>(x, dtype, msg, n, (hipStream_t)stream)
                   : mx_pack_t<mxe5m2_t>(x, dtype, msg, n, (hipStream_t)stream);
}

// out[i] = post * sum_k q_k[i] * 2^X_k over nmsg messages laid out msg_stride bytes apart (fp32 out, message
// order; post = 1 or AVG's fused 1 / world).
int flexar_mx_unpack_sum_scaled(const void* msgs, size_t msg_stride, int nmsg, size_t n, int wire, float post,
                                float* out, void* stream) {
  if (!msgs || !out || nmsg < 1) { set_error("mx unpack: null argument or no message"); return FLEXAR_ERR_INVALID; }
  if (wire != 4 && wire != 5) { set_error("mx unpack: wire must be 4 (e4m3) or 5 (e5m2)"); return FLEXAR_ERR_INVALID; }
  if (msg_stride < n + (n + kMxBlock - 1) / kMxBlock) { set_error("mx unpack: message stride too small"); return FLEXAR_ERR_INVALID; }
  if (n == 0) return 0;
  if (wire == 4) mx_unpack_launch<mxe4m3_t>(msgs, msg_stride, nmsg, n, post, out, (hipStream_t)stream);
  else mx_unpack_launch<mxe5m2_t>(msgs, msg_stride, nmsg, n, post, out, (hipStream_t)stream);
  FXM_CHECK_LAUNCH();
  return 0;
}

int flexar_mx_unpack_sum(const void* msgs, size_t msg_stride, int nmsg, size_t n, int wire, float* out,
                         void* stream) {
  return flexar_mx_unpack_sum_scaled(msgs, msg_stride, nmsg, n, wire, 1.0f, out, stream);
}

}  // extern "C"
