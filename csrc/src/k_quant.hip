// fp8 (OCP e4m3) gradient compression kernels for the compressed allreduce path (BASELINE config #5):
//   amax       |x|max of a fp32/bf16/fp16 buffer -> kAmaxParts per-workgroup partial maxima (no atomics:
//              one shared address taking an atomic from every workgroup serialises at the memory side,
//              measured 23 us for 26 MB on MI355X; the partials are reduced by their consumers instead)
//   quantize   q = e4m3(clamp(x * s, +-448)),   s = num / max(partials)   (read on device: no host sync)
//   dequantize x = q / s
// Each is ONE pass over HBM with one 16-byte vector of the wide type per lane and step (coalesced), gfx950
// packed conversions (v_cvt_pk_fp8_f32 / v_cvt_pk_f32_fp8) and no intermediate buffers — replacing the
// abs / max / mul / cast / cast / div / copy chain of separate elementwise kernels. The partials array is
// what the compressed allreduce exchanges with its MAX allreduce (1 KiB: the LL protocol).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "flexar/flexar.h"
#include "flexar/types.hpp"
#include "internal.hpp"

namespace flexar {

constexpr int kQThreads = 256;
constexpr int kAmaxThreads = 1024;  // 16 waves per CU: enough loads in flight with one workgroup per CU
constexpr int kAmaxParts = FLEXAR_AMAX_PARTIALS;
constexpr int kQUnroll = 4;         // independent 16-B vectors in flight per lane

// Coalescing: a lane owns ONE 16-byte vector of the wide type per step (PER = 16 / sizeof(T) elements),
// so every wave-instruction covers 1 KiB contiguous on the wide side and 64 x PER bytes on the fp8 side.
typedef unsigned int q_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int q_u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) q_u32x4 g_q_u32x4;

template <typename T>
struct QVec {
  static constexpr int PER = 16 / sizeof(T);  // elements per 16-B vector: 4 (fp32) or 8 (bf16 / fp16)
  __device__ static __forceinline__ void load(const char* x, uint64_t v, float (&f)[PER]) {
    q_u32x4 r = __builtin_nontemporal_load((const g_q_u32x4*)(x + v * 16));
    T e[PER];
    __builtin_memcpy(e, &r, 16);
#pragma unroll
    for (int k = 0; k < PER; ++k) f[k] = Elem<T>::load(e[k]);
  }
  __device__ static __forceinline__ void store(char* x, uint64_t v, const float (&f)[PER]) {
    T e[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) e[k] = Elem<T>::store(f[k]);
    q_u32x4 r;
    __builtin_memcpy(&r, e, 16);
    *(g_q_u32x4*)(x + v * 16) = r;
  }
};

__device__ __forceinline__ float sat448(float x) { return __builtin_fminf(__builtin_fmaxf(x, -448.0f), 448.0f); }
// 4 floats -> 4 e4m3 bytes (RNE, saturated first), gfx950 packed conversion
__device__ __forceinline__ unsigned int pack4(float a, float b, float c, float d) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(sat448(a), sat448(b), 0, false);
  return (unsigned int)__builtin_amdgcn_cvt_pk_fp8_f32(sat448(c), sat448(d), lo, true);
}
__device__ __forceinline__ void unpack4(unsigned int w, float inv, float* f) {
  auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false);
  auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
  f[0] = lo[0] * inv;
  f[1] = lo[1] * inv;
  f[2] = hi[0] * inv;
  f[3] = hi[1] * inv;
}

// s = num / max(partials): every workgroup reduces the kAmaxParts partials itself (1 KiB, L2-served)
__device__ __forceinline__ float block_scale(const float* parts, float num) {
  __shared__ float red[kQThreads / 64];
  __shared__ float s_out;
  float m = 0.0f;
  for (int i = threadIdx.x; i < kAmaxParts; i += blockDim.x) m = fmaxf(m, parts[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = red[0];
    for (int w = 1; w < (int)(blockDim.x / 64); ++w) b = fmaxf(b, red[w]);
    s_out = b > 0.0f ? num / b : 1.0f;
  }
  __syncthreads();
  return s_out;
}

template <typename T>
__global__ void __launch_bounds__(kAmaxThreads) amax_kernel(const char* x, uint64_t n, float* parts) {
  using V = QVec<T>;
  float m = 0.0f;
  const uint64_t nv = n / V::PER;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; v + (kQUnroll - 1) * stride < nv; v += kQUnroll * stride) {
    float f[kQUnroll][V::PER];
#pragma unroll
    for (int u = 0; u < kQUnroll; ++u) V::load(x, v + u * stride, f[u]);
#pragma unroll
    for (int u = 0; u < kQUnroll; ++u)
#pragma unroll
      for (int k = 0; k < V::PER; ++k) m = fmaxf(m, fabsf(f[u][k]));
  }
  for (; v < nv; v += stride) {
    float f[V::PER];
    V::load(x, v, f);
#pragma unroll
    for (int k = 0; k < V::PER; ++k) m = fmaxf(m, fabsf(f[k]));
  }
  for (uint64_t i = nv * V::PER + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    m = fmaxf(m, fabsf(Elem<T>::load(reinterpret_cast<const T*>(x)[i])));
  // wave (64 lanes) then workgroup; one plain store per workgroup
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wmax[kAmaxThreads / 64];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = wmax[0];
    for (int w = 1; w < kAmaxThreads / 64; ++w) b = fmaxf(b, wmax[w]);
    parts[blockIdx.x] = b;
  }
}

template <typename T>
__device__ __forceinline__ void quant_vec(const char* x, uint8_t* q, uint64_t v, float s) {
  using V = QVec<T>;
  float f[V::PER];
  V::load(x, v, f);
  if constexpr (V::PER == 4) {
    *(__attribute__((address_space(1))) unsigned int*)(q + v * 4) = pack4(f[0] * s, f[1] * s, f[2] * s, f[3] * s);
  } else {
    q_u32x2 w = {pack4(f[0] * s, f[1] * s, f[2] * s, f[3] * s), pack4(f[4] * s, f[5] * s, f[6] * s, f[7] * s)};
    *(__attribute__((address_space(1))) q_u32x2*)(q + v * 8) = w;
  }
}

template <typename T>
__global__ void __launch_bounds__(kQThreads) quantize_kernel(const char* x, uint8_t* q, uint64_t n, const float* amax,
                                                             float num) {
  using V = QVec<T>;
  const float s = block_scale(amax, num);
  const uint64_t nv = n / V::PER;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; v + (kQUnroll - 1) * stride < nv; v += kQUnroll * stride) {
#pragma unroll
    for (int u = 0; u < kQUnroll; ++u) quant_vec<T>(x, q, v + u * stride, s);
  }
  for (; v < nv; v += stride) quant_vec<T>(x, q, v, s);
  for (uint64_t i = nv * V::PER + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    q[i] = Elem<fp8e4m3_t>::store(Elem<T>::load(reinterpret_cast<const T*>(x)[i]) * s).bits;
}

template <typename T>
__device__ __forceinline__ void dequant_vec(const uint8_t* q, char* x, uint64_t v, float inv) {
  using V = QVec<T>;
  float f[V::PER];
  if constexpr (V::PER == 4) {
    unpack4(*(const __attribute__((address_space(1))) unsigned int*)(q + v * 4), inv, f);
  } else {
    q_u32x2 w = *(const __attribute__((address_space(1))) q_u32x2*)(q + v * 8);
    unpack4(w.x, inv, f);
    unpack4(w.y, inv, f + 4);
  }
  V::store(x, v, f);
}

template <typename T>
__global__ void __launch_bounds__(kQThreads) dequantize_kernel(const uint8_t* q, char* x, uint64_t n, const float* amax,
                                                               float num) {
  using V = QVec<T>;
  const float inv = 1.0f / block_scale(amax, num);
  const uint64_t nv = n / V::PER;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; v + (kQUnroll - 1) * stride < nv; v += kQUnroll * stride) {
#pragma unroll
    for (int u = 0; u < kQUnroll; ++u) dequant_vec<T>(q, x, v + u * stride, inv);
  }
  for (; v < nv; v += stride) dequant_vec<T>(q, x, v, inv);
  for (uint64_t i = nv * V::PER + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    reinterpret_cast<T*>(x)[i] = Elem<T>::store(Elem<fp8e4m3_t>::load(fp8e4m3_t{q[i]}) * inv);
}

static int qgrid(uint64_t n) {  // 4 elements per lane and step at least, kQUnroll steps per lane
  uint64_t g = (n / 4 + (uint64_t)kQThreads * kQUnroll - 1) / ((uint64_t)kQThreads * kQUnroll);
  if (g < 1) g = 1;
  return (int)(g > 2048 ? 2048 : g);  // grid-stride beyond 8 workgroups per CU
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace flexar

using namespace flexar;

#define FXQ_CHECK_LAUNCH()                                                                      \
  do {                                                                                          \
    hipError_t e_ = hipGetLastError();                                                          \
    if (e_ != hipSuccess) {                                                                     \
      set_error(std::string("quant kernel launch: ") + hipGetErrorString(e_));                  \
      return FLEXAR_ERR_HIP;                                                                    \
    }                                                                                           \
  } while (0)

#define FXQ_DISPATCH(dtype, KERNEL, ...)                                                        \
  switch (dtype) {                                                                              \
    case FLEXAR_FLOAT32: hipLaunchKernelGGL(KERNEL<float>, __VA_ARGS__); break;                 \
    case FLEXAR_BFLOAT16: hipLaunchKernelGGL(KERNEL<bf16_t>, __VA_ARGS__); break;               \
    case FLEXAR_FLOAT16: hipLaunchKernelGGL(KERNEL<f16_t>, __VA_ARGS__); break;                 \
    default: set_error("fp8 compression: dtype must be float32, bfloat16 or float16");         \
      return FLEXAR_ERR_UNSUPPORTED;                                                            \
  }

extern "C" {

// parts_out: FLEXAR_AMAX_PARTIALS device floats, every one written (one per workgroup).
int flexar_amax(const void* x, size_t n, int dtype, float* parts_out, void* stream) {
  if (!x || !parts_out) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (!aligned16(x)) { set_error("fp8 compression needs 16-byte aligned buffers"); return FLEXAR_ERR_INVALID; }
  FXQ_DISPATCH(dtype, amax_kernel, dim3(kAmaxParts), dim3(kAmaxThreads), 0, (hipStream_t)stream, (const char*)x,
               (uint64_t)n, parts_out)
  FXQ_CHECK_LAUNCH();
  return 0;
}

// q[i] = e4m3(x[i] * num / amax) (saturating), amax = max of the FLEXAR_AMAX_PARTIALS device floats
// (e.g. after a MAX allreduce of the partials).
int flexar_quantize_fp8(const void* x, int dtype, void* q, size_t n, const float* amax, float num, void* stream) {
  if (!x || !q || !amax) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (!aligned16(x) || !aligned16(q)) { set_error("fp8 compression needs 16-byte aligned buffers"); return FLEXAR_ERR_INVALID; }
  if (n == 0) return 0;
  FXQ_DISPATCH(dtype, quantize_kernel, dim3(qgrid(n)), dim3(kQThreads), 0, (hipStream_t)stream, (const char*)x,
               (uint8_t*)q, (uint64_t)n, amax, num)
  FXQ_CHECK_LAUNCH();
  return 0;
}

// x[i] = e4m3_to_f32(q[i]) * amax / num
int flexar_dequantize_fp8(const void* q, void* x, int dtype, size_t n, const float* amax, float num, void* stream) {
  if (!x || !q || !amax) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (!aligned16(x) || !aligned16(q)) { set_error("fp8 compression needs 16-byte aligned buffers"); return FLEXAR_ERR_INVALID; }
  if (n == 0) return 0;
  FXQ_DISPATCH(dtype, dequantize_kernel, dim3(qgrid(n)), dim3(kQThreads), 0, (hipStream_t)stream, (const uint8_t*)q,
               (char*)x, (uint64_t)n, amax, num)
  FXQ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
