// OCP MX fp8 message codec for the hierarchical communicator's cross-node step
// (allreduce_over_mpi_amd/parallel/hierarchical.py _cross_all_reduce_mx):
//   pack         msg = [q_0 .. q_{n-1} | X_0 .. X_{ceil(n/32)-1}]: one e8m0 byte X per 32-element block
//                (the smallest exponent with amax <= fp8_max * 2^X, types.hpp mx_scale_byte) and the fp8 values
//                q = rne(x / 2^X) - the layout the cross-node all-gather carries, in one HBM pass;
//   unpack_sum   out[i] = sum over messages k, in order, of q_k[i] * 2^X_k - the dequantise-and-sum of every
//                node's message in one pass, fp32 accumulation.
// Both are bit-identical to ops.quant.mx_quantize / mx_dequantize + the node-order sum (the torch reference
// and CPU fallback). A 32-element block is 32 consecutive lanes: its amax is an integer max over the
// sign-cleared f32 bits through 5 xor-shuffles inside the half-wave, and one lane stores the scale byte.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "flexar/flexar.h"
#include "flexar/types.hpp"
#include "internal.hpp"

namespace flexar {

constexpr int kMxcThreads = 256;

static int mxc_grid(uint64_t n) {
  const uint64_t g = (n + kMxcThreads - 1) / kMxcThreads;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));  // >= 64 workgroups per XCD for large n
}

template <typename T, typename W>
__global__ void __launch_bounds__(kMxcThreads) mx_pack_kernel(const T* __restrict__ x, uint8_t* __restrict__ msg,
                                                              uint64_t n) {
  constexpr bool E4 = sizeof(W) == 1 && __is_same(W, mxe4m3_t);
  const uint64_t n32 = (n + kMxBlock - 1) / kMxBlock * kMxBlock;
  const uint64_t stride = (uint64_t)gridDim.x * kMxcThreads;  // a multiple of 32: blocks never split
  uint8_t* sb = msg + n;
  for (uint64_t i = (uint64_t)blockIdx.x * kMxcThreads + threadIdx.x; i < n32; i += stride) {
    const float v = i < n ? (float)Elem<T>::load(x[i]) : 0.0f;
    uint32_t am = __float_as_uint(v) & 0x7fffffffu;
#pragma unroll
    for (int o = kMxBlock / 2; o > 0; o >>= 1) am = max(am, (uint32_t)__shfl_xor((int)am, o));
    const uint32_t xr = mx_scale_byte(am, E4);
    if (i < n) msg[i] = Elem<W>::store(v / mx_scale_value(xr)).bits;
    if ((i & (kMxBlock - 1)) == 0) sb[i / kMxBlock] = (uint8_t)xr;
  }
}

template <typename W>
__global__ void __launch_bounds__(kMxcThreads) mx_unpack_sum_kernel(const uint8_t* __restrict__ msgs,
                                                                    uint64_t msg_stride, int nmsg, uint64_t n,
                                                                    float* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kMxcThreads;
  for (uint64_t i = (uint64_t)blockIdx.x * kMxcThreads + threadIdx.x; i < n; i += stride) {
    const uint8_t* m = msgs;
    float acc = (float)Elem<W>::load(W{m[i]}) * mx_scale_value(m[n + i / kMxBlock]);
    for (int k = 1; k < nmsg; ++k) {
      m += msg_stride;
      acc += (float)Elem<W>::load(W{m[i]}) * mx_scale_value(m[n + i / kMxBlock]);
    }
    out[i] = acc;
  }
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

template <typename W>
static int mx_pack_t(const void* x, int dtype, void* msg, uint64_t n, hipStream_t s) {
  const int g = mxc_grid((n + kMxBlock - 1) / kMxBlock * kMxBlock);
  switch (dtype) {
    case FLEXAR_FLOAT32: hipLaunchKernelGGL((mx_pack_kernel<float, W>), g, kMxcThreads, 0, s, (const float*)x, (uint8_t*)msg, n); break;
    case FLEXAR_BFLOAT16: hipLaunchKernelGGL((mx_pack_kernel<bf16_t, W>), g, kMxcThreads, 0, s, (const bf16_t*)x, (uint8_t*)msg, n); break;
    case FLEXAR_FLOAT16: hipLaunchKernelGGL((mx_pack_kernel<f16_t, W>), g, kMxcThreads, 0, s, (const f16_t*)x, (uint8_t*)msg, n); break;
    default: set_error("mx pack: dtype must be float32, bfloat16 or float16"); return FLEXAR_ERR_UNSUPPORTED;
  }
  FXM_CHECK_LAUNCH();
  return 0;
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

// out[i] = sum_k q_k[i] * 2^X_k over nmsg messages laid out msg_stride bytes apart (fp32 out, message order).
int flexar_mx_unpack_sum(const void* msgs, size_t msg_stride, int nmsg, size_t n, int wire, float* out,
                         void* stream) {
  if (!msgs || !out || nmsg < 1) { set_error("mx unpack: null argument or no message"); return FLEXAR_ERR_INVALID; }
  if (wire != 4 && wire != 5) { set_error("mx unpack: wire must be 4 (e4m3) or 5 (e5m2)"); return FLEXAR_ERR_INVALID; }
  if (msg_stride < n + (n + kMxBlock - 1) / kMxBlock) { set_error("mx unpack: message stride too small"); return FLEXAR_ERR_INVALID; }
  if (n == 0) return 0;
  const int g = mxc_grid(n);
  if (wire == 4)
    hipLaunchKernelGGL((mx_unpack_sum_kernel<mxe4m3_t>), g, kMxcThreads, 0, (hipStream_t)stream, (const uint8_t*)msgs,
                       (uint64_t)msg_stride, nmsg, (uint64_t)n, out);
  else
    hipLaunchKernelGGL((mx_unpack_sum_kernel<mxe5m2_t>), g, kMxcThreads, 0, (hipStream_t)stream, (const uint8_t*)msgs,
                       (uint64_t)msg_stride, nmsg, (uint64_t)n, out);
  FXM_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
