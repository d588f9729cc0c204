// Instantiation helper included by each k_<dtype>.hip.
#pragma once

#include <atomic>
#include <string>

#include "internal.hpp"
#include "launch.hpp"

namespace flexar {

template <typename K>
inline int query_kernel(K kern, const LaunchArgs& a, int threads = kExecThreads) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, threads, 0) != hipSuccess) {
    (void)hipGetLastError();
    set_error("occupancy query failed");
    return FLEXAR_ERR_HIP;
  }
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kern)) != hipSuccess) {
    (void)hipGetLastError();
    fa.numRegs = 0;
    fa.localSizeBytes = 0;
  }
  if (a.occ_out) *a.occ_out = occ;
  if (a.regs_out) *a.regs_out = fa.numRegs;
  if (a.scratch_out) *a.scratch_out = (int)fa.localSizeBytes;
  return 0;
}

// HIP keeps a failed call's error for the thread until it is read; one left by an unrelated, ignored call
// must not be reported as this launch's failure (the check after the launch reads only its own error).
inline void clear_stale_error() { (void)hipGetLastError(); }

template <typename T, typename OP>
inline int launch_one(const LaunchArgs& a) {
  if (a.kind != LAUNCH_QUERY) clear_stale_error();
  switch (a.kind) {
    case LAUNCH_QUERY:
      if (a.query == 1) {
        if (sizeof(T) > 4) return FLEXAR_ERR_UNSUPPORTED;
        return query_kernel(ll_kernel<T, OP>, a);
      }
      if (a.query == 2) return query_kernel(a.proto == PM_WT ? reduce_kernel<T, OP, PM_WT> : reduce_kernel<T, OP, PM_FENCE>, a);
      return query_kernel(a.proto == PM_WT ? exec_kernel<T, OP, PM_WT>
                                           : a.proto == PM_FENCE_NTS ? exec_kernel<T, OP, PM_FENCE_NTS>
                                                                     : exec_kernel<T, OP, PM_FENCE>, a);
    case LAUNCH_EXEC:
      if (a.proto == PM_WT)
        hipLaunchKernelGGL((exec_kernel<T, OP, PM_WT>), dim3(a.grid), dim3(kExecThreads), 0, a.stream, a.ctx);
      else if (a.proto == PM_FENCE_NTS)
        hipLaunchKernelGGL((exec_kernel<T, OP, PM_FENCE_NTS>), dim3(a.grid), dim3(kExecThreads), 0, a.stream, a.ctx);
      else
        hipLaunchKernelGGL((exec_kernel<T, OP, PM_FENCE>), dim3(a.grid), dim3(kExecThreads), 0, a.stream, a.ctx);
      break;
    case LAUNCH_GROUP:
      if (a.proto == PM_WT)
        hipLaunchKernelGGL((exec_group_kernel<T, OP, PM_WT>), dim3(a.grid * a.nranks), dim3(kExecThreads), 0,
                           a.stream, a.d_ctxs, (uint32_t)a.grid);
      else if (a.proto == PM_FENCE_NTS)
        hipLaunchKernelGGL((exec_group_kernel<T, OP, PM_FENCE_NTS>), dim3(a.grid * a.nranks), dim3(kExecThreads), 0,
                           a.stream, a.d_ctxs, (uint32_t)a.grid);
      else
        hipLaunchKernelGGL((exec_group_kernel<T, OP, PM_FENCE>), dim3(a.grid * a.nranks), dim3(kExecThreads), 0,
                           a.stream, a.d_ctxs, (uint32_t)a.grid);
      break;
    case LAUNCH_REDUCE:
      if (a.proto == PM_WT)
        hipLaunchKernelGGL((reduce_kernel<T, OP, PM_WT>), dim3(a.grid), dim3(kExecThreads), 0, a.stream, a.srcs,
                           a.nsrc, a.dst, a.dst2, a.n, a.scale, a.vec);
      else
        hipLaunchKernelGGL((reduce_kernel<T, OP, PM_FENCE>), dim3(a.grid), dim3(kExecThreads), 0, a.stream, a.srcs,
                           a.nsrc, a.dst, a.dst2, a.n, a.scale, a.vec);
      break;
    case LAUNCH_LL:
      if (sizeof(T) > 4) return FLEXAR_ERR_UNSUPPORTED;
      hipLaunchKernelGGL((ll_kernel<T, OP>), dim3(a.grid), dim3(kExecThreads), 0, a.stream, a.ctx);
      break;
    case LAUNCH_LL_GROUP:
      if (sizeof(T) > 4) return FLEXAR_ERR_UNSUPPORTED;
      hipLaunchKernelGGL((ll_group_kernel<T, OP>), dim3(a.grid * a.nranks), dim3(kExecThreads), 0, a.stream,
                         a.d_ctxs, (uint32_t)a.grid);
      break;
    default:
      return FLEXAR_ERR_INVALID;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("kernel launch: ") + hipGetErrorString(e));
    return FLEXAR_ERR_HIP;
  }
  return 0;
}

template <typename T>
inline int launch_float(int op, const LaunchArgs& a) {
  switch (op) {
    case FLEXAR_SUM: case FLEXAR_AVG: return launch_one<T, OpSum>(a);
    case FLEXAR_PROD: return launch_one<T, OpProd>(a);
    case FLEXAR_MAX: return launch_one<T, OpMax>(a);
    case FLEXAR_MIN: return launch_one<T, OpMin>(a);
    default: return FLEXAR_ERR_UNSUPPORTED;
  }
}

template <typename T>
inline int launch_int(int op, const LaunchArgs& a) {
  switch (op) {
    case FLEXAR_SUM: return launch_one<T, OpSum>(a);
    case FLEXAR_PROD: return launch_one<T, OpProd>(a);
    case FLEXAR_MAX: return launch_one<T, OpMax>(a);
    case FLEXAR_MIN: return launch_one<T, OpMin>(a);
    case FLEXAR_BAND: return launch_one<T, OpBand>(a);
    case FLEXAR_BOR: return launch_one<T, OpBor>(a);
    case FLEXAR_BXOR: return launch_one<T, OpBxor>(a);
    default: return FLEXAR_ERR_UNSUPPORTED;
  }
}

}  // namespace flexar

namespace flexar {

// Workgroups of `kern` (at `threads`) the current device keeps resident at once, cached per kernel and device.
template <typename K>
inline int resident_blocks(K kern, int threads, std::atomic<int>* cache) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) { (void)hipGetLastError(); return 0; }
  int v = cache[dev].load(std::memory_order_relaxed);
  if (v > 0) return v;
  int occ = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, threads, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  v = occ * cus;
  cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

// Typed-program executor launch (exec_mx_kernel<T, W, PM, KMAX>); "+nts" runs the fence protocol.
template <typename T, typename W, int KMAX>
inline int launch_typed_k(const LaunchArgs& a) {
  const bool wt = a.proto == PM_WT;
  if (a.kind != LAUNCH_QUERY) clear_stale_error();
  // FLEXAR_TYPED_THREADS = 256: 2-3 times the workgroups of half the size (a multiple of the channel count still),
  // never more than the device keeps resident (every workgroup waits on its peers' workgroup of the same index)
  int g = a.grid;
  if (typed_grid_mul<KMAX>() > 1 && a.kind != LAUNCH_QUERY) {
    static std::atomic<int> res_cache[2][2][16];  // [group][wt][device]
    const int ranks = a.kind == LAUNCH_GROUP ? a.nranks : 1;
    const int res = a.kind == LAUNCH_GROUP
                        ? resident_blocks(wt ? exec_mx_group_kernel<T, W, PM_WT, KMAX> : exec_mx_group_kernel<T, W, PM_FENCE, KMAX>,
                                          kTypedThreads, res_cache[0][wt])
                        : resident_blocks(wt ? exec_mx_kernel<T, W, PM_WT, KMAX> : exec_mx_kernel<T, W, PM_FENCE, KMAX>,
                                          kTypedThreads, res_cache[1][wt]);
    for (int m = typed_grid_mul<KMAX>(); m > 1; --m)
      if (a.grid * m <= (int)kMaxGridBlocks && a.grid * m * ranks <= res) { g = a.grid * m; break; }
  }
  switch (a.kind) {
    case LAUNCH_QUERY:
      return query_kernel(wt ? exec_mx_kernel<T, W, PM_WT, KMAX> : exec_mx_kernel<T, W, PM_FENCE, KMAX>, a,
                          kTypedThreads);
    case LAUNCH_EXEC:
      if (wt) hipLaunchKernelGGL((exec_mx_kernel<T, W, PM_WT, KMAX>), dim3(g), dim3(kTypedThreads), 0, a.stream, a.ctx);
      else hipLaunchKernelGGL((exec_mx_kernel<T, W, PM_FENCE, KMAX>), dim3(g), dim3(kTypedThreads), 0, a.stream, a.ctx);
      break;
    case LAUNCH_GROUP:
      if (wt)
        hipLaunchKernelGGL((exec_mx_group_kernel<T, W, PM_WT, KMAX>), dim3(g * a.nranks), dim3(kTypedThreads), 0,
                           a.stream, a.d_ctxs, (uint32_t)g);
      else
        hipLaunchKernelGGL((exec_mx_group_kernel<T, W, PM_FENCE, KMAX>), dim3(g * a.nranks), dim3(kTypedThreads), 0,
                           a.stream, a.d_ctxs, (uint32_t)g);
      break;
    default:
      return FLEXAR_ERR_INVALID;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("kernel launch: ") + hipGetErrorString(e));
    return FLEXAR_ERR_HIP;
  }
  return 0;
}
// fp8 wire kernels (global and MX scales) come in two fan-in classes (xfer_op_typed KMAX): programs whose
// XFERs read at most 4 operands (flat schedules of <= 4 ranks) launch the narrow one
template <typename T, typename W>
inline int launch_typed(const LaunchArgs& a) {
  if constexpr (sizeof(W) == 1) {
    if (a.max_fanin > 0 && a.max_fanin <= 4) return launch_typed_k<T, W, 4>(a);
  }
  return launch_typed_k<T, W, kMaxSrc>(a);
}

}  // namespace flexar

#define FX_DEFINE_FLOAT_LAUNCH(T, NAME) \
  namespace flexar {                    \
  int launch_##NAME(int op, const LaunchArgs& a) { return launch_float<T>(op, a); } \
  }
#define FX_DEFINE_INT_LAUNCH(T, NAME) \
  namespace flexar {                  \
  int launch_##NAME(int op, const LaunchArgs& a) { return launch_int<T>(op, a); } \
  }
