// Per-dtype kernel launchers. Each dtype's kernels are instantiated in their own
// translation unit (k_<dtype>.hip) so the gfx950 build parallelises.
#pragma once

#include <hip/hip_runtime.h>

#include "device_exec.hpp"

namespace flexar {

// LAUNCH_QUERY launches nothing: it reports the occupancy (workgroups per CU) and the VGPR count of the
// kernel that `proto` / `query` select (query 0 = executor, 1 = LL, 2 = standalone reduce).
enum LaunchKind { LAUNCH_EXEC = 0, LAUNCH_GROUP = 1, LAUNCH_REDUCE = 2, LAUNCH_LL = 3, LAUNCH_LL_GROUP = 4,
                  LAUNCH_QUERY = 5 };

struct LaunchArgs {
  int kind = LAUNCH_EXEC;
  DevCtx ctx;                      // EXEC
  const DevCtx* d_ctxs = nullptr;  // GROUP
  int nranks = 1;                  // GROUP
  int grid = 1;
  hipStream_t stream = nullptr;
  SrcTable srcs;                   // REDUCE
  int nsrc = 0;
  char* dst = nullptr;
  char* dst2 = nullptr;            // REDUCE: optional second destination
  uint64_t n = 0;
  float scale = 1.0f;
  int vec = 1;
  int proto = PM_FENCE;  // executor protocol mode (PM_*: "+nts", "+wt")
  int query = 0;         // QUERY: which kernel
  int* occ_out = nullptr;
  int* regs_out = nullptr;
};

// Defined in k_<dtype>.hip; returns 0 or a FLEXAR_ERR_* code.
#define FX_DECLARE_LAUNCH(NAME) int launch_##NAME(int op, const LaunchArgs& a);
FX_DECLARE_LAUNCH(f32)
FX_DECLARE_LAUNCH(f16)
FX_DECLARE_LAUNCH(bf16)
FX_DECLARE_LAUNCH(f64)
FX_DECLARE_LAUNCH(e4m3)
FX_DECLARE_LAUNCH(e5m2)
FX_DECLARE_LAUNCH(i8)
FX_DECLARE_LAUNCH(u8)
FX_DECLARE_LAUNCH(i16)
FX_DECLARE_LAUNCH(u16)
FX_DECLARE_LAUNCH(i32)
FX_DECLARE_LAUNCH(u32)
FX_DECLARE_LAUNCH(i64)
FX_DECLARE_LAUNCH(u64)
FX_DECLARE_LAUNCH(boolean)
#undef FX_DECLARE_LAUNCH

inline int launch_dtype(int dtype, int op, const LaunchArgs& a) {
  switch (dtype) {
    case FLEXAR_FLOAT32: return launch_f32(op, a);
    case FLEXAR_FLOAT16: return launch_f16(op, a);
    case FLEXAR_BFLOAT16: return launch_bf16(op, a);
    case FLEXAR_FLOAT64: return launch_f64(op, a);
    case FLEXAR_FP8_E4M3: return launch_e4m3(op, a);
    case FLEXAR_FP8_E5M2: return launch_e5m2(op, a);
    case FLEXAR_INT8: return launch_i8(op, a);
    case FLEXAR_UINT8: return launch_u8(op, a);
    case FLEXAR_INT16: return launch_i16(op, a);
    case FLEXAR_UINT16: return launch_u16(op, a);
    case FLEXAR_INT32: return launch_i32(op, a);
    case FLEXAR_UINT32: return launch_u32(op, a);
    case FLEXAR_INT64: return launch_i64(op, a);
    case FLEXAR_UINT64: return launch_u64(op, a);
    case FLEXAR_BOOL: return launch_boolean(op, a);
    default: return FLEXAR_ERR_UNSUPPORTED;
  }
}

}  // namespace flexar
