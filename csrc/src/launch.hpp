// Per-dtype kernel launchers. Each dtype's kernels are instantiated in their own
// translation unit (k_<dtype>.hip) so the gfx950 build parallelises.
#pragma once

#include <hip/hip_runtime.h>

#include "crumbs.hpp"
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
  int* scratch_out = nullptr;  // private segment bytes per lane
  int max_fanin = 0;     // typed programs: the widest XFER fan-in (Program::max_nsrc; 0 = unknown, widest kernel)
  int wire = 0;          // EXEC / GROUP / QUERY of a typed program (Program::wire): 1 fp32, 2 e4m3, 3 e5m2,
                         // 4 / 5 MX e4m3 / e5m2
  // breadcrumb of this launch (crumbs.hpp): the spec / purpose, the device epoch it runs as, its bytes
  const char* tag = nullptr;
  uint64_t epoch = 0;
  uint64_t bytes = 0;
};

// Typed-program executors (exec_mx_kernel), SUM/AVG only: fp32 partials for 16/8-bit dtypes
// (k_mx_acc*.hip) and an fp8 wire for 32/16-bit floats (k_mx_wire_*.hip), one translation unit per
// input dtype so the gfx950 build parallelises.
int launch_mx_acc_bf16(const LaunchArgs& a);  // 16/8-bit dtypes with fp32 partials
int launch_mx_acc_f16(const LaunchArgs& a);
int launch_mx_acc_e4m3(const LaunchArgs& a);
int launch_mx_acc_e5m2(const LaunchArgs& a);
int launch_mx_wire_f32(const LaunchArgs& a);          // fp32 over e4m3 / e5m2 (a.wire)
int launch_mx_wire_bf16(const LaunchArgs& a);
int launch_mx_wire_f16(const LaunchArgs& a);
int launch_mxb_wire_f32(const LaunchArgs& a);         // OCP MX block-scaled fp8 wire (a.wire 4 / 5)
int launch_mxb_wire_bf16(const LaunchArgs& a);
int launch_mxb_wire_f16(const LaunchArgs& a);
inline int launch_mx(int dtype, const LaunchArgs& a) {
  if (a.wire >= 4) {
    switch (dtype) {
      case FLEXAR_FLOAT32: return launch_mxb_wire_f32(a);
      case FLEXAR_BFLOAT16: return launch_mxb_wire_bf16(a);
      case FLEXAR_FLOAT16: return launch_mxb_wire_f16(a);
      default: return FLEXAR_ERR_UNSUPPORTED;
    }
  }
  if (a.wire == 1) {
    switch (dtype) {
      case FLEXAR_BFLOAT16: return launch_mx_acc_bf16(a);
      case FLEXAR_FLOAT16: return launch_mx_acc_f16(a);
      case FLEXAR_FP8_E4M3: return launch_mx_acc_e4m3(a);
      case FLEXAR_FP8_E5M2: return launch_mx_acc_e5m2(a);
      default: return FLEXAR_ERR_UNSUPPORTED;
    }
  }
  switch (dtype) {
    case FLEXAR_FLOAT32: return launch_mx_wire_f32(a);
    case FLEXAR_BFLOAT16: return launch_mx_wire_bf16(a);
    case FLEXAR_FLOAT16: return launch_mx_wire_f16(a);
    default: return FLEXAR_ERR_UNSUPPORTED;
  }
}

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

inline void launch_crumb(int dtype, int op, const LaunchArgs& a) {
  CrumbArgs c;
  c.type = CRUMB_LAUNCH;
  c.launch_kind = (uint8_t)a.kind;
  c.proto = (uint8_t)a.proto;
  c.wire = (uint8_t)a.wire;
  const bool grouped = a.kind == LAUNCH_GROUP || a.kind == LAUNCH_LL_GROUP;
  c.rank = grouped ? (int16_t)-1 : (a.kind == LAUNCH_REDUCE ? (int16_t)-1 : (int16_t)a.ctx.rank);
  c.nranks = (int16_t)(grouped ? a.nranks : a.ctx.nranks);
  c.dtype = (int16_t)dtype;
  c.op = (int16_t)op;
  c.grid = (uint32_t)(grouped ? a.grid * a.nranks : a.grid);
  c.epoch = a.epoch;
  c.bytes = a.bytes;
  c.what = a.kind == LAUNCH_REDUCE ? "reduce" : grouped ? "group" : "executor";
  c.label = a.tag;
  crumb(c);
}

inline int launch_dtype(int dtype, int op, const LaunchArgs& a) {
  if (a.kind != LAUNCH_QUERY) launch_crumb(dtype, op, a);
  if (a.wire && (a.kind == LAUNCH_EXEC || a.kind == LAUNCH_GROUP || a.kind == LAUNCH_QUERY)) {
    if (op != FLEXAR_SUM && op != FLEXAR_AVG) return FLEXAR_ERR_UNSUPPORTED;
    return launch_mx(dtype, a);
  }
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
