// Element types, conversions and reduction functors shared by the host
// executor (CPU path / simulator) and the gfx950 device kernels.
//
// Parity: the reference supports SUM and BAND on integer/float/double types
// (allreduce_over_mpi/mpi_mod.hpp:825-874) via reduce_sum / reduce_band
// (mpi_mod.hpp:245-660, hand-unrolled per fan-in, OpenMP). Here one functor
// family covers SUM/PROD/MAX/MIN/AVG/BAND/BOR/BXOR, and 16/8-bit floats
// (bf16, fp16, OCP fp8 e4m3/e5m2) accumulate in fp32 and round once.
#pragma once

#include <stdint.h>
#include <string.h>

#include "flexar/flexar.h"

#if defined(__HIPCC__)
#define FX_HD __host__ __device__
#define FX_INLINE __forceinline__
#else
#define FX_HD
#define FX_INLINE inline __attribute__((always_inline))
#endif

namespace flexar {

// ---- storage types -------------------------------------------------------
struct bf16_t { uint16_t bits; };
struct f16_t { uint16_t bits; };
struct fp8e4m3_t { uint8_t bits; };
struct fp8e5m2_t { uint8_t bits; };
// OCP MX block-scaled fp8 on the links (AlgoSpec::wire 4 / 5, "+mxe4m3" / "+mxe5m2"): the element bits
// are those of fp8e4m3_t / fp8e5m2_t, and every kMxBlock consecutive elements share one e8m0 scale byte
// (device_exec.hpp xfer_mxb, host_exec.hpp host_xfer_mxb). Distinct types select the block-scaled executor.
struct mxe4m3_t { uint8_t bits; };
struct mxe5m2_t { uint8_t bits; };

FX_HD FX_INLINE uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
FX_HD FX_INLINE float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

// ---- bf16 ----------------------------------------------------------------
FX_HD FX_INLINE float bf16_to_f32(uint16_t b) { return u2f(((uint32_t)b) << 16); }
FX_HD FX_INLINE uint16_t f32_to_bf16(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  // v_cvt_pk_bf16_f32 (RNE, keeps NaN a NaN — MI355X_MICROARCH.md correctness table)
  __bf16 h = (__bf16)f;
  uint16_t r; memcpy(&r, &h, 2); return r;
#else
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
#endif
}

// ---- fp16 ----------------------------------------------------------------
FX_HD FX_INLINE float f16_to_f32(uint16_t h) {
#if defined(__HIP_DEVICE_COMPILE__)
  _Float16 x; memcpy(&x, &h, 2); return (float)x;
#else
  uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ffu;
  if (e == 0) {
    if (m == 0) return u2f(s);
    float v = (float)m * (1.0f / 16777216.0f);  // m * 2^-24
    return (s ? -v : v);
  }
  if (e == 31) return u2f(s | 0x7f800000u | (m << 13));
  return u2f(s | ((e + 112) << 23) | (m << 13));
#endif
}
FX_HD FX_INLINE uint16_t f32_to_f16(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  _Float16 x = (_Float16)f; uint16_t r; memcpy(&r, &x, 2); return r;
#else
  uint32_t u = f2u(f);
  uint32_t s = (u >> 16) & 0x8000u;
  uint32_t a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return (uint16_t)(s | 0x7e00u);
  if (a >= 0x477ff000u) return (uint16_t)(s | 0x7c00u);  // overflow -> inf (IEEE RNE)
  if (a < 0x38800000u) {                                   // subnormal / zero
    // value * 2^24 rounded to nearest even
    float v = u2f(a) * 16777216.0f;
    uint32_t m = (uint32_t)v;
    float rem = v - (float)m;
    if (rem > 0.5f || (rem == 0.5f && (m & 1u))) m++;
    return (uint16_t)(s | m);
  }
  uint32_t e = (a >> 23) - 112, m = a & 0x7fffffu;
  uint32_t h = (e << 10) | (m >> 13);
  uint32_t rest = m & 0x1fffu;
  if (rest > 0x1000u || (rest == 0x1000u && (h & 1u))) h++;
  return (uint16_t)(s | h);
#endif
}

// ---- OCP fp8 (software reference; the device path uses v_cvt_*_fp8) -------
FX_HD FX_INLINE float fp8_decode(uint8_t v, int ebits, int mbits, int bias, bool has_inf) {
  uint32_t s = (v >> 7) & 1u;
  uint32_t e = (v >> mbits) & ((1u << ebits) - 1u);
  uint32_t m = v & ((1u << mbits) - 1u);
  float r;
  if (has_inf) {  // e5m2: IEEE-like
    if (e == (1u << ebits) - 1u) return u2f((s << 31) | (m ? 0x7fc00000u : 0x7f800000u));
  } else {        // e4m3fn: only S.1111.111 is NaN
    if (e == (1u << ebits) - 1u && m == (1u << mbits) - 1u) return u2f((s << 31) | 0x7fc00000u);
  }
  if (e == 0) {
    r = (float)m / (float)(1u << mbits);
    // * 2^(1-bias)
    float sc = 1.0f;
    for (int i = 0; i < bias - 1; ++i) sc *= 0.5f;
    r *= sc;
  } else {
    r = u2f(((e - bias + 127u) << 23) | (m << (23 - mbits)));
  }
  return s ? -r : r;
}
// Saturating round-to-nearest-even encode (OCP "satfinite").
FX_HD FX_INLINE uint8_t fp8_encode(float f, int ebits, int mbits, int bias, float maxv) {
  uint32_t u = f2u(f);
  uint8_t s = (uint8_t)((u >> 24) & 0x80u);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint8_t)(s | 0x7f);  // NaN (e4m3: S1111111, e5m2: S11111xx)
  float a = u2f(u & 0x7fffffffu);
  if (a > maxv) a = maxv;
  // smallest normal exponent = 1 - bias
  int emin = 1 - bias;
  uint32_t au = f2u(a);
  int e = (int)(au >> 23) - 127;
  if (a == 0.0f) return s;
  if (e < emin) {  // subnormal in fp8: quantum 2^(emin - mbits)
    float q = 1.0f;
    for (int i = 0; i < mbits - emin; ++i) q *= 2.0f;  // 1/quantum
    float v = a * q;
    uint32_t m = (uint32_t)v;
    float rem = v - (float)m;
    if (rem > 0.5f || (rem == 0.5f && (m & 1u))) m++;
    // m may round up to 1<<mbits => smallest normal, encoding continues naturally
    return (uint8_t)(s | m);
  }
  uint32_t mant = au & 0x7fffffu;
  uint32_t sh = 23 - mbits;
  uint32_t q = ((uint32_t)(e + bias) << mbits) | (mant >> sh);
  uint32_t rest = mant & ((1u << sh) - 1u), half = 1u << (sh - 1);
  if (rest > half || (rest == half && (q & 1u))) q++;
  return (uint8_t)(s | q);
}
#if defined(__HIP_DEVICE_COMPILE__)
// gfx950 converts OCP fp8 natively (v_cvt_f32_fp8 / v_cvt_pk_fp8_f32); saturate first (satfinite).
__device__ FX_INLINE float e4m3_to_f32(uint8_t v) { return __builtin_amdgcn_cvt_f32_fp8((int)v, 0); }
__device__ FX_INLINE float e5m2_to_f32(uint8_t v) { return __builtin_amdgcn_cvt_f32_bf8((int)v, 0); }
__device__ FX_INLINE uint8_t f32_to_e4m3(float f) {
  if (f != f) return 0x7f;  // keep NaN a NaN (fmin/fmax would map it to a bound)
  f = __builtin_fminf(__builtin_fmaxf(f, -448.0f), 448.0f);
  return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(f, f, 0, false) & 0xff);
}
__device__ FX_INLINE uint8_t f32_to_e5m2(float f) {
  if (f != f) return 0x7f;
  f = __builtin_fminf(__builtin_fmaxf(f, -57344.0f), 57344.0f);
  return (uint8_t)(__builtin_amdgcn_cvt_pk_bf8_f32(f, f, 0, false) & 0xff);
}
#else
inline float e4m3_to_f32(uint8_t v) { return fp8_decode(v, 4, 3, 7, false); }
inline float e5m2_to_f32(uint8_t v) { return fp8_decode(v, 5, 2, 15, true); }
inline uint8_t f32_to_e4m3(float f) { return fp8_encode(f, 4, 3, 7, 448.0f); }
inline uint8_t f32_to_e5m2(float f) { return fp8_encode(f, 5, 2, 15, 57344.0f); }
#endif

// ---- per-type traits: storage <-> accumulator ---------------------------------
template <typename T> struct Elem;
#define FX_SIMPLE_ELEM(T, ACC, FLT)                                   \
  template <> struct Elem<T> {                                        \
    using acc = ACC;                                                  \
    static constexpr bool is_float = FLT;                             \
    FX_HD static FX_INLINE acc load(T v) { return (acc)v; }           \
    FX_HD static FX_INLINE T store(acc v) { return (T)v; }            \
  };
FX_SIMPLE_ELEM(float, float, true)
FX_SIMPLE_ELEM(double, double, true)
FX_SIMPLE_ELEM(int8_t, int8_t, false)
FX_SIMPLE_ELEM(uint8_t, uint8_t, false)
FX_SIMPLE_ELEM(int16_t, int16_t, false)
FX_SIMPLE_ELEM(uint16_t, uint16_t, false)
FX_SIMPLE_ELEM(int32_t, int32_t, false)
FX_SIMPLE_ELEM(uint32_t, uint32_t, false)
FX_SIMPLE_ELEM(int64_t, int64_t, false)
FX_SIMPLE_ELEM(uint64_t, uint64_t, false)
#undef FX_SIMPLE_ELEM
struct bool_t { uint8_t v; };
template <> struct Elem<bool_t> {
  using acc = uint8_t;
  static constexpr bool is_float = false;
  FX_HD static FX_INLINE acc load(bool_t v) { return v.v != 0; }
  FX_HD static FX_INLINE bool_t store(acc v) { return bool_t{(uint8_t)(v != 0)}; }
};
template <> struct Elem<bf16_t> {
  using acc = float;
  static constexpr bool is_float = true;
  FX_HD static FX_INLINE acc load(bf16_t v) { return bf16_to_f32(v.bits); }
  FX_HD static FX_INLINE bf16_t store(acc v) { return bf16_t{f32_to_bf16(v)}; }
};
template <> struct Elem<f16_t> {
  using acc = float;
  static constexpr bool is_float = true;
  FX_HD static FX_INLINE acc load(f16_t v) { return f16_to_f32(v.bits); }
  FX_HD static FX_INLINE f16_t store(acc v) { return f16_t{f32_to_f16(v)}; }
};
template <> struct Elem<fp8e4m3_t> {
  using acc = float;
  static constexpr bool is_float = true;
  FX_HD static FX_INLINE acc load(fp8e4m3_t v) { return e4m3_to_f32(v.bits); }
  FX_HD static FX_INLINE fp8e4m3_t store(acc v) { return fp8e4m3_t{f32_to_e4m3(v)}; }
};
template <> struct Elem<fp8e5m2_t> {
  using acc = float;
  static constexpr bool is_float = true;
  FX_HD static FX_INLINE acc load(fp8e5m2_t v) { return e5m2_to_f32(v.bits); }
  FX_HD static FX_INLINE fp8e5m2_t store(acc v) { return fp8e5m2_t{f32_to_e5m2(v)}; }
};
template <> struct Elem<mxe4m3_t> {
  using acc = float;
  static constexpr bool is_float = true;
  FX_HD static FX_INLINE acc load(mxe4m3_t v) { return e4m3_to_f32(v.bits); }
  FX_HD static FX_INLINE mxe4m3_t store(acc v) { return mxe4m3_t{f32_to_e4m3(v)}; }
};
template <> struct Elem<mxe5m2_t> {
  using acc = float;
  static constexpr bool is_float = true;
  FX_HD static FX_INLINE acc load(mxe5m2_t v) { return e5m2_to_f32(v.bits); }
  FX_HD static FX_INLINE mxe5m2_t store(acc v) { return mxe5m2_t{f32_to_e5m2(v)}; }
};

// ---- OCP MX block scales (e8m0) -------------------------------------------
// A block's scale is 2^X with X the smallest exponent such that amax <= fp8_max * 2^X, fp8_max = 1.75 *
// 2^emax (e4m3: 448, emax 8; e5m2: 57344, emax 15): every element / 2^X is then within the fp8 range, so
// the quantisation never saturates (the gfx950 scaled converts turn an overflow into NaN) and the largest
// element keeps fp8's full relative precision. `amax_bits` = the f32 bits of the block's largest
// magnitude, taken as an unsigned maximum over sign-cleared bits (NaN and inf count as the largest);
// returned: the biased e8m0 byte X + 127, clamped to [1, 254] (a normal f32 scale).
constexpr uint32_t kMxBlock = 32;
FX_HD FX_INLINE uint32_t mx_scale_byte(uint32_t amax_bits, bool e4m3) {
  const int e = (int)(amax_bits >> 23) - (e4m3 ? 8 : 15) + ((amax_bits & 0x7fffffu) > 0x600000u ? 1 : 0);
  return (uint32_t)(e < 1 ? 1 : (e > 254 ? 254 : e));
}
FX_HD FX_INLINE float mx_scale_value(uint32_t byte) { return u2f(byte << 23); }

// ---- reduction functors (operate on the accumulator type) ---------------------
// Integer SUM/PROD wrap (computed in the unsigned domain: no signed-overflow UB).
template <typename A> struct Unsigned { using type = A; };
template <> struct Unsigned<int8_t> { using type = uint8_t; };
template <> struct Unsigned<int16_t> { using type = uint16_t; };
template <> struct Unsigned<int32_t> { using type = uint32_t; };
template <> struct Unsigned<int64_t> { using type = uint64_t; };

struct OpSum {
  template <typename A> FX_HD static FX_INLINE A apply(A a, A b) {
    using U = typename Unsigned<A>::type;
    return (A)(U)((U)a + (U)b);
  }
};
template <> FX_HD FX_INLINE float OpSum::apply<float>(float a, float b) { return a + b; }
template <> FX_HD FX_INLINE double OpSum::apply<double>(double a, double b) { return a + b; }
struct OpProd {
  template <typename A> FX_HD static FX_INLINE A apply(A a, A b) {
    using U = typename Unsigned<A>::type;
    return (A)(U)((U)a * (U)b);
  }
};
template <> FX_HD FX_INLINE float OpProd::apply<float>(float a, float b) { return a * b; }
template <> FX_HD FX_INLINE double OpProd::apply<double>(double a, double b) { return a * b; }
struct OpMax { template <typename A> FX_HD static FX_INLINE A apply(A a, A b) { return a > b ? a : b; } };
struct OpMin { template <typename A> FX_HD static FX_INLINE A apply(A a, A b) { return a < b ? a : b; } };
struct OpBand { template <typename A> FX_HD static FX_INLINE A apply(A a, A b) { return (A)(a & b); } };
struct OpBor { template <typename A> FX_HD static FX_INLINE A apply(A a, A b) { return (A)(a | b); } };
struct OpBxor { template <typename A> FX_HD static FX_INLINE A apply(A a, A b) { return (A)(a ^ b); } };

inline size_t dtype_size(int dt) {
  switch (dt) {
    case FLEXAR_FLOAT32: case FLEXAR_INT32: case FLEXAR_UINT32: return 4;
    case FLEXAR_FLOAT16: case FLEXAR_BFLOAT16: case FLEXAR_INT16: case FLEXAR_UINT16: return 2;
    case FLEXAR_FLOAT64: case FLEXAR_INT64: case FLEXAR_UINT64: return 8;
    case FLEXAR_FP8_E4M3: case FLEXAR_FP8_E5M2: case FLEXAR_INT8: case FLEXAR_UINT8: case FLEXAR_BOOL: return 1;
    default: return 0;
  }
}
inline bool dtype_is_float(int dt) {
  return dt == FLEXAR_FLOAT32 || dt == FLEXAR_FLOAT16 || dt == FLEXAR_BFLOAT16 || dt == FLEXAR_FLOAT64 ||
         dt == FLEXAR_FP8_E4M3 || dt == FLEXAR_FP8_E5M2;
}
// Bitwise ops are defined for integer/bool types only (reference: BAND on integer types,
// mpi_mod.hpp:849-868); MAX/MIN/PROD/SUM/AVG for every type (AVG: floats only).
inline bool op_supported(int dt, int op) {
  if (dt < 0 || dt >= FLEXAR_NUM_DTYPES || op < 0 || op >= FLEXAR_NUM_OPS) return false;
  bool bitwise = (op == FLEXAR_BAND || op == FLEXAR_BOR || op == FLEXAR_BXOR);
  if (bitwise) return !dtype_is_float(dt);
  if (op == FLEXAR_AVG) return dtype_is_float(dt);
  return true;
}
inline const char* dtype_name(int dt) {
  static const char* n[] = {"float32", "float16", "bfloat16", "float64", "fp8_e4m3", "fp8_e5m2", "int8", "uint8",
                            "int16", "uint16", "int32", "uint32", "int64", "uint64", "bool"};
  return (dt >= 0 && dt < FLEXAR_NUM_DTYPES) ? n[dt] : "?";
}
inline const char* op_name(int op) {
  static const char* n[] = {"sum", "prod", "max", "min", "avg", "band", "bor", "bxor"};
  return (op >= 0 && op < FLEXAR_NUM_OPS) ? n[op] : "?";
}

// Dispatch helper: calls F::template run<T, OP>(args...) for a runtime (dtype, op).
template <typename F, typename... Args>
inline int dispatch_dtype_op(int dt, int op, Args&&... args) {
  if (!op_supported(dt, op)) return FLEXAR_ERR_UNSUPPORTED;
#define FX_OPS_FLOAT(T)                                                                      \
  switch (op) {                                                                              \
    case FLEXAR_SUM: case FLEXAR_AVG: return F::template run<T, OpSum>(args...);            \
    case FLEXAR_PROD: return F::template run<T, OpProd>(args...);                            \
    case FLEXAR_MAX: return F::template run<T, OpMax>(args...);                              \
    case FLEXAR_MIN: return F::template run<T, OpMin>(args...);                              \
    default: return FLEXAR_ERR_UNSUPPORTED;                                                  \
  }
#define FX_OPS_INT(T)                                                                        \
  switch (op) {                                                                              \
    case FLEXAR_SUM: return F::template run<T, OpSum>(args...);                              \
    case FLEXAR_PROD: return F::template run<T, OpProd>(args...);                            \
    case FLEXAR_MAX: return F::template run<T, OpMax>(args...);                              \
    case FLEXAR_MIN: return F::template run<T, OpMin>(args...);                              \
    case FLEXAR_BAND: return F::template run<T, OpBand>(args...);                            \
    case FLEXAR_BOR: return F::template run<T, OpBor>(args...);                              \
    case FLEXAR_BXOR: return F::template run<T, OpBxor>(args...);                            \
    default: return FLEXAR_ERR_UNSUPPORTED;                                                  \
  }
  switch (dt) {
    case FLEXAR_FLOAT32: FX_OPS_FLOAT(float)
    case FLEXAR_FLOAT16: FX_OPS_FLOAT(f16_t)
    case FLEXAR_BFLOAT16: FX_OPS_FLOAT(bf16_t)
    case FLEXAR_FLOAT64: FX_OPS_FLOAT(double)
    case FLEXAR_FP8_E4M3: FX_OPS_FLOAT(fp8e4m3_t)
    case FLEXAR_FP8_E5M2: FX_OPS_FLOAT(fp8e5m2_t)
    case FLEXAR_INT8: FX_OPS_INT(int8_t)
    case FLEXAR_UINT8: FX_OPS_INT(uint8_t)
    case FLEXAR_INT16: FX_OPS_INT(int16_t)
    case FLEXAR_UINT16: FX_OPS_INT(uint16_t)
    case FLEXAR_INT32: FX_OPS_INT(int32_t)
    case FLEXAR_UINT32: FX_OPS_INT(uint32_t)
    case FLEXAR_INT64: FX_OPS_INT(int64_t)
    case FLEXAR_UINT64: FX_OPS_INT(uint64_t)
    case FLEXAR_BOOL: FX_OPS_INT(bool_t)
    default: return FLEXAR_ERR_UNSUPPORTED;
  }
#undef FX_OPS_FLOAT
#undef FX_OPS_INT
}

}  // namespace flexar
