// Typed executors, fp32 partial sums for bf16 / fp16 ("+f32": ring / tree schedules round once).
#include "kernels_impl.hpp"

namespace flexar {
int launch_mx_acc16(int dtype, const LaunchArgs& a) {
  return dtype == FLEXAR_BFLOAT16 ? launch_typed<bf16_t, float>(a) : launch_typed<f16_t, float>(a);
}
}  // namespace flexar
