// Typed executors, fp32 partial sums for OCP fp8 inputs ("+f32": ring / tree schedules round once).
#include "kernels_impl.hpp"

namespace flexar {
int launch_mx_acc8(int dtype, const LaunchArgs& a) {
  return dtype == FLEXAR_FP8_E4M3 ? launch_typed<fp8e4m3_t, float>(a) : launch_typed<fp8e5m2_t, float>(a);
}
}  // namespace flexar
