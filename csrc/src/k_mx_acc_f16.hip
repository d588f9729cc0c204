// Typed executors, fp32 partial sums for f16 inputs ("+f32": ring / tree schedules round once).
#include "kernels_impl.hpp"

namespace flexar {
int launch_mx_acc_f16(const LaunchArgs& a) { return launch_typed<f16_t, float>(a); }
}  // namespace flexar
