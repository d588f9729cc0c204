// Typed executors, fp32 partial sums for e5m2 inputs ("+f32": ring / tree schedules round once).
#include "kernels_impl.hpp"

namespace flexar {
int launch_mx_acc_e5m2(const LaunchArgs& a) { return launch_typed<fp8e5m2_t, float>(a); }
}  // namespace flexar
