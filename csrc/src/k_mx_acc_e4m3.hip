// Typed executors, fp32 partial sums for e4m3 inputs ("+f32": ring / tree schedules round once).
#include "kernels_impl.hpp"

namespace flexar {
int launch_mx_acc_e4m3(const LaunchArgs& a) { return launch_typed<fp8e4m3_t, float>(a); }
}  // namespace flexar
