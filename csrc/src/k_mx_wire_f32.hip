// Typed executors, f32 inputs over an fp8 wire ("+e4m3" / "+e5m2": flat schedule, the pre-scale from
// the global amax fused into the first transfer, the post-scale into the last).
#include "kernels_impl.hpp"

namespace flexar {
int launch_mx_wire_f32(const LaunchArgs& a) {
  return a.wire == 3 ? launch_typed<float, fp8e5m2_t>(a) : launch_typed<float, fp8e4m3_t>(a);
}
}  // namespace flexar
