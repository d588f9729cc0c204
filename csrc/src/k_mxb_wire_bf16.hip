// Typed executors, bf16 inputs over an OCP MX block-scaled fp8 wire ("+mxe4m3" / "+mxe5m2": flat
// schedule, one e8m0 scale per 32-element block, no amax pass; device_exec.hpp xfer_mxb).
#include "kernels_impl.hpp"

namespace flexar {
int launch_mxb_wire_bf16(const LaunchArgs& a) {
  return a.wire == 5 ? launch_typed<bf16_t, mxe5m2_t>(a) : launch_typed<bf16_t, mxe4m3_t>(a);
}
}  // namespace flexar
