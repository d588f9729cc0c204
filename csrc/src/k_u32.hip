// gfx950 kernels (executor, group executor, reduction) for dtype uint32_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(uint32_t, u32)
