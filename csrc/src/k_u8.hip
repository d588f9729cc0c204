// gfx950 kernels (executor, group executor, reduction) for dtype uint8_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(uint8_t, u8)
