// gfx950 kernels (executor, group executor, reduction) for dtype uint16_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(uint16_t, u16)
