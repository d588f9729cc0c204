// gfx950 kernels (executor, group executor, reduction) for dtype int16_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(int16_t, i16)
