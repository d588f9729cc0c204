// gfx950 kernels (executor, group executor, reduction) for dtype int8_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(int8_t, i8)
