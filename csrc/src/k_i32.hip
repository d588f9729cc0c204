// gfx950 kernels (executor, group executor, reduction) for dtype int32_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(int32_t, i32)
