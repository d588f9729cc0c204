// gfx950 kernels (executor, group executor, reduction) for dtype int64_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(int64_t, i64)
