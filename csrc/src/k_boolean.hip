// gfx950 kernels (executor, group executor, reduction) for dtype bool_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(bool_t, boolean)
