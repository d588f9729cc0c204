// gfx950 kernels (executor, group executor, reduction) for dtype f16_t.
#include "kernels_impl.hpp"
FX_DEFINE_FLOAT_LAUNCH(f16_t, f16)
