// gfx950 kernels (executor, group executor, reduction) for dtype fp8e4m3_t.
#include "kernels_impl.hpp"
FX_DEFINE_FLOAT_LAUNCH(fp8e4m3_t, e4m3)
