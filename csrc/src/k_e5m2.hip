// gfx950 kernels (executor, group executor, reduction) for dtype fp8e5m2_t.
#include "kernels_impl.hpp"
FX_DEFINE_FLOAT_LAUNCH(fp8e5m2_t, e5m2)
