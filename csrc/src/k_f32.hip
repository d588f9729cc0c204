// gfx950 kernels (executor, group executor, reduction) for dtype float.
#include "kernels_impl.hpp"
FX_DEFINE_FLOAT_LAUNCH(float, f32)
