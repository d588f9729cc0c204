// gfx950 kernels (executor, group executor, reduction) for dtype double.
#include "kernels_impl.hpp"
FX_DEFINE_FLOAT_LAUNCH(double, f64)
