// gfx950 kernels (executor, group executor, reduction) for dtype bf16_t.
#include "kernels_impl.hpp"
FX_DEFINE_FLOAT_LAUNCH(bf16_t, bf16)
