// gfx950 kernels (executor, group executor, reduction) for dtype uint64_t.
#include "kernels_impl.hpp"
FX_DEFINE_INT_LAUNCH(uint64_t, u64)
