// Semantics of gfx950's scaled fp8 conversions (v_cvt_scalef32_pk_fp8_f32 / _bf16 and back), measured on the
// device: which way the f32 scale applies, whether only its exponent counts, saturation and rounding.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probes/scaled_cvt_probe.hip -o bin/scaled_cvt_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short s2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));

struct Case { float a, b, scale; };

__global__ void probe(const Case* cs, int n, float* out) {
  const int t = threadIdx.x;
  if (t >= n) return;
  const Case c = cs[t];
  // f32 -> e4m3 with scale, decoded without scale: shows x / scale or x * scale
  const s2 q = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(s2{0, 0}, c.a, c.b, c.scale, false);
  const f2 plain = __builtin_amdgcn_cvt_pk_f32_fp8((int)(unsigned short)q[0], false);
  // e4m3 (encoded without scale) -> f32 with scale
  const int e = __builtin_amdgcn_cvt_pk_fp8_f32(c.a, c.b, 0, false);
  const f2 up = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8((unsigned)e, c.scale, false);
  // bf16 -> e4m3 with scale, and e4m3 -> bf16 with scale
  const bf2 x = {(__bf16)c.a, (__bf16)c.b};
  const s2 qb = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(s2{0, 0}, x, c.scale, false);
  const f2 plainb = __builtin_amdgcn_cvt_pk_f32_fp8((int)(unsigned short)qb[0], false);
  const bf2 upb = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((unsigned)e, c.scale, false);
  float* o = out + t * 8;
  o[0] = plain.x; o[1] = plain.y; o[2] = up.x; o[3] = up.y;
  o[4] = plainb.x; o[5] = plainb.y; o[6] = (float)upb.x; o[7] = (float)upb.y;
}

int main() {
  const Case h[] = {{1.0f, 3.0f, 2.0f},   {1.0f, 3.0f, 3.0f},  {1.0f, 3.0f, 0.5f},  {448.0f, 500.0f, 1.0f},
                    {896.0f, 1e6f, 2.0f}, {1.0625f, 1.09375f, 1.0f}, {1.03125f, 1.09375f, 1.0f},
                    {0.001f, -2.5f, 0.25f}, {100.f, -100.f, 1.5f}};
  const int n = sizeof(h) / sizeof(h[0]);
  Case* d = nullptr;
  float* o = nullptr;
  if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&o, n * 8 * sizeof(float)) != hipSuccess) return 1;
  if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, n, o);
  float r[64 * 8];
  if (hipMemcpy(r, o, n * 8 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int i = 0; i < n; ++i) {
    const float* v = r + i * 8;
    printf("{\"a\": %g, \"b\": %g, \"scale\": %g, \"f32_to_fp8_decoded_plain\": [%g, %g], "
           "\"fp8_to_f32_scaled\": [%g, %g], \"bf16_to_fp8_decoded_plain\": [%g, %g], \"fp8_to_bf16_scaled\": [%g, %g]}\n",
           h[i].a, h[i].b, h[i].scale, v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
  }
  return 0;
}
