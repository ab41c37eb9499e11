// Semantics of the gfx950 scaled fp8 conversions used by the attention backward staging:
// v_cvt_scalef32_pk_fp8_bf16 / _f32 (is the scale multiplied or divided? rounding? saturation?)
// against v_cvt_pk_fp8_f32 of x*s and x/s, and v_dot2c_f32_bf16 against an fp32 dot.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

__global__ void probe(const float* x, int n, float s, unsigned* o) {
  const int i = threadIdx.x;
  if (i >= n) return;
  const float a = x[i], b = x[(i + 1) % n];
  // bf16 of a, b (truncation-free: inputs are bf16-exact)
  unsigned ua, ub;
  memcpy(&ua, &a, 4); memcpy(&ub, &b, 4);
  const unsigned w = (ua >> 16) | (ub & 0xffff0000u);
  const bf16x2 bb = __builtin_bit_cast(bf16x2, w);
  const s16x2 c1 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16((s16x2){0, 0}, bb, s, false);
  // word_sel = true: the high half written, the low half kept from `old` (= c1)?
  const s16x2 c3 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(c1, bb, s, true);
  const s16x2 c4 = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(c1, a, b, s, true);
  const s16x2 c2 = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32((s16x2){0, 0}, a, b, s, false);
  const int m = __builtin_amdgcn_cvt_pk_fp8_f32(a * s, b * s, 0, false);
  const int d = __builtin_amdgcn_cvt_pk_fp8_f32(a / s, b / s, 0, false);
  const float dot = __builtin_amdgcn_fdot2_f32_bf16(bb, bb, 1.0f, false);
  const float ref = 1.0f + a * a + b * b;
  unsigned r[6] = {(unsigned)__builtin_bit_cast(unsigned, c1) & 0xffffu,
                   (unsigned)__builtin_bit_cast(unsigned, c2) & 0xffffu, (unsigned)__builtin_bit_cast(unsigned, c3),
                   (unsigned)__builtin_bit_cast(unsigned, c4), 0, 0};
  (void)m; (void)d;
  memcpy(&r[4], &dot, 4);
  memcpy(&r[5], &ref, 4);
  for (int k = 0; k < 6; ++k) o[i * 6 + k] = r[k];
}

int main() {
  const float xs[] = {1.0f, -1.5f, 3.0f, 0.375f, 100.0f, 448.0f, 500.0f, -1000.0f, 0.0078125f, 7.0f, 0.0f, 240.0f,
                      1.0e-3f, 2.5f, -0.75f, 3.5f};
  const int n = sizeof(xs) / sizeof(xs[0]);
  const float scales[] = {1.0f, 4.0f, 0.25f};
  float* dx;
  unsigned* dout;
  hipMalloc(&dx, sizeof(xs));
  hipMalloc(&dout, n * 6 * 4);
  hipMemcpy(dx, xs, sizeof(xs), hipMemcpyHostToDevice);
  for (float s : scales) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dx, n, s, dout);
    unsigned h[16 * 6];
    hipMemcpy(h, dout, n * 6 * 4, hipMemcpyDeviceToHost);
    printf("scale %g\n", s);
    for (int i = 0; i < n; ++i) {
      float dot, ref;
      memcpy(&dot, &h[i * 6 + 4], 4);
      memcpy(&ref, &h[i * 6 + 5], 4);
      printf("  x=(%g,%g) scalef_bf16=%04x scalef_f32=%04x hi_bf16(old=lo)=%08x hi_f32(old=lo)=%08x dot2=%g ref=%g\n", xs[i], xs[(i + 1) % n],
             h[i * 6], h[i * 6 + 1], h[i * 6 + 2], h[i * 6 + 3], dot, ref);
    }
  }
  hipFree(dx);
  hipFree(dout);
  return 0;
}
