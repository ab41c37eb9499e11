// Precision of v_dot2c_f32_bf16 on gfx950 vs fp32 products/sum, random bf16 inputs (as the
// attention backward's delta = rowsum(dO * O) would use it).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <cstring>

__global__ void k(const uint32_t* a, const uint32_t* b, float* out, float* ref, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float acc = 0.f, r = 0.f;
  for (int e = 0; e < 32; ++e) {
    const uint32_t x = a[i * 32 + e], y = b[i * 32 + e];
    asm volatile("v_dot2c_f32_bf16 %0, %1, %2" : "+v"(acc) : "v"(x), "v"(y));
    r += __uint_as_float(x << 16) * __uint_as_float(y << 16) + __uint_as_float(x & 0xffff0000u) * __uint_as_float(y & 0xffff0000u);
  }
  out[i] = acc;
  ref[i] = r;
}

static uint32_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u >> 16; }
int main() {
  const int n = 256;
  uint32_t *ha = new uint32_t[n * 32], *hb = new uint32_t[n * 32];
  uint64_t s = 12345;
  auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return ((s >> 33) % 20000) / 10000.0f - 1.0f; };
  for (int i = 0; i < n * 32; ++i) {
    ha[i] = bf(rnd() * 3.f) | (bf(rnd() * 3.f) << 16);
    hb[i] = bf(rnd()) | (bf(rnd()) << 16);
  }
  uint32_t *da, *db; float *dout, *dref;
  hipMalloc(&da, n * 32 * 4); hipMalloc(&db, n * 32 * 4); hipMalloc(&dout, n * 4); hipMalloc(&dref, n * 4);
  hipMemcpy(da, ha, n * 32 * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, n * 32 * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, da, db, dout, dref, n);
  float ho[n], hr[n];
  hipMemcpy(ho, dout, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hr, dref, n * 4, hipMemcpyDeviceToHost);
  double maxrel = 0; int worst = 0;
  for (int i = 0; i < n; ++i) {
    const double rel = fabs(ho[i] - hr[i]) / (fabs(hr[i]) + 1e-6);
    if (rel > maxrel) { maxrel = rel; worst = i; }
  }
  printf("max rel err %g at %d: dot2 %.8g ref %.8g\n", maxrel, worst, ho[worst], hr[worst]);
  for (int i = 0; i < 8; ++i) printf("  %d: dot2 %.8g ref %.8g\n", i, ho[i], hr[i]);
  return 0;
}
