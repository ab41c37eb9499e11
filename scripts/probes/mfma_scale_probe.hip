// Probe of the per-lane E8M0 block-scale operands of v_mfma_scale_f32_32x32x64_f8f6f4
// (gfx950). A = B = all e4m3 1.0; workgroup L raises the scale of lane L alone (2^10 instead
// of 2^0) on the A operand (then on the B operand). D[m][n] = sum_k A B sa sb, so the
// entries that change show which output rows (A) / columns (B) -- and by the size of the
// change, how many of the 64 k -- lane L's scale covers. Prints one line per lane.
//   hipcc --offload-arch=gfx950 -O2 scripts/probes/mfma_scale_probe.hip -o build/mfma_scale_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// half = 1: the operand carrying the probed scale holds data (1.0) only in lanes 0..31 (zeros
// in 32..63): a lane whose raised scale still changes D then scales data held by lanes 0..31
__global__ void probe(float* out, int on_b, int half) {
  const int lane = threadIdx.x, L = blockIdx.x;
  const int one4 = 0x38383838;  // four e4m3 1.0
  const int d = (half && lane >= 32) ? 0 : one4;
  const i32x8 ones = {one4, one4, one4, one4, one4, one4, one4, one4};
  const i32x8 part = {d, d, d, d, d, d, d, d};
  const int s = lane == L ? 137 : 127;
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(on_b ? ones : part, on_b ? part : ones, c, 0, 0, 0,
                                                       on_b ? 127 : s, 0, on_b ? s : 127);
  for (int r = 0; r < 16; ++r) {
    const int m = 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3), n = lane & 31;
    out[L * 1024 + m * 32 + n] = c[r];
  }
}

int main() {
  float* d;
  if (hipMalloc(&d, 64 * 1024 * sizeof(float))) return 1;
  static float h[64 * 1024];
  for (int it = 0; it < 4; ++it) {
    const int on_b = it & 1, half = it >> 1;
    hipLaunchKernelGGL(probe, dim3(64), dim3(64), 0, 0, d, on_b, half);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost)) return 2;
    const float base = half ? 32.f : 64.f;
    printf("== scale on %s operand, data %s: lane L -> changed D entries (value)\n", on_b ? "B" : "A",
           half ? "only in lanes 0..31" : "in all lanes");
    for (int L = 0; L < 64; ++L) {
      int cnt = 0, m0 = -1, n0 = -1, m1 = -1, n1 = -1;
      float v = 0.f;
      for (int i = 0; i < 1024; ++i)
        if (h[L * 1024 + i] != base) {
          if (cnt == 0) { m0 = i / 32; n0 = i % 32; v = h[L * 1024 + i]; }
          m1 = i / 32; n1 = i % 32;
          ++cnt;
        }
      printf("lane %2d: %4d entries changed, first (m %2d, n %2d) last (m %2d, n %2d), value %g\n", L, cnt, m0, n0,
             m1, n1, v);
    }
  }
  return 0;
}
