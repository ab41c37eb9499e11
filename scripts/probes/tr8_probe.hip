// Probe of ds_read_b64_tr_b8 lane semantics (gfx950): which (row, column) byte of the
// LDS image each lane receives, for lane addresses row = lane / 2, column = 8 * (lane % 2)
// (a 32-row x 16-byte window, row stride 64 B). Prints one line per lane.
//   hipcc --offload-arch=gfx950 -O2 scripts/probes/tr8_probe.hip -o build/tr8_probe && build/tr8_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v2i __attribute__((ext_vector_type(2)));

__global__ void probe(v2i* out_row, v2i* out_col) {
  __shared__ __attribute__((aligned(16))) unsigned char srow[64 * 64], scol[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) {
    srow[i] = (unsigned char)(i / 64);
    scol[i] = (unsigned char)(i % 64);
  }
  __syncthreads();
  const int lane = threadIdx.x;
  const int off = (lane >> 1) * 64 + (lane & 1) * 8;
  typedef v2i __attribute__((address_space(3))) * lp;
  v2i a = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lp)((__attribute__((address_space(3))) unsigned char*)(uintptr_t)(uint32_t)(uintptr_t)(srow + off)));
  v2i b = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lp)((__attribute__((address_space(3))) unsigned char*)(uintptr_t)(uint32_t)(uintptr_t)(scol + off)));
  out_row[lane] = a;
  out_col[lane] = b;
}

int main() {
  v2i *dr, *dc;
  if (hipMalloc(&dr, 64 * sizeof(v2i)) || hipMalloc(&dc, 64 * sizeof(v2i))) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dr, dc);
  v2i hr[64], hc[64];
  if (hipMemcpy(hr, dr, sizeof(hr), hipMemcpyDeviceToHost) || hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost)) return 2;
  for (int l = 0; l < 64; ++l) {
    const unsigned char* r = (const unsigned char*)&hr[l];
    const unsigned char* c = (const unsigned char*)&hc[l];
    printf("lane %2d:", l);
    for (int e = 0; e < 8; ++e) printf(" (r%2d,c%2d)", r[e], c[e]);
    printf("\n");
  }
  return 0;
}
