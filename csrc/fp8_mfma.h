// Shared helpers of the block-scaled fp8 MFMA attention kernels (attention_f8.hip,
// attention_bwd_f8.hip): fp8 row images, the 32x32x64 operand k layout and its tr8 reads.
//
// Operand K layout of v_mfma_scale_f32_32x32x64_f8f6f4 (probe: scripts/probes/mfma_scale_probe.hip):
// byte b of lane (row, half hh) is k = 16 hh + b for b < 16 and k = 32 + 16 hh + (b - 16)
// otherwise; lane (row, hh)'s E8M0 scale covers the k block [32 hh, 32 hh + 32).
#pragma once
#include "pdt_common.h"

namespace pdt_f8 {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// fp8 row image [rows][64 B]: 16-B chunk c of row r at chunk c ^ ((r >> 2) & 3)
__device__ __forceinline__ int k8_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// largest e with amax * 2^e <= 448 (0 for an all-zero block)
__device__ __forceinline__ int pow2_exp(float amax) {
  if (!(amax > 0.f)) return 0;
  int e = max(min((int)floorf(__log2f(448.f / amax)), 100), -100);
  if (ldexpf(amax, e) > 448.f) --e;  // (the fast log2 may round up at an exact power of two)
  return e;
}

__device__ __forceinline__ uint32_t e4m3x4(float a, float b, float c, float d) { return pdt_cvt4_f8<0>(a, b, c, d); }
// in range by construction (pow2-scaled from the block's own |max|, or 256 P): no clamp
__device__ __forceinline__ uint32_t e4m3x4_ir(float a, float b, float c, float d) {
  return pdt_cvt4_e4m3_inrange(a, b, c, d);
}

// the 32-byte A / B fragment of a row image: row `row`, bytes 32 hh .. 32 hh + 31
__device__ __forceinline__ i32x8 row_frag(const char* img, int row, int hh) {
  const u32x4 a = *reinterpret_cast<const u32x4*>(img + k8_off(row, 2 * hh));
  const u32x4 b = *reinterpret_cast<const u32x4*>(img + k8_off(row, 2 * hh + 1));
  return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}

__device__ __forceinline__ i32x2 tr8(const char* a) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32(
      (i32x2 __attribute__((address_space(3)))*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(
          uintptr_t)a));
}

// Order of the 32 rows of one tile inside a packed 32x32 accumulator operand: a lane's 16
// accumulator values of tile t (rows 8 (r >> 2) + 4 hh + (r & 3)) packed as bytes 0..15
// (tile t) / 16..31 (tile t + 1) give k -> 32 (k >> 5) + pi(k & 31) for both tiles.
__device__ __forceinline__ int pi_q(int p) { return 8 * ((p & 15) >> 2) + 4 * (p >> 4) + (p & 3); }

// the image row holding MFMA k of lane half hh's 4 tr8 reads: read r, row jj of the read
// (bytes 8 r + jj): k block r >> 1, position 16 hh + 8 (r & 1) + jj within it
template <bool PI>
__device__ __forceinline__ int kb_row(int r, int jj, int hh) {
  const int pos = 16 * hh + 8 * (r & 1) + jj;
  return 32 * (r >> 1) + (PI ? pi_q(pos) : pos);
}

// Transposed 32x32x64 operand from a row image: lane (16-lane group g, j) gets column
// 16 (g & 1) + j of the 16-byte column block `chunk`, for the 64 k rows row0 + kb_row(..)
// (4 tr8 reads of 8 rows; lane pair j >> 1 addresses one row, byte half j & 1).
template <bool PI>
__device__ __forceinline__ i32x8 tr_frag(const char* img, int row0, int chunk, int j, int hh) {
  i32x8 out;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = row0 + kb_row<PI>(r, j >> 1, hh);
    const i32x2 v = tr8(img + k8_off(row, chunk) + 8 * (j & 1));
    out[2 * r] = v[0];
    out[2 * r + 1] = v[1];
  }
  return out;
}

__device__ __forceinline__ f32x16 mfma8(const i32x8& a, const i32x8& b, const f32x16& c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

}  // namespace pdt_f8
