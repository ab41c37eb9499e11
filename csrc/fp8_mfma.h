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

// gfx950 scaled converts: v_cvt_scalef32_pk_fp8_{bf16,f32} round x / sdiv to e4m3 (they DIVIDE
// by the scale operand: scripts/probes/cvt_scale_probe.hip; bit-identical to cvt(x * 2^e) for
// sdiv = 2^-e). One instruction per pair instead of unpack + multiply + convert.
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// four bf16 (two packed words) -> four e4m3 codes of x / sdiv, element order kept
__device__ __forceinline__ uint32_t e4m3x4_bf16(uint32_t w0, uint32_t w1, float sdiv) {
  s16x2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(s16x2{0, 0}, __builtin_bit_cast(bf16x2v, w0), sdiv, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, __builtin_bit_cast(bf16x2v, w1), sdiv, true);
  return __builtin_bit_cast(uint32_t, r);
}
// four floats -> four e4m3 codes of x / sdiv (in range by construction)
__device__ __forceinline__ uint32_t e4m3x4_div(float a, float b, float c, float d, float sdiv) {
  s16x2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(s16x2{0, 0}, a, b, sdiv, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, c, d, sdiv, true);
  return __builtin_bit_cast(uint32_t, r);
}
// running |x|max of packed bf16 pairs on the bits: magnitudes compare as u16 (v_pk_max_u16)
__device__ __forceinline__ uint32_t absmax_bf16x2(uint32_t m, uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, m),
                                                                __builtin_bit_cast(u16x2, w & 0x7fff7fffu)));
}
// acc + sum over the 8 bf16 of a * b (fp32 products and sums, v_dot2c_f32_bf16 x 4). The operands
// are bit-cast as WHOLE vectors and split with swizzles: hipcc 7.2 miscompiles
// __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, v[e]), ...) in an unrolled loop --
// it loads one dword and feeds element 0 to all four calls. (An inline-asm v_dot2c also works
// but hides its latency from the hazard recognizer: a following DPP read got 1 nop, not 2.)
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
__device__ __forceinline__ float dot8_bf16(const u32x4& a, const u32x4& b, float acc) {
  const bf16x8v x = __builtin_bit_cast(bf16x8v, a), y = __builtin_bit_cast(bf16x8v, b);
  acc = __builtin_amdgcn_fdot2_f32_bf16(x.s01, y.s01, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(x.s23, y.s23, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(x.s45, y.s45, acc, false);
  return __builtin_amdgcn_fdot2_f32_bf16(x.s67, y.s67, acc, false);
}
// the float value of the larger of the two magnitudes
__device__ __forceinline__ float absmax_bf16x2_value(uint32_t m) {
  const uint32_t hi = m >> 16, lo = m & 0xffffu;
  return __uint_as_float((hi > lo ? hi : lo) << 16);
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
