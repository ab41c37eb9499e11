// Fused (flash-style) multi-head attention for ViT on MI355X MFMA, bf16 in /
// fp32 softmax, head dim 64, non-causal, any sequence length (ViT-B/16: 197).
//
// Layout: Q, K, V are read in place from the qkv projection output
// [B, T, 3, H, 64] (row stride ld elements), O is written as [B, T, H*64]
// (the proj GEMM's input, no transpose pass), gradients dQ/dK/dV are written
// into a [B, T, 3, H, 64] buffer (the qkv GEMM's output gradient).
//
// Forward, one workgroup = 64 queries of one (b, h), one wave = 16 queries:
//   S^T = K Q^T with mfma_f32_16x16x32_bf16 (K rows = A operand, Q = B operand)
//   puts 4 keys x 1 query in every lane (query = lane & 15), so the running
//   row max / sum reduce over the 4 lanes {l, l^16, l^32, l^48} only; the
//   exponentiated probabilities are ALREADY the B operand of O^T = V^T P^T
//   (k index permuted consistently on both operands), and V^T comes from the
//   hardware-transposing LDS read ds_read_b64_tr_b16. The O^T accumulator has
//   the same query-per-lane layout as the softmax state: rescales need no
//   cross-lane traffic.
// Backward: dK/dV kernel (one workgroup per 64 keys, 16 keys per wave, loops
// over all query tiles) and a dQ kernel (one workgroup per 64 queries) -- the
// probabilities are recomputed from Q, K and the saved log-sum-exp, no atomics.
#include "pdt_common.h"
#include <stdlib.h>

namespace {

constexpr int D = 64;     // head dim
constexpr int TILE = 64;  // keys (or queries) per LDS tile

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// [64 rows][64 bf16] tile, 128-B rows. Two images:
//  * row image (ds_read_b128 of 8 contiguous d): chunk XOR ((row >> 1) & 7)
//  * transposed image (ds_read_b64_tr_b16): 32-B segment XOR seg_swz(row)
__device__ __forceinline__ int row_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int seg_swz(int row) { return ((row >> 1) & 1) | ((row >> 2) & 2); }
__device__ __forceinline__ int tr_off(int row, int byte_in_row) {
  int seg = byte_in_row >> 5;
  return row * 128 + ((seg ^ seg_swz(row)) << 5) + (byte_in_row & 31);
}

// stage a [64][64] bf16 tile (rows r0.., valid rows < nvalid, zero otherwise) into LDS
template <bool TR>
__device__ __forceinline__ void stage_tile(char* lds, const u16* src, long ld, int r0, int nvalid, int tid) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {  // 512 chunks of 16 B over 256 threads
    const int q = tid + it * 256;
    const int row = q >> 3, ch = q & 7;
    u32x4 v = {0, 0, 0, 0};
    if (r0 + row < nvalid) v = *reinterpret_cast<const u32x4*>(src + (long)(r0 + row) * ld + ch * 8);
    const int off = TR ? tr_off(row, ch * 16) : row_off(row, ch);
    *reinterpret_cast<u32x4*>(lds + off) = v;
  }
}

__device__ __forceinline__ bf16x8 ld_row_frag(const char* lds, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds + row_off(row, chunk));
}

// A/B fragment whose 8 k-elements are rows {kb0 + 0..3} and {kb1 + 0..3} (per
// 16-lane group: kb += 4*g) of column block col0..col0+15 of a transposed image.
__device__ __forceinline__ bf16x8 tr_frag2(const char* lds, int kb0, int kb1, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int cb = (col0 + 4 * p) * 2;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)(
          lds + tr_off(kb0 + 4 * g + q, cb))));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)(
          lds + tr_off(kb1 + 4 * g + q, cb))));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// reductions over lanes l, l^16, l^32, l^48 (permlane swaps, see pdt_common.h)
__device__ __forceinline__ float xor_max4(float v) { return xor32_reduce(xor16_reduce(v, MaxOp{}), MaxOp{}); }
__device__ __forceinline__ float xor_sum4(float v) { return xor32_reduce(xor16_reduce(v, AddOp{}), AddOp{}); }

__device__ __forceinline__ bf16x8 pack_p(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (__bf16)a[0]; r[1] = (__bf16)a[1]; r[2] = (__bf16)a[2]; r[3] = (__bf16)a[3];
  r[4] = (__bf16)b[0]; r[5] = (__bf16)b[1]; r[6] = (__bf16)b[2]; r[7] = (__bf16)b[3];
  return r;
}

struct AttnParams {
  const u16* qkv;   // [B, T, 3, H, 64]
  u16* out;         // [B, T, H*64]
  float* lse;       // [B*H, T]  (log2-domain of scaled scores)
  int B, T, H;
  long ld;          // row stride of qkv (3*H*64)
  long ldo;         // row stride of out (H*64)
  float c;          // softmax scale * log2(e)
};

__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE * D * 2];
  char* Ks = smem;
  char* Vs = smem + TILE * D * 2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int q0 = blockIdx.x * TILE + wave * 16;
  const u16* base = p.qkv + (long)b * p.T * p.ld + h * D;
  const u16* Qg = base;
  const u16* Kg = base + p.H * D;
  const u16* Vg = base + 2 * p.H * D;
  // Q fragments (B operand of S^T): Q[q0 + (lane&15)][32kk + 8g .. +7]
  const int qrow = q0 + (lane & 15);
  bf16x8 qf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    u32x4 v = {0, 0, 0, 0};
    if (qrow < p.T) v = *reinterpret_cast<const u32x4*>(Qg + (long)qrow * p.ld + 32 * kk + 8 * g);
    qf[kk] = __builtin_bit_cast(bf16x8, v);
  }
  float m = -INFINITY, l = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < p.T; k0 += TILE) {
    __syncthreads();
    stage_tile<false>(Ks, Kg, p.ld, k0, p.T, tid);
    stage_tile<true>(Vs, Vg, p.ld, k0, p.T, tid);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(Ks, 16 * t + (lane & 15), 4 * kk + g), qf[kk],
                                                       s[t], 0, 0, 0);
    }
    // s[t][r] = S[key = k0 + 16t + 4g + r][q = qrow]
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * t + 4 * g + r;
        float v = key < p.T ? s[t][r] * p.c : -INFINITY;
        s[t][r] = v;
        mt = fmaxf(mt, v);
      }
    mt = xor_max4(mt);
    const float mn = fmaxf(m, mt);
    const float alpha = exp2f(m - mn);  // m = -inf first: exp2(-inf) = 0
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float e = exp2f(s[t][r] - mn);
        s[t][r] = e;
        ls += e;
      }
    l = l * alpha + xor_sum4(ls);
    m = mn;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    // O^T[d][q] += sum_key V^T[d][key] P^T[key][q]  (two 32-key steps)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pf = pack_p(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_frag2(Vs, 32 * ks, 32 * ks + 16, 16 * dt, lane), pf,
                                                        o[dt], 0, 0, 0);
    }
  }
  // o[dt][r] = O^T[d = 16dt + 4g + r][q = qrow]
  if (qrow < p.T) {
    const float inv = 1.f / l;
    u16* orow = p.out + ((long)b * p.T + qrow) * p.ldo + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      uint2 w;
      w.x = pack2bf(o[dt][0] * inv, o[dt][1] * inv);
      w.y = pack2bf(o[dt][2] * inv, o[dt][3] * inv);
      *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * g) = w;
    }
    if (g == 0) p.lse[(long)bh * p.T + qrow] = m + log2f(l);
  }
}

struct AttnBwdParams {
  const u16* qkv;   // [B, T, 3, H, 64]
  const u16* dout;  // [B, T, H*64]
  const float* lse; // [B*H, T]
  const float* delta;  // [B*H, T] = rowsum(dO * O)
  u16* dqkv;        // [B, T, 3, H, 64]
  int B, T, H;
  long ld, ldo;
  float c;          // scale * log2(e)
  float scale;
};

// delta[bh][q] = sum_d dO[q][d] * O[q][d]; 8 lanes (16 B each) per (b, t, h) row
__global__ void __launch_bounds__(256) attn_delta_kernel(const u16* __restrict__ dout, const u16* __restrict__ out,
                                                         float* __restrict__ delta, int B, int T, int H, long ldo) {
  const long row = ((long)blockIdx.x * 256 + threadIdx.x) >> 3;  // over B*T*H (b, t, h)
  const int part = threadIdx.x & 7;
  const bool ok = row < (long)B * T * H;
  const long rr = ok ? row : 0;
  const int h = rr % H;
  const long bt = rr / H;
  const long off = bt * ldo + h * D + part * 8;
  float v = 0.f;
  if (ok) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(dout + off);
    const u32x4 b = *reinterpret_cast<const u32x4*>(out + off);
#pragma unroll
    for (int e = 0; e < 4; ++e) v += lo_bf(a[e]) * lo_bf(b[e]) + hi_bf(a[e]) * hi_bf(b[e]);
  }
  v = row8_sum(v);  // the 8 lanes of this row (DPP)
  if (ok && part == 0) {
    const int b = bt / T, t = bt % T;
    delta[((long)b * H + h) * T + t] = v;
  }
}

// dK, dV: one workgroup per 64 keys of one (b, h); wave = 16 keys.
// S = Q K^T with Q rows as A operand -> lane holds S[q = 16u + 4g + r][key = lane&15]
__global__ void __launch_bounds__(256) attn_bwd_dkdv_kernel(AttnBwdParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE * D * 2];
  char* Qs = smem;                    // transposed image (B operand of dK via tr reads)
  char* dOs = smem + TILE * D * 2;    // row image + tr image? -> two separate uses below
  __shared__ __attribute__((aligned(16))) char dOt[TILE * D * 2];
  __shared__ __attribute__((aligned(16))) char Qr[TILE * D * 2];
  __shared__ float lse_s[TILE], dl_s[TILE];  // per-query softmax stats of the current q tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int kbase = blockIdx.x * TILE + wave * 16;
  const int key = kbase + (lane & 15);
  const u16* base = p.qkv + (long)b * p.T * p.ld + h * D;
  const u16* Qg = base;
  const u16* Kg = base + p.H * D;
  const u16* Vg = base + 2 * p.H * D;
  const u16* dOg = p.dout + (long)b * p.T * p.ldo + h * D;
  // K, V fragments as B operands (k = d): K[key][8g + j + 32kk]
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    u32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
    if (key < p.T) {
      a = *reinterpret_cast<const u32x4*>(Kg + (long)key * p.ld + 32 * kk + 8 * g);
      c = *reinterpret_cast<const u32x4*>(Vg + (long)key * p.ld + 32 * kk + 8 * g);
    }
    kf[kk] = __builtin_bit_cast(bf16x8, a);
    vf[kk] = __builtin_bit_cast(bf16x8, c);
  }
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* lse = p.lse + (long)bh * p.T;
  const float* dl = p.delta + (long)bh * p.T;

  for (int q0 = 0; q0 < p.T; q0 += TILE) {
    __syncthreads();
    stage_tile<false>(Qr, Qg, p.ld, q0, p.T, tid);     // rows: A operand of S
    stage_tile<true>(Qs, Qg, p.ld, q0, p.T, tid);      // transposed: B operand of dK
    stage_tile<false>(dOs, dOg, p.ldo, q0, p.T, tid);  // rows: A operand of dP
    stage_tile<true>(dOt, dOg, p.ldo, q0, p.T, tid);   // transposed: B operand of dV
    if (tid < TILE) {
      const int q = q0 + tid;
      lse_s[tid] = q < p.T ? lse[q] : 0.f;
      dl_s[tid] = q < p.T ? dl[q] : 0.f;
    }
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s[u] = dp[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        s[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(Qr, 16 * u + (lane & 15), 4 * kk + g), kf[kk],
                                                       s[u], 0, 0, 0);
        dp[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(dOs, 16 * u + (lane & 15), 4 * kk + g),
                                                        vf[kk], dp[u], 0, 0, 0);
      }
    }
    // s[u][r] = S[q = q0 + 16u + 4g + r][key], same for dp
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * u + 4 * g + r;
        float pr = 0.f, ds = 0.f;
        if (q0 + ql < p.T && key < p.T) {
          pr = exp2f(s[u][r] * p.c - lse_s[ql]);
          ds = pr * (dp[u][r] - dl_s[ql]);
        }
        s[u][r] = pr;
        dp[u][r] = ds;
      }
    // dV^T[d][key] += dO^T[d][q] P[q][key] ; dK^T[d][key] += Q^T[d][q] dS[q][key]
    // A operand = transposed dO / Q tile (rows d, k = q permuted), B = P / dS (k = q, col = key)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pf = pack_p(s[2 * ks], s[2 * ks + 1]);
      const bf16x8 sf = pack_p(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_frag2(dOt, 32 * ks, 32 * ks + 16, 16 * dt, lane), pf,
                                                         dv[dt], 0, 0, 0);
        dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_frag2(Qs, 32 * ks, 32 * ks + 16, 16 * dt, lane), sf,
                                                         dk[dt], 0, 0, 0);
      }
    }
  }
  // dk[dt][r] = dK^T[d = 16dt + 4g + r][key]
  if (key < p.T) {
    u16* drow = p.dqkv + ((long)b * p.T + key) * p.ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      uint2 wk, wv;
      wk.x = pack2bf(dk[dt][0] * p.scale, dk[dt][1] * p.scale);
      wk.y = pack2bf(dk[dt][2] * p.scale, dk[dt][3] * p.scale);
      wv.x = pack2bf(dv[dt][0], dv[dt][1]);
      wv.y = pack2bf(dv[dt][2], dv[dt][3]);
      *reinterpret_cast<uint2*>(drow + p.H * D + 16 * dt + 4 * g) = wk;
      *reinterpret_cast<uint2*>(drow + 2 * p.H * D + 16 * dt + 4 * g) = wv;
    }
  }
}

// dQ: one workgroup per 64 queries; wave = 16 queries; S^T orientation (as forward).
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(AttnBwdParams p) {
  __shared__ __attribute__((aligned(16))) char smem[3 * TILE * D * 2];
  char* Kr = smem;                    // row image (A operand of S^T)
  char* Kt = smem + TILE * D * 2;     // transposed (A operand of dQ^T)
  char* Vr = smem + 2 * TILE * D * 2; // row image (A operand of dP^T)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int qrow = blockIdx.x * TILE + wave * 16 + (lane & 15);
  const u16* base = p.qkv + (long)b * p.T * p.ld + h * D;
  const u16* Qg = base;
  const u16* Kg = base + p.H * D;
  const u16* Vg = base + 2 * p.H * D;
  const u16* dOg = p.dout + (long)b * p.T * p.ldo + h * D;
  bf16x8 qf[2], of[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    u32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
    if (qrow < p.T) {
      a = *reinterpret_cast<const u32x4*>(Qg + (long)qrow * p.ld + 32 * kk + 8 * g);
      c = *reinterpret_cast<const u32x4*>(dOg + (long)qrow * p.ldo + 32 * kk + 8 * g);
    }
    qf[kk] = __builtin_bit_cast(bf16x8, a);
    of[kk] = __builtin_bit_cast(bf16x8, c);
  }
  const float lq = qrow < p.T ? p.lse[(long)bh * p.T + qrow] : 0.f;
  const float dq_delta = qrow < p.T ? p.delta[(long)bh * p.T + qrow] : 0.f;
  f32x4 dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < p.T; k0 += TILE) {
    __syncthreads();
    stage_tile<false>(Kr, Kg, p.ld, k0, p.T, tid);
    stage_tile<true>(Kt, Kg, p.ld, k0, p.T, tid);
    stage_tile<false>(Vr, Vg, p.ld, k0, p.T, tid);
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(Kr, 16 * t + (lane & 15), 4 * kk + g), qf[kk],
                                                       s[t], 0, 0, 0);
        dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(Vr, 16 * t + (lane & 15), 4 * kk + g), of[kk],
                                                        dp[t], 0, 0, 0);
      }
    }
    // s[t][r] = S[key = k0 + 16t + 4g + r][q = qrow]
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + 16 * t + 4 * g + r;
        float ds = 0.f;
        if (k < p.T && qrow < p.T) {
          float pr = exp2f(s[t][r] * p.c - lq);
          ds = pr * (dp[t][r] - dq_delta);
        }
        s[t][r] = ds;
      }
    // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 sf = pack_p(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_frag2(Kt, 32 * ks, 32 * ks + 16, 16 * dt, lane), sf,
                                                         dq[dt], 0, 0, 0);
    }
  }
  if (qrow < p.T) {
    u16* drow = p.dqkv + ((long)b * p.T + qrow) * p.ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      uint2 w;
      w.x = pack2bf(dq[dt][0] * p.scale, dq[dt][1] * p.scale);
      w.y = pack2bf(dq[dt][2] * p.scale, dq[dt][3] * p.scale);
      *reinterpret_cast<uint2*>(drow + 16 * dt + 4 * g) = w;
    }
  }
}

// ============================================================================
// Whole-sequence kernels (T <= 16*NKT <= 256, e.g. ViT's 197 tokens): one
// workgroup per (b, h) stages the ENTIRE K/V (forward), Q/dO (dK/dV) or K/V
// (dQ) of the head into LDS once, then every wave loops over its 16-row
// subtiles with no further barriers -- the tiled kernels above pay a
// global->LDS round trip and two barriers per 64-row tile for 16 MFMAs.
// The softmax of a 16-query subtile is taken over all keys at once.
// ============================================================================

// stage rows [0, 16*NKT) of a head (zero beyond T) as a row or transposed image
template <bool TR, int NKT, int NTH>
__device__ __forceinline__ void stage_seq(char* lds, const u16* src, long ld, int T, int tid) {
  constexpr int CH = NKT * 16 * 8;  // 16-B chunks
#pragma unroll
  for (int it = 0; it < (CH + NTH - 1) / NTH; ++it) {
    const int q = tid + it * NTH;
    if (q < CH) {
      const int row = q >> 3, ch = q & 7;
      u32x4 v = {0, 0, 0, 0};
      if (row < T) v = *reinterpret_cast<const u32x4*>(src + (long)row * ld + ch * 8);
      *reinterpret_cast<u32x4*>(lds + (TR ? tr_off(row, ch * 16) : row_off(row, ch))) = v;
    }
  }
}

// Per-lane LDS offsets. A 16-row subtile's row-image fragment (rows 16t + (lane&15),
// chunk 4kk + g) and a transposed-image fragment pair (rows 32x + 4g + q and
// +16, column block 16dt) are a lane constant plus an immediate: the XOR
// swizzles only see bits of (lane&15) / (g, q) -- so no per-read address math.
__device__ __forceinline__ int row_lane_off(int lane, int kk) {
  const int l = lane & 15, g = lane >> 4;
  return l * 128 + (((4 * kk + g) ^ ((l >> 1) & 7)) << 4);
}
__device__ __forceinline__ int tr_lane_off(int lane, int dt) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int sw = ((q >> 1) & 1) | (((g >> 1) & 1) << 1);  // seg_swz(32x + 16h + 4g + q)
  return (4 * g + q) * 128 + ((dt ^ sw) << 5) + 8 * pp;
}
// The same transposed-read fragment taken from a ROW image (row_off swizzle) instead of
// a separate transposed image: the backward kernels then stage each matrix once
// (half the LDS -> two workgroups per CU). Byte column 32dt + 8pp of row 4g + q sits in
// 16-B chunk 2dt + (pp >> 1), swizzled by ((row >> 1) & 7) -- bits of (g, q) only, and
// unchanged by the +16 / +32x row offsets frag_tr adds.
__device__ __forceinline__ int tr_row_lane_off(int lane, int dt) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int row = 4 * g + q;
  return row * 128 + (((2 * dt + (pp >> 1)) ^ ((row >> 1) & 7)) << 4) + 8 * (pp & 1);
}
__device__ __forceinline__ bf16x8 frag_row(const char* img, int off, int t) {
  return *reinterpret_cast<const bf16x8*>(img + off + t * 2048);
}
__device__ __forceinline__ bf16x8 frag_tr(const char* img, int off, int x) {
  const char* a = img + off + x * 4096;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)a));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)(a + 2048)));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// forward: NT = number of 16-key subtiles (exact: ceil(T/16)); keys >= T only
// occur in subtile NT-1, so only that one is masked
template <int NT>
__global__ void __launch_bounds__(256) attn_fwd_seq_kernel(AttnParams p) {
  constexpr int NE = (NT + 1) & ~1;  // staged subtiles (even: 32-key PV steps)
  __shared__ __attribute__((aligned(16))) char smem[2 * NE * 16 * 128];
  char* Ks = smem;
  char* Vs = smem + NE * 16 * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const u16* base = p.qkv + (long)b * p.T * p.ld + h * D;
  stage_seq<false, NE, 256>(Ks, base + p.H * D, p.ld, p.T, tid);
  stage_seq<true, NE, 256>(Vs, base + 2 * p.H * D, p.ld, p.T, tid);
  const int r0 = row_lane_off(lane, 0), r1 = row_lane_off(lane, 1);
  int to[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) to[dt] = tr_lane_off(lane, dt);
  const int klast = 16 * (NT - 1) + 4 * g;  // first key of this lane in the last subtile
  // Q fragments of this wave's first subtile are fetched while K/V stage; each
  // iteration prefetches the next subtile's before computing the current one
  auto load_q = [&](int qs, u32x4* v) {
    const int qrow = qs * 16 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v[kk] = u32x4{0, 0, 0, 0};
      if (qs < NT && qrow < p.T) v[kk] = *reinterpret_cast<const u32x4*>(base + (long)qrow * p.ld + 32 * kk + 8 * g);
    }
  };
  u32x4 qn[2];
  load_q(wave, qn);
  __syncthreads();
  for (int qs = wave; qs < NT; qs += 4) {
    const int qrow = qs * 16 + (lane & 15);
    bf16x8 qf[2];
    qf[0] = __builtin_bit_cast(bf16x8, qn[0]);
    qf[1] = __builtin_bit_cast(bf16x8, qn[1]);
    load_q(qs + 4, qn);
    f32x4 s[NE];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Ks, r0, t), qf[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Ks, r1, t), qf[1], s[t], 0, 0, 0);
    }
    if (NE > NT) s[NE - 1] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (klast + r >= p.T) s[NT - 1][r] = -INFINITY;
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NT; ++t) m = fmaxf(m, fmaxf(fmaxf(s[t][0], s[t][1]), fmaxf(s[t][2], s[t][3])));
    m = xor_max4(m);
    const float cm = m * p.c;
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < NE; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = fast_exp2(fmaf(s[t][r], p.c, -cm));
        s[t][r] = e;
        l += e;
      }
    l = xor_sum4(l);
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NE / 2; ++ks) {
      const bf16x8 pf = pack_p(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(Vs, to[dt], ks), pf, o[dt], 0, 0, 0);
    }
    if (qrow < p.T) {
      const float inv = 1.f / l;
      u16* orow = p.out + ((long)b * p.T + qrow) * p.ldo + h * D;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        uint2 w;
        w.x = pack2bf(o[dt][0] * inv, o[dt][1] * inv);
        w.y = pack2bf(o[dt][2] * inv, o[dt][3] * inv);
        *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * g) = w;
      }
      if (g == 0) p.lse[(long)bh * p.T + qrow] = cm + log2f(l);
    }
  }
}

// delta[q] = sum_d dO[q][d] O[q][d] for the 16-query subtile of this lane group:
// each of the 4 lanes sharing a query sums 16 of the 64 dims
__device__ __forceinline__ float row_delta(const u16* dOrow, const u16* Orow, int g) {
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(dOrow + 16 * g + 8 * c);
    const u32x4 o = *reinterpret_cast<const u32x4*>(Orow + 16 * g + 8 * c);
#pragma unroll
    for (int e = 0; e < 4; ++e) v += lo_bf(a[e]) * lo_bf(o[e]) + hi_bf(a[e]) * hi_bf(o[e]);
  }
  return xor_sum4(v);
}

struct AttnSeqBwdParams {
  const u16* qkv;
  const u16* out;   // forward output O [B, T, H*64]
  const u16* dout;  // [B, T, H*64]
  const float* lse; // [B*H, T]
  u16* dqkv;
  int B, T, H;
  long ld, ldo;
  float c, scale;
  // optional: e5m2 codes of d(qkv) (bf16-rounded, same layout) for the qkv projection's fp8
  // data / weight gradients, delayed scale q8_meta[0]; per-workgroup max |d(qkv)| ->
  // q8_part[bh] (dK/dV kernel) and q8_part[B*H + bh] (dQ kernel)
  uint8_t* q8;
  const float* q8_meta;
  float* q8_part;
};

// 4 bf16 (packed) -> 4 e5m2 codes with scale s (saturating), updating |max|
__device__ __forceinline__ uint32_t q8_e5m2(uint2 w, float s, float& mx) {
  const float f0 = lo_bf(w.x), f1 = hi_bf(w.x), f2 = lo_bf(w.y), f3 = hi_bf(w.y);
  mx = fmaxf(mx, fmaxf(fmaxf(fabsf(f0), fabsf(f1)), fmaxf(fabsf(f2), fabsf(f3))));
  return pdt_cvt4_f8<1>(f0 * s, f1 * s, f2 * s, f3 * s);
}

// block max of a per-thread value -> part[slot] (all threads of the block call this)
__device__ __forceinline__ void q8_block_max(float mx, float* part, long slot, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  mx = warp_max(mx);
  __syncthreads();
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = red[0];
    for (int w = 1; w < nw; ++w) m = fmaxf(m, red[w]);
    part[slot] = m;
  }
}

// dK, dV: one workgroup (8 waves) per (b, h); wave w owns key subtiles w, w+8.
// Per query subtile u: S = Q K^T (q on the register axis, key on the lane),
// P = exp2(c S - lse), dS = P (dP - delta); dV^T += dO^T P, dK^T += Q^T dS.
// SINGLE: Q and dO staged once (row images serve the transposed reads too): 2 images
// instead of 4 -> 2 workgroups per CU
template <int NT, bool SINGLE>
__global__ void __launch_bounds__(512) attn_bwd_dkdv_seq_kernel(AttnSeqBwdParams p) {
  constexpr int NE = (NT + 1) & ~1;
  constexpr int IMG = NE * 16 * 128;
  constexpr int NIMG = SINGLE ? 2 : 4;
  __shared__ __attribute__((aligned(16))) char smem[NIMG * IMG + 2 * NE * 16 * 4];
  char* Qr = smem;
  char* dOr = smem + IMG;
  char* Qt = SINGLE ? Qr : smem + 2 * IMG;
  char* dOt = SINGLE ? dOr : smem + 3 * IMG;
  float* lse_s = reinterpret_cast<float*>(smem + NIMG * IMG);  // pre-negated: -lse
  float* dl_s = lse_s + NE * 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const u16* base = p.qkv + (long)b * p.T * p.ld + h * D;
  const u16* dOg = p.dout + (long)b * p.T * p.ldo + h * D;
  const u16* Og = p.out + (long)b * p.T * p.ldo + h * D;
  stage_seq<false, NE, 512>(Qr, base, p.ld, p.T, tid);
  stage_seq<false, NE, 512>(dOr, dOg, p.ldo, p.T, tid);
  if (!SINGLE) {
    stage_seq<true, NE, 512>(Qt, base, p.ld, p.T, tid);
    stage_seq<true, NE, 512>(dOt, dOg, p.ldo, p.T, tid);
  }
  // per-query stats: -lse (so P = exp2(fma(S, c, -lse))) and delta (8 lanes per query);
  // rows >= T get -inf -> P = 0
  for (int i = tid; i < NE * 16 * 8; i += 512) {
    const int q = i >> 3, part = i & 7;
    float v = 0.f;
    if (q < p.T) {
      const u32x4 a = *reinterpret_cast<const u32x4*>(dOg + (long)q * p.ldo + part * 8);
      const u32x4 o = *reinterpret_cast<const u32x4*>(Og + (long)q * p.ldo + part * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) v += lo_bf(a[e]) * lo_bf(o[e]) + hi_bf(a[e]) * hi_bf(o[e]);
    }
    v = row8_sum(v);  // the 8 lanes of this query (DPP)
    if (part == 0) {
      dl_s[q] = v;
      lse_s[q] = q < p.T ? -p.lse[(long)bh * p.T + q] : -INFINITY;
    }
  }
  const int r0 = row_lane_off(lane, 0), r1 = row_lane_off(lane, 1);
  int to[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) to[dt] = SINGLE ? tr_row_lane_off(lane, dt) : tr_lane_off(lane, dt);
  __shared__ float q8red[8];
  float q8max = 0.f;
  __syncthreads();
  for (int kt = wave; kt < NT; kt += 8) {
    const int key = kt * 16 + (lane & 15);
    const bool kok = key < p.T;
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
      if (kok) {
        a = *reinterpret_cast<const u32x4*>(base + p.H * D + (long)key * p.ld + 32 * kk + 8 * g);
        c = *reinterpret_cast<const u32x4*>(base + 2 * p.H * D + (long)key * p.ld + 32 * kk + 8 * g);
      }
      kf[kk] = __builtin_bit_cast(bf16x8, a);
      vf[kk] = __builtin_bit_cast(bf16x8, c);
    }
    const float kmask = kok ? 1.f : 0.f;  // padded keys: P = dS = 0 (their K/V rows are zero)
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int qp = 0; qp < NE / 2; ++qp) {
      f32x4 pp[2], dsp[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int u = 2 * qp + h2;
        f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dpv = f32x4{0.f, 0.f, 0.f, 0.f};
        if (u < NT) {
          sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Qr, r0, u), kf[0], sv, 0, 0, 0);
          sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Qr, r1, u), kf[1], sv, 0, 0, 0);
          dpv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(dOr, r0, u), vf[0], dpv, 0, 0, 0);
          dpv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(dOr, r1, u), vf[1], dpv, 0, 0, 0);
        }
        // sv[r] = S[q = 16u + 4g + r][key]; stats of those 4 queries in one 16-B LDS read each
        const f32x4 nl = *reinterpret_cast<const f32x4*>(lse_s + 16 * u + 4 * g);
        const f32x4 dl = *reinterpret_cast<const f32x4*>(dl_s + 16 * u + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pr = fast_exp2(fmaf(sv[r], p.c, nl[r])) * kmask;
          sv[r] = pr;
          dpv[r] = pr * (dpv[r] - dl[r]);
        }
        pp[h2] = sv;
        dsp[h2] = dpv;
      }
      const bf16x8 pf = pack_p(pp[0], pp[1]);
      const bf16x8 sf = pack_p(dsp[0], dsp[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(dOt, to[dt], qp), pf, dv[dt], 0, 0, 0);
        dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(Qt, to[dt], qp), sf, dk[dt], 0, 0, 0);
      }
    }
    if (kok) {
      const long roff = ((long)b * p.T + key) * p.ld + h * D;
      u16* drow = p.dqkv + roff;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        uint2 wk, wv;
        wk.x = pack2bf(dk[dt][0] * p.scale, dk[dt][1] * p.scale);
        wk.y = pack2bf(dk[dt][2] * p.scale, dk[dt][3] * p.scale);
        wv.x = pack2bf(dv[dt][0], dv[dt][1]);
        wv.y = pack2bf(dv[dt][2], dv[dt][3]);
        *reinterpret_cast<uint2*>(drow + p.H * D + 16 * dt + 4 * g) = wk;
        *reinterpret_cast<uint2*>(drow + 2 * p.H * D + 16 * dt + 4 * g) = wv;
        if (p.q8 != nullptr) {
          const float s8 = p.q8_meta[0];
          *reinterpret_cast<uint32_t*>(p.q8 + roff + p.H * D + 16 * dt + 4 * g) = q8_e5m2(wk, s8, q8max);
          *reinterpret_cast<uint32_t*>(p.q8 + roff + 2 * p.H * D + 16 * dt + 4 * g) = q8_e5m2(wv, s8, q8max);
        }
      }
    }
  }
  if (p.q8 != nullptr) q8_block_max(q8max, p.q8_part, bh, q8red);
}

// dQ: one workgroup (8 waves) per (b, h); wave w owns query subtiles w, w+8.
template <int NT, bool SINGLE>
__global__ void __launch_bounds__(512) attn_bwd_dq_seq_kernel(AttnSeqBwdParams p) {
  constexpr int NE = (NT + 1) & ~1;
  constexpr int IMG = NE * 16 * 128;
  __shared__ __attribute__((aligned(16))) char smem[(SINGLE ? 2 : 3) * IMG];
  char* Kr = smem;
  char* Vr = smem + IMG;
  char* Kt = SINGLE ? Kr : smem + 2 * IMG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const u16* base = p.qkv + (long)b * p.T * p.ld + h * D;
  const u16* dOg = p.dout + (long)b * p.T * p.ldo + h * D;
  const u16* Og = p.out + (long)b * p.T * p.ldo + h * D;
  stage_seq<false, NE, 512>(Kr, base + p.H * D, p.ld, p.T, tid);
  stage_seq<false, NE, 512>(Vr, base + 2 * p.H * D, p.ld, p.T, tid);
  if (!SINGLE) stage_seq<true, NE, 512>(Kt, base + p.H * D, p.ld, p.T, tid);
  const int r0 = row_lane_off(lane, 0), r1 = row_lane_off(lane, 1);
  int to[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) to[dt] = SINGLE ? tr_row_lane_off(lane, dt) : tr_lane_off(lane, dt);
  const int klast = 16 * (NT - 1) + 4 * g;
  __shared__ float q8red[8];
  float q8max = 0.f;
  __syncthreads();
  for (int qs = wave; qs < NT; qs += 8) {
    const int qrow = qs * 16 + (lane & 15);
    const bool qok = qrow < p.T;
    const int qr = qok ? qrow : 0;
    bf16x8 qf[2], of[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
      if (qok) {
        a = *reinterpret_cast<const u32x4*>(base + (long)qrow * p.ld + 32 * kk + 8 * g);
        c = *reinterpret_cast<const u32x4*>(dOg + (long)qrow * p.ldo + 32 * kk + 8 * g);
      }
      qf[kk] = __builtin_bit_cast(bf16x8, a);
      of[kk] = __builtin_bit_cast(bf16x8, c);
    }
    const float delta = qok ? row_delta(dOg + (long)qr * p.ldo, Og + (long)qr * p.ldo, g) : 0.f;
    const float nlq = qok ? -p.lse[(long)bh * p.T + qrow] : -INFINITY;
    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int kp = 0; kp < NE / 2; ++kp) {
      f32x4 dsp[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int t = 2 * kp + h2;
        f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dpv = f32x4{0.f, 0.f, 0.f, 0.f};
        if (t < NT) {
          sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Kr, r0, t), qf[0], sv, 0, 0, 0);
          sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Kr, r1, t), qf[1], sv, 0, 0, 0);
          dpv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Vr, r0, t), of[0], dpv, 0, 0, 0);
          dpv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Vr, r1, t), of[1], dpv, 0, 0, 0);
        }
        // sv[r] = S[key = 16t + 4g + r][q = qrow]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float ds = fast_exp2(fmaf(sv[r], p.c, nlq)) * (dpv[r] - delta);
          if (t >= NT - 1 && (t >= NT || klast + r >= p.T)) ds = 0.f;  // padded keys (last subtile only)
          sv[r] = ds;
        }
        dsp[h2] = sv;
      }
      const bf16x8 sf = pack_p(dsp[0], dsp[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(Kt, to[dt], kp), sf, dq[dt], 0, 0, 0);
    }
    if (qok) {
      const long roff = ((long)b * p.T + qrow) * p.ld + h * D;
      u16* drow = p.dqkv + roff;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        uint2 w;
        w.x = pack2bf(dq[dt][0] * p.scale, dq[dt][1] * p.scale);
        w.y = pack2bf(dq[dt][2] * p.scale, dq[dt][3] * p.scale);
        *reinterpret_cast<uint2*>(drow + 16 * dt + 4 * g) = w;
        if (p.q8 != nullptr)
          *reinterpret_cast<uint32_t*>(p.q8 + roff + 16 * dt + 4 * g) = q8_e5m2(w, p.q8_meta[0], q8max);
      }
    }
  }
  if (p.q8 != nullptr) q8_block_max(q8max, p.q8_part, (long)p.B * p.H + bh, q8red);
}

}  // namespace

// whole-sequence kernel instantiation for T <= 256 (16-row subtiles)
static int seq_nkt(int T) {
  const int n = (T + 15) / 16;
  return n <= 16 ? n : 0;
}

#define PDT_SEQ_SWITCH(N, CALL) \
  switch (N) {                  \
    case 1: CALL(1); break;     \
    case 2: CALL(2); break;     \
    case 3: CALL(3); break;     \
    case 4: CALL(4); break;     \
    case 5: CALL(5); break;     \
    case 6: CALL(6); break;     \
    case 7: CALL(7); break;     \
    case 8: CALL(8); break;     \
    case 9: CALL(9); break;     \
    case 10: CALL(10); break;   \
    case 11: CALL(11); break;   \
    case 12: CALL(12); break;   \
    case 13: CALL(13); break;   \
    case 14: CALL(14); break;   \
    case 15: CALL(15); break;   \
    default: CALL(16); break;   \
  }

// PDT_ATTN_BWD_SINGLE=0: the two-image (row + transposed) backward staging, for A/B runs
static int g_attn_bwd_single = -1;
static int attn_bwd_single() {
  if (g_attn_bwd_single < 0) {
    const char* e = getenv("PDT_ATTN_BWD_SINGLE");
    g_attn_bwd_single = (e && e[0] == '0') ? 0 : 1;
  }
  return g_attn_bwd_single;
}
PDT_API int pdt_attn_set_bwd_single(int on) {
  g_attn_bwd_single = on ? 1 : 0;
  return 0;
}

static int attn_seq_disabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PDT_ATTN_TILED");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v;
}

PDT_API int pdt_attn_fwd(const void* qkv, void* out, float* lse, int B, int T, int H, float scale, hipStream_t st) {
  AttnParams p;
  p.qkv = (const u16*)qkv;
  p.out = (u16*)out;
  p.lse = lse;
  p.B = B; p.T = T; p.H = H;
  p.ld = 3L * H * D;
  p.ldo = (long)H * D;
  p.c = scale * 1.4426950408889634f;
  const int nkt = attn_seq_disabled() ? 0 : seq_nkt(T);
  if (nkt) {
    dim3 g(B * H);
#define FWD_SEQ(N) hipLaunchKernelGGL(attn_fwd_seq_kernel<N>, g, dim3(256), 0, st, p)
    PDT_SEQ_SWITCH(nkt, FWD_SEQ)
#undef FWD_SEQ
    PDT_RETURN_LAUNCH();
  }
  dim3 grid((T + TILE - 1) / TILE, B * H);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, st, p);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_fp8_meta_roll_partial(float* meta, const float* partial, int nblk, int fmt, float* dq_out,
                                      hipStream_t st);

static int attn_bwd_impl(const void* qkv, const void* out, const void* dout, const float* lse, float* delta,
                         void* dqkv, int B, int T, int H, float scale, void* q8, float* q8_meta, float* q8_part,
                         float* q8_dq, hipStream_t st);

PDT_API int pdt_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, float* delta,
                         void* dqkv, int B, int T, int H, float scale, hipStream_t st) {
  return attn_bwd_impl(qkv, out, dout, lse, delta, dqkv, B, T, H, scale, nullptr, nullptr, nullptr, nullptr, st);
}

// pdt_attn_bwd that also writes the e5m2 codes of d(qkv) for the qkv projection's fp8
// gradient GEMMs (delayed scale q8_meta[0]), rolls that history (q8_part: 2*B*H floats) and
// writes the codes' dequant factor to q8_dq. Whole-sequence kernels only (T <= 256): -1 else.
PDT_API int pdt_attn_bwd_q8(const void* qkv, const void* out, const void* dout, const float* lse, float* delta,
                            void* dqkv, int B, int T, int H, float scale, void* q8, float* q8_meta, float* q8_part,
                            float* q8_dq, hipStream_t st) {
  if (!q8 || !q8_meta || !q8_part || attn_seq_disabled() || !seq_nkt(T)) return -1;
  return attn_bwd_impl(qkv, out, dout, lse, delta, dqkv, B, T, H, scale, q8, q8_meta, q8_part, q8_dq, st);
}

static int attn_bwd_impl(const void* qkv, const void* out, const void* dout, const float* lse, float* delta,
                         void* dqkv, int B, int T, int H, float scale, void* q8, float* q8_meta, float* q8_part,
                         float* q8_dq, hipStream_t st) {
  const int nkt = attn_seq_disabled() ? 0 : seq_nkt(T);
  if (nkt) {
    AttnSeqBwdParams q;
    q.q8 = (uint8_t*)q8;
    q.q8_meta = q8_meta;
    q.q8_part = q8_part;
    q.qkv = (const u16*)qkv;
    q.out = (const u16*)out;
    q.dout = (const u16*)dout;
    q.lse = lse;
    q.dqkv = (u16*)dqkv;
    q.B = B; q.T = T; q.H = H;
    q.ld = 3L * H * D;
    q.ldo = (long)H * D;
    q.c = scale * 1.4426950408889634f;
    q.scale = scale;
    dim3 g(B * H);
#define SEQ_BWD(N)                                                                     \
  if (attn_bwd_single()) {                                                             \
    hipLaunchKernelGGL((attn_bwd_dkdv_seq_kernel<N, true>), g, dim3(512), 0, st, q);   \
    hipLaunchKernelGGL((attn_bwd_dq_seq_kernel<N, true>), g, dim3(512), 0, st, q);     \
  } else {                                                                             \
    hipLaunchKernelGGL((attn_bwd_dkdv_seq_kernel<N, false>), g, dim3(512), 0, st, q);  \
    hipLaunchKernelGGL((attn_bwd_dq_seq_kernel<N, false>), g, dim3(512), 0, st, q);    \
  }
    PDT_SEQ_SWITCH(nkt, SEQ_BWD)
#undef SEQ_BWD
    if (q8 == nullptr) PDT_RETURN_LAUNCH();
    const int e = (int)hipGetLastError();
    if (e) return e;
    return pdt_fp8_meta_roll_partial(q8_meta, q8_part, 2 * B * H, 1, q8_dq, st);
  }
  const long rows = (long)B * T * H;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, st, (const u16*)dout,
                     (const u16*)out, delta, B, T, H, (long)H * D);
  int e = (int)hipGetLastError();
  if (e) return e;
  AttnBwdParams p;
  p.qkv = (const u16*)qkv;
  p.dout = (const u16*)dout;
  p.lse = lse;
  p.delta = delta;
  p.dqkv = (u16*)dqkv;
  p.B = B; p.T = T; p.H = H;
  p.ld = 3L * H * D;
  p.ldo = (long)H * D;
  p.c = scale * 1.4426950408889634f;
  p.scale = scale;
  dim3 grid((T + TILE - 1) / TILE, B * H);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, grid, dim3(256), 0, st, p);
  e = (int)hipGetLastError();
  if (e) return e;
  hipLaunchKernelGGL(attn_bwd_dq_kernel, grid, dim3(256), 0, st, p);
  PDT_RETURN_LAUNCH();
}
