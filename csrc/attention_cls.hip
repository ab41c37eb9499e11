// Class-token attention: the last ViT block's attention for the ONE query the network's output
// depends on (the classifier reads only token 0 of the final block), against all T keys /
// values. Forward and backward for a packed qkv tensor [B][T][3][H][64] (bf16).
//
//   s_t = (q . k_t) / 8,  p = softmax(s),  o = sum_t p_t v_t                     (per b, h)
//   backward: dv_t = p_t do,  dp_t = do . v_t,  ds_t = p_t (dp_t - do . o),
//             dq = sum_t ds_t k_t / 8,  dk_t = ds_t q / 8     (dq of every other token = 0)
//
// One 256-thread workgroup per (b, h): thread t owns key t (T <= 256) for the dot products and
// the per-key gradient rows; the 64-wide sums over keys (o, dq) run as 64 columns x 4 key
// slices through LDS. fp32 softmax and accumulation; bf16 in and out. The work is tiny
// (B*H*T*64*4 MACs) -- what matters is that the block's other 196 query rows are never formed.
#include "pdt_common.h"

namespace {

constexpr int CT = 256;  // threads = max keys
constexpr int HD = 64;   // head dim

__device__ __forceinline__ void load_row(const u16* src, float (&r)[HD]) {
#pragma unroll
  for (int c = 0; c < HD / 8; ++c) {
    const u32x4 w = *reinterpret_cast<const u32x4*>(src + c * 8);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r[c * 8 + 2 * e] = lo_bf(w[e]);
      r[c * 8 + 2 * e + 1] = hi_bf(w[e]);
    }
  }
}

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  v = is_max ? warp_max(v) : warp_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < CT / 64; ++w) r = is_max ? fmaxf(r, red[w]) : r + red[w];
  return r;
}

// LDS layout (one array: floats): q/do [64] | p [256] | partial sums [4][64] | reduce [4]
constexpr int L_VEC = 0, L_P = HD, L_PART = HD + CT, L_RED = HD + CT + 4 * HD, L_TOTAL = L_RED + 8;

__global__ void __launch_bounds__(CT) cls_attn_fwd_kernel(const u16* __restrict__ qkv, u16* __restrict__ o,
                                                           float* __restrict__ lse, int T, int H) {
  __shared__ float sm[L_TOTAL];
  const int bh = blockIdx.x, b = bh / H, h = bh % H, tid = threadIdx.x;
  const int D = H * HD;
  const size_t row = (size_t)3 * D;  // elements per token row of qkv
  const u16* base = qkv + (size_t)b * T * row;
  if (tid < HD) sm[L_VEC + tid] = bf2f(base[h * HD + tid]) * 0.125f;  // q (token 0), scaled
  __syncthreads();
  float s = -INFINITY;
  if (tid < T) {
    float k[HD];
    load_row(base + tid * row + D + h * HD, k);
    float acc = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) acc = fmaf(sm[L_VEC + d], k[d], acc);
    s = acc;
  }
  const float mx = block_reduce(s, sm + L_RED, true);
  const float e = tid < T ? __expf(s - mx) : 0.f;
  const float sum = block_reduce(e, sm + L_RED, false);
  const float inv = 1.f / sum;
  sm[L_P + tid] = e * inv;
  __syncthreads();
  // o[d] = sum_t p_t v_t[d]: column d, key slice t % 4
  const int d = tid & (HD - 1), sl = tid >> 6;
  float acc = 0.f;
  for (int t = sl; t < T; t += 4) acc = fmaf(sm[L_P + t], bf2f(base[t * row + 2 * D + h * HD + d]), acc);
  sm[L_PART + sl * HD + d] = acc;
  __syncthreads();
  if (tid < HD) {
    const float v = sm[L_PART + tid] + sm[L_PART + HD + tid] + sm[L_PART + 2 * HD + tid] + sm[L_PART + 3 * HD + tid];
    o[(size_t)b * D + h * HD + tid] = f2bf(v);
  }
  if (tid == 0) lse[bh] = mx + __logf(sum);
}

__global__ void __launch_bounds__(CT) cls_attn_bwd_kernel(const u16* __restrict__ qkv, const u16* __restrict__ o,
                                                           const u16* __restrict__ dout, const float* __restrict__ lse,
                                                           u16* __restrict__ dqkv, int T, int H) {
  __shared__ float sm[L_TOTAL + HD];  // + q [64]
  const int bh = blockIdx.x, b = bh / H, h = bh % H, tid = threadIdx.x;
  const int D = H * HD;
  const size_t row = (size_t)3 * D;
  const u16* base = qkv + (size_t)b * T * row;
  u16* dbase = dqkv + (size_t)b * T * row;
  float* qs = sm + L_TOTAL;
  if (tid < HD) {
    qs[tid] = bf2f(base[h * HD + tid]) * 0.125f;
    sm[L_VEC + tid] = bf2f(dout[(size_t)b * D + h * HD + tid]);  // do
  }
  // Di = do . o (o as stored, bf16)
  float di_part = tid < HD ? bf2f(dout[(size_t)b * D + h * HD + tid]) * bf2f(o[(size_t)b * D + h * HD + tid]) : 0.f;
  const float Di = block_reduce(di_part, sm + L_RED, false);  // (its barriers also publish qs / do)
  const float L = lse[bh];
  float ds = 0.f;
  if (tid < T) {
    float k[HD], v[HD];
    load_row(base + tid * row + D + h * HD, k);
    load_row(base + tid * row + 2 * D + h * HD, v);
    float sc = 0.f, dp = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) {
      sc = fmaf(qs[d], k[d], sc);
      dp = fmaf(sm[L_VEC + d], v[d], dp);
    }
    const float p = __expf(sc - L);
    ds = p * (dp - Di);
    // dk_t = ds q / 8 (qs already holds q / 8), dv_t = p do; dq of token t > 0 = 0
    u16* dr = dbase + tid * row;
#pragma unroll
    for (int c = 0; c < HD / 8; ++c) {
      u32x4 wk, wv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int dd = c * 8 + 2 * e;
        wk[e] = pack2bf(ds * qs[dd], ds * qs[dd + 1]);
        wv[e] = pack2bf(p * sm[L_VEC + dd], p * sm[L_VEC + dd + 1]);
      }
      *reinterpret_cast<u32x4*>(dr + D + h * HD + c * 8) = wk;
      *reinterpret_cast<u32x4*>(dr + 2 * D + h * HD + c * 8) = wv;
      if (tid > 0) *reinterpret_cast<u32x4*>(dr + h * HD + c * 8) = u32x4{0u, 0u, 0u, 0u};
    }
  }
  sm[L_P + tid] = ds;
  __syncthreads();
  // dq[d] = sum_t ds_t k_t[d] / 8
  const int d = tid & (HD - 1), sl = tid >> 6;
  float acc = 0.f;
  for (int t = sl; t < T; t += 4) acc = fmaf(sm[L_P + t], bf2f(base[t * row + D + h * HD + d]), acc);
  sm[L_PART + sl * HD + d] = acc;
  __syncthreads();
  if (tid < HD) {
    const float v = sm[L_PART + tid] + sm[L_PART + HD + tid] + sm[L_PART + 2 * HD + tid] + sm[L_PART + 3 * HD + tid];
    dbase[h * HD + tid] = f2bf(v * 0.125f);
  }
}

}  // namespace

// qkv [B][T][3][H][64] bf16 -> o [B][H*64] (token 0's attention output), lse [B*H] fp32
PDT_API int pdt_cls_attn_fwd(const void* qkv, void* o, float* lse, int B, int T, int H, hipStream_t st) {
  if (B <= 0 || T <= 0 || T > CT || H <= 0) return -1;
  hipLaunchKernelGGL(cls_attn_fwd_kernel, dim3(B * H), dim3(CT), 0, st, (const u16*)qkv, (u16*)o, lse, T, H);
  PDT_RETURN_LAUNCH();
}

// dqkv [B][T][3][H][64] (every element written) from the token-0 output gradient dout [B][H*64]
PDT_API int pdt_cls_attn_bwd(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv, int B,
                             int T, int H, hipStream_t st) {
  if (B <= 0 || T <= 0 || T > CT || H <= 0) return -1;
  hipLaunchKernelGGL(cls_attn_bwd_kernel, dim3(B * H), dim3(CT), 0, st, (const u16*)qkv, (const u16*)o,
                     (const u16*)dout, lse, (u16*)dqkv, T, H);
  PDT_RETURN_LAUNCH();
}
