// Class-token attention: the last ViT block's attention for the ONE query the network's output
// depends on (the classifier reads only token 0 of the final block), against all T keys /
// values. Forward and backward for a packed qkv tensor [B][T][3][H][64] (bf16).
//
//   s_t = (q . k_t) / 8,  p = softmax(s),  o = sum_t p_t v_t                     (per b, h)
//   backward: dv_t = p_t do,  dp_t = do . v_t,  ds_t = p_t (dp_t - do . o),
//             dq = sum_t ds_t k_t / 8,  dk_t = ds_t q / 8     (dq of every other token = 0)
//
// One 256-thread workgroup per (b, h). Lane roles: 8 lanes per token (tid = 8 tg + c: token
// group tg = 0..31, 16-B chunk c = dims 8c .. 8c + 7), so every load / store of a wave covers 8
// whole 128-B head rows instead of 64 lanes each touching a different row; the 64-wide dot
// products are 8-FMA partials reduced over the 8 lanes, the sums over keys (o, dq) over the
// token groups (lane bits 3-5, then the 4 waves through LDS). fp32 softmax and accumulation;
// bf16 in and out. The work is tiny (B*H*T*64*4 MACs) -- what matters is that the block's
// other 196 query rows are never formed.
#include "pdt_common.h"

namespace {

constexpr int CT = 256;  // threads
constexpr int HD = 64;   // head dim
constexpr int TG = CT / 8;  // token groups per pass

__device__ __forceinline__ void unpack8f(const u32x4& w, float (&r)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    r[2 * e] = lo_bf(w[e]);
    r[2 * e + 1] = hi_bf(w[e]);
  }
}

// sum over the 8 lanes of a token group (lanes 8 tg .. 8 tg + 7)
__device__ __forceinline__ float sum8(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
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

// the 8-dim chunk sums acc[8] of all token groups -> out[64] (LDS part[4][64]; caller syncs after)
__device__ __forceinline__ void chunk_sum_to_lds(float (&acc)[8], float* part) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c = tid & 7;
#pragma unroll
  for (int e = 0; e < 8; ++e) {  // token groups of this wave: lane bits 3, 4, 5
    acc[e] += __shfl_xor(acc[e], 8, 64);
    acc[e] += __shfl_xor(acc[e], 16, 64);
    acc[e] += __shfl_xor(acc[e], 32, 64);
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) part[wave * HD + c * 8 + e] = acc[e];
  }
}

// LDS layout (floats): scores / probabilities [256] | partial sums [4][64] | reduce [8]
constexpr int L_P = 0, L_PART = CT, L_RED = CT + 4 * HD, L_TOTAL = L_RED + 8;

__global__ void __launch_bounds__(CT) cls_attn_fwd_kernel(const u16* __restrict__ qkv, u16* __restrict__ o,
                                                           float* __restrict__ lse, int T, int H) {
  __shared__ float sm[L_TOTAL];
  const int bh = blockIdx.x, b = bh / H, h = bh % H, tid = threadIdx.x;
  const int tg = tid >> 3, c = tid & 7;
  const int D = H * HD;
  const size_t row = (size_t)3 * D;  // elements per token row of qkv
  const u16* base = qkv + (size_t)b * T * row;
  float qc[8];  // q (token 0), scaled, dims 8c .. 8c + 7
  unpack8f(*reinterpret_cast<const u32x4*>(base + h * HD + c * 8), qc);
#pragma unroll
  for (int e = 0; e < 8; ++e) qc[e] *= 0.125f;
  float smax = -INFINITY;
  for (int t = tg; t < T; t += TG) {
    float kc[8];
    unpack8f(*reinterpret_cast<const u32x4*>(base + t * row + D + h * HD + c * 8), kc);
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = fmaf(qc[e], kc[e], acc);
    acc = sum8(acc);
    if (c == 0) sm[L_P + t] = acc;
    smax = fmaxf(smax, acc);
  }
  const float mx = block_reduce(smax, sm + L_RED, true);  // (its barriers publish the scores)
  float esum = 0.f;
  for (int t = tid; t < T; t += CT) {
    const float e = __expf(sm[L_P + t] - mx);
    sm[L_P + t] = e;
    esum += e;
  }
  const float sum = block_reduce(esum, sm + L_RED, false);  // (and the exponentials)
  const float inv = 1.f / sum;
  // o[d] = sum_t p_t v_t[d]
  float oa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int t = tg; t < T; t += TG) {
    float vc[8];
    unpack8f(*reinterpret_cast<const u32x4*>(base + t * row + 2 * D + h * HD + c * 8), vc);
    const float pt = sm[L_P + t] * inv;
#pragma unroll
    for (int e = 0; e < 8; ++e) oa[e] = fmaf(pt, vc[e], oa[e]);
  }
  chunk_sum_to_lds(oa, sm + L_PART);
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
  __shared__ float sm[L_TOTAL];
  const int bh = blockIdx.x, b = bh / H, h = bh % H, tid = threadIdx.x;
  const int tg = tid >> 3, c = tid & 7;
  const int D = H * HD;
  const size_t row = (size_t)3 * D;
  const u16* base = qkv + (size_t)b * T * row;
  u16* dbase = dqkv + (size_t)b * T * row;
  float qs[8], dc[8], oc[8];  // q / 8, do, o (as stored, bf16) of dims 8c .. 8c + 7
  unpack8f(*reinterpret_cast<const u32x4*>(base + h * HD + c * 8), qs);
  unpack8f(*reinterpret_cast<const u32x4*>(dout + (size_t)b * D + h * HD + c * 8), dc);
  unpack8f(*reinterpret_cast<const u32x4*>(o + (size_t)b * D + h * HD + c * 8), oc);
  float di = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    qs[e] *= 0.125f;
    di = fmaf(dc[e], oc[e], di);
  }
  const float Di = sum8(di);  // do . o (every token group holds it)
  const float L = lse[bh];
  // per key t: p = exp(q.k/8 - L), ds = p (do.v - Di); dk_t = ds q / 8, dv_t = p do; dq of t > 0 = 0
  float dq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int t = tg; t < T; t += TG) {
    float kc[8], vc[8];
    unpack8f(*reinterpret_cast<const u32x4*>(base + t * row + D + h * HD + c * 8), kc);
    unpack8f(*reinterpret_cast<const u32x4*>(base + t * row + 2 * D + h * HD + c * 8), vc);
    float sc = 0.f, dp = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc = fmaf(qs[e], kc[e], sc);
      dp = fmaf(dc[e], vc[e], dp);
    }
    sc = sum8(sc);
    dp = sum8(dp);
    const float p = __expf(sc - L);
    const float ds = p * (dp - Di);
    u16* dr = dbase + t * row + h * HD + c * 8;
    u32x4 wk, wv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wk[e] = pack2bf(ds * qs[2 * e], ds * qs[2 * e + 1]);
      wv[e] = pack2bf(p * dc[2 * e], p * dc[2 * e + 1]);
    }
    *reinterpret_cast<u32x4*>(dr + D) = wk;
    *reinterpret_cast<u32x4*>(dr + 2 * D) = wv;
    if (t > 0) *reinterpret_cast<u32x4*>(dr) = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) dq[e] = fmaf(ds, kc[e], dq[e]);
  }
  // dq[d] = sum_t ds_t k_t[d] / 8 (token 0's q row: the only nonzero dq)
  chunk_sum_to_lds(dq, sm + L_PART);
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
  if (((uintptr_t)qkv) & 15) return -5;  // 16-B chunk loads
  hipLaunchKernelGGL(cls_attn_fwd_kernel, dim3(B * H), dim3(CT), 0, st, (const u16*)qkv, (u16*)o, lse, T, H);
  PDT_RETURN_LAUNCH();
}

// dqkv [B][T][3][H][64] (every element written) from the token-0 output gradient dout [B][H*64]
PDT_API int pdt_cls_attn_bwd(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv, int B,
                             int T, int H, hipStream_t st) {
  if (B <= 0 || T <= 0 || T > CT || H <= 0) return -1;
  if ((((uintptr_t)qkv) | ((uintptr_t)o) | ((uintptr_t)dout) | ((uintptr_t)dqkv)) & 15) return -5;
  hipLaunchKernelGGL(cls_attn_bwd_kernel, dim3(B * H), dim3(CT), 0, st, (const u16*)qkv, (const u16*)o,
                     (const u16*)dout, lse, (u16*)dqkv, T, H);
  PDT_RETURN_LAUNCH();
}
