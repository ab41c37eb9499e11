// Fused training-mode BatchNorm(+residual)(+ReLU) for NHWC bf16 activations.
//
// Replaces the stock chain  BN-fwd(mean/var, norm) -> add -> relu  and its
// backward  relu-bwd -> add-bwd -> BN-bwd(dscale/dbias, dx)  (SURVEY §2.6(b):
// these memory-bound passes cost about as much as the convs at 8 TB/s).
//
// Forward : y (conv output) -> per-channel partial (sum, sumsq)   [bn_stats]
//           (or taken from the conv epilogue)  -> finalize         [bn_finalize]
//           a = act(y * scale + shift (+ res))  one read, one write [bn_apply]
// Backward: dz = dA * relu'(.)  ; partial (sum dz, sum dz*(y-mean)) [bn_bwd_reduce]
//           -> dgamma, dbeta, and dy = k1*dz + k2*y + k3            [bn_bwd_finalize]
//           dy (and dres = dz for the residual branch) in one pass   [bn_bwd_apply]
//
// All element passes move 16 B per lane (8 channels); channel parameters are
// read as 2x f32x4. Partial sums are [2][R][C] fp32 (R partial rows) and are
// combined in fp64 by the finalize kernels (deterministic, no atomics).
#include "pdt_common.h"
#include <stdlib.h>

namespace {

constexpr int NT = 256;

__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
  f[0] = lo_bf(v[0]); f[1] = hi_bf(v[0]);
  f[2] = lo_bf(v[1]); f[3] = hi_bf(v[1]);
  f[4] = lo_bf(v[2]); f[5] = hi_bf(v[2]);
  f[6] = lo_bf(v[3]); f[7] = hi_bf(v[3]);
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  return u32x4{pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7])};
}

__device__ __forceinline__ void load8f(const float* p, float* f) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}

// -------------------------------------------------------------------- stats
// grid: G blocks; block b handles rows b, b+G, ... in passes of RP rows.
__global__ void __launch_bounds__(NT) bn_stats_kernel(const u16* __restrict__ y, float* __restrict__ part, long M,
                                                      int C) {
  __shared__ float red[2][NT][8];
  const int cpr = C / 8;               // chunks per row
  const int rp = NT / cpr;             // rows per pass
  const int t = threadIdx.x;
  const int ch = t % cpr, rr = t / cpr;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rr < rp) {
    for (long r = (long)blockIdx.x * rp + rr; r < M; r += (long)gridDim.x * rp) {
      u32x4 v = *reinterpret_cast<const u32x4*>(y + r * C + ch * 8);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += f[k];
        q[k] += f[k] * f[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][t][k] = s[k];
    red[1][t][k] = q[k];
  }
  __syncthreads();
  // reduce over rr for each ch
  if (t < cpr) {
    float as[8] = {0, 0, 0, 0, 0, 0, 0, 0}, aq[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < rp; ++j) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        as[k] += red[0][j * cpr + t][k];
        aq[k] += red[1][j * cpr + t][k];
      }
    }
    const long R = gridDim.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      part[(long)blockIdx.x * C + t * 8 + k] = as[k];
      part[(R + blockIdx.x) * C + t * 8 + k] = aq[k];
    }
  }
}

// Parallel first stage of the partial-row reduction: [2][R][C] -> [2][G][C].
// grid (ceil(C/64), G); 256 threads = 64 channels x 4 row groups; each thread
// sums rows y*4+rg, y*4+rg + 4G, ... in fp32, then the 4 row groups combine in LDS.
__global__ void __launch_bounds__(256) rows_reduce_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                          int R, int C, int G) {
  __shared__ float red[2][4][64];
  const int t = threadIdx.x, cl = t & 63, rg = t >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int g = blockIdx.y;
  float s = 0.f, q = 0.f;
  if (c < C) {
    // 8 rows per trip, all loads issued before the adds (latency, not bandwidth, bounds this)
    int r = g * 4 + rg;
    const int step = 4 * G;
    for (; r + 7 * step < R; r += 8 * step) {
      float a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = part[(long)(r + u * step) * C + c];
        b[u] = part[(long)(R + r + u * step) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s += a[u];
        q += b[u];
      }
    }
    for (; r < R; r += step) {
      s += part[(long)r * C + c];
      q += part[(long)(R + r) * C + c];
    }
  }
  red[0][rg][cl] = s;
  red[1][rg][cl] = q;
  __syncthreads();
  if (rg == 0 && c < C) {
    out[(long)g * C + c] = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    out[(long)(G + g) * C + c] = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
  }
}

// Block-parallel finalize: 256 threads = 64 channels x 4 row groups; rows are
// summed in fp64 and combined through LDS (R <= 256 after rows_reduce).
__device__ __forceinline__ void sum_rows64(const float* __restrict__ part, int R, int C, int c, int rg,
                                           double* sh_s, double* sh_q, double& s, double& q) {
  const int cl = threadIdx.x & 63;
  double a = 0, b = 0;
  if (c < C) {
    int r = rg;
    for (; r + 28 < R; r += 32) {  // 8 rows per trip, loads first
      float x[8], y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        x[u] = part[(long)(r + 4 * u) * C + c];
        y[u] = part[(long)(R + r + 4 * u) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a += x[u];
        b += y[u];
      }
    }
    for (; r < R; r += 4) {
      a += part[(long)r * C + c];
      b += part[(long)(R + r) * C + c];
    }
  }
  sh_s[rg * 64 + cl] = a;
  sh_q[rg * 64 + cl] = b;
  __syncthreads();
  s = sh_s[cl] + sh_s[64 + cl] + sh_s[128 + cl] + sh_s[192 + cl];
  q = sh_q[cl] + sh_q[64 + cl] + sh_q[128 + cl] + sh_q[192 + cl];
}

struct FwdFin {
  double count;
  float eps, momentum;
  const float* gamma;
  const float* beta;
  float *mean_out, *invstd_out, *scale, *shift, *running_mean, *running_var;
  long* nbt;
};

struct BwdFin {
  double count;
  const float *gamma, *mean, *invstd;
  float *dgamma, *dbeta, *k1, *k2, *k3;
  int accumulate;
};

// outputs: mean, invstd (saved for backward), scale = gamma*invstd, shift = beta - mean*scale,
// running stats updated in place (unbiased variance) and num_batches_tracked += 1.
__device__ __forceinline__ void fwd_finalize_channel(const FwdFin& f, int c, double s, double q) {
  const double count = f.count;
  const float momentum = f.momentum;
  const float* gamma = f.gamma;
  const float* beta = f.beta;
  double mean = s / count;
  double var = q / count - mean * mean;
  if (var < 0) var = 0;
  float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  f.mean_out[c] = (float)mean;
  f.invstd_out[c] = invstd;
  f.scale[c] = g * invstd;
  f.shift[c] = b - (float)mean * g * invstd;
  if (f.running_mean) {
    double unb = count > 1 ? var * count / (count - 1) : var;
    f.running_mean[c] = (1.f - momentum) * f.running_mean[c] + momentum * (float)mean;
    f.running_var[c] = (1.f - momentum) * f.running_var[c] + momentum * (float)unb;
  }
}

// dgamma = sum(dz*(y-mean))*invstd, dbeta = sum(dz); dy = k1*dz + k2*y + k3
__device__ __forceinline__ void bwd_finalize_channel(const BwdFin& f, int c, double s, double q) {
  double is = f.invstd[c], g = f.gamma ? f.gamma[c] : 1.0, mu = f.mean[c];
  double dg = q * is, db = s;
  if (f.dgamma) f.dgamma[c] = (float)(f.accumulate ? f.dgamma[c] + dg : dg);
  if (f.dbeta) f.dbeta[c] = (float)(f.accumulate ? f.dbeta[c] + db : db);
  double a1 = g * is;
  double a2 = -g * is * is * is * q / f.count;
  double a3 = -g * is * s / f.count - a2 * mu;
  f.k1[c] = (float)a1;
  f.k2[c] = (float)a2;
  f.k3[c] = (float)a3;
}

__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ part, int R, int C, FwdFin f) {
  __shared__ double sh_s[256], sh_q[256];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  double s, q;
  sum_rows64(part, R, C, c, rg, sh_s, sh_q, s, q);
  if (blockIdx.x == 0 && threadIdx.x == 0 && f.nbt) f.nbt[0] += 1;
  if (rg != 0 || c >= C) return;
  fwd_finalize_channel(f, c, s, q);
}

__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(const float* __restrict__ part, int R, int C, BwdFin f) {
  __shared__ double sh_s[256], sh_q[256];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  double s, q;
  sum_rows64(part, R, C, c, rg, sh_s, sh_q, s, q);
  if (rg != 0 || c >= C) return;
  bwd_finalize_channel(f, c, s, q);
}

// -------------------------------------------------------------------- apply
// MASK: also write the ReLU mask as one bit per element (byte i = chunk i's 8
// channels): the backward then reads 1/16 of the bytes instead of `out`.
// NTS: nontemporal (streaming) stores of the element pass outputs
template <typename T>
__device__ __forceinline__ void st_pol(T* p, const T& v, bool nts) {
  if (nts) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// RAFF: the residual is itself a raw conv output whose BatchNorm affine is applied
// here (r*rscale + rshift) -- the ResNet downsample branch's BN apply folded into
// the block's bn3 apply (its output is never written or re-read).
template <bool RES, bool RELU, bool MASK = false, int U = 1, bool NTS = false, bool RAFF = false>
__global__ void __launch_bounds__(NT) bn_apply_kernel(const u16* __restrict__ y, const u16* __restrict__ res,
                                                      u16* __restrict__ out, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, long n8, int C,
                                                      uint8_t* __restrict__ mask,
                                                      const float* __restrict__ rscale = nullptr,
                                                      const float* __restrict__ rshift = nullptr) {
  // the host sizes the grid so the stride is a multiple of C/8: a thread's 8
  // channels never change, so the per-channel coefficients are loaded once
  const int cpr = C / 8;
  const int ch = (int)((blockIdx.x * NT + threadIdx.x) % (uint32_t)cpr) * 8;
  float sc[8], sh[8], rsc[8], rsh[8];
  load8f(scale + ch, sc);
  load8f(shift + ch, sh);
  if (RAFF) {
    load8f(rscale + ch, rsc);
    load8f(rshift + ch, rsh);
  }
  const uint32_t S = gridDim.x * NT;
  auto body = [&](uint32_t i, const u32x4& yv, const u32x4& rv) {
    float f[8];
    unpack8(yv, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = f[k] * sc[k] + sh[k];
    if (RES) {
      float r[8];
      unpack8(rv, r);
      if (RAFF) {
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] += r[k] * rsc[k] + rsh[k];
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] += r[k];
      }
    }
    if (RELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = fmaxf(f[k], 0.f);
    }
    const u32x4 o = pack8(f);
    st_pol(reinterpret_cast<u32x4*>(out) + i, o, NTS);
    if (MASK) {
      uint32_t m = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // mask of the ROUNDED output (what backward's act > 0 saw)
        m |= ((o[e] & 0x7fffu) != 0 && !(o[e] & 0x8000u)) ? (1u << (2 * e)) : 0u;
        m |= ((o[e] & 0x7fff0000u) != 0 && !(o[e] & 0x80000000u)) ? (1u << (2 * e + 1)) : 0u;
      }
      mask[i] = (uint8_t)m;
    }
  };
  uint32_t i = blockIdx.x * NT + threadIdx.x;
  // U chunks per trip, every load issued before any is consumed (memory-level
  // parallelism); the tail runs one chunk per trip (no per-load predicates)
  for (; U > 1 && i + (U - 1) * S < (uint32_t)n8; i += U * S) {
    u32x4 yv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      yv[u] = reinterpret_cast<const u32x4*>(y)[i + u * S];
      if (RES) rv[u] = reinterpret_cast<const u32x4*>(res)[i + u * S];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) body(i + u * S, yv[u], RES ? rv[u] : yv[u]);
  }
  for (; i < (uint32_t)n8; i += S) {
    const u32x4 yv = reinterpret_cast<const u32x4*>(y)[i];
    const u32x4 rv = RES ? reinterpret_cast<const u32x4*>(res)[i] : yv;
    body(i, yv, rv);
  }
}

// -------------------------------------------------------------------- backward
// relu mask: if `act` (saved output) is given, mask = act > 0; else if RELU,
// mask = y*scale+shift > 0 (exact when there is no residual).
// USE_MASK: the ReLU mask comes from the forward's bit mask (takes precedence over USE_ACT)
// ResNet stem: the BN-backward passes read the BN output gradient dA straight from
// the max-pool's output gradient and argmax bytes (csrc/pool.hip: maxpool_bwd_kernel
// gathers the same way), so the full-resolution dA is never written or read.
struct PoolSrc {
  const u16* dout;     // [N][Ho][Wo][C] pool output gradient
  const uint8_t* idx;  // [N][Ho][Wo][C] argmax (kh*k + kw) per element
  int H, W, Ho, Wo, k, s, p;
};

__device__ inline void pool_grad8(const PoolSrc& ps, uint32_t pix, int cc, int cpr, float (&acc)[8]) {
  const uint32_t w = pix % (uint32_t)ps.W, r = pix / (uint32_t)ps.W;
  const int h = r % (uint32_t)ps.H, n = r / (uint32_t)ps.H;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const int oh_lo = max(h + ps.p - ps.k + ps.s, 0) / ps.s, oh_hi = min((h + ps.p) / ps.s, ps.Ho - 1);
  const int ow_lo = max((int)w + ps.p - ps.k + ps.s, 0) / ps.s, ow_hi = min(((int)w + ps.p) / ps.s, ps.Wo - 1);
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int kh = h + ps.p - oh * ps.s;
    if (kh < 0 || kh >= ps.k) continue;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int kw = (int)w + ps.p - ow * ps.s;
      if (kw < 0 || kw >= ps.k) continue;
      const uint32_t o = (((uint32_t)n * ps.Ho + oh) * ps.Wo + ow) * cpr + cc;
      const uint2 bi = reinterpret_cast<const uint2*>(ps.idx)[o];
      float g[8];
      unpack8(reinterpret_cast<const u32x4*>(ps.dout)[o], g);
      const uint32_t me = (uint32_t)(kh * ps.k + kw);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t b = ((j < 4 ? bi.x : bi.y) >> (8 * (j & 3))) & 0xffu;
        if (b == me) acc[j] += g[j];
      }
    }
  }
}

template <bool RELU, bool USE_ACT, bool USE_MASK = false, bool POOL = false>
__global__ void __launch_bounds__(NT) bn_bwd_reduce_kernel(const u16* __restrict__ dA, const u16* __restrict__ y,
                                                           const u16* __restrict__ act,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           float* __restrict__ part, long M, int C,
                                                           const uint8_t* __restrict__ mask, PoolSrc ps = {}) {
  __shared__ float red[2][NT][8];
  const int cpr = C / 8;
  const int rp = NT / cpr;
  const int t = threadIdx.x;
  const int ch = t % cpr, rr = t / cpr;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rr < rp) {
    float mu[8], sc[8], sh[8];
    load8f(mean + ch * 8, mu);
    if (RELU && !USE_ACT && !USE_MASK) {
      load8f(scale + ch * 8, sc);
      load8f(shift + ch * 8, sh);
    }
    for (long r = (long)blockIdx.x * rp + rr; r < M; r += (long)gridDim.x * rp) {
      const long off = r * C + ch * 8;
      float g[8], yv[8];
      if (POOL)
        pool_grad8(ps, (uint32_t)r, ch, cpr, g);
      else
        unpack8(*reinterpret_cast<const u32x4*>(dA + off), g);
      unpack8(*reinterpret_cast<const u32x4*>(y + off), yv);
      if (RELU) {
        if (USE_MASK) {
          const uint32_t m = mask[off >> 3];
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] = (m >> k) & 1u ? g[k] : 0.f;
        } else if (USE_ACT) {
          float a[8];
          unpack8(*reinterpret_cast<const u32x4*>(act + off), a);
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] = a[k] > 0.f ? g[k] : 0.f;
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] = (yv[k] * sc[k] + sh[k]) > 0.f ? g[k] : 0.f;
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += g[k];
        q[k] += g[k] * (yv[k] - mu[k]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][t][k] = s[k];
    red[1][t][k] = q[k];
  }
  __syncthreads();
  if (t < cpr) {
    float as[8] = {0, 0, 0, 0, 0, 0, 0, 0}, aq[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < rp; ++j) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        as[k] += red[0][j * cpr + t][k];
        aq[k] += red[1][j * cpr + t][k];
      }
    }
    const long R = gridDim.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      part[(long)blockIdx.x * C + t * 8 + k] = as[k];
      part[(R + blockIdx.x) * C + t * 8 + k] = aq[k];
    }
  }
}

template <bool RELU, bool USE_ACT, bool DRES, bool USE_MASK = false, bool POOL = false, int U = 1, bool NTS = false>
__global__ void __launch_bounds__(NT) bn_bwd_apply_kernel(const u16* __restrict__ dA, const u16* __restrict__ y,
                                                          const u16* __restrict__ act,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ k1, const float* __restrict__ k2,
                                                          const float* __restrict__ k3, u16* __restrict__ dy,
                                                          u16* __restrict__ dres, long n8, int C,
                                                          const uint8_t* __restrict__ mask, PoolSrc ps = {}) {
  const int cpr = C / 8;
  const int ch = (int)((blockIdx.x * NT + threadIdx.x) % (uint32_t)cpr) * 8;  // invariant (see bn_apply)
  float a1[8], a2[8], a3[8], sc[8], sh[8];
  load8f(k1 + ch, a1);
  load8f(k2 + ch, a2);
  load8f(k3 + ch, a3);
  if (RELU && !USE_MASK && !USE_ACT) {
    load8f(scale + ch, sc);
    load8f(shift + ch, sh);
  }
  const uint32_t S = gridDim.x * NT;
  // g: dA chunk (already gathered for POOL), yq: y chunk, gate: act chunk or mask byte
  auto body = [&](uint32_t i, float (&g)[8], const u32x4& yq, const u32x4& aq, uint32_t m) {
    float yv[8];
    unpack8(yq, yv);
    if (RELU) {
      if (USE_MASK) {
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = (m >> k) & 1u ? g[k] : 0.f;
      } else if (USE_ACT) {
        float a[8];
        unpack8(aq, a);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = a[k] > 0.f ? g[k] : 0.f;
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = (yv[k] * sc[k] + sh[k]) > 0.f ? g[k] : 0.f;
      }
    }
    if (DRES) st_pol(reinterpret_cast<u32x4*>(dres) + i, pack8(g), NTS);
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = a1[k] * g[k] + a2[k] * yv[k] + a3[k];
    st_pol(reinterpret_cast<u32x4*>(dy) + i, pack8(g), NTS);
  };
  uint32_t i = blockIdx.x * NT + threadIdx.x;
  if constexpr (!POOL && U > 1) {
    // U chunks per trip, all loads first (see bn_apply_kernel)
    for (; i + (U - 1) * S < (uint32_t)n8; i += U * S) {
      u32x4 gq[U], yq[U], aq[U];
      uint32_t mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        gq[u] = reinterpret_cast<const u32x4*>(dA)[i + u * S];
        yq[u] = reinterpret_cast<const u32x4*>(y)[i + u * S];
        if (RELU && USE_MASK) mb[u] = mask[i + u * S];
        else mb[u] = 0;
        if (RELU && !USE_MASK && USE_ACT) aq[u] = reinterpret_cast<const u32x4*>(act)[i + u * S];
        else aq[u] = yq[u];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float g[8];
        unpack8(gq[u], g);
        body(i + u * S, g, yq[u], aq[u], mb[u]);
      }
    }
  }
  for (; i < (uint32_t)n8; i += S) {
    float g[8];
    if (POOL)
      pool_grad8(ps, i / (uint32_t)cpr, ch / 8, cpr, g);
    else
      unpack8(reinterpret_cast<const u32x4*>(dA)[i], g);
    const u32x4 yq = reinterpret_cast<const u32x4*>(y)[i];
    const u32x4 aq = (RELU && !USE_MASK && USE_ACT) ? reinterpret_cast<const u32x4*>(act)[i] : yq;
    const uint32_t m = (RELU && USE_MASK) ? (uint32_t)mask[i] : 0u;
    body(i, g, yq, aq, m);
  }
}

// elementwise trip unroll of bn_apply / bn_bwd_apply (PDT_BN_UNROLL=1|2|4, default 1;
// pdt_bn_set_unroll for in-process A/B runs). Measured at ResNet-50 stage 1, bs 1024
// (scripts/bench_bn.py, one MI355X): apply 4.49 / 4.38 / 4.45 TB/s and backward apply
// 4.91 / 4.47 / 4.44 TB/s for U = 1 / 2 / 4 -- the grid-stride loop already keeps
// enough bytes in flight; deeper trips only cost occupancy.
int g_bn_unroll = -1;
int bn_unroll() {
  if (g_bn_unroll < 0) {
    const char* e = getenv("PDT_BN_UNROLL");
    int u = e ? atoi(e) : 1;
    g_bn_unroll = (u == 1 || u == 2 || u == 4 || u == 11) ? u : 1;
  }
  return g_bn_unroll;
}

int gcd_i(int a, int b) { return b ? gcd_i(b, a % b) : a; }

// grid for the element passes: <= 4096 blocks, rounded so that the grid
// stride (blocks * NT chunks) is a multiple of C/8 (channel-invariant threads)
int grid_for(long n8, int C) {
  long b = (n8 + NT - 1) / NT;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  const int cpr = C / 8;
  const int f = cpr / gcd_i(cpr, NT);
  b = (b + f - 1) / f * f;
  return (int)b;
}

}  // namespace

PDT_API int pdt_bn_set_unroll(int u) {  // 1 / 2 / 4: trip unroll; 11: unroll 1 + nontemporal stores
  if (u != 1 && u != 2 && u != 4 && u != 11) return -1;
  g_bn_unroll = u;
  return 0;
}

PDT_API int pdt_bn_stats_blocks(long M, int C) {
  int cpr = C / 8;
  int rp = NT / cpr;
  long b = (M + rp - 1) / rp;
  // several blocks per CU, each streaming many rows (PDT_BN_BLOCKS overrides the cap)
  static int cap = -1;
  if (cap < 0) {
    const char* e = getenv("PDT_BN_BLOCKS");
    cap = e ? atoi(e) : 512;
    if (cap < 1) cap = 512;
  }
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

PDT_API int pdt_bn_stats(const void* y, float* part, long M, int C, int blocks, hipStream_t st) {
  if (C % 8 || C / 8 > NT) return -1;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(blocks), dim3(NT), 0, st, (const u16*)y, part, M, C);
  PDT_RETURN_LAUNCH();
}

// Number of floats of extra workspace the finalize calls need after the
// [2][R][C] partial block (stage-1 output of the parallel row reduction).
// stage-1 row groups: enough blocks to fill the chip for narrow C, few enough
// rows left for the finalize's single pass
static int rows_groups(int R, int C) {
  if (R <= 256) return 0;
  return (R > 2048 && C <= 256) ? 128 : 64;
}

PDT_API long pdt_rows_reduce_workspace(int R, int C) {
  const int G = rows_groups(R, C);
  return G ? 2L * G * C : 0;
}


// Stage 1 of the partial-row reduction when R > 256 (a separate launch: a
// single-launch "last block finalizes" variant needs a device-scope release
// fence per block, which on the multi-XCD MI355X writes back L2 -- measured
// ~2.4x slower than the two launches).
static const float* rows_reduce(const float* part, int* R, int C, hipStream_t st) {
  const int G = rows_groups(*R, C);
  if (G == 0) return part;
  float* out = const_cast<float*>(part) + 2L * (*R) * C;  // workspace tail
  hipLaunchKernelGGL(rows_reduce_kernel, dim3((C + 63) / 64, G), dim3(256), 0, st, part, out, *R, C, G);
  *R = G;
  return out;
}

PDT_API int pdt_bn_finalize(const float* part, int R, int C, double count, float eps, float momentum,
                            const float* gamma, const float* beta, float* mean, float* invstd, float* scale,
                            float* shift, float* running_mean, float* running_var, long* num_batches_tracked,
                            hipStream_t st) {
  FwdFin f{count, eps, momentum, gamma, beta, mean, invstd, scale, shift, running_mean, running_var,
           num_batches_tracked};
  part = rows_reduce(part, &R, C, st);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, st, part, R, C, f);
  PDT_RETURN_LAUNCH();
}

// mask (optional, relu only): [M*C/8] bytes, bit k of byte i = (out[8i+k] > 0)
PDT_API int pdt_bn_apply(const void* y, const void* res, void* out, const float* scale, const float* shift, long M,
                         int C, int relu, void* mask, hipStream_t st) {
  if (C % 8) return -1;
  if (mask && !relu) return -2;
  long n8 = M * C / 8;
  dim3 g(grid_for(n8, C)), b(NT);
  const u16* Y = (const u16*)y;
  const u16* R = (const u16*)res;
  u16* O = (u16*)out;
  uint8_t* MK = (uint8_t*)mask;
  const int un = bn_unroll();
#define APPLY(R_, U_, M_)                                                                                   \
  do {                                                                                                      \
    if (un == 4) hipLaunchKernelGGL((bn_apply_kernel<R_, U_, M_, 4>), g, b, 0, st, Y, R, O, scale, shift, n8, C, MK); \
    else if (un == 11) hipLaunchKernelGGL((bn_apply_kernel<R_, U_, M_, 1, true>), g, b, 0, st, Y, R, O, scale, shift, n8, C, MK); \
    else if (un == 2) hipLaunchKernelGGL((bn_apply_kernel<R_, U_, M_, 2>), g, b, 0, st, Y, R, O, scale, shift, n8, C, MK); \
    else hipLaunchKernelGGL((bn_apply_kernel<R_, U_, M_, 1>), g, b, 0, st, Y, R, O, scale, shift, n8, C, MK); \
  } while (0)
  if (res) {
    if (relu) { if (mask) APPLY(true, true, true); else APPLY(true, true, false); }
    else APPLY(true, false, false);
  } else {
    if (relu) { if (mask) APPLY(false, true, true); else APPLY(false, true, false); }
    else APPLY(false, false, false);
  }
#undef APPLY
  PDT_RETURN_LAUNCH();
}

// out = relu?(y*scale + shift + (r*rscale + rshift)): a residual that is the raw output
// of another conv whose BN affine (rscale, rshift) is applied here
PDT_API int pdt_bn_apply_res_affine(const void* y, const void* r, void* out, const float* scale, const float* shift,
                                    const float* rscale, const float* rshift, long M, int C, int relu, void* mask,
                                    hipStream_t st) {
  if (C % 8 || !r || !rscale || !rshift) return -1;
  if (mask && !relu) return -2;
  long n8 = M * C / 8;
  dim3 g(grid_for(n8, C)), b(NT);
  const u16* Y = (const u16*)y;
  const u16* R = (const u16*)r;
  u16* O = (u16*)out;
  uint8_t* MK = (uint8_t*)mask;
  if (relu && mask)
    hipLaunchKernelGGL((bn_apply_kernel<true, true, true, 1, false, true>), g, b, 0, st, Y, R, O, scale, shift, n8, C,
                       MK, rscale, rshift);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<true, true, false, 1, false, true>), g, b, 0, st, Y, R, O, scale, shift, n8, C,
                       MK, rscale, rshift);
  else
    hipLaunchKernelGGL((bn_apply_kernel<true, false, false, 1, false, true>), g, b, 0, st, Y, R, O, scale, shift, n8,
                       C, MK, rscale, rshift);
  PDT_RETURN_LAUNCH();
}

// ReLU mask source (relu != 0): bit mask if given, else act > 0 if given, else recomputed from y
PDT_API int pdt_bn_bwd_reduce(const void* dA, const void* y, const void* act, const float* mean,
                              const float* scale, const float* shift, float* part, long M, int C, int relu,
                              int blocks, const void* mask, hipStream_t st) {
  if (C % 8 || C / 8 > NT) return -1;
  const u16 *G = (const u16*)dA, *Y = (const u16*)y, *A = (const u16*)act;
  const uint8_t* MK = (const uint8_t*)mask;
  dim3 g(blocks), b(NT);
#define RED(R_, U_, M_) \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<R_, U_, M_>), g, b, 0, st, G, Y, A, mean, scale, shift, part, M, C, MK)
  if (!relu) RED(false, false, false);
  else if (mask) RED(true, false, true);
  else if (act) RED(true, true, false);
  else RED(true, false, false);
#undef RED
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_bn_bwd_finalize(const float* part, int R, int C, double count, const float* gamma,
                                const float* mean, const float* invstd, float* dgamma, float* dbeta, float* k1,
                                float* k2, float* k3, int accumulate, hipStream_t st) {
  BwdFin f{count, gamma, mean, invstd, dgamma, dbeta, k1, k2, k3, accumulate};
  part = rows_reduce(part, &R, C, st);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, st, part, R, C, f);
  PDT_RETURN_LAUNCH();
}

// ResNet downsample blocks: the block-output gradient dA feeds TWO BatchNorm backwards -- bn3
// of the main branch and the shortcut's BN -- both gated by the block's ReLU bit mask. One
// pass reads dA and the mask once and writes both input gradients:
//   dy1 = (k1a*g + k2a*y1 + k3a),  dy2 = (k1b*g + k2b*y2 + k3b),  g = dA masked
__global__ void __launch_bounds__(NT) bn_bwd_apply_dual_kernel(
    const u16* __restrict__ dA, const uint8_t* __restrict__ mask, const u16* __restrict__ y1,
    const float* __restrict__ k1a, const float* __restrict__ k2a, const float* __restrict__ k3a, u16* __restrict__ dy1,
    const u16* __restrict__ y2, const float* __restrict__ k1b, const float* __restrict__ k2b,
    const float* __restrict__ k3b, u16* __restrict__ dy2, long n8, int C) {
  const int cpr = C / 8;
  const int ch = (int)((blockIdx.x * NT + threadIdx.x) % (uint32_t)cpr) * 8;  // invariant (see bn_apply)
  float a1[8], a2[8], a3[8], b1[8], b2[8], b3[8];
  load8f(k1a + ch, a1);
  load8f(k2a + ch, a2);
  load8f(k3a + ch, a3);
  load8f(k1b + ch, b1);
  load8f(k2b + ch, b2);
  load8f(k3b + ch, b3);
  const uint32_t S = gridDim.x * NT;
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < (uint32_t)n8; i += S) {
    const u32x4 gq = reinterpret_cast<const u32x4*>(dA)[i];
    const u32x4 yq1 = reinterpret_cast<const u32x4*>(y1)[i];
    const u32x4 yq2 = reinterpret_cast<const u32x4*>(y2)[i];
    const uint32_t m = mask[i];
    float g[8], v1[8], v2[8], o1[8], o2[8];
    unpack8(gq, g);
    unpack8(yq1, v1);
    unpack8(yq2, v2);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float gg = (m >> k) & 1u ? g[k] : 0.f;
      o1[k] = a1[k] * gg + a2[k] * v1[k] + a3[k];
      o2[k] = b1[k] * gg + b2[k] * v2[k] + b3[k];
    }
    reinterpret_cast<u32x4*>(dy1)[i] = pack8(o1);
    reinterpret_cast<u32x4*>(dy2)[i] = pack8(o2);
  }
}

PDT_API int pdt_bn_bwd_apply_dual(const void* dA, const void* mask, const void* y1, const float* k1a,
                                  const float* k2a, const float* k3a, void* dy1, const void* y2, const float* k1b,
                                  const float* k2b, const float* k3b, void* dy2, long M, int C, hipStream_t st) {
  if (C % 8 || !mask) return -1;
  const long n8 = M * C / 8;
  hipLaunchKernelGGL(bn_bwd_apply_dual_kernel, dim3(grid_for(n8, C)), dim3(NT), 0, st, (const u16*)dA,
                     (const uint8_t*)mask, (const u16*)y1, k1a, k2a, k3a, (u16*)dy1, (const u16*)y2, k1b, k2b, k3b,
                     (u16*)dy2, n8, C);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_bn_bwd_apply(const void* dA, const void* y, const void* act, const float* scale,
                             const float* shift, const float* k1, const float* k2, const float* k3, void* dy,
                             void* dres, long M, int C, int relu, const void* mask, hipStream_t st) {
  if (C % 8) return -1;
  long n8 = M * C / 8;
  dim3 g(grid_for(n8, C)), b(NT);
  const u16 *G = (const u16*)dA, *Y = (const u16*)y, *A = (const u16*)act;
  u16 *DY = (u16*)dy, *DR = (u16*)dres;
  const uint8_t* MK = (const uint8_t*)mask;
  const int un = bn_unroll();
#define BWD_LAUNCH(R_, U_, D_, M_)                                                                                   \
  do {                                                                                                               \
    if (un == 4)                                                                                                     \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<R_, U_, D_, M_, false, 4>), g, b, 0, st, G, Y, A, scale, shift, k1, k2, \
                         k3, DY, DR, n8, C, MK, PoolSrc{});                                                          \
    else if (un == 11)                                                                                               \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<R_, U_, D_, M_, false, 1, true>), g, b, 0, st, G, Y, A, scale, shift, k1, \
                         k2, k3, DY, DR, n8, C, MK, PoolSrc{});                                                      \
    else if (un == 2)                                                                                                \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<R_, U_, D_, M_, false, 2>), g, b, 0, st, G, Y, A, scale, shift, k1, k2, \
                         k3, DY, DR, n8, C, MK, PoolSrc{});                                                          \
    else                                                                                                             \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<R_, U_, D_, M_, false, 1>), g, b, 0, st, G, Y, A, scale, shift, k1, k2, \
                         k3, DY, DR, n8, C, MK, PoolSrc{});                                                          \
  } while (0)
#define BWD_APPLY(R_, U_, D_) BWD_LAUNCH(R_, U_, D_, false)
#define BWD_APPLY_M(D_) BWD_LAUNCH(true, false, D_, true)
  if (!relu) {
    if (dres) BWD_APPLY(false, false, true); else BWD_APPLY(false, false, false);
  } else if (mask) {
    if (dres) BWD_APPLY_M(true); else BWD_APPLY_M(false);
  } else if (act) {
    if (dres) BWD_APPLY(true, true, true); else BWD_APPLY(true, true, false);
  } else {
    if (dres) BWD_APPLY(true, false, true); else BWD_APPLY(true, false, false);
  }
#undef BWD_APPLY
#undef BWD_APPLY_M
#undef BWD_LAUNCH
  PDT_RETURN_LAUNCH();
}

// Stem BN(+ReLU) backward with dA gathered from the max-pool gradient (PoolSrc):
// reduce + apply over y [N][H][W][C] (ReLU mask recomputed from y*scale+shift).
PDT_API int pdt_bn_bwd_reduce_pool(const void* dout, const void* idx, const void* y, const float* mean,
                                   const float* scale, const float* shift, float* part, int N, int H, int W, int C,
                                   int Ho, int Wo, int k, int s, int p, int blocks, hipStream_t st) {
  const long M = (long)N * H * W;
  if (C % 8 || C / 8 > NT || M * (C / 8) >= (1L << 31) || (long)N * Ho * Wo * (C / 8) >= (1L << 31)) return -1;
  PoolSrc ps{(const u16*)dout, (const uint8_t*)idx, H, W, Ho, Wo, k, s, p};
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<true, false, false, true>), dim3(blocks), dim3(NT), 0, st, nullptr,
                     (const u16*)y, nullptr, mean, scale, shift, part, M, C, nullptr, ps);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_bn_bwd_apply_pool(const void* dout, const void* idx, const void* y, const float* scale,
                                  const float* shift, const float* k1, const float* k2, const float* k3, void* dy,
                                  int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p, hipStream_t st) {
  const long n8 = (long)N * H * W * (C / 8);
  if (C % 8 || n8 >= (1L << 31) || (long)N * Ho * Wo * (C / 8) >= (1L << 31)) return -1;
  PoolSrc ps{(const u16*)dout, (const uint8_t*)idx, H, W, Ho, Wo, k, s, p};
  hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false, false, false, true>), dim3(grid_for(n8, C)), dim3(NT), 0, st,
                     nullptr, (const u16*)y, nullptr, scale, shift, k1, k2, k3, (u16*)dy, nullptr, n8, C, nullptr,
                     ps);
  PDT_RETURN_LAUNCH();
}
