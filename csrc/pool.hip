// Pooling for NHWC bf16: max-pool (k x k, stride s, pad p) with a saved uint8
// argmax, gather-form backward (no atomics), and global average pool.
// Reference op: F.max_pool2d in the LeNet (/root/reference/model/model.py:16-17);
// ResNet stem max-pool 3x3 s2 p1 and the final global average pool.
#include "pdt_common.h"

namespace {
constexpr int NT = 256;

__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
  f[0] = lo_bf(v[0]); f[1] = hi_bf(v[0]); f[2] = lo_bf(v[1]); f[3] = hi_bf(v[1]);
  f[4] = lo_bf(v[2]); f[5] = hi_bf(v[2]); f[6] = lo_bf(v[3]); f[7] = hi_bf(v[3]);
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  return u32x4{pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7])};
}

// one thread = 8 channels of one output pixel. AFF: the input is a pre-BatchNorm
// conv output and every window element is first mapped through the BN affine
// + ReLU (relu(x * scale[c] + shift[c]), fp32) -- the ResNet stem's BN-apply
// pass and its full-resolution activation are never materialised.
template <bool AFF, typename IdxT>
__global__ void maxpool_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, uint8_t* __restrict__ idx,
                                   int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p,
                                   const float* __restrict__ scale, const float* __restrict__ shift) {
  const IdxT cpr = C / 8;
  const IdxT total = (IdxT)N * Ho * Wo * cpr;
  for (IdxT t = (IdxT)blockIdx.x * NT + threadIdx.x; t < total; t += (IdxT)gridDim.x * NT) {
    int cc = t % cpr;
    IdxT pix = t / cpr;
    int ow = pix % (IdxT)Wo;
    IdxT r = pix / (IdxT)Wo;
    int oh = r % (IdxT)Ho;
    int n = r / (IdxT)Ho;
    float best[8], sc[8], sh[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    if (AFF) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { sc[j] = scale[cc * 8 + j]; sh[j] = shift[cc * 8 + j]; }
    }
    auto take = [&](const u32x4 v, int w) __attribute__((always_inline)) {
      float f[8];
      unpack8(v, f);
      if (AFF) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j] * sc[j] + sh[j], 0.f);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (f[j] > best[j] || (f[j] != f[j])) { best[j] = f[j]; bi[j] = (uint8_t)w; }
    };
    if (k == 3) {
      // the ResNet stem's window: all 9 loads issued before the first is used (out-of-window
      // taps read the window's centre pixel and are skipped) -- a load under a per-tap
      // condition is branched around and waited for on its own
      const int ih0 = oh * s - p, iw0 = ow * s - p;
      const int ihc = min(max(ih0 + 1, 0), H - 1), iwc = min(max(iw0 + 1, 0), W - 1);
      u32x4 v[9];
#pragma unroll
      for (int w = 0; w < 9; ++w) {
        const int ih = ih0 + w / 3, iw = iw0 + w % 3;
        const bool ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        v[w] = *reinterpret_cast<const u32x4*>(x + (((IdxT)n * H + (ok ? ih : ihc)) * W + (ok ? iw : iwc)) * C + cc * 8);
      }
#pragma unroll
      for (int w = 0; w < 9; ++w) {
        const int ih = ih0 + w / 3, iw = iw0 + w % 3;
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) take(v[w], w);
      }
    } else {
      for (int kh = 0; kh < k; ++kh) {
        int ih = oh * s - p + kh;
        if ((unsigned)ih >= (unsigned)H) continue;
        for (int kw = 0; kw < k; ++kw) {
          int iw = ow * s - p + kw;
          if ((unsigned)iw >= (unsigned)W) continue;
          take(*reinterpret_cast<const u32x4*>(x + (((IdxT)n * H + ih) * W + iw) * C + cc * 8), kh * k + kw);
        }
      }
    }
    reinterpret_cast<u32x4*>(y)[t] = pack8(best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    reinterpret_cast<uint2*>(idx)[t] = packed;
  }
}

// gather: each input pixel sums the gradients of the windows whose argmax it is.
// Index math in IdxT: 32-bit when the tensor has < 2^31 chunks (the ResNet stem at
// batch 512 has 51M), since 64-bit division is a long software sequence per thread.
template <typename IdxT>
__global__ void maxpool_bwd_kernel(const u16* __restrict__ dy, const uint8_t* __restrict__ idx, u16* __restrict__ dx,
                                   int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p) {
  const IdxT cpr = C / 8;
  const IdxT total = (IdxT)N * H * W * cpr;
  for (IdxT t = (IdxT)blockIdx.x * NT + threadIdx.x; t < total; t += (IdxT)gridDim.x * NT) {
    int cc = t % cpr;
    IdxT pix = t / cpr;
    int w = pix % (IdxT)W;
    IdxT r = pix / (IdxT)W;
    int h = r % (IdxT)H;
    int n = r / (IdxT)H;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int oh_lo = (h + p - k + s) / s; if (h + p - k + 1 < 0) oh_lo = 0;
    int oh_hi = (h + p) / s;
    int ow_lo = (w + p - k + s) / s; if (w + p - k + 1 < 0) ow_lo = 0;
    int ow_hi = (w + p) / s;
    for (int oh = max(oh_lo, 0); oh <= min(oh_hi, Ho - 1); ++oh) {
      int kh = h + p - oh * s;
      if (kh < 0 || kh >= k) continue;
      for (int ow = max(ow_lo, 0); ow <= min(ow_hi, Wo - 1); ++ow) {
        int kw = w + p - ow * s;
        if (kw < 0 || kw >= k) continue;
        IdxT o = ((((IdxT)n * Ho + oh) * Wo + ow) * cpr + cc);
        uint2 bi = reinterpret_cast<const uint2*>(idx)[o];
        float g[8];
        unpack8(reinterpret_cast<const u32x4*>(dy)[o], g);
        const uint8_t me = (uint8_t)(kh * k + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          uint32_t word = j < 4 ? bi.x : bi.y;
          uint8_t b = (word >> (8 * (j & 3))) & 0xff;
          if (b == me) acc[j] += g[j];
        }
      }
    }
    reinterpret_cast<u32x4*>(dx)[t] = pack8(acc);
  }
}

// The ResNet stem's 3x3 / stride-2 / pad-1 pool. Input rows / cols 2a and 2a + 1 take their
// gradient from windows a and a + 1 only (2a: window a at offset 1; 2a + 1: window a at
// offset 2 and window a + 1 at offset 0), so one thread owns an input QUAD (2a..2a+1) x
// (2b..2b+1) x 8 channels: it reads the 4 windows (a..a+1) x (b..b+1) once and writes 4
// chunks -- no divergent window loops, ~2.2x fewer loads than the per-pixel gather. One
// workgroup per quad row (n, a). Windows are summed in the generic kernel's (oh, ow)
// order (bit-identical). CPR = C / 8.
template <int CPR>
__global__ void __launch_bounds__(NT) maxpool_bwd_k3s2_kernel(const u16* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx, u16* __restrict__ dx,
                                                              int H, int W, int Ho, int Wo) {
  const int Hq = (H + 1) >> 1, Wq = (W + 1) >> 1;
  const int n = blockIdx.x / Hq, a = blockIdx.x - n * Hq;
  for (int t = threadIdx.x; t < Wq * CPR; t += NT) {
    const int b = t / CPR, cc = t - b * CPR;
    // windows (a + i, b + j), i, j in {0, 1}; missing ones (past the last row / col) read as 0
    float g[2][2][8];
    uint32_t bi[2][2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = a + i < Ho && b + j < Wo;
        const size_t o = (((size_t)n * Ho + (ok ? a + i : a)) * Wo + (ok ? b + j : b)) * CPR + cc;
        const uint2 v = ok ? reinterpret_cast<const uint2*>(idx)[o] : uint2{0xffffffffu, 0xffffffffu};
        bi[i][j][0] = v.x;
        bi[i][j][1] = v.y;
        if (ok) {
          unpack8(reinterpret_cast<const u32x4*>(dy)[o], g[i][j]);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) g[i][j][e] = 0.f;
        }
      }
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const int h = 2 * a + dh;
      if (h >= H) break;
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int w = 2 * b + dw;
        if (w >= W) continue;
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (dh == 0 && i == 1) continue;  // row 2a: window a only
          const int kh = dh == 0 ? 1 : (i == 0 ? 2 : 0);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (dw == 0 && j == 1) continue;
            const int kw = dw == 0 ? 1 : (j == 0 ? 2 : 0);
            const uint32_t me = (uint32_t)(kh * 3 + kw);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (((bi[i][j][e >> 2] >> (8 * (e & 3))) & 0xffu) == me) acc[e] += g[i][j][e];
          }
        }
        reinterpret_cast<u32x4*>(dx)[(((size_t)n * H + h) * W + w) * CPR + cc] = pack8(acc);
      }
    }
  }
}

// The same k3 s2 p1 quad-gather backward for the ResNet stem, fused with the stem BatchNorm's
// backward REDUCTION: while dA is formed (and stored: the stem weight gradient reads it), each
// thread also reads y at the pixels it writes and accumulates, per channel,
//   s = sum g,  q = sum g * (y - mean),  g = dA (bf16 as stored) gated by relu(y*scale + shift)
// -- exactly bn_bwd_reduce_kernel's partials, without its second full read of dA. Grid-stride
// over quad rows; one partial row per workgroup (part[2][gridDim.x][64], pdt_bn_bwd_finalize).
__global__ void __launch_bounds__(NT) maxpool_bwd_k3s2_bnred_kernel(
    const u16* __restrict__ dy, const uint8_t* __restrict__ idx, u16* __restrict__ dx, const u16* __restrict__ yb,
    const float* __restrict__ mean, const float* __restrict__ scale, const float* __restrict__ shift,
    float* __restrict__ part, int N, int H, int W, int Ho, int Wo) {
  constexpr int CPR = 8;  // C = 64
  __shared__ float red[2][NT][8];
  const int Hq = (H + 1) >> 1, Wq = (W + 1) >> 1;
  const int cc = threadIdx.x % CPR;  // NT % CPR == 0: a thread's channel chunk is fixed
  float mu[8], sc[8], sh[8], s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = mean[cc * 8 + e];
    sc[e] = scale[cc * 8 + e];
    sh[e] = shift[cc * 8 + e];
    s[e] = q[e] = 0.f;
  }
  for (int row = blockIdx.x; row < N * Hq; row += gridDim.x) {
    const int n = row / Hq, a = row - n * Hq;
    for (int t = threadIdx.x; t < Wq * CPR; t += NT) {
      const int b = t / CPR;
      u32x4 gq[2][2];  // window gradients, packed (unpacked per use: fewer VGPRs, more waves)
      uint32_t bi[2][2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bool ok = a + i < Ho && b + j < Wo;
          const size_t o = (((size_t)n * Ho + (ok ? a + i : a)) * Wo + (ok ? b + j : b)) * CPR + cc;
          const uint2 v = ok ? reinterpret_cast<const uint2*>(idx)[o] : uint2{0xffffffffu, 0xffffffffu};
          bi[i][j][0] = v.x;
          bi[i][j][1] = v.y;
          gq[i][j] = ok ? reinterpret_cast<const u32x4*>(dy)[o] : u32x4{0u, 0u, 0u, 0u};
        }
      // y of the (up to) four pixels this item writes, loaded with the window reads (all loads
      // of the item in flight together: the kernel is load-latency bound)
      u32x4 yq[2][2];
#pragma unroll
      for (int dh = 0; dh < 2; ++dh)
#pragma unroll
        for (int dw = 0; dw < 2; ++dw) {
          const int h = 2 * a + dh, w = 2 * b + dw;
          yq[dh][dw] = (h < H && w < W) ? reinterpret_cast<const u32x4*>(yb)[(((size_t)n * H + h) * W + w) * CPR + cc]
                                        : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        const int h = 2 * a + dh;
        if (h >= H) break;
#pragma unroll
        for (int dw = 0; dw < 2; ++dw) {
          const int w = 2 * b + dw;
          if (w >= W) continue;
          float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            if (dh == 0 && i == 1) continue;
            const int kh = dh == 0 ? 1 : (i == 0 ? 2 : 0);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              if (dw == 0 && j == 1) continue;
              const int kw = dw == 0 ? 1 : (j == 0 ? 2 : 0);
              const uint32_t me = (uint32_t)(kh * 3 + kw);
              float g[8];
              unpack8(gq[i][j], g);
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (((bi[i][j][e >> 2] >> (8 * (e & 3))) & 0xffu) == me) acc[e] += g[e];
            }
          }
          const size_t po = (((size_t)n * H + h) * W + w) * CPR + cc;
          const u32x4 pk = pack8(acc);
          reinterpret_cast<u32x4*>(dx)[po] = pk;
          float gv[8], yv[8];
          unpack8(pk, gv);
          unpack8(yq[dh][dw], yv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gg = (yv[e] * sc[e] + sh[e]) > 0.f ? gv[e] : 0.f;
            s[e] += gg;
            q[e] += gg * (yv[e] - mu[e]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][threadIdx.x][e] = s[e];
    red[1][threadIdx.x][e] = q[e];
  }
  __syncthreads();
  if (threadIdx.x < 2 * 64) {  // (sum | sumsq) x 64 channels: thread = (half, channel)
    const int half = threadIdx.x >> 6, c = threadIdx.x & 63, ch = c >> 3, e = c & 7;
    float acc = 0.f;
    for (int t = ch; t < NT; t += CPR) acc += red[half][t][e];
    part[((size_t)half * gridDim.x + blockIdx.x) * 64 + c] = acc;
  }
}

// x [N][HW][C] -> y [N][C]  (bf16 out, fp32 sum)
__global__ void avgpool_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, int N, int HW, int C) {
  const int cpr = C / 8;
  int t = blockIdx.x * NT + threadIdx.x;
  if (t >= N * cpr) return;
  int n = t / cpr, cc = t % cpr;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < HW; ++i) {
    float f[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + ((long)n * HW + i) * C + cc * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f[j];
  }
  const float inv = 1.f / HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  reinterpret_cast<u32x4*>(y)[t] = pack8(acc);
}

__global__ void avgpool_bwd_kernel(const u16* __restrict__ dy, u16* __restrict__ dx, int N, int HW, int C) {
  const int cpr = C / 8;
  long total = (long)N * HW * cpr;
  const float inv = 1.f / HW;
  for (long t = (long)blockIdx.x * NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    int cc = t % cpr;
    long n = t / ((long)HW * cpr);
    float g[8];
    unpack8(reinterpret_cast<const u32x4*>(dy)[n * cpr + cc], g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= inv;
    reinterpret_cast<u32x4*>(dx)[t] = pack8(g);
  }
}

int grid_for(long n) {
  long b = (n + NT - 1) / NT;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}
}  // namespace

PDT_API int pdt_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int Ho, int Wo, int k,
                            int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255) return -1;
  long total = (long)N * Ho * Wo * (C / 8);
  if ((long)N * H * W * C < (1L << 31))  // 32-bit index math (element offsets of the input fit)
    hipLaunchKernelGGL((maxpool_fwd_kernel<false, uint32_t>), dim3(grid_for(total)), dim3(NT), 0, st, (const u16*)x,
                       (u16*)y, (uint8_t*)idx, N, H, W, C, Ho, Wo, k, s, p, nullptr, nullptr);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<false, long>), dim3(grid_for(total)), dim3(NT), 0, st, (const u16*)x,
                       (u16*)y, (uint8_t*)idx, N, H, W, C, Ho, Wo, k, s, p, nullptr, nullptr);
  PDT_RETURN_LAUNCH();
}

// max-pool of relu(x * scale + shift) (per-channel fp32 BN affine), argmax as above
PDT_API int pdt_maxpool_fwd_affine(const void* x, void* y, void* idx, const float* scale, const float* shift, int N,
                                   int H, int W, int C, int Ho, int Wo, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255 || !scale || !shift) return -1;
  long total = (long)N * Ho * Wo * (C / 8);
  if ((long)N * H * W * C < (1L << 31))  // 32-bit index math (element offsets of the input fit)
    hipLaunchKernelGGL((maxpool_fwd_kernel<true, uint32_t>), dim3(grid_for(total)), dim3(NT), 0, st, (const u16*)x,
                       (u16*)y, (uint8_t*)idx, N, H, W, C, Ho, Wo, k, s, p, scale, shift);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<true, long>), dim3(grid_for(total)), dim3(NT), 0, st, (const u16*)x,
                       (u16*)y, (uint8_t*)idx, N, H, W, C, Ho, Wo, k, s, p, scale, shift);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_maxpool_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                            int k, int s, int p, hipStream_t st) {
  if (C % 8) return -1;
  long total = (long)N * H * W * (C / 8);
  const char* e = getenv("PDT_MAXPOOL_BWD_ROW");  // "0": always the generic gather kernel (A/B, tests)
  const bool row_ok = !(e && e[0] == '0');
  if (row_ok && k == 3 && s == 2 && p == 1 && Ho == (H + 1) / 2 && Wo == (W + 1) / 2 && C == 64 &&
      (long)N * ((H + 1) / 2) < (1L << 31)) {
    hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel<8>, dim3(N * ((H + 1) / 2)), dim3(NT), 0, st, (const u16*)dy,
                       (const uint8_t*)idx, (u16*)dx, H, W, Ho, Wo);
    PDT_RETURN_LAUNCH();
  }
  if (total < (1L << 31))
    hipLaunchKernelGGL(maxpool_bwd_kernel<uint32_t>, dim3(grid_for(total)), dim3(NT), 0, st, (const u16*)dy,
                       (const uint8_t*)idx, (u16*)dx, N, H, W, C, Ho, Wo, k, s, p);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<long>, dim3(grid_for(total)), dim3(NT), 0, st, (const u16*)dy,
                       (const uint8_t*)idx, (u16*)dx, N, H, W, C, Ho, Wo, k, s, p);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_avgpool_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  int total = N * (C / 8);
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((total + NT - 1) / NT), dim3(NT), 0, st, (const u16*)x, (u16*)y, N,
                     HW, C);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_avgpool_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  long total = (long)N * HW * (C / 8);
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for(total)), dim3(NT), 0, st, (const u16*)dy, (u16*)dx, N, HW,
                     C);
  PDT_RETURN_LAUNCH();
}

// Stem max-pool backward (k3 s2 p1, 64 channels) fused with the stem BN backward reduction
// (see maxpool_bwd_k3s2_bnred_kernel): writes dx and part[2][blocks][64]; -5 when not covered.
PDT_API int pdt_maxpool_bwd_bnred(const void* dy, const void* idx, void* dx, const void* y, const float* mean,
                                  const float* scale, const float* shift, float* part, int N, int H, int W, int C,
                                  int Ho, int Wo, int blocks, hipStream_t st) {
  // (64-bit offsets: no element-count limit)
  if (C != 64 || Ho != (H + 1) / 2 || Wo != (W + 1) / 2 || blocks < 1 || (long)N * ((H + 1) / 2) >= (1L << 31))
    return -5;
  hipLaunchKernelGGL(maxpool_bwd_k3s2_bnred_kernel, dim3(blocks), dim3(NT), 0, st, (const u16*)dy, (const uint8_t*)idx,
                     (u16*)dx, (const u16*)y, mean, scale, shift, part, N, H, W, Ho, Wo);
  PDT_RETURN_LAUNCH();
}
