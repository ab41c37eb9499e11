// LayerNorm (bf16 in/out, fp32 statistics) and GELU(tanh) backward for the
// ViT-B/16 path (BASELINE config #5).
//
// Forward: one wave64 per row; each lane owns D/256 chunks of four bf16
// (8-byte loads), row mean / rstd by wave shuffles; y = (x-mean)*rstd*g + b.
// Backward: same row mapping; dx = rstd * (dxhat - mean(dxhat) - xhat*mean(dxhat*xhat)),
// dxhat = dy*g; per-block column partials of (dy*xhat, dy) are written to a
// [2][blocks][D] buffer and summed by a second, deterministic pass.
#include "pdt_common.h"

namespace {

constexpr int WPB = 4;  // waves (rows) per block

__device__ __forceinline__ void ld4(const u16* p, float* f) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
}
__device__ __forceinline__ void st4(u16* p, const float* f) {
  uint2 v;
  v.x = pack2bf(f[0], f[1]);
  v.y = pack2bf(f[2], f[3]);
  *reinterpret_cast<uint2*>(p) = v;
}

// F8: also write the e4m3 codes of the (bf16-rounded) output with the delayed scale
// meta[0] of the consuming fp8 GEMM, and the block's |y| max to amax_part[blockIdx.x]
// (rolled into that GEMM's amax history by pdt_fp8_meta_roll_partial) -- the
// activation-quantisation pass of the fp8 path folded into the producer.
template <int CH, bool F8 = false>  // chunks of 4 per lane: D = 256*CH
__global__ void __launch_bounds__(64 * WPB) ln_fwd_kernel(const u16* __restrict__ x, const float* __restrict__ g,
                                                          const float* __restrict__ b, u16* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int rows, float eps, uint8_t* __restrict__ q8 = nullptr,
                                                          const float* __restrict__ meta = nullptr,
                                                          float* __restrict__ amax_part = nullptr,
                                                          const u16* __restrict__ radd = nullptr,
                                                          u16* __restrict__ xsum = nullptr) {
  const int lane = threadIdx.x & 63;
  int row = blockIdx.x * WPB + (threadIdx.x >> 6);
  __shared__ float red[WPB];
  if (!F8 && row >= rows) return;
  // F8: a wave past the last row recomputes row rows-1 (same values) so every wave
  // reaches the block's amax barrier; its stores are the same bytes as that row's
  if (F8 && row >= rows) row = rows - 1;
  float amax = 0.f;
  constexpr int D = 256 * CH;
  const u16* xr = x + (long)row * D;
  float v[CH][4];
  float s = 0.f;
  // all of the row's x (and residual) chunks are loaded before any is used, each path in one
  // block: with the residual branch inside the chunk loop (or between the x and r loads) hipcc
  // waited for the x loads before issuing the r loads
  uint2 xw[CH], rw[CH];
  if (radd != nullptr) {  // residual add of a pre-norm block: xsum = bf16(x + r), normalised
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      xw[c] = *reinterpret_cast<const uint2*>(xr + (c * 64 + lane) * 4);
      rw[c] = *reinterpret_cast<const uint2*>(radd + (long)row * D + (c * 64 + lane) * 4);
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const float r[4] = {lo_bf(rw[c].x), hi_bf(rw[c].x), lo_bf(rw[c].y), hi_bf(rw[c].y)};
      const float xv[4] = {lo_bf(xw[c].x), hi_bf(xw[c].x), lo_bf(xw[c].y), hi_bf(xw[c].y)};
#pragma unroll
      for (int e = 0; e < 4; ++e) v[c][e] = bf2f(f2bf(xv[e] + r[e]));
      st4(xsum + (long)row * D + (c * 64 + lane) * 4, v[c]);
    }
  } else {
#pragma unroll
    for (int c = 0; c < CH; ++c) xw[c] = *reinterpret_cast<const uint2*>(xr + (c * 64 + lane) * 4);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      v[c][0] = lo_bf(xw[c].x); v[c][1] = hi_bf(xw[c].x);
      v[c][2] = lo_bf(xw[c].y); v[c][3] = hi_bf(xw[c].y);
    }
  }
#pragma unroll
  for (int c = 0; c < CH; ++c) s += v[c][0] + v[c][1] + v[c][2] + v[c][3];
  const float mean = warp_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[c][e] - mean;
      q = fmaf(d, d, q);  // (explicit: hipcc contracted some of these per instantiation, not all)
    }
  const float rstd = rsqrtf(fmaf(warp_sum(q), 1.f / D, eps));
  u16* yr = y + (long)row * D;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 64 + lane) * 4;
    f32x4 gg = *reinterpret_cast<const f32x4*>(g + col);
    f32x4 bb = *reinterpret_cast<const f32x4*>(b + col);
    float o[4];
#pragma unroll
    // (explicit fma: every instantiation rounds alike, whatever hipcc would contract)
    for (int e = 0; e < 4; ++e) o[e] = fmaf((v[c][e] - mean) * rstd, gg[e], bb[e]);
    if (!F8 || y != nullptr) st4(yr + col, o);  // (F8: y == nullptr -- the codes are the only consumer's input)
    if (F8) {
      const float s = meta[0];
      float r[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        r[e] = bf2f(f2bf(o[e]));  // quantise exactly what the bf16 output holds
        amax = fmaxf(amax, fabsf(r[e]));
      }
      *reinterpret_cast<uint32_t*>(q8 + (long)row * D + col) = pdt_cvt4_f8<0>(r[0] * s, r[1] * s, r[2] * s, r[3] * s);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  if (F8) {
    amax = warp_max(amax);
    if (lane == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    if (threadIdx.x == 0) {
      float m = red[0];
#pragma unroll
      for (int w = 1; w < WPB; ++w) m = fmaxf(m, red[w]);
      amax_part[blockIdx.x] = m;
    }
  }
}

// F8: also write the e5m2 codes of dx (bf16-rounded) with the delayed scale q8_meta[0]
// of the fp8 GEMM that consumes this gradient, and the block's max |dx| to
// q8_part[blockIdx.x] (the e5m2 quantisation pass of that GEMM folded in here).
template <int CH, bool F8 = false>
__global__ void __launch_bounds__(64 * WPB) ln_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ x,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in, u16* __restrict__ dx,
                                                          float* __restrict__ part, int rows, int rows_per_block,
                                                          const u16* __restrict__ addend,
                                                          uint8_t* __restrict__ q8 = nullptr,
                                                          const float* __restrict__ q8_meta = nullptr,
                                                          float* __restrict__ q8_part = nullptr,
                                                          float* __restrict__ cpart = nullptr) {
  // cpart (optional): per-block column sums of dx as stored (bf16) -> cpart[blockIdx.x][D]: the
  // bias gradient of the layer whose output gradient dx is, formed where dx is written
  constexpr int D = 256 * CH;
  __shared__ float red[2][WPB][D];
  __shared__ float q8red[WPB];
  float q8max = 0.f;
  const float q8s = F8 ? q8_meta[0] : 0.f;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float dg[CH][4], db[CH][4], cs[CH][4];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) dg[c][e] = db[c][e] = cs[c][e] = 0.f;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  // Rows are software-pipelined: the next row's operands are loaded at the top of this row's
  // iteration and stay in flight through its arithmetic and stores. The empty asm with the
  // loaded registers as "+v" operands is the one wait per row: after it every use sees plain
  // registers, so hipcc does not fold the in-flight next-row loads into a later wait (with
  // loads and stores both pending it waits for zero -- which, at a wait for this row's data
  // placed after the prefetch, would have drained the prefetch too).
  uint2 nx[CH], ndy[CH], nad[CH];
  float nmean = 0.f, nrstd = 0.f;
  // (without an addend the third stream re-reads dy -- a valid address, its values unused --
  // so the prefetch is one branch-free block of loads)
  const u16* aptr = addend != nullptr ? addend : dy;
  auto fetch = [&](int rr) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const long off = (long)rr * D + (c * 64 + lane) * 4;
      nx[c] = *reinterpret_cast<const uint2*>(x + off);
      ndy[c] = *reinterpret_cast<const uint2*>(dy + off);
      nad[c] = *reinterpret_cast<const uint2*>(aptr + off);
    }
    nmean = mean_in[rr];
    nrstd = rstd_in[rr];
  };
  // gamma is per column: loaded once (a load issued after the prefetch and waited for inside
  // the row would retire the prefetch with it -- vmcnt counts in order)
  f32x4 gv[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) gv[c] = *reinterpret_cast<const f32x4*>(g + (c * 64 + lane) * 4);
  if (r0 + w < r1) fetch(r0 + w);
  for (int row = r0 + w; row < r1; row += WPB) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("" : "+v"(nx[c]), "+v"(ndy[c]), "+v"(nad[c])::"memory");
    asm volatile("" : "+v"(nmean), "+v"(nrstd)::"memory");
    uint2 cx[CH], cdy[CH], cad[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      cx[c] = nx[c];
      cdy[c] = ndy[c];
      cad[c] = nad[c];
    }
    const float mean = nmean, rstd = nrstd;
    if (row + WPB < r1) fetch(row + WPB);
    float xh[CH][4], gy[CH][4], ad[CH][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const float xv[4] = {lo_bf(cx[c].x), hi_bf(cx[c].x), lo_bf(cx[c].y), hi_bf(cx[c].y)};
      const float dv[4] = {lo_bf(cdy[c].x), hi_bf(cdy[c].x), lo_bf(cdy[c].y), hi_bf(cdy[c].y)};
      ad[c][0] = lo_bf(cad[c].x); ad[c][1] = hi_bf(cad[c].x);
      ad[c][2] = lo_bf(cad[c].y); ad[c][3] = hi_bf(cad[c].y);
      const f32x4 gg = gv[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[c][e] = (xv[e] - mean) * rstd;
        gy[c][e] = dv[e] * gg[e];
        s1 += gy[c][e];
        s2 += gy[c][e] * xh[c][e];
        dg[c][e] += dv[e] * xh[c][e];
        db[c][e] += dv[e];
      }
    }
    const float m1 = warp_sum(s1) * (1.f / D), m2 = warp_sum(s2) * (1.f / D);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = rstd * (gy[c][e] - m1 - xh[c][e] * m2);
      if (addend != nullptr) {  // residual-branch gradient of the same tensor: dx += addend
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] += ad[c][e];
      }
      st4(dx + (long)row * D + (c * 64 + lane) * 4, o);
      if (cpart != nullptr) {
#pragma unroll
        for (int e = 0; e < 4; ++e) cs[c][e] += bf2f(f2bf(o[e]));
      }
      if (F8) {
        float r[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          r[e] = bf2f(f2bf(o[e]));  // quantise exactly what the bf16 gradient holds
          q8max = fmaxf(q8max, fabsf(r[e]));
        }
        *reinterpret_cast<uint32_t*>(q8 + (long)row * D + (c * 64 + lane) * 4) =
            pdt_cvt4_f8<1>(r[0] * q8s, r[1] * q8s, r[2] * q8s, r[3] * q8s);
      }
    }
  }
  if (F8) {
    q8max = warp_max(q8max);
    if (lane == 0) q8red[w] = q8max;
  }
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[0][w][(c * 64 + lane) * 4 + e] = dg[c][e];
      red[1][w][(c * 64 + lane) * 4 + e] = db[c][e];
    }
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += 64 * WPB) {
    float a = 0.f, bsum = 0.f;
#pragma unroll
    for (int k = 0; k < WPB; ++k) {
      a += red[0][k][col];
      bsum += red[1][k][col];
    }
    part[(long)blockIdx.x * D + col] = a;
    part[(long)(gridDim.x + blockIdx.x) * D + col] = bsum;
  }
  if (cpart != nullptr) {
    __syncthreads();  // red[0] is read above
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[0][w][(c * 64 + lane) * 4 + e] = cs[c][e];
    __syncthreads();
    for (int col = threadIdx.x; col < D; col += 64 * WPB) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < WPB; ++k) a += red[0][k][col];
      cpart[(long)blockIdx.x * D + col] = a;
    }
  }
  if (F8 && threadIdx.x == 0) {  // q8red was written before the barrier above
    float m = q8red[0];
#pragma unroll
    for (int k = 1; k < WPB; ++k) m = fmaxf(m, q8red[k]);
    q8_part[blockIdx.x] = m;
  }
}

// out[c] (+)= sum_r part[r][c]  for the two halves (dgamma, dbeta);
// 1024 threads = 64 columns x 16 row groups, 8 rows per trip with every load issued
// before the adds (12 workgroups for D = 768: latency, not bandwidth, bounds this),
// combined through LDS in a fixed order.
constexpr int CS_RG = 16;
__global__ void __launch_bounds__(64 * CS_RG) colsum_f32_kernel(const float* __restrict__ part, float* __restrict__ dg,
                                                                float* __restrict__ db, int R, int D, int accumulate) {
  __shared__ float sa[CS_RG][64], sb[CS_RG][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float a = 0.f, b = 0.f;
  if (c < D) {
    int r = rg;
    for (; r + 7 * CS_RG < R; r += 8 * CS_RG) {
      float x[8], y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        x[u] = part[(long)(r + u * CS_RG) * D + c];
        y[u] = part[(long)(R + r + u * CS_RG) * D + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a += x[u];
        b += y[u];
      }
    }
    for (; r < R; r += CS_RG) {
      a += part[(long)r * D + c];
      b += part[(long)(R + r) * D + c];
    }
  }
  sa[rg][cl] = a;
  sb[rg][cl] = b;
  __syncthreads();
  if (rg == 0 && c < D) {
    a = 0.f;
    b = 0.f;
#pragma unroll
    for (int g = 0; g < CS_RG; ++g) {
      a += sa[g][cl];
      b += sb[g][cl];
    }
    dg[c] = accumulate ? dg[c] + a : a;
    db[c] = accumulate ? db[c] + b : b;
  }
}

// GELU (tanh approximation) backward: dz = dy * gelu'(z)
__global__ void gelu_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ z, u16* __restrict__ dz,
                                long n8) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    u32x4 a = reinterpret_cast<const u32x4*>(dy)[i], b = reinterpret_cast<const u32x4*>(z)[i], o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float r[2];
      float gv[2] = {lo_bf(a[k]), hi_bf(a[k])}, zv[2] = {lo_bf(b[k]), hi_bf(b[k])};
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float x = zv[e];
        const float u = 0.7978845608f * (x + 0.044715f * x * x * x);
        const float t = pdt_tanh(u);
        const float du = 0.7978845608f * (1.f + 3.f * 0.044715f * x * x);
        r[e] = gv[e] * (0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du);
      }
      o[k] = pack2bf(r[0], r[1]);
    }
    reinterpret_cast<u32x4*>(dz)[i] = o;
  }
}

}  // namespace

PDT_API int pdt_ln_fwd(const void* x, const float* g, const float* b, void* y, float* mean, float* rstd, int rows,
                       int D, float eps, hipStream_t st) {
  dim3 grid((rows + WPB - 1) / WPB), blk(64 * WPB);
  switch (D) {
    case 256: hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, blk, 0, st, (const u16*)x, g, b, (u16*)y, mean, rstd, rows, eps); break;
    case 512: hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, blk, 0, st, (const u16*)x, g, b, (u16*)y, mean, rstd, rows, eps); break;
    case 768: hipLaunchKernelGGL(ln_fwd_kernel<3>, grid, blk, 0, st, (const u16*)x, g, b, (u16*)y, mean, rstd, rows, eps); break;
    case 1024: hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, blk, 0, st, (const u16*)x, g, b, (u16*)y, mean, rstd, rows, eps); break;
    default: return -1;
  }
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_fp8_meta_roll_partial(float* meta, const float* partial, int nblk, int fmt, float* dq_out,
                                      hipStream_t st);

PDT_API int pdt_ln_fwd_f8_blocks(int rows) { return (rows + WPB - 1) / WPB; }

// LayerNorm of xsum = bf16(x + r) (written to xsum): the residual add of a pre-norm block moved
// out of the producing GEMM's epilogue (so a library GEMM can produce x). q (optional, with
// meta / amax_part / dq_out as pdt_ln_fwd_f8): the e4m3 codes of the output as well; with q,
// y may be null (codes only: the consuming fp8 GEMM reads nothing else).
PDT_API int pdt_ln_add_fwd(const void* x, const void* r, void* xsum, const float* g, const float* b, void* y,
                           float* mean, float* rstd, int rows, int D, float eps, void* q, float* meta,
                           float* amax_part, float* dq_out, hipStream_t st) {
  if (!r || !xsum || (q && (!meta || !amax_part)) || (!q && !y)) return -1;
  const int nb = (rows + WPB - 1) / WPB;
  dim3 grid(nb), blk(64 * WPB);
#define LA(CH_, F_) hipLaunchKernelGGL((ln_fwd_kernel<CH_, F_>), grid, blk, 0, st, (const u16*)x, g, b, (u16*)y, mean, \
                                       rstd, rows, eps, (uint8_t*)q, (const float*)meta, amax_part, (const u16*)r,   \
                                       (u16*)xsum)
  if (q) {
    switch (D) {
      case 256: LA(1, true); break;
      case 512: LA(2, true); break;
      case 768: LA(3, true); break;
      case 1024: LA(4, true); break;
      default: return -1;
    }
  } else {
    switch (D) {
      case 256: LA(1, false); break;
      case 512: LA(2, false); break;
      case 768: LA(3, false); break;
      case 1024: LA(4, false); break;
      default: return -1;
    }
  }
#undef LA
  int e = (int)hipGetLastError();
  if (e || !q) return e;
  return pdt_fp8_meta_roll_partial(meta, amax_part, nb, 0, dq_out, st);
}

// LayerNorm forward that also emits the e4m3 codes of its output for the next fp8 GEMM
// (delayed scale meta[0]) and rolls that GEMM's amax history; amax_part holds
// pdt_ln_fwd_f8_blocks(rows) floats; dq_out receives the codes' dequant factor. y may be null
// (codes only).
PDT_API int pdt_ln_fwd_f8(const void* x, const float* g, const float* b, void* y, float* mean, float* rstd, int rows,
                          int D, float eps, void* q, float* meta, float* amax_part, float* dq_out, hipStream_t st) {
  const int nb = (rows + WPB - 1) / WPB;
  dim3 grid(nb), blk(64 * WPB);
#define LF(CH_) hipLaunchKernelGGL((ln_fwd_kernel<CH_, true>), grid, blk, 0, st, (const u16*)x, g, b, (u16*)y, mean, \
                                   rstd, rows, eps, (uint8_t*)q, (const float*)meta, amax_part)
  switch (D) {
    case 256: LF(1); break;
    case 512: LF(2); break;
    case 768: LF(3); break;
    case 1024: LF(4); break;
    default: return -1;
  }
#undef LF
  int e = (int)hipGetLastError();
  if (e) return e;
  return pdt_fp8_meta_roll_partial(meta, amax_part, nb, 0, dq_out, st);
}

// rows per LayerNorm-backward block: 64, doubled until at most PDT_LN_BWD_MAXB (512) blocks
static int ln_rows_per_block(int rows) {
  static int maxb = -1;
  if (maxb < 0) {
    const char* e = getenv("PDT_LN_BWD_MAXB");
    maxb = e ? atoi(e) : 512;
    if (maxb < 64) maxb = 512;
  }
  int rpb = 64;
  while ((rows + rpb - 1) / rpb > maxb) rpb *= 2;
  return rpb;
}

PDT_API int pdt_ln_bwd_blocks(int rows) {
  int rpb = ln_rows_per_block(rows);
  int b = (rows + rpb - 1) / rpb;
  return b < 1 ? 1 : b;
}

// addend (optional, bf16 [rows][D]): dx = LN backward + addend (a residual branch's
// gradient of the same input, summed in the same pass)
PDT_API int pdt_ln_bwd(const void* dy, const void* x, const float* g, const float* mean, const float* rstd, void* dx,
                       float* dg, float* db, float* part, int rows, int D, int accumulate, const void* addend,
                       hipStream_t st) {
  const int blocks = pdt_ln_bwd_blocks(rows);
  const int rpb = ln_rows_per_block(rows);
  dim3 grid(blocks), blk(64 * WPB);
  const u16 *DY = (const u16*)dy, *X = (const u16*)x;
  u16* DX = (u16*)dx;
  const u16* AD = (const u16*)addend;
  switch (D) {
    case 256: hipLaunchKernelGGL(ln_bwd_kernel<1>, grid, blk, 0, st, DY, X, g, mean, rstd, DX, part, rows, rpb, AD); break;
    case 512: hipLaunchKernelGGL(ln_bwd_kernel<2>, grid, blk, 0, st, DY, X, g, mean, rstd, DX, part, rows, rpb, AD); break;
    case 768: hipLaunchKernelGGL(ln_bwd_kernel<3>, grid, blk, 0, st, DY, X, g, mean, rstd, DX, part, rows, rpb, AD); break;
    case 1024: hipLaunchKernelGGL(ln_bwd_kernel<4>, grid, blk, 0, st, DY, X, g, mean, rstd, DX, part, rows, rpb, AD); break;
    default: return -1;
  }
  int e = (int)hipGetLastError();
  if (e) return e;
  hipLaunchKernelGGL(colsum_f32_kernel, dim3((D + 63) / 64), dim3(64 * CS_RG), 0, st, part, dg, db, blocks, D,
                     accumulate);
  PDT_RETURN_LAUNCH();
}

// LayerNorm backward that also emits the e5m2 codes of dx for the fp8 GEMM consuming that
// gradient (delayed scale q8_meta[0]), rolls its amax history and writes the codes'
// dequant factor to q8_dq; q8_part holds pdt_ln_bwd_blocks(rows) floats.
PDT_API int pdt_ln_bwd_f8(const void* dy, const void* x, const float* g, const float* mean, const float* rstd,
                          void* dx, float* dg, float* db, float* part, int rows, int D, int accumulate,
                          const void* addend, void* q8, float* q8_meta, float* q8_part, float* q8_dq, hipStream_t st) {
  const int blocks = pdt_ln_bwd_blocks(rows);
  const int rpb = ln_rows_per_block(rows);
  dim3 grid(blocks), blk(64 * WPB);
  const u16 *DY = (const u16*)dy, *X = (const u16*)x;
  u16* DX = (u16*)dx;
  const u16* AD = (const u16*)addend;
  uint8_t* Q = (uint8_t*)q8;
#define LB8(CH_) hipLaunchKernelGGL((ln_bwd_kernel<CH_, true>), grid, blk, 0, st, DY, X, g, mean, rstd, DX, part, rows, \
                                    rpb, AD, Q, (const float*)q8_meta, q8_part)
  switch (D) {
    case 256: LB8(1); break;
    case 512: LB8(2); break;
    case 768: LB8(3); break;
    case 1024: LB8(4); break;
    default: return -1;
  }
#undef LB8
  int e = (int)hipGetLastError();
  if (e) return e;
  hipLaunchKernelGGL(colsum_f32_kernel, dim3((D + 63) / 64), dim3(64 * CS_RG), 0, st, part, dg, db, blocks, D,
                     accumulate);
  return pdt_fp8_meta_roll_partial(q8_meta, q8_part, blocks, 1, q8_dq, st);
}

PDT_API int pdt_wgrad_reduce_rows(const float* rows, float* out, int nrows, int n, float scale, int accumulate,
                                  float* work, hipStream_t stream);
PDT_API long pdt_reduce_rows_work(int nrows, int n);

// pdt_ln_bwd_f8 + the column sums of dx (bf16 as stored) into bias_out [D] (= or += with
// bias_acc): the bias gradient of the fp8 layer that produced the LayerNorm's input, so its
// weight-gradient kernel does not re-read dx for it. cpart: pdt_ln_bwd_blocks(rows) * D floats
// + pdt_reduce_rows_work(pdt_ln_bwd_blocks(rows), D) behind them (the reduce's workspace).
PDT_API int pdt_ln_bwd_f8_db(const void* dy, const void* x, const float* g, const float* mean, const float* rstd,
                             void* dx, float* dg, float* db, float* part, int rows, int D, int accumulate,
                             const void* addend, void* q8, float* q8_meta, float* q8_part, float* q8_dq,
                             float* cpart, float* bias_out, int bias_acc, hipStream_t st) {
  if (!cpart || !bias_out) return -1;
  const int blocks = pdt_ln_bwd_blocks(rows);
  const int rpb = ln_rows_per_block(rows);
  dim3 grid(blocks), blk(64 * WPB);
  const u16 *DY = (const u16*)dy, *X = (const u16*)x;
  u16* DX = (u16*)dx;
  const u16* AD = (const u16*)addend;
  uint8_t* Q = (uint8_t*)q8;
#define LB8(CH_) hipLaunchKernelGGL((ln_bwd_kernel<CH_, true>), grid, blk, 0, st, DY, X, g, mean, rstd, DX, part, rows, \
                                    rpb, AD, Q, (const float*)q8_meta, q8_part, cpart)
  switch (D) {
    case 256: LB8(1); break;
    case 512: LB8(2); break;
    case 768: LB8(3); break;
    case 1024: LB8(4); break;
    default: return -1;
  }
#undef LB8
  int e = (int)hipGetLastError();
  if (e) return e;
  hipLaunchKernelGGL(colsum_f32_kernel, dim3((D + 63) / 64), dim3(64 * CS_RG), 0, st, part, dg, db, blocks, D,
                     accumulate);
  e = pdt_wgrad_reduce_rows(cpart, bias_out, blocks, D, 1.f, bias_acc, cpart + (long)blocks * D, st);
  if (e) return e;
  return pdt_fp8_meta_roll_partial(q8_meta, q8_part, blocks, 1, q8_dq, st);
}

PDT_API int pdt_gelu_bwd(const void* dy, const void* z, void* dz, long n, hipStream_t st) {
  if (n % 8) return -1;
  long n8 = n / 8;
  long b = (n8 + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3((int)b), dim3(256), 0, st, (const u16*)dy, (const u16*)z, (u16*)dz, n8);
  PDT_RETURN_LAUNCH();
}
