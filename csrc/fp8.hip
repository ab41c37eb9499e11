// FP8 (OCP e4m3fn / e5m2) quantization for the fp8 GEMM path with per-tensor
// "current" scaling, no host round trip:
//
//   pdt_amax_partial : grid-stride |x| max -> partial[nblk]   (no atomics, no memset)
//   pdt_cast_fp8     : every block re-reduces the <= 1024 partials (4 KB, L2),
//                      scale = FP8_MAX / amax, writes q = sat(x * scale) as fp8
//                      and block 0 writes dq = 1 / scale (the GEMM epilogue's
//                      dequant factor); optional [R][C] -> [C][R] transpose
//                      (weights for the dgrad GEMM) through a 64x64 LDS tile.
//
// The conversions are the gfx950 packed converts v_cvt_pk_fp8_f32 /
// v_cvt_pk_bf8_f32 (round to nearest even); inputs are clamped to the format's
// finite range first, so nothing overflows to NaN.
#include <cstdlib>
#include <mutex>

#include "pdt_common.h"

namespace {

constexpr int AMAX_BLOCKS = 1024;

template <bool BF16>
__device__ __forceinline__ float ld(const void* p, long i) {
  if (BF16) return bf2f(reinterpret_cast<const u16*>(p)[i]);
  return reinterpret_cast<const float*>(p)[i];
}

template <bool BF16>
__global__ void __launch_bounds__(256) amax_partial_kernel(const void* __restrict__ x, long n,
                                                           float* __restrict__ partial) {
  __shared__ float red[4];
  float m = 0.f;
  const long stride = (long)gridDim.x * 256 * 8;
  for (long base = ((long)blockIdx.x * 256 + threadIdx.x) * 8; base < n; base += stride) {
    if (BF16 && base + 8 <= n) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const u16*>(x) + base);
#pragma unroll
      for (int e = 0; e < 4; ++e) m = fmaxf(m, fmaxf(fabsf(lo_bf(v[e])), fabsf(hi_bf(v[e]))));
    } else {
      for (long i = base; i < base + 8 && i < n; ++i) m = fmaxf(m, fabsf(ld<BF16>(x, i)));
    }
  }
  m = warp_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// amax from the partials; every thread of the block gets it
__device__ __forceinline__ float block_amax(const float* __restrict__ partial, int nblk) {
  __shared__ float red[16];  // up to 1024 threads
  float m = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
  const int B = blockDim.x;
  int i = threadIdx.x;
  for (; i + 3 * B < nblk; i += 4 * B) {  // four independent loads in flight
    m = fmaxf(m, partial[i]);
    m1 = fmaxf(m1, partial[i + B]);
    m2 = fmaxf(m2, partial[i + 2 * B]);
    m3 = fmaxf(m3, partial[i + 3 * B]);
  }
  for (; i < nblk; i += B) m = fmaxf(m, partial[i]);
  m = fmaxf(fmaxf(m, m1), fmaxf(m2, m3));
  m = warp_max(m);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float r = red[0];
  for (int w = 1; w < (B + 63) / 64; ++w) r = fmaxf(r, red[w]);
  return r;
}

template <int FMT>
__device__ __forceinline__ uint32_t cvt4(float a, float b, float c, float d) {
  return pdt_cvt4_f8<FMT>(a, b, c, d);
}

template <int FMT>
__device__ __forceinline__ float scale_from(float amax) {
  constexpr float FMAX = FMT == 0 ? 448.f : 57344.f;
  return amax > 0.f ? FMAX / amax : 1.f;
}

template <bool BF16, int FMT>
__global__ void __launch_bounds__(256) cast_fp8_kernel(const void* __restrict__ x, long n,
                                                       const float* __restrict__ partial, int nblk,
                                                       uint8_t* __restrict__ q, float* __restrict__ dq) {
  const float s = scale_from<FMT>(block_amax(partial, nblk));
  if (blockIdx.x == 0 && threadIdx.x == 0) dq[0] = 1.f / s;
  const long stride = (long)gridDim.x * 256 * 8;
  for (long base = ((long)blockIdx.x * 256 + threadIdx.x) * 8; base < n; base += stride) {
    float v[8];
    if (BF16 && base + 8 <= n) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(reinterpret_cast<const u16*>(x) + base);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = lo_bf(w[e]);
        v[2 * e + 1] = hi_bf(w[e]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = base + e < n ? ld<BF16>(x, base + e) : 0.f;
    }
    if (base + 8 <= n) {
      uint2 o;
      o.x = cvt4<FMT>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
      o.y = cvt4<FMT>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
      *reinterpret_cast<uint2*>(q + base) = o;
    } else {
      for (long i = base; i < n; ++i) q[i] = (uint8_t)(cvt4<FMT>(v[i - base] * s, 0.f, 0.f, 0.f) & 0xff);
    }
  }
}

// [R][C] fp32 -> fp8 [C][R] with the tensor's scale (64x64 tiles, 256 threads).
// q_rows (optional): the same codes in [R][C] layout from the same tile (one read of the
// fp32 weight for both the forward and the data-gradient operand), dq: 1 / scale.
template <int FMT>
__global__ void __launch_bounds__(256) cast_fp8_t_kernel(const float* __restrict__ x, int R, int C,
                                                         const float* __restrict__ partial, int nblk,
                                                         uint8_t* __restrict__ q, uint8_t* __restrict__ q_rows = nullptr,
                                                         float* __restrict__ dq = nullptr) {
  __shared__ float tile[64][65];
  const float s = scale_from<FMT>(block_amax(partial, nblk));
  if (dq != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) dq[0] = 1.f / s;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? x[(long)r * C + c] * s : 0.f;
  }
  __syncthreads();
  if (q_rows != nullptr) {  // [R][C] codes: row r0 + i, 4-byte groups of columns
    for (int i = threadIdx.x; i < 64 * 16; i += 256) {
      const int rr = i >> 4, g = (i & 15) * 4;
      const int r = r0 + rr, c = c0 + g;
      if (r < R && c + 3 < C) {
        *reinterpret_cast<uint32_t*>(q_rows + (long)r * C + c) =
            cvt4<FMT>(tile[rr][g], tile[rr][g + 1], tile[rr][g + 2], tile[rr][g + 3]);
      } else if (r < R) {
        for (int e = 0; e < 4 && c + e < C; ++e)
          q_rows[(long)r * C + c + e] = (uint8_t)(cvt4<FMT>(tile[rr][g + e], 0.f, 0.f, 0.f) & 0xff);
      }
    }
  }
  // out row = c (64 of them), 64 bytes each: thread -> (row, 4-byte group)
  for (int i = threadIdx.x; i < 64 * 16; i += 256) {
    const int oc = i >> 4, g = (i & 15) * 4;
    const int c = c0 + oc, r = r0 + g;
    if (c < C && r + 3 < R) {
      *reinterpret_cast<uint32_t*>(q + (long)c * R + r) =
          cvt4<FMT>(tile[g][oc], tile[g + 1][oc], tile[g + 2][oc], tile[g + 3][oc]);
    } else if (c < C) {
      for (int e = 0; e < 4 && r + e < R; ++e)
        q[(long)c * R + r + e] = (uint8_t)(cvt4<FMT>(tile[g + e][oc], 0.f, 0.f, 0.f) & 0xff);
    }
  }
}

// ---------------------------------------------------------------------------
// Delayed scaling (one pass): quantize with the scale derived from an amax
// history, record this tensor's amax for the next steps. Per-tensor state
// (fp32 words):
//   [0] scale in use         [1] dq of the LAST cast (1/scale, read by the GEMM)
//   [2] amax of this cast    (uint bits, atomicMax; non-negative floats order as uints)
//   [3] unused               [4] history index     [5 .. 5+H) amax history
// A one-block roll kernel then moves [2] into the history and sets the next scale.
constexpr int HIST = 16;

template <bool BF16, int FMT>
__global__ void __launch_bounds__(256) cast_fp8_delayed_kernel(const void* __restrict__ x, long n,
                                                               float* __restrict__ meta, uint8_t* __restrict__ q) {
  __shared__ float red[4];
  const float s = meta[0];
  float m = 0.f;
  const long stride = (long)gridDim.x * 256 * 8;
  for (long base = ((long)blockIdx.x * 256 + threadIdx.x) * 8; base < n; base += stride) {
    float v[8];
    if (BF16 && base + 8 <= n) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(reinterpret_cast<const u16*>(x) + base);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = lo_bf(w[e]);
        v[2 * e + 1] = hi_bf(w[e]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = base + e < n ? ld<BF16>(x, base + e) : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
    if (base + 8 <= n) {
      uint2 o;
      o.x = cvt4<FMT>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
      o.y = cvt4<FMT>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
      *reinterpret_cast<uint2*>(q + base) = o;
    } else {
      for (long i = base; i < n; ++i) q[i] = (uint8_t)(cvt4<FMT>(v[i - base] * s, 0.f, 0.f, 0.f) & 0xff);
    }
  }
  m = warp_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(reinterpret_cast<unsigned int*>(meta) + 2, __float_as_uint(bm));  // order-free -> deterministic
  }
}

// The MLP fc1 epilogue as a pass after a library GEMM (hipBLASLt has no GELU-derivative or
// fp8 side output): y = the bf16 pre-activation (bias included) ->
//   aux = gelu'(y) (bf16), q = fp8(bf16(gelu(y)) * scale) with the delayed scale, amax recorded,
//   a_out (optional, may alias y) = gelu(y) (bf16)
// -- the same values the fused conv_nt act-4 + q8 epilogue writes. n % 8 == 0.
template <int FMT>
__global__ void __launch_bounds__(256) gelu_dual_cast_kernel(const u16* __restrict__ y, long n,
                                                             float* __restrict__ meta, uint8_t* __restrict__ q,
                                                             u16* __restrict__ aux, u16* a_out) {
  __shared__ float red[4];
  const float s = meta[0];
  float m = 0.f;
  const long stride = (long)gridDim.x * 256 * 8;
  for (long base = ((long)blockIdx.x * 256 + threadIdx.x) * 8; base < n; base += stride) {
    const u32x4 w = *reinterpret_cast<const u32x4*>(y + base);
    u32x4 gq, dq;
    float g[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float g0, g1, d0, d1;
      pdt_gelu_dual(lo_bf(w[e]), g0, d0);
      pdt_gelu_dual(hi_bf(w[e]), g1, d1);
      gq[e] = pack2bf(g0, g1);
      dq[e] = pack2bf(d0, d1);
      g[2 * e] = lo_bf(gq[e]);
      g[2 * e + 1] = hi_bf(gq[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(g[e]));
    if (aux != nullptr) *reinterpret_cast<u32x4*>(aux + base) = dq;
    if (a_out != nullptr) *reinterpret_cast<u32x4*>(a_out + base) = gq;
    uint2 o;
    o.x = cvt4<FMT>(g[0] * s, g[1] * s, g[2] * s, g[3] * s);
    o.y = cvt4<FMT>(g[4] * s, g[5] * s, g[6] * s, g[7] * s);
    *reinterpret_cast<uint2*>(q + base) = o;
  }
  m = warp_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(reinterpret_cast<unsigned int*>(meta) + 2, __float_as_uint(bm));
  }
}

// cast_fp8_delayed_kernel of a bf16 [rows][cols] gradient that also forms its column sums
// (the producing nn.Linear's bias gradient) from the bf16 values it reads anyway: block b owns
// rows [b * rpb, (b + 1) * rpb), a thread owns 8-column chunks (every chunk of the band is one
// thread's, so no in-block combine) -> cpart[b][cols]. cols % 8 == 0.
// GG: x is a GEMM's (g W) and zz the GELU pre-activation of the same shape -- the values cast
// and summed are x * gelu'(zz) (the MLP fc1 output gradient, when the fc2 data gradient runs on
// the library GEMM without the act-3 epilogue).
// RG > 1 row groups (RG * cols / 8 <= blockDim): thread (g, c8) walks rows r0 + g, r0 + g + RG,
// ... -- a block keeps RG times the loads in flight (96 threads per band at cols = 768 left the
// cast latency-bound at ~1.7 TB/s); the groups' column sums are added in group order through LDS.
template <int FMT, bool GG = false>
__global__ void __launch_bounds__(1024) cast_fp8_delayed_cs_kernel(const u16* __restrict__ x, int rows, int cols,
                                                                   int rpb, float* __restrict__ meta,
                                                                   uint8_t* __restrict__ q, float* __restrict__ cpart,
                                                                   const u16* __restrict__ zz = nullptr, int RG = 1) {
  __shared__ float red[16];
  // [RG][c8n][8] column partials (RG * c8n <= 1024): dynamic, sized by the launcher only when
  // RG > 1 -- an RG == 1 launch reserves no LDS for it (a static 32 KB array cost them occupancy)
  extern __shared__ f32x4 csh[];
  const float s = meta[0];
  const int c8n = cols / 8;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  float m = 0.f;
  const int g = RG > 1 ? (int)threadIdx.x / c8n : 0;
  const int c8first = RG > 1 ? (int)threadIdx.x - g * c8n : (int)threadIdx.x;
  const int c8step = RG > 1 ? c8n : (int)blockDim.x;  // RG > 1: one chunk per thread
  for (int c8 = c8first; c8 < c8n && g < RG; c8 += c8step) {  // (one trip when cols <= 8 * blockDim)
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int r = r0 + g;
    auto row = [&](const u32x4& w, const u32x4& zw, long base) __attribute__((always_inline)) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = lo_bf(w[e]);
        v[2 * e + 1] = hi_bf(w[e]);
      }
      if constexpr (GG) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float g0, g1, d0, d1;
          pdt_gelu_dual(lo_bf(zw[e]), g0, d0);
          pdt_gelu_dual(hi_bf(zw[e]), g1, d1);
          v[2 * e] *= d0;
          v[2 * e + 1] *= d1;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        m = fmaxf(m, fabsf(v[e]));
        cs[e] += v[e];
      }
      uint2 o;
      o.x = cvt4<FMT>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
      o.y = cvt4<FMT>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
      *reinterpret_cast<uint2*>(q + base) = o;
    };
    for (; r + 3 * RG < r1; r += 4 * RG) {  // four rows' loads in flight before any is used
      u32x4 w[4], zw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        w[u] = *reinterpret_cast<const u32x4*>(x + (long)(r + u * RG) * cols + c8 * 8);
        if constexpr (GG) zw[u] = *reinterpret_cast<const u32x4*>(zz + (long)(r + u * RG) * cols + c8 * 8);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) row(w[u], zw[u], (long)(r + u * RG) * cols + c8 * 8);
    }
    for (; r < r1; r += RG) {
      const long base = (long)r * cols + c8 * 8;
      u32x4 zw{};
      if constexpr (GG) zw = *reinterpret_cast<const u32x4*>(zz + base);
      row(*reinterpret_cast<const u32x4*>(x + base), zw, base);
    }
    if (RG > 1) {
      csh[2 * threadIdx.x] = f32x4{cs[0], cs[1], cs[2], cs[3]};
      csh[2 * threadIdx.x + 1] = f32x4{cs[4], cs[5], cs[6], cs[7]};
    } else {
      float* cp = cpart + (long)blockIdx.x * cols + c8 * 8;
      *reinterpret_cast<f32x4*>(cp) = f32x4{cs[0], cs[1], cs[2], cs[3]};
      *reinterpret_cast<f32x4*>(cp + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
    }
  }
  if (RG > 1) {  // the band's column sums: row groups added in group order
    __syncthreads();
    if ((int)threadIdx.x < c8n) {
      f32x4 a = csh[2 * threadIdx.x], b = csh[2 * threadIdx.x + 1];
      for (int k = 1; k < RG; ++k) {
        a += csh[2 * (k * c8n + threadIdx.x)];
        b += csh[2 * (k * c8n + threadIdx.x) + 1];
      }
      float* cp = cpart + (long)blockIdx.x * cols + threadIdx.x * 8;
      *reinterpret_cast<f32x4*>(cp) = a;
      *reinterpret_cast<f32x4*>(cp + 4) = b;
    }
  }
  m = warp_max(m);
  const int nw = (blockDim.x + 63) / 64;
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float bm = red[0];
    for (int k = 1; k < nw; ++k) bm = fmaxf(bm, red[k]);
    atomicMax(reinterpret_cast<unsigned int*>(meta) + 2, __float_as_uint(bm));  // order-free -> deterministic
  }
}

// history roll, one tiny launch after the cast (a last-block roll inside the
// cast would need a device-scope release fence per block: an L2 write-back on
// the multi-XCD part)
// dq_out (optional): this cast's dequant factor 1/scale in a caller-owned slot that later
// casts do not overwrite (meta[1] is rewritten by the tensor's next cast)
template <int FMT>
__global__ void fp8_meta_roll_kernel(float* __restrict__ meta, float* __restrict__ dq_out) {
  if (threadIdx.x != 0) return;
  if (dq_out) dq_out[0] = 1.f / meta[0];
  unsigned int* mu = reinterpret_cast<unsigned int*>(meta);
  const float cur = __uint_as_float(mu[2]);
  const int idx = (int)mu[4];
  meta[5 + idx % HIST] = cur;
  mu[4] = (unsigned)(idx + 1);
  float h = 0.f;
  for (int i = 0; i < HIST; ++i) h = fmaxf(h, meta[5 + i]);
  meta[1] = 1.f / meta[0];
  meta[0] = scale_from<FMT>(h);
  mu[2] = 0u;
}

// the same roll for a producer kernel that wrote per-block amax partials instead of
// the atomicMax slot (the LayerNorm forward's fused fp8 output)
template <int FMT>
__global__ void __launch_bounds__(1024) fp8_meta_roll_part_kernel(float* __restrict__ meta,
                                                                const float* __restrict__ partial, int nblk,
                                                                float* __restrict__ dq_out) {
  const float a = block_amax(partial, nblk);
  if (threadIdx.x != 0) return;
  if (dq_out) dq_out[0] = 1.f / meta[0];
  unsigned int* mu = reinterpret_cast<unsigned int*>(meta);
  const float cur = fmaxf(a, __uint_as_float(mu[2]));
  const int idx = (int)mu[4];
  meta[5 + idx % HIST] = cur;
  mu[4] = (unsigned)(idx + 1);
  float h = 0.f;
  for (int i = 0; i < HIST; ++i) h = fmaxf(h, meta[5 + i]);
  meta[1] = 1.f / meta[0];
  meta[0] = scale_from<FMT>(h);
  mu[2] = 0u;
}

int nblocks(long n) {
  long b = (n + 256 * 8 - 1) / (256 * 8);
  if (b > AMAX_BLOCKS) b = AMAX_BLOCKS;
  return b < 1 ? 1 : (int)b;
}

}  // namespace

PDT_API int pdt_amax_blocks(long n) { return nblocks(n); }

PDT_API int pdt_amax_partial(const void* x, int bf16, long n, float* partial, hipStream_t st) {
  const int nb = nblocks(n);
  if (bf16)
    hipLaunchKernelGGL(amax_partial_kernel<true>, dim3(nb), dim3(256), 0, st, x, n, partial);
  else
    hipLaunchKernelGGL(amax_partial_kernel<false>, dim3(nb), dim3(256), 0, st, x, n, partial);
  PDT_RETURN_LAUNCH();
}

// fmt: 0 = e4m3fn, 1 = e5m2
PDT_API int pdt_cast_fp8(const void* x, int bf16, long n, const float* partial, int fmt, void* q, float* dq,
                         hipStream_t st) {
  const int nb = nblocks(n);
  uint8_t* qo = (uint8_t*)q;
  if (bf16) {
    if (fmt == 0) hipLaunchKernelGGL((cast_fp8_kernel<true, 0>), dim3(nb), dim3(256), 0, st, x, n, partial, nb, qo, dq);
    else hipLaunchKernelGGL((cast_fp8_kernel<true, 1>), dim3(nb), dim3(256), 0, st, x, n, partial, nb, qo, dq);
  } else {
    if (fmt == 0) hipLaunchKernelGGL((cast_fp8_kernel<false, 0>), dim3(nb), dim3(256), 0, st, x, n, partial, nb, qo, dq);
    else hipLaunchKernelGGL((cast_fp8_kernel<false, 1>), dim3(nb), dim3(256), 0, st, x, n, partial, nb, qo, dq);
  }
  PDT_RETURN_LAUNCH();
}

// fp32 [R][C] -> e4m3 [C][R]; the partials must come from pdt_amax_partial over the same R*C values
PDT_API int pdt_cast_fp8_t(const float* x, int R, int C, const float* partial, void* q, hipStream_t st) {
  const int nb = nblocks((long)R * C);
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(cast_fp8_t_kernel<0>, grid, dim3(256), 0, st, x, R, C, partial, nb, (uint8_t*)q);
  PDT_RETURN_LAUNCH();
}

// fp32 [R][C] -> e4m3 [R][C] AND [C][R] in one pass (the weight's forward and data-gradient
// operands), dq = 1 / scale; the partials must come from pdt_amax_partial over the same values
PDT_API int pdt_cast_fp8_dual(const float* x, int R, int C, const float* partial, void* q, void* qt, float* dq,
                              hipStream_t st) {
  const int nb = nblocks((long)R * C);
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(cast_fp8_t_kernel<0>, grid, dim3(256), 0, st, x, R, C, partial, nb, (uint8_t*)qt, (uint8_t*)q,
                     dq);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_fp8_meta_words() { return 5 + HIST; }

// one-pass delayed-scaling cast; meta must be initialised by pdt_fp8_meta_seed
PDT_API int pdt_cast_fp8_delayed(const void* x, int bf16, long n, float* meta, int fmt, void* q, float* dq_out,
                                 hipStream_t st) {
  const int nb = nblocks(n);
  uint8_t* qo = (uint8_t*)q;
#define CD(B_, F_) hipLaunchKernelGGL((cast_fp8_delayed_kernel<B_, F_>), dim3(nb), dim3(256), 0, st, x, n, meta, qo)
  if (bf16) { if (fmt == 0) CD(true, 0); else CD(true, 1); }
  else { if (fmt == 0) CD(false, 0); else CD(false, 1); }
#undef CD
  if (fmt == 0) hipLaunchKernelGGL(fp8_meta_roll_kernel<0>, dim3(1), dim3(64), 0, st, meta, dq_out);
  else hipLaunchKernelGGL(fp8_meta_roll_kernel<1>, dim3(1), dim3(64), 0, st, meta, dq_out);
  PDT_RETURN_LAUNCH();
}

// y [n] bf16 -> aux = gelu'(y) if given, q = fp8 codes of gelu(y) (delayed scale, history rolled,
// dq_out = this cast's dequant factor), a_out = gelu(y) if given (may be y itself). Without aux the
// caller keeps y itself (the pre-activation) for the backward's act-3 epilogue.
PDT_API int pdt_gelu_dual_cast_fp8(const void* y, long n, float* meta, int fmt, void* q, void* aux, void* a_out,
                                   float* dq_out, hipStream_t st) {
  if (n % 8 != 0 || !y || !meta || !q) return -1;
  const int nb = nblocks(n);
  const u16* Y = (const u16*)y;
  if (fmt == 0) {
    hipLaunchKernelGGL(gelu_dual_cast_kernel<0>, dim3(nb), dim3(256), 0, st, Y, n, meta, (uint8_t*)q, (u16*)aux,
                       (u16*)a_out);
    hipLaunchKernelGGL(fp8_meta_roll_kernel<0>, dim3(1), dim3(64), 0, st, meta, dq_out);
  } else {
    hipLaunchKernelGGL(gelu_dual_cast_kernel<1>, dim3(nb), dim3(256), 0, st, Y, n, meta, (uint8_t*)q, (u16*)aux,
                       (u16*)a_out);
    hipLaunchKernelGGL(fp8_meta_roll_kernel<1>, dim3(1), dim3(64), 0, st, meta, dq_out);
  }
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_wgrad_reduce_rows(const float* rows, float* out, int nrows, int n, float scale, int accumulate,
                                  float* work, hipStream_t stream);
PDT_API long pdt_reduce_rows_work(int nrows, int n);

// block shape of the column-summing casts: one thread per 8-column chunk, times up to 8 row groups
// (PDT_CAST_CS_RG=1: the previous one-row-walker-per-chunk shape, for A/B runs)
static void cs_block(int cols, int* nt, int* rg) {
  static int env = -1;
  if (env < 0) {
    const char* e = getenv("PDT_CAST_CS_RG");
    env = e ? atoi(e) : 0;
  }
  const int c8n = cols / 8;
  int g = c8n <= 1024 ? 1024 / c8n : 1;
  if (g > 8) g = 8;
  if (env >= 1 && env < g) g = env;
  if (g < 1) g = 1;
  const int n = g > 1 ? c8n * g : c8n;
  *nt = ((n + 63) / 64) * 64;
  if (*nt > 1024) *nt = 1024;
  *rg = g;
}

// row bands of pdt_cast_fp8_delayed_cs (its cpart holds that many rows of cols floats, followed
// by pdt_reduce_rows_work(bands, cols) floats of reduce workspace)
PDT_API int pdt_cast_cs_bands(int rows) {
  int rpb = 64;
  while ((rows + rpb - 1) / rpb > 2048) rpb *= 2;
  return (rows + rpb - 1) / rpb;
}

// bands actually launched: pdt_cast_cs_bands(rows) is the bound the caller sized cpart for;
// above one round of resident blocks it is rounded DOWN to whole rounds (the ViT qkv gradient,
// 201 728 x 2304: 1 576 bands of 896 threads at 2 per CU = 3.08 rounds, the fourth 8 % full).
// Fewer bands never need more cpart: the reduce workspace grows with the band count.
// PDT_CAST_CS_ROUNDS=0: the bound itself (A/B runs).
// The occupancy answer is cached per (kernel, threads, LDS bytes): the query is host time on
// every cast launch otherwise (the step is partly host-issue-bound).
static int cs_blocks_per_cu(const void* kern, int nt, size_t sh) {
  struct Ent {
    const void* k;
    int nt;
    size_t sh;
    int per;
  };
  static Ent cache[32];
  static int n = 0;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  for (int i = 0; i < n; ++i)
    if (cache[i].k == kern && cache[i].nt == nt && cache[i].sh == sh) return cache[i].per;
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, nt, sh) != hipSuccess) per = 0;
  if (n < 32) cache[n++] = Ent{kern, nt, sh, per};
  return per;
}

static size_t cs_lds_bytes(int cols, int rg) { return rg > 1 ? (size_t)rg * (cols / 8) * 2 * sizeof(f32x4) : 0; }

static int cs_launch_bands(const void* kern, int rows, int nt, size_t sh) {
  static int env = -1;
  if (env < 0) {
    const char* e = getenv("PDT_CAST_CS_ROUNDS");
    env = e ? atoi(e) : 1;
  }
  const int nb = pdt_cast_cs_bands(rows);
  if (env == 0) return nb;
  const int per = cs_blocks_per_cu(kern, nt, sh);
  if (per < 1) return nb;
  const int slots = per * pdt_num_cus();
  return nb > slots ? nb / slots * slots : nb;
}

// pdt_cast_fp8_delayed for a bf16 [rows][cols] gradient + its column sums into bias_out (=)
PDT_API int pdt_cast_fp8_delayed_cs(const void* x, int rows, int cols, float* meta, int fmt, void* q, float* dq_out,
                                    float* cpart, float* bias_out, hipStream_t st) {
  if (cols % 8 != 0 || rows < 1 || !cpart || !bias_out) return -1;
  const u16* X = (const u16*)x;
  int nt, rg;
  cs_block(cols, &nt, &rg);
  const size_t sh = cs_lds_bytes(cols, rg);
  const int nb = cs_launch_bands(
      fmt == 0 ? (const void*)cast_fp8_delayed_cs_kernel<0> : (const void*)cast_fp8_delayed_cs_kernel<1>, rows, nt,
      sh);
  const int rpb = (rows + nb - 1) / nb;
  if (fmt == 0)
    hipLaunchKernelGGL(cast_fp8_delayed_cs_kernel<0>, dim3(nb), dim3(nt), sh, st, X, rows, cols, rpb, meta,
                       (uint8_t*)q, cpart, nullptr, rg);
  else
    hipLaunchKernelGGL(cast_fp8_delayed_cs_kernel<1>, dim3(nb), dim3(nt), sh, st, X, rows, cols, rpb, meta,
                       (uint8_t*)q, cpart, nullptr, rg);
  if (fmt == 0) hipLaunchKernelGGL(fp8_meta_roll_kernel<0>, dim3(1), dim3(64), 0, st, meta, dq_out);
  else hipLaunchKernelGGL(fp8_meta_roll_kernel<1>, dim3(1), dim3(64), 0, st, meta, dq_out);
  const int e = (int)hipGetLastError();
  if (e) return e;
  return pdt_wgrad_reduce_rows(cpart, bias_out, nb, cols, 1.f, 0, cpart + (long)nb * cols, st);
}

// pdt_cast_fp8_delayed_cs of x * gelu'(z) (x, z bf16 [rows][cols]): the MLP fc1 output gradient
// from the fc2 data gradient's plain GEMM output, cast + bias sums in the same pass
PDT_API int pdt_cast_fp8_gelu_grad_cs(const void* x, const void* z, int rows, int cols, float* meta, int fmt,
                                      void* q, float* dq_out, float* cpart, float* bias_out, hipStream_t st) {
  if (cols % 8 != 0 || rows < 1 || !z || !cpart || !bias_out) return -1;
  int nt, rg;
  cs_block(cols, &nt, &rg);
  const size_t sh = cs_lds_bytes(cols, rg);
  const int nb = cs_launch_bands(fmt == 0 ? (const void*)cast_fp8_delayed_cs_kernel<0, true>
                                          : (const void*)cast_fp8_delayed_cs_kernel<1, true>,
                                 rows, nt, sh);
  const int rpb = (rows + nb - 1) / nb;
  if (fmt == 0)
    hipLaunchKernelGGL((cast_fp8_delayed_cs_kernel<0, true>), dim3(nb), dim3(nt), sh, st, (const u16*)x, rows, cols,
                       rpb, meta, (uint8_t*)q, cpart, (const u16*)z, rg);
  else
    hipLaunchKernelGGL((cast_fp8_delayed_cs_kernel<1, true>), dim3(nb), dim3(nt), sh, st, (const u16*)x, rows, cols,
                       rpb, meta, (uint8_t*)q, cpart, (const u16*)z, rg);
  if (fmt == 0) hipLaunchKernelGGL(fp8_meta_roll_kernel<0>, dim3(1), dim3(64), 0, st, meta, dq_out);
  else hipLaunchKernelGGL(fp8_meta_roll_kernel<1>, dim3(1), dim3(64), 0, st, meta, dq_out);
  const int e = (int)hipGetLastError();
  if (e) return e;
  return pdt_wgrad_reduce_rows(cpart, bias_out, nb, cols, 1.f, 0, cpart + (long)nb * cols, st);
}

// threads of the one-block partial-amax roll: 1024 for the long partial lists of the LayerNorm
// forward (a 256-thread block walked them in ~24 us); PDT_ROLL_NT overrides (256 / 512 / 1024)
static int roll_threads(int nblk) {
  static const int nt = [] {
    const char* e = getenv("PDT_ROLL_NT");
    const int v = e ? atoi(e) : 1024;
    return (v == 256 || v == 512) ? v : 1024;
  }();
  return nblk <= 1024 ? 256 : nt;
}

// roll after a fused producer (pdt_ln_fwd_f8): partial[nblk] holds its per-block amaxes
PDT_API int pdt_fp8_meta_roll_partial(float* meta, const float* partial, int nblk, int fmt, float* dq_out,
                                      hipStream_t st) {
  if (fmt == 0)
    hipLaunchKernelGGL(fp8_meta_roll_part_kernel<0>, dim3(1), dim3(roll_threads(nblk)), 0, st, meta, partial, nblk,
                       dq_out);
  else
    hipLaunchKernelGGL(fp8_meta_roll_part_kernel<1>, dim3(1), dim3(roll_threads(nblk)), 0, st, meta, partial, nblk,
                       dq_out);
  PDT_RETURN_LAUNCH();
}

namespace {
template <int FMT>
__global__ void fp8_meta_seed_kernel(const float* __restrict__ partial, int nblk, float* __restrict__ meta) {
  const float a = block_amax(partial, nblk);
  if (threadIdx.x == 0) {
    unsigned int* mu = reinterpret_cast<unsigned int*>(meta);
    for (int i = 0; i < HIST; ++i) meta[5 + i] = 0.f;
    meta[5] = a;
    mu[4] = 1u;
    mu[2] = 0u;
    mu[3] = 0u;
    meta[0] = scale_from<FMT>(a);
    meta[1] = 1.f / meta[0];
  }
}
}  // namespace

// seed the history with the exact amax of a first tensor (from pdt_amax_partial)
PDT_API int pdt_fp8_meta_seed(const float* partial, long n, int fmt, float* meta, hipStream_t st) {
  const int nb = nblocks(n);
  if (fmt == 0) hipLaunchKernelGGL(fp8_meta_seed_kernel<0>, dim3(1), dim3(256), 0, st, partial, nb, meta);
  else hipLaunchKernelGGL(fp8_meta_seed_kernel<1>, dim3(1), dim3(256), 0, st, partial, nb, meta);
  PDT_RETURN_LAUNCH();
}
