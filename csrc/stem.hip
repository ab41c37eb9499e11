// ResNet stem forward (7x7 / stride 2 / pad 3 conv over <= 4 input channels, 64 output
// channels) as a halo-patch implicit GEMM with the BatchNorm statistics in the epilogue.
//
// Why: the generic implicit GEMM runs the stem as the space-to-depth GEMM (K = 256, see
// native_ops._s2d_weight) and gathers 32 taps x 16 B per output pixel through L2; at 2048
// images that GEMM took 1.64 ms for 842 GFLOP and 4.1 GB of compulsory traffic (a ~0.75 ms
// floor). Here a workgroup owns 8 output rows of one image (8 x 112 pixels x 64 channels)
// and stages the 21 input rows they read ONCE into LDS; every tap's A fragment is then a
// ds_read of that patch at a (row, pair) offset.
//
// Space-to-depth view (native_ops._s2d_weight): the NHWC input padded to 4 channels is read
// as PAIRS of horizontally adjacent pixels (16 B = 2 px x 4 ch), and
//   y[n, oh, ow, co] = sum_{kh < 7, t < 4} sum_{j < 8} X[n, 2oh + kh - 3, pair ow + t - 2, j]
//                                                     * W'[co, (kh * 4 + t) * 8 + j]
// (kh = 7 is the zero row of the padded 8x8 kernel: skipped, K = 224 per pixel).
//
// Layout: patch [21 (24 allocated) rows][128 slots] of 16-B pairs (slot s = pair s - 2; slots past the image
// are zero), double-buffered; the weight [64 co][32 chunks] with chunk c of row co at physical
// chunk c ^ (co & 15) (a B fragment's 16 rows hit 16 distinct bank groups). A fragments are
// 16 consecutive slots per 16-lane group: conflict-free without a swizzle.
//
// Waves: 8, wave w computes output row oh0 + w (7 blocks of 16 pixels x 4 blocks of 16
// channels, the swapped-operand MFMA so a lane holds 4 consecutive channels of one pixel).
// Persistent: one workgroup per CU walks tiles (image, 8-row band); the next band's patch is
// DMA'd into the other buffer while this one computes, and this band's output stores are
// issued AFTER that DMA, so the next band's counted vmcnt wait retires the patch without
// waiting for the stores (the store stream of band i overlaps the MFMAs of band i + 1).
// BatchNorm statistics: each lane accumulates its 16 channels' sum / sum of squares over every
// band it computes (fp32, from the accumulators as the generic epilogue does); one partial row
// per (workgroup, wave) at the end, reduced by pdt_bn_finalize.
#include "pdt_common.h"

namespace {

constexpr int NW = 8, NTH = NW * 64;
constexpr int ROWS = 2 * NW + 5;     // input rows a band reads (2 * 8 output rows + 7 - 2)
constexpr int PROWS = 24;            // patch rows allocated: PROWS * SLOTS = 6 DMA passes of 512 x 16 B
constexpr int SLOTS = 128;           // 16-B pair slots per patch row (116 used)
constexpr int PATCH = PROWS * SLOTS * 16;
constexpr int WBYTES = 64 * 32 * 16;  // weight: 64 rows x 32 chunks x 16 B
constexpr int LP = PROWS * SLOTS / NTH;             // patch DMA instructions per thread (6)
static_assert(PROWS * SLOTS % NTH == 0 && PROWS >= ROWS, "whole DMA passes");
constexpr int LW = 64 * 32 / NTH;                   // weight DMA instructions per thread (4)
constexpr int WO = 112, MI = WO / 16;               // output row width, 16-pixel blocks

static __device__ __attribute__((aligned(64))) u32x4 stem_zero[4];

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct StemParams {
  const u16* x;     // [N][H][W][4] bf16 (NHWC padded to 4 channels): pairs [N][H][W/2][8]
  const u16* w;     // [64][256] bf16 space-to-depth weight
  u16* y;           // [N][H/2][W/2][64]
  float* part;      // [2][R][64]: per (workgroup, wave) sum / sum of squares; R = grid * 8
  const void* zero;
  int N, H, W;      // W / 2 == 112 (one output row = 7 x 16 pixels)
  int ntiles, R;
};

__global__ void __launch_bounds__(NTH, 1) stem_fwd_kernel(StemParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PATCH + WBYTES];
  char* const sw = smem + 2 * PATCH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ho = p.H / 2, bands = Ho / NW, Wp = p.W / 2;  // Wp: pairs per input row (= WO)

  // weight -> LDS once (lane-linear image, swizzle on the source: physical chunk pc of row co
  // holds logical chunk pc ^ (co & 15))
#pragma unroll
  for (int l = 0; l < LW; ++l) {
    const int q = tid + NTH * l;
    const int co = q >> 5, pc = q & 31;
    const void* src = p.w + co * 256 + ((pc ^ (co & 15)) * 8);
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sw + (64 * wave + NTH * l) * 16),
                                     16, 0, 0);
  }
  auto issue_patch = [&](int tile, int buf) __attribute__((always_inline)) {
    const bool live = tile < p.ntiles;
    const int n = live ? tile / bands : 0, band = live ? tile - (tile / bands) * bands : 0;
    const int ih0 = 2 * band * NW - 3;
    char* sp = smem + buf * PATCH;
#pragma unroll
    for (int l = 0; l < LP; ++l) {
      const int q = tid + NTH * l;
      const int r = q >> 7, s = q & (SLOTS - 1);
      const int ih = ih0 + r, pr = s - 2;
      const bool ok = live && r < ROWS && (unsigned)ih < (unsigned)p.H && (unsigned)pr < (unsigned)Wp;
      const void* src = ok ? (const void*)(p.x + (((size_t)n * p.H + ih) * Wp + pr) * 8) : p.zero;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sp + (64 * wave + NTH * l) * 16),
                                       16, 0, 0);
    }
  };

  // per-lane statistics of its 16 channels (co = j * 16 + (lane >> 4) * 4 + r)
  float ssum[4][4], ssq[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) ssum[j][r] = ssq[j][r] = 0.f;


  int tile = blockIdx.x;
  if (tile < p.ntiles) issue_patch(tile, 0);
  bool first = true;
  for (int it = 0; tile < p.ntiles; ++it, tile += gridDim.x) {
    const int buf = it & 1;
    // retire this band's patch (and at the first band the weight); the previous band's
    // output stores (issued after this DMA) stay in flight
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MI * 2) : "memory");
    first = false;
    __builtin_amdgcn_s_barrier();  // every wave's DMA landed; the other buffer's readers are done
    asm volatile("" ::: "memory");
    issue_patch(tile + gridDim.x, buf ^ 1);

    const int n = tile / bands, band = tile - n * bands;
    const int oh = band * NW + wave;
    const char* sp = smem + buf * PATCH;
    f32x4 acc[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      // B fragment: weight row co = j * 16 + (lane & 15), logical chunk kh * 4 + (lane >> 4)
      bf16x8 bq[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = j * 16 + (lane & 15);
        const int c = kh * 4 + (lane >> 4);
        bq[j] = *reinterpret_cast<const bf16x8*>(sw + co * 512 + ((c ^ (co & 15)) << 4));
      }
      const char* prow = sp + (2 * wave + kh) * (SLOTS * 16);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        // pixel ow = 16 i + (lane & 15), tap t = lane >> 4: slot ow + t (pair ow + t - 2)
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(prow + (16 * i + (lane & 15) + (lane >> 4)) * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j], af, acc[i][j], 0, 0, 0);
      }
    }
    // epilogue: statistics, then 16-B stores (lanes l and l ^ 16 exchange quads of blocks j, j + 1)
    u16* yrow = p.y + (((size_t)n * Ho + oh) * WO) * 64;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ssum[j][r] += acc[i][j][r];
          ssq[j][r] = fmaf(acc[i][j][r], acc[i][j][r], ssq[j][r]);
        }
      const int ow = 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const uint32_t a0 = pack2bf(acc[i][j][0], acc[i][j][1]), a1 = pack2bf(acc[i][j][2], acc[i][j][3]);
        const uint32_t b0 = pack2bf(acc[i][j + 1][0], acc[i][j + 1][1]),
                       b1 = pack2bf(acc[i][j + 1][2], acc[i][j + 1][3]);
        const auto r0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
        const bool odd = (lane >> 4) & 1;
        const u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
        const int co = (odd ? j + 1 : j) * 16 + (lane >> 5) * 8;
        *reinterpret_cast<u32x4*>(yrow + (size_t)ow * 64 + co) = v;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA / store outlives the workgroup
  // partial row (workgroup, wave): the 16 lanes of a DPP row hold 16 pixels of the same channels
  const int prow = blockIdx.x * NW + wave;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float s[4], q[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[r] = row16_sum(ssum[j][r]);
      q[r] = row16_sum(ssq[j][r]);
    }
    if ((lane & 15) < 8) {
      const int r = lane & 3;
      const float sv = (r & 2) ? ((r & 1) ? s[3] : s[2]) : ((r & 1) ? s[1] : s[0]);
      const float qv = (r & 2) ? ((r & 1) ? q[3] : q[2]) : ((r & 1) ? q[1] : q[0]);
      const int co = j * 16 + (lane >> 4) * 4 + r;
      p.part[(size_t)(((lane & 15) < 4 ? 0 : p.R) + prow) * 64 + co] = (lane & 15) < 4 ? sv : qv;
    }
  }
}

}  // namespace

// Applicability (0 = ok) and the number of statistics partial rows of the halo stem.
PDT_API int pdt_stem_fwd_rows(int N, int H, int W, int Cout) {
  if (Cout != 64 || H % (2 * NW) != 0 || W != 2 * WO || N < 1) return -5;
  const int ntiles = N * (H / 2 / NW);
  return (ntiles < 256 ? ntiles : 256) * NW;
}

// y = stem conv of x (see the header), BN partial statistics into part[2][R][64],
// R = pdt_stem_fwd_rows(...). -5: geometry not covered (the caller takes the generic path).
PDT_API int pdt_stem_fwd(const void* x4, const void* w256, void* y, float* part, int N, int H, int W, int Cout,
                         hipStream_t stream) {
  const int R = pdt_stem_fwd_rows(N, H, W, Cout);
  if (R < 0) return R;
  // (every global offset is 64-bit: no element-count limit)
  static const void* zcache[PDT_MAX_DEV] = {};
  StemParams p;
  p.x = (const u16*)x4;
  p.w = (const u16*)w256;
  p.y = (u16*)y;
  p.part = part;
  p.zero = pdt_symbol_addr(HIP_SYMBOL(stem_zero), zcache);
  if (p.zero == nullptr) return PDT_ERR_SYMBOL;
  p.N = N; p.H = H; p.W = W;
  p.ntiles = N * (H / 2 / NW);
  p.R = R;
  hipLaunchKernelGGL(stem_fwd_kernel, dim3(R / NW), dim3(NTH), 0, stream, p);
  PDT_RETURN_LAUNCH();
}

// ============================================================================
// Stem weight gradient with the stem BatchNorm's backward apply in its dY staging:
//
//   dW'[co][k] = sum_m dy[m][co] * X[m][k],   dy = k1 * (y*scale + shift > 0 ? dA : 0) + k2 * y + k3
//
// (X, W' in the space-to-depth view of the forward above; dy is bn_bwd_apply's output, never
// written to memory). The generic weight gradient re-gathers X per tap chunk from L2 (32 x 16 B
// per pixel) and ran at 2.95 ms for 7.4 GB of compulsory traffic at 2048 images. Here a
// workgroup walks bands of 4 output rows of one image: the band's dA / y (448 pixels x 64
// channels) are loaded into registers one band ahead, turned into dy and written to an LDS
// tile, and its 13 input rows are DMA'd into a patch (double-buffered); both operands are
// pixel-major, so MFMA fragments come through the transposing ds_read_b64_tr_b16 --
// 16x16x16 MFMAs, reduction over 16 pixels per step: dy^T (4 blocks of 16 channels) x X
// (14 blocks of 16 k = two taps of one kernel row each; kh = 7 is the zero row).
// Wave w accumulates output row w of each band over every band of the workgroup (64 x 224
// fp32 = 56 accumulators, one wave per SIMD, in AGPRs) and writes its own slab row;
// pdt_wgrad_reduce sums the slabs. (8 waves, two per SIMD over k halves, spilled 19 VGPRs and
// ran 2.33 vs 2.05 ms at 2048 images.)
namespace {

constexpr int WB = 4;                  // output rows per band
constexpr int WNW = 4, WNTH = WNW * 64;
constexpr int WROWS = 2 * WB + 5;      // input rows a band reads (13)
constexpr int WPROWS = 16;             // allocated: 16 x 128 slots = 8 DMA passes of 256 x 16 B
constexpr int WPATCH = WPROWS * SLOTS * 16;
constexpr int WPX = WB * WO;           // band pixels (448)
constexpr int DYT = WPX * 128;         // dy tile bytes
constexpr int WLP = WPROWS * SLOTS / WNTH;
constexpr int WLC = WPX * 8 / WNTH;    // 16-B dA / y chunks per thread per band (14)

struct StemWgParams {
  const u16* x;      // [N][H][W][4] bf16 = pairs [N][H][W/2][8]
  const u16* dA;     // [N][H/2][W/2][64]: the gradient at the stem BN's output (before its backward)
  const u16* y;      // [N][H/2][W/2][64]: the stem conv output
  const float* bnc;  // [5][64]: k1, k2, k3, scale, shift
  float* slab;       // [grid * 4][64][256]
  const void* zero;
  int N, H, W, ntiles;
};

// dy-tile byte offset of (pixel row, 16-B chunk c of 8 channels): 32-B segment XOR (row >> 1) & 3,
// so a transposed read's 32-lane half (rows 4g + q, g = 0..1, one segment) hits 8 distinct
// 32-B bank groups
__device__ __forceinline__ int dyt_off(int row, int byte) {
  return row * 128 + ((((byte >> 5) ^ ((row >> 1) & 3))) << 5) + (byte & 31);
}

__device__ __forceinline__ bf16x4 tr4(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(
      (__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)p));
}

__global__ void __launch_bounds__(WNTH, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) stem_wgrad_kernel(StemWgParams p) {
  __shared__ __attribute__((aligned(16))) char smem[DYT + 2 * WPATCH];
  __shared__ float coef[5 * 64];  // k1, k2, k3, scale, shift (read at each apply: registers go to the prefetch)
  char* const dyt = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ho = p.H / 2, bands = Ho / WB, Wp = p.W / 2;
  for (int i = tid; i < 5 * 64; i += WNTH) coef[i] = p.bnc[i];
  // this thread's channel chunk (8 channels) is the same for all its dy chunks
  const int cc = tid & 7;
  u32x4 ra[WLC], ry[WLC];
  auto load_regs = [&](int tile) __attribute__((always_inline)) {
    const bool live = tile < p.ntiles;
    const int n = live ? tile / bands : 0, band = live ? tile - (tile / bands) * bands : 0;
    const size_t base = (((size_t)n * Ho + band * WB) * WO) * 64 + cc * 8;
#pragma unroll
    for (int l = 0; l < WLC; ++l) {
      const int px = (tid >> 3) + (WNTH / 8) * l;
      // (loads issued unconditionally -- the zero page past the last tile: a load under even a
      // wave-uniform condition is branched around and waited for on its own)
      ra[l] = *reinterpret_cast<const u32x4*>(live ? (const void*)(p.dA + base + (size_t)px * 64) : p.zero);
      ry[l] = *reinterpret_cast<const u32x4*>(live ? (const void*)(p.y + base + (size_t)px * 64) : p.zero);
    }
  };
  auto issue_patch = [&](int tile, int buf) __attribute__((always_inline)) {
    const bool live = tile < p.ntiles;
    const int n = live ? tile / bands : 0, band = live ? tile - (tile / bands) * bands : 0;
    const int ih0 = 2 * band * WB - 3;
    char* sp = smem + DYT + buf * WPATCH;
#pragma unroll
    for (int l = 0; l < WLP; ++l) {
      const int q = tid + WNTH * l;
      const int r = q >> 7, s = q & (SLOTS - 1);
      const int ih = ih0 + r, pr = s - 2;
      const bool ok = live && r < WROWS && (unsigned)ih < (unsigned)p.H && (unsigned)pr < (unsigned)Wp;
      const void* src = ok ? (const void*)(p.x + (((size_t)n * p.H + ih) * Wp + pr) * 8) : p.zero;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sp + (64 * wave + WNTH * l) * 16),
                                       16, 0, 0);
    }
  };

  f32x4 acc[4][14];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int kb = 0; kb < 14; ++kb) acc[cb][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;

  int tile = blockIdx.x;
  load_regs(tile);
  issue_patch(tile, 0);
  for (int it = 0; tile < p.ntiles; ++it, tile += gridDim.x) {
    const int buf = it & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this band's dA / y registers and patch
    __builtin_amdgcn_s_barrier();                      // every wave is done with the previous band's tiles
    asm volatile("" ::: "memory");
    // dy = BN backward apply -> LDS tile (bf16)
    float k1[8], k2[8], k3[8], sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      k1[e] = coef[cc * 8 + e];
      k2[e] = coef[64 + cc * 8 + e];
      k3[e] = coef[128 + cc * 8 + e];
      sc[e] = coef[192 + cc * 8 + e];
      sh[e] = coef[256 + cc * 8 + e];
    }
#pragma unroll
    for (int l = 0; l < WLC; ++l) {
      const int px = (tid >> 3) + (WNTH / 8) * l;
      float d[8], yv[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        d[2 * e] = lo_bf(ra[l][e]); d[2 * e + 1] = hi_bf(ra[l][e]);
        yv[2 * e] = lo_bf(ry[l][e]); yv[2 * e + 1] = hi_bf(ry[l][e]);
      }
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 2 * e + h;
          const float gk = (yv[k] * sc[k] + sh[k]) > 0.f ? d[k] : 0.f;
          v[h] = k1[k] * gk + k2[k] * yv[k] + k3[k];
        }
        o[e] = pack2bf(v[0], v[1]);
      }
      *reinterpret_cast<u32x4*>(dyt + dyt_off(px, cc * 16)) = o;
    }
    // the next band: registers and patch (the other buffer, last read before the barrier above)
    load_regs(tile + gridDim.x);
    issue_patch(tile + gridDim.x, buf ^ 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // dy tile visible
    asm volatile("" ::: "memory");
    const char* sp = smem + DYT + buf * WPATCH;
#pragma unroll 1
    for (int s = 0; s < WO / 16; ++s) {
      const int m0 = wave * WO + 16 * s;       // band pixel of this step's first row
      const int ow = 16 * s + 4 * g + q;       // this lane's pixel (row of the stored matrices)
      bf16x4 af[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) af[cb] = tr4(dyt + dyt_off(m0 + 4 * g + q, cb * 32 + pp * 8));
#pragma unroll
      for (int kb = 0; kb < 14; ++kb) {
        const int kh = kb >> 1, t0 = 2 * (kb & 1);
        const bf16x4 xf = tr4(sp + (2 * wave + kh) * (SLOTS * 16) + (ow + t0 + (pp >> 1)) * 16 + (pp & 1) * 8);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[cb][kb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af[cb], xf, acc[cb][kb], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  // slab row (workgroup, wave): D[co][k], lane holds co = cb*16 + 4*(lane >> 4) + r, k = kb*16 + (lane & 15)
  float* out = p.slab + (size_t)(blockIdx.x * WNW + wave) * 64 * 256;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = cb * 16 + 4 * (lane >> 4) + r;
#pragma unroll
      for (int kb = 0; kb < 14; ++kb) out[co * 256 + kb * 16 + (lane & 15)] = acc[cb][kb][r];
      out[co * 256 + 224 + (lane & 15)] = 0.f;  // kh = 7: the zero row of the padded kernel
      out[co * 256 + 240 + (lane & 15)] = 0.f;
    }
}

}  // namespace

static int pdt_stem_wgrad_splits_v1(int N, int H, int W, int Cout);
constexpr int KB2 = 7;  // 16-column k blocks per v2 wave (half of the 14)

// ---------------------------------------------------------------------------- v2
// The same weight gradient with every operand DMA'd (no register prefetch): bands of 2 output
// rows; per band the raw dA and y tiles (224 px x 64 ch each) and the 9 input rows go global ->
// LDS by LDS-DMA into one of two buffer sets, and the NEXT band's DMA is issued right after the
// barrier that opens a band -- before this band's dA is turned into dy in place -- so the loads
// stay in flight through the conversion and the MFMAs (v1 issued its register prefetch only
// after staging: HBM idled for this CU while it converted). 4 waves: wave w = output row w & 1
// of the band, k half w >> 1 (64 co x 112 k, 28 accumulators). The dy tile keeps v1's 32-B
// segment swizzle: the DMA lane at physical chunk c of pixel row r loads logical chunk
// swz(r, c) (the XOR is an involution), and the converter rewrites its own chunk in place.
namespace {

constexpr int V2B = 2;                  // output rows per band
constexpr int V2PX = V2B * WO;          // 224 band pixels
constexpr int V2RAW = V2PX * 128;       // one raw tile (dA or y): 28 KB
constexpr int V2ROWS = 2 * V2B + 5;     // 9 input rows
constexpr int V2PROWS = 10;             // allocated: 10 x 128 slots = 5 passes of 256 x 16 B
constexpr int V2PATCH = V2PROWS * SLOTS * 16;
constexpr int V2SET = 2 * V2RAW + V2PATCH;  // one buffer set: dA (-> dy), y, patch = 76 KB
constexpr int V2LR = V2PX * 8 / WNTH;   // raw-tile DMA passes per tensor (7)
constexpr int V2LP = V2PROWS * SLOTS / WNTH;  // patch DMA passes (5)
static_assert(2 * V2SET <= 160 * 1024 - 2048, "two buffer sets in LDS");

// logical 16-B chunk held by physical chunk c of dy-tile row r (dyt_off's segment swizzle)
__device__ __forceinline__ int v2_chunk(int r, int c) { return ((((c >> 1) ^ ((r >> 1) & 3))) << 1) | (c & 1); }

__global__ void __launch_bounds__(WNTH, 1) stem_wgrad2_kernel(StemWgParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * V2SET];
  __shared__ float coef[5 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ho = p.H / 2, bands = Ho / V2B, Wp = p.W / 2;
  for (int i = tid; i < 5 * 64; i += WNTH) coef[i] = p.bnc[i];

  auto issue = [&](int tile, int set) __attribute__((always_inline)) {
    const bool live = tile < p.ntiles;
    const int n = live ? tile / bands : 0, band = live ? tile - (tile / bands) * bands : 0;
    char* sa = smem + set * V2SET;
    const size_t base = (((size_t)n * Ho + band * V2B) * WO) * 64;
#pragma unroll
    for (int l = 0; l < V2LR; ++l) {
      const int q = tid + WNTH * l;
      const int px = q >> 3, c = v2_chunk(px, q & 7);
      const size_t off = base + (size_t)px * 64 + c * 8;
      const void* sd = live ? (const void*)(p.dA + off) : p.zero;
      const void* sy = live ? (const void*)(p.y + off) : p.zero;
      __builtin_amdgcn_global_load_lds(sd, (__attribute__((address_space(3))) void*)(sa + (64 * wave + WNTH * l) * 16),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds(sy, (__attribute__((address_space(3))) void*)(sa + V2RAW +
                                                                                      (64 * wave + WNTH * l) * 16),
                                       16, 0, 0);
    }
    const int ih0 = 2 * band * V2B - 3;
    char* sp = sa + 2 * V2RAW;
#pragma unroll
    for (int l = 0; l < V2LP; ++l) {
      const int q = tid + WNTH * l;
      const int r = q >> 7, s = q & (SLOTS - 1);
      const int ih = ih0 + r, pr = s - 2;
      const bool ok = live && r < V2ROWS && (unsigned)ih < (unsigned)p.H && (unsigned)pr < (unsigned)Wp;
      const void* src = ok ? (const void*)(p.x + (((size_t)n * p.H + ih) * Wp + pr) * 8) : p.zero;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sp + (64 * wave + WNTH * l) * 16),
                                       16, 0, 0);
    }
  };

  __syncthreads();  // coef table
  float c_k1[8], c_k2[8], c_k3[8], c_sc[8], c_sh[8];
  {
    const int c8 = v2_chunk(tid >> 3, tid & 7) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      c_k1[k] = coef[c8 + k];
      c_k2[k] = coef[64 + c8 + k];
      c_k3[k] = coef[128 + c8 + k];
      c_sc[k] = coef[192 + c8 + k];
      c_sh[k] = coef[256 + c8 + k];
    }
  }
  const int wr = wave & 1, kh0 = (wave >> 1) * KB2;
  f32x4 acc[4][KB2];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int kb = 0; kb < KB2; ++kb) acc[cb][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;

  int tile = blockIdx.x;
  issue(tile, 0);
  for (int it = 0; tile < p.ntiles; ++it, tile += gridDim.x) {
    const int set = it & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this band's raw tiles and patch (own DMA)
    __builtin_amdgcn_s_barrier();                      // everyone's landed; the other set's readers are done
    asm volatile("" ::: "memory");
    issue(tile + gridDim.x, set ^ 1);                  // next band: in flight through convert + MFMAs
    char* const dyt = smem + set * V2SET;
    const char* const yt = dyt + V2RAW;
    // dA -> dy in place (each thread its own chunks: pixel rows (tid >> 3) + 32 l all share
    // the swizzle bits (row >> 1) & 3, so the logical channel chunk -- and the coefficients,
    // loaded once -- are the same for all of them)
#pragma unroll
    for (int l = 0; l < V2LR; ++l) {
      const int qq = tid + WNTH * l;
      u32x4* dp = reinterpret_cast<u32x4*>(dyt + qq * 16);
      const u32x4 da = *dp, yy = *reinterpret_cast<const u32x4*>(yt + qq * 16);
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 2 * e + h;
          const float d = h ? hi_bf(da[e]) : lo_bf(da[e]);
          const float yv = h ? hi_bf(yy[e]) : lo_bf(yy[e]);
          const float gk = (yv * c_sc[k] + c_sh[k]) > 0.f ? d : 0.f;
          v[h] = c_k1[k] * gk + c_k2[k] * yv + c_k3[k];
        }
        o[e] = pack2bf(v[0], v[1]);
      }
      *dp = o;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // dy tile complete
    asm volatile("" ::: "memory");
    const char* sp = dyt + 2 * V2RAW;
#pragma unroll 1
    for (int s = 0; s < WO / 16; ++s) {
      const int m0 = wr * WO + 16 * s;
      const int ow = 16 * s + 4 * g + q;
      bf16x4 af[4];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) af[cb] = tr4(dyt + dyt_off(m0 + 4 * g + q, cb * 32 + pp * 8));
#pragma unroll
      for (int kb = 0; kb < KB2; ++kb) {
        const int kh = (kh0 + kb) >> 1, t0 = 2 * ((kh0 + kb) & 1);
        const bf16x4 xf = tr4(sp + (2 * wr + kh) * (SLOTS * 16) + (ow + t0 + (pp >> 1)) * 16 + (pp & 1) * 8);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[cb][kb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af[cb], xf, acc[cb][kb], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* out = p.slab + (size_t)(blockIdx.x * 2 + wr) * 64 * 256;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = cb * 16 + 4 * (lane >> 4) + r;
#pragma unroll
      for (int kb = 0; kb < KB2; ++kb) out[co * 256 + (kh0 + kb) * 16 + (lane & 15)] = acc[cb][kb][r];
      if (kh0 != 0) {
        out[co * 256 + 224 + (lane & 15)] = 0.f;
        out[co * 256 + 240 + (lane & 15)] = 0.f;
      }
    }
}

}  // namespace

// v2 (variant 1 of pdt_stem_wgrad_v): slab rows = grid * 2
PDT_API int pdt_stem_wgrad_splits_v(int N, int H, int W, int Cout, int variant) {
  if (variant == 0) return pdt_stem_wgrad_splits_v1(N, H, W, Cout);
  if (variant != 1 || Cout != 64 || H % (2 * V2B) != 0 || W != 2 * WO || N < 1) return -5;
  const int ntiles = N * (H / 2 / V2B);
  return (ntiles < 256 ? ntiles : 256) * 2;
}

// Slab rows (splits) of the halo stem weight gradient; -5 when the geometry is not covered.
PDT_API int pdt_stem_wgrad_splits(int N, int H, int W, int Cout) { return pdt_stem_wgrad_splits_v(N, H, W, Cout, 0); }
static int pdt_stem_wgrad_splits_v1(int N, int H, int W, int Cout) {
  if (Cout != 64 || H % (2 * WB) != 0 || W != 2 * WO || N < 1) return -5;
  const int ntiles = N * (H / 2 / WB);
  return (ntiles < 256 ? ntiles : 256) * WNW;
}

// slab[splits][64][256] = per-wave partials of the stem weight gradient (space-to-depth layout)
// with the BN backward apply formed from dA, y and bnc = [k1; k2; k3; scale; shift] ([5][64]);
// reduce with pdt_wgrad_reduce(slab, out, nullptr, nullptr, splits, 64, 256, ...).
PDT_API int pdt_stem_wgrad_v(const void* x4, const void* dA, const void* y, const float* bnc, float* slab, int N,
                             int H, int W, int Cout, int variant, hipStream_t stream);

PDT_API int pdt_stem_wgrad(const void* x4, const void* dA, const void* y, const float* bnc, float* slab, int N, int H,
                           int W, int Cout, hipStream_t stream) {
  return pdt_stem_wgrad_v(x4, dA, y, bnc, slab, N, H, W, Cout, 0, stream);
}

// variant 0: v1 (register prefetch, 4-row bands), 1: v2 (all-DMA double-buffered, 2-row bands)
PDT_API int pdt_stem_wgrad_v(const void* x4, const void* dA, const void* y, const float* bnc, float* slab, int N,
                             int H, int W, int Cout, int variant, hipStream_t stream) {
  const int splits = pdt_stem_wgrad_splits_v(N, H, W, Cout, variant);
  if (splits < 0) return splits;
  // (every global offset is 64-bit: no element-count limit)
  static const void* zcache[PDT_MAX_DEV] = {};
  StemWgParams p;
  p.x = (const u16*)x4;
  p.dA = (const u16*)dA;
  p.y = (const u16*)y;
  p.bnc = bnc;
  p.slab = slab;
  p.zero = pdt_symbol_addr(HIP_SYMBOL(stem_zero), zcache);
  if (p.zero == nullptr) return PDT_ERR_SYMBOL;
  p.N = N; p.H = H; p.W = W;
  if (variant == 1) {
    p.ntiles = N * (H / 2 / V2B);
    hipLaunchKernelGGL(stem_wgrad2_kernel, dim3(splits / 2), dim3(WNTH), 0, stream, p);
  } else {
    p.ntiles = N * (H / 2 / WB);
    hipLaunchKernelGGL(stem_wgrad_kernel, dim3(splits / WNW), dim3(WNTH), 0, stream, p);
  }
  PDT_RETURN_LAUNCH();
}
