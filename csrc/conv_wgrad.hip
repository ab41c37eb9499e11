// Weight-gradient implicit GEMM for NHWC bf16 convolutions (and plain "TN"
// GEMMs such as nn.Linear's dW) on MI355X MFMA, split over the pixel (K)
// dimension.
//
//   dW[co, tap*C + c] = sum_m dY[m, co] * X[n, oh*sh + oh0 + dh*th, ow*sw + ow0 + dw*tw, c]
//
// Both operands arrive "K-outer" (pixel rows, channels contiguous), so tiles
// are staged into LDS exactly as they come from HBM -- [64 pixel rows][BM|BN
// channels] -- and MFMA fragments are read with the CDNA4 hardware-transpose
// LDS read (ds_read_b64_tr_b16): per 16-lane group a 4-row x 16-column block
// is delivered column-major, i.e. four consecutive k of one channel per lane;
// two such reads give the 8-element bf16 fragment of mfma_f32_16x16x32_bf16.
// 32-byte segments of each LDS row are XOR-swizzled by a function of the row
// so the eight rows a 32-lane half touches fall on distinct banks.
//
// Each workgroup computes a BM x BN tile over a contiguous slice of the
// pixels and writes an fp32 partial slab; pdt_wgrad_reduce sums the slabs in
// a fixed order (bitwise deterministic, no atomics) and writes / accumulates
// the fp32 gradient.
//
// Workgroup shapes: 4 waves (2x2, up to 128x128, two workgroups per CU) or
// 8 waves (256x128 as 4x2, 128x256 as 2x4, 256x256 as 2x4 with a 128x64 tile
// per wave; one workgroup per CU). The 8-wave tiles halve the L2->LDS bytes
// per MFMA of the 128x128 tile: the big 3x3 weight gradients (No = 9*Cin up
// to 4608) are otherwise bound by the staging traffic, not the matrix cores.
#include "pdt_common.h"
#include <stdlib.h>
#include <type_traits>

namespace pdt_nt {  // the 3x3 halo-patch weight gradient (conv3x3_halo.hip), variant id WG_NVAR
int halo_wgrad_plan(int M, int Mo, int C, int Hs, int Ws, int* splits, int* tps);
int run_halo_wgrad(const void* dy, const void* x, float* slab, int M, int Mo, int C, int Hs, int Ws, int splits,
                   int tps, hipStream_t st);
}  // namespace pdt_nt

namespace {

struct WGParams {
  const u16* dy;     // [M][ldy] (co contiguous)
  const u16* x;      // NHWC source [N][Hs][Ws][C]
  float* slab;       // [splits][Mo][No]
  int M;             // pixels (K of the GEMM)
  int Mo, No;        // Mo = Cout, No = ntaps*C
  int ldy;
  int Hs, Ws, C;
  int pix;           // elements per source pixel in memory (= C; C/2 for the space-to-depth stem)
  int Hm, Wm;        // output grid of the forward conv
  int sh, sw, oh0, ow0, dh, dw, ntw;
  int ktiles_per_split, splits;
  int xcd;           // 1: XCD-aware block mapping (PDT_WGRAD_XCD=0 disables, for A/B runs)
  float* bslab;      // optional [splits][Mo]: per-split column sums of dY (nn.Linear bias gradient),
                     // accumulated by the tn == 0 blocks from the dY tiles they stage anyway
  // BNA instantiations: `dy` is dA, the gradient at a BN+ReLU unit's output, and the unit's
  // BatchNorm backward apply is computed while staging it (no dy tensor is written):
  //   dY = k1 * (y*scale + shift > 0 ? dA : 0) + k2 * y + k3   (csrc/bn_act.hip bn_bwd_apply)
  const u16* bn_y;   // [M][ldy] the unit's pre-BN conv output
  const float* bn_c; // [5][Mo]: k1, k2, k3, scale, shift
  FastDiv div_Wm, div_HWm, div_C, div_ntw;
  const void* zero;  // 16 zero bytes: the source of padding / out-of-range chunks (every load is issued)
};

constexpr int BK = 64;
constexpr int NT = 256;

static __device__ __attribute__((aligned(64))) u32x4 wg_zero_chunk[4];

// XOR applied to the 32-B segment index of an LDS row. A transposed read's
// 32-lane half touches rows {8g + q : g = 0,1, q = 0..3} (+4) in one logical
// segment; for rows of >= 256 B (a whole bank row or more) the swizzle gives
// those 8 rows 8 distinct values mod 8 -> 8 distinct 32-B bank groups.
template <int RB>
__device__ __forceinline__ int seg_swz(int row) {
  if (RB >= 256) return (row & 3) | ((row >> 1) & 4);
  return ((row >> 1) & 1) | ((row >> 2) & 2);  // RB == 128
}

template <int RB>
__device__ __forceinline__ int lds_off(int row, int byte_in_row) {
  int seg = byte_in_row >> 5;
  return row * RB + ((seg ^ seg_swz<RB>(row)) << 5) + (byte_in_row & 31);
}

template <int RB>
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int krow0, int col0, int lane) {
  // lane = 16*g + 4*q + p :  rows krow0 + 8g + q (+4), columns col0 + 4p .. +3
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int r1 = krow0 + 8 * g + q;
  const int cb = (col0 + 4 * pp) * 2;
  typedef __bf16 __attribute__((address_space(3))) * lptr;
  const char* a1 = base + lds_off<RB>(r1, cb);
  const char* a2 = base + lds_off<RB>(r1 + 4, cb);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(
      (__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)a1));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bf16x4 __attribute__((address_space(3)))*)(
      (__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)a2));
  (void)sizeof(lptr);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// PF = register prefetch slots (NSTAGE == 2 only): with PF = 2 the global loads
// of tile k+3 are issued right after tile k's barrier and land in LDS two
// compute phases later (PF = 1: one), so a workgroup keeps ~2x the bytes in
// flight -- the large weight gradients are load-latency bound otherwise.
template <int BM, int BN, int NSTAGE, int NTH = NT, int WM = 2, int PF = 1, bool BIAS = false, bool BNA = false>
__global__ void __launch_bounds__(NTH, NTH == NT ? 2 : 1) wgrad_kernel(WGParams p) {
  static_assert(!BNA || (PF == 1 && !BIAS), "the staged BN-backward apply: single register slot, no bias");
  constexpr int WN = NTH / 64 / WM;    // waves along the (tap, c) columns
  constexpr int RBA = BM * 2;   // bytes per A row (co)
  constexpr int RBB = BN * 2;   // bytes per B row (tap,c)
  constexpr int A_BYTES = BK * RBA;
  constexpr int B_BYTES = BK * RBB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int ACH = BM / 8;          // 16-B chunks per A row
  constexpr int AROWS = NTH / ACH;     // rows covered per pass
  constexpr int NA = BK / AROWS;       // A chunks per thread
  constexpr int BCH = BN / 8;
  constexpr int BROWS = NTH / BCH;
  constexpr int NB = BK / BROWS;
  constexpr int MI = BM / (WM * 16);   // co 16-tiles per wave
  constexpr int NI = BN / (WN * 16);   // tc 16-tiles per wave
  static_assert(NA >= 1 && NB >= 1 && MI >= 1 && NI >= 1 && WM * WN * 64 == NTH, "wgrad tile shape");
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int ntm = (p.Mo + BM - 1) / BM, ntn = (p.No + BN - 1) / BN;
  const int ntiles = ntm * ntn;
  // XCD-aware: a contiguous run of logical ids (= the tiles of one or a few
  // pixel splits) stays on one XCD, so the dY / X slices those tiles share are
  // fetched into that XCD's L2 once instead of once per XCD
  const int bid = p.xcd ? (int)xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int tile = bid % ntiles;  // consecutive blocks: same split, different tiles
  const int split = bid / ntiles;
  const int tm = tile / ntn, tn = tile % ntn;
  const int co0 = tm * BM, tc0 = tn * BN;

  const int nk_total = (p.M + BK - 1) / BK;
  const int kt_begin = split * p.ktiles_per_split;
  const int kt_end = min(nk_total, kt_begin + p.ktiles_per_split);

  // A (dY) chunk of this thread: column chunk cA, rows rA0 + AROWS*i
  const int cA = tid % ACH, rA0 = tid / ACH;
  const int coA = co0 + cA * 8;
  const bool okA = coA < p.Mo;
  // B (X gather) chunk: fixed column -> fixed (tap, c)
  const int cB = tid % BCH, rB0 = tid / BCH;
  const int colB = tc0 + cB * 8;
  const bool okB = colB < p.No;
  int tap = fdiv(okB ? colB : 0, p.div_C);
  const int cB_ch = (okB ? colB : 0) - tap * p.C;
  const int th = fdiv(tap, p.div_ntw), tw = tap - th * p.ntw;
  const int offh = p.oh0 + p.dh * th, offw = p.ow0 + p.dw * tw;

  u32x4 ra[NA], rb[NB];
  // BNA: the y chunks beside the dA chunks, row validity, this thread's 8 channels' coefficients
  u32x4 ry[BNA ? NA : 1];
  bool rv[BNA ? NA : 1];
  float c1[BNA ? 8 : 1], c2[BNA ? 8 : 1], c3[BNA ? 8 : 1], csc[BNA ? 8 : 1], csh[BNA ? 8 : 1];
  if constexpr (BNA) {
    const int c0 = okA ? coA : 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      c1[e] = p.bn_c[c0 + e];
      c2[e] = p.bn_c[p.Mo + c0 + e];
      c3[e] = p.bn_c[2 * p.Mo + c0 + e];
      csc[e] = p.bn_c[3 * p.Mo + c0 + e];
      csh[e] = p.bn_c[4 * p.Mo + c0 + e];
    }
  }
  // bias gradient on the matrix cores: the tn == 0 blocks also multiply their
  // dY fragments by a fragment of ones (the wn == 0 waves' sums are written) (D[tc][co] = sum_m dY[m][co]
  // in every tc lane), MI extra MFMAs per 16*NI; they run their OWN copy of the
  // k-loop (compile-time DB below) so the other blocks' loop is the plain one.
  // (Summing the staged registers on the VALU instead cost every block 20-30 %.)
  const bool dobias = BIAS && tn == 0;  // block-uniform (the loop copies hold barriers)
  f32x4 bacc[BIAS ? MI : 1];
#pragma unroll
  for (int i = 0; i < (BIAS ? MI : 1); ++i) bacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_into = [&](int kt, u32x4 (&ra)[NA], u32x4 (&rb)[NB]) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      // every load is issued (padding from the zero page): a load under a per-chunk condition
      // is branched around and waited for one by one
      int m = k0 + rA0 + AROWS * i;
      const bool ok = okA && m < p.M;
      ra[i] = *reinterpret_cast<const u32x4*>(ok ? (const void*)(p.dy + (size_t)m * p.ldy + coA) : p.zero);
      if constexpr (BNA) {
        rv[i] = ok;
        ry[i] = *reinterpret_cast<const u32x4*>(ok ? (const void*)(p.bn_y + (size_t)m * p.ldy + coA) : p.zero);
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int m = k0 + rB0 + BROWS * i;
      bool ok = okB && m < p.M;
      uint32_t mm = ok ? m : 0;
      uint32_t img = fdiv(mm, p.div_HWm);
      uint32_t rem = mm - img * (uint32_t)(p.Hm * p.Wm);
      uint32_t oh = fdiv(rem, p.div_Wm);
      uint32_t ow = rem - oh * p.Wm;
      int ih = (int)(oh * p.sh) + offh, iw = (int)(ow * p.sw) + offw;
      ok = ok && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws;
      rb[i] = *reinterpret_cast<const u32x4*>(
          ok ? (const void*)(p.x + ((size_t)(img * p.Hs + ih) * p.Ws + iw) * p.pix + cB_ch) : p.zero);
    }
  };
  auto load_tile = [&](int kt) { load_into(kt, ra, rb); };
  auto store_from_db = [&](auto, int buf, const u32x4 (&ra)[NA], const u32x4 (&rb)[NB]) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      u32x4 v = ra[i];
      if constexpr (BNA) {  // dY from dA and y (rows past M stay zero)
        float g[8], y[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          g[2 * e] = lo_bf(v[e]); g[2 * e + 1] = hi_bf(v[e]);
          y[2 * e] = lo_bf(ry[i][e]); y[2 * e + 1] = hi_bf(ry[i][e]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          g[k] = (y[k] * csc[k] + csh[k]) > 0.f ? g[k] : 0.f;
          g[k] = c1[k] * g[k] + c2[k] * y[k] + c3[k];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = rv[i] ? pack2bf(g[2 * e], g[2 * e + 1]) : 0u;
      }
      *reinterpret_cast<u32x4*>(sa + lds_off<RBA>(rA0 + AROWS * i, cA * 16)) = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      *reinterpret_cast<u32x4*>(sb + lds_off<RBB>(rB0 + BROWS * i, cB * 16)) = rb[i];
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](auto, const char* sa) {
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bfr[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = tr_frag<RBB>(sb, kk * 32, wn * (BN / WN) + j * 16, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bf16x8 af = tr_frag<RBA>(sa, kk * 32, wm * (BM / WM) + i * 16, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af, acc[i][j], 0, 0, 0);
      }
    }
  };

  auto kloop = [&](auto db) {
  auto store_from = [&](int buf, const u32x4 (&ra)[NA], const u32x4 (&rb)[NB]) { store_from_db(db, buf, ra, rb); };
  auto store_tile = [&](int buf) { store_from(buf, ra, rb); };
  if constexpr (PF == 2) {
    static_assert(NSTAGE == 2, "deep prefetch uses the 2-stage LDS ring");
    // slot A = (ra, rb), slot B = (rb2 pair); loop unrolled by 2 so slots stay compile-time
    u32x4 ra2[NA], rb2[NB];
    const int n = kt_end - kt_begin;
    if (n > 0) {
      load_into(kt_begin, ra, rb);
      store_from(0, ra, rb);
    }
    if (n > 1) load_into(kt_begin + 1, ra2, rb2);
    if (n > 2) load_into(kt_begin + 2, ra, rb);
    __syncthreads();
    for (int i = 0; i < n; i += 2) {
      // tile i in LDS stage 0, tile i+1 in slot B, tile i+2 in flight to slot A
      compute(db, smem);
      if (i + 1 < n) store_from(1, ra2, rb2);
      __syncthreads();
      if (i + 3 < n) load_into(kt_begin + i + 3, ra2, rb2);
      if (i + 1 >= n) break;
      // tile i+1 in LDS stage 1, tile i+2 in slot A, tile i+3 in flight to slot B
      compute(db, smem + STAGE);
      if (i + 2 < n) store_from(0, ra, rb);
      __syncthreads();
      if (i + 4 < n) load_into(kt_begin + i + 4, ra, rb);
    }
  } else {
  if (kt_begin < kt_end) {
    load_tile(kt_begin);
    store_tile(0);
  }
  __syncthreads();
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int cur = NSTAGE == 2 ? ((kt - kt_begin) & 1) : 0;
    if (kt + 1 < kt_end) load_tile(kt + 1);
    // B fragments for the whole k-step, A fragments one 16-row tile at a time
    // (the 128x64-per-wave tile would otherwise hold 12 fragments at once)
    compute(db, smem + cur * STAGE);
    if (NSTAGE == 2) {
      if (kt + 1 < kt_end) store_tile(cur ^ 1);
      __syncthreads();
    } else if (kt + 1 < kt_end) {
      __syncthreads();
      store_tile(0);
      __syncthreads();
    }
  }
  }
  };
  kloop(std::integral_constant<bool, false>{});

  if constexpr (BIAS) {
    if (dobias) {
      // column sums of dY[k-range of this split][co0, co0 + BM): thread = (16-B chunk, row phase)
      constexpr int CPR = BM / 8, RPP = NTH / CPR;
      const int cc = tid % CPR, rr = tid / CPR;
      const int co = co0 + cc * 8;
      float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (co < p.Mo) {
        const int m1 = min(p.M, kt_end * BK);
        int m = kt_begin * BK + rr;
        for (; m + 3 * RPP < m1; m += 4 * RPP) {  // 4 rows in flight
          u32x4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const u32x4*>(p.dy + (size_t)(m + u * RPP) * p.ldy + co);
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bs[2 * e] += lo_bf(v[u][e]);
              bs[2 * e + 1] += hi_bf(v[u][e]);
            }
        }
        for (; m < m1; m += RPP) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(p.dy + (size_t)m * p.ldy + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bs[2 * e] += lo_bf(v[e]);
            bs[2 * e + 1] += hi_bf(v[e]);
          }
        }
      }
      __syncthreads();  // operand stages are free
      float* red = reinterpret_cast<float*>(smem);  // [NTH][8]
#pragma unroll
      for (int k = 0; k < 8; ++k) red[tid * 8 + k] = bs[k];
      __syncthreads();
      if (tid < CPR && co < p.Mo) {
        float t8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < RPP; ++j)
#pragma unroll
          for (int k = 0; k < 8; ++k) t8[k] += red[(j * CPR + tid) * 8 + k];
        float* bo = p.bslab + (size_t)split * p.Mo + co;
        *reinterpret_cast<f32x4*>(bo) = f32x4{t8[0], t8[1], t8[2], t8[3]};
        *reinterpret_cast<f32x4*>(bo + 4) = f32x4{t8[4], t8[5], t8[6], t8[7]};
      }
    }
  }

  float* out = p.slab + (size_t)split * p.Mo * p.No;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    int co = co0 + wm * (BM / WM) + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      int tc = tc0 + wn * (BN / WN) + j * 16 + (lane >> 4) * 4;
      if (co < p.Mo && tc < p.No) {
        *reinterpret_cast<f32x4*>(out + (size_t)co * p.No + tc) = acc[i][j];
      }
    }
  }
}

// Two-stage deterministic slab reduction.
// stage 1: grid (ceil(n4/256), G): block (x, g) sums slabs g, g+G, g+2G, ... for
//          256 float4 columns -> part[g][n4]   (G = 1 writes the output directly)
// stage 2: out = (accumulate ? out : 0) + scale * sum_g part[g]
__global__ void wgrad_reduce1_kernel(const float* __restrict__ slab, float* __restrict__ dst, long n4, int splits,
                                     int G, float scale, int accumulate, int final_stage) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int g = blockIdx.y;
  const f32x4* s = reinterpret_cast<const f32x4*>(slab) + i;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  int k = g;
  for (; k + G < splits; k += 2 * G) {
    a += s[(long)k * n4];
    b += s[(long)(k + G) * n4];
  }
  if (k < splits) a += s[(long)k * n4];
  a += b;
  f32x4* o = reinterpret_cast<f32x4*>(dst) + (final_stage ? i : (long)g * n4 + i);
  if (final_stage) {
    a *= scale;
    if (accumulate) a += *o;
  }
  *o = a;
}

}  // namespace

// Variants (autotuned per shape from Python; -1 = heuristic: tile from Mo/No, 2 stages, ~1024 WGs):
//   0..11 : v = tile * 3 + cfg, 4-wave tiles {64x64, 64x128, 128x64, 128x128} (Mo x No);
//           cfg 0 = 2 LDS stages / ~1024 workgroups, 1 = 1 stage / ~1024, 2 = 1 stage / ~2048
//   12..17: 8-wave tiles, 2 LDS stages: 256x128 and 128x256 (64x64 per wave) at ~512 and ~1024
//           workgroups; 256x256 (128x64 per wave, 128 KB LDS) at ~256 and ~512
struct WGVar {
  int BM, BN, NS, NTH, target;
};
//   18..27: NS = 3 marks the 2-stage ring with 2 register prefetch slots (PF = 2)
constexpr int WG_NVAR = 28;
constexpr WGVar WG_VARS[WG_NVAR] = {
    {64, 64, 2, 256, 1024},   {64, 64, 1, 256, 1024},   {64, 64, 1, 256, 2048},
    {64, 128, 2, 256, 1024},  {64, 128, 1, 256, 1024},  {64, 128, 1, 256, 2048},
    {128, 64, 2, 256, 1024},  {128, 64, 1, 256, 1024},  {128, 64, 1, 256, 2048},
    {128, 128, 2, 256, 1024}, {128, 128, 1, 256, 1024}, {128, 128, 1, 256, 2048},
    {256, 128, 2, 512, 512},  {128, 256, 2, 512, 512},  {256, 128, 2, 512, 1024},
    {128, 256, 2, 512, 1024}, {256, 256, 2, 512, 256},  {256, 256, 2, 512, 512},
    {64, 128, 3, 256, 1024},  {128, 64, 3, 256, 1024},  {128, 128, 3, 256, 1024},
    {128, 128, 3, 256, 2048}, {64, 64, 3, 256, 2048},   {256, 128, 3, 512, 512},
    {128, 256, 3, 512, 512},  {256, 128, 3, 512, 1024}, {128, 256, 3, 512, 1024},
    {256, 256, 3, 512, 512},
};
static WGVar wg_variant(int v, int Mo, int No) {
  if (v < 0 || v >= WG_NVAR) return WGVar{Mo <= 64 ? 64 : 128, No <= 64 ? 64 : 128, 2, 256, 1024};
  return WG_VARS[v];
}

// + 1: the 3x3 halo-patch kernel (id WG_NVAR; NOT_APPLICABLE (-5) outside stride-1 3x3 geometry)
// + 2: the 256x256 ping-pong ring (id WG_RING, csrc/wgrad_ring.hip; Mo, No multiples of 256)
constexpr int WG_RING = WG_NVAR + 1;
PDT_API int pdt_wgrad_num_variants() { return WG_NVAR + 2; }
PDT_API int pdt_wgrad_halo_id() { return WG_NVAR; }
PDT_API int pdt_wgrad_ring_id() { return WG_RING; }
PDT_API int pdt_wgrad_ring_ok(int Mo, int No, int C, int pix);
PDT_API int pdt_wgrad_ring_launch(const void* dy, const void* x, float* slab, int M, int Mo, int No, int ldy,
                                  int Hs, int Ws, int C, int Hm, int Wm, int sh, int sw, int oh0, int ow0, int dh,
                                  int dw, int ntw, int splits, int ktiles_per_split, int pix, hipStream_t st);

// the ring's split plan: one workgroup per CU, so the dispatch-wave model -- splits s <= the
// k-tiles / 8 minimising (waves of tiles*s over the CUs) x (k-tiles per split)
static int wgrad_ring_plan(int M, int Mo, int No, int* ktiles_per_split) {
  const int tiles = (Mo / 256) * (No / 256);
  const int nk = (M + BK - 1) / BK;
  const long slots = pdt_num_cus();
  int splits = 1;
  long best_cost = -1;
  for (int s = 1; s <= nk; ++s) {
    const int kps = (nk + s - 1) / s;
    if (s > 1 && kps < 8) break;
    const int se = (nk + kps - 1) / kps;
    const long cost = (((long)tiles * se + slots - 1) / slots) * kps;
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      splits = s;
    }
  }
  const int kps = (nk + splits - 1) / splits;
  *ktiles_per_split = kps;
  return (nk + kps - 1) / kps;
}

// the BN-backward-apply instantiations: the 4-wave, 1/2-stage tiles (variants 0..11)
static void launch_wg_bna(const WGVar& w, dim3 grid, const WGParams& p, hipStream_t stream) {
#define WG_LAUNCH_B(a, b, c) hipLaunchKernelGGL((wgrad_kernel<a, b, c, NT, 2, 1, false, true>), grid, dim3(NT), 0, stream, p)
  if (w.NS == 2) {
    if (w.BM == 64 && w.BN == 64) WG_LAUNCH_B(64, 64, 2);
    else if (w.BM == 64) WG_LAUNCH_B(64, 128, 2);
    else if (w.BN == 64) WG_LAUNCH_B(128, 64, 2);
    else WG_LAUNCH_B(128, 128, 2);
  } else {
    if (w.BM == 64 && w.BN == 64) WG_LAUNCH_B(64, 64, 1);
    else if (w.BM == 64) WG_LAUNCH_B(64, 128, 1);
    else if (w.BN == 64) WG_LAUNCH_B(128, 64, 1);
    else WG_LAUNCH_B(128, 128, 1);
  }
#undef WG_LAUNCH_B
}

template <bool BIAS>
static void launch_wg(const WGVar& w, dim3 grid, const WGParams& p, hipStream_t stream) {
  const int BM = w.BM, BN = w.BN, NS = w.NS;
#define WG_LAUNCH(a, b, c) hipLaunchKernelGGL((wgrad_kernel<a, b, c, NT, 2, 1, BIAS>), grid, dim3(NT), 0, stream, p)
#define WG_LAUNCH8(a, b, wm) hipLaunchKernelGGL((wgrad_kernel<a, b, 2, 512, wm, 1, BIAS>), grid, dim3(512), 0, stream, p)
#define WG_LAUNCH_PF(a, b, t, wm) hipLaunchKernelGGL((wgrad_kernel<a, b, 2, t, wm, 2, BIAS>), grid, dim3(t), 0, stream, p)
  if (NS == 3) {
    if (w.NTH == 512) {
      if (BM == 256 && BN == 256) WG_LAUNCH_PF(256, 256, 512, 2);
      else if (BM == 256) WG_LAUNCH_PF(256, 128, 512, 4);
      else WG_LAUNCH_PF(128, 256, 512, 2);
    } else {
      if (BM == 64 && BN == 64) WG_LAUNCH_PF(64, 64, 256, 2);
      else if (BM == 64) WG_LAUNCH_PF(64, 128, 256, 2);
      else if (BN == 64) WG_LAUNCH_PF(128, 64, 256, 2);
      else WG_LAUNCH_PF(128, 128, 256, 2);
    }
  } else if (w.NTH == 512) {
    if (BM == 256 && BN == 256) WG_LAUNCH8(256, 256, 2);
    else if (BM == 256) WG_LAUNCH8(256, 128, 4);
    else WG_LAUNCH8(128, 256, 2);
  } else if (NS == 2) {
    if (BM == 64 && BN == 64) WG_LAUNCH(64, 64, 2);
    else if (BM == 64) WG_LAUNCH(64, 128, 2);
    else if (BN == 64) WG_LAUNCH(128, 64, 2);
    else WG_LAUNCH(128, 128, 2);
  } else {
    if (BM == 64 && BN == 64) WG_LAUNCH(64, 64, 1);
    else if (BM == 64) WG_LAUNCH(64, 128, 1);
    else if (BN == 64) WG_LAUNCH(128, 64, 1);
    else WG_LAUNCH(128, 128, 1);
  }
#undef WG_LAUNCH
#undef WG_LAUNCH8
#undef WG_LAUNCH_PF
}

// the kernel launch_wg / launch_wg_bna start for a variant (for the occupancy query)
template <bool BIAS, bool BNA>
static const void* wg_kernel(const WGVar& w) {
#define KP(a, b, c, t, wm, pf) return reinterpret_cast<const void*>(&wgrad_kernel<a, b, c, t, wm, pf, BIAS, BNA>)
  const int BM = w.BM, BN = w.BN, NS = w.NS;
  if constexpr (!BNA) {
    if (NS == 3) {
      if (w.NTH == 512) {
        if (BM == 256 && BN == 256) KP(256, 256, 2, 512, 2, 2);
        if (BM == 256) KP(256, 128, 2, 512, 4, 2);
        KP(128, 256, 2, 512, 2, 2);
      }
      if (BM == 64 && BN == 64) KP(64, 64, 2, NT, 2, 2);
      if (BM == 64) KP(64, 128, 2, NT, 2, 2);
      if (BN == 64) KP(128, 64, 2, NT, 2, 2);
      KP(128, 128, 2, NT, 2, 2);
    }
    if (w.NTH == 512) {
      if (BM == 256 && BN == 256) KP(256, 256, 2, 512, 2, 1);
      if (BM == 256) KP(256, 128, 2, 512, 4, 1);
      KP(128, 256, 2, 512, 2, 1);
    }
  }
  if (NS == 2) {
    if (BM == 64 && BN == 64) KP(64, 64, 2, NT, 2, 1);
    if (BM == 64) KP(64, 128, 2, NT, 2, 1);
    if (BN == 64) KP(128, 64, 2, NT, 2, 1);
    KP(128, 128, 2, NT, 2, 1);
  }
  if (BM == 64 && BN == 64) KP(64, 64, 1, NT, 2, 1);
  if (BM == 64) KP(64, 128, 1, NT, 2, 1);
  if (BN == 64) KP(128, 64, 1, NT, 2, 1);
  KP(128, 128, 1, NT, 2, 1);
#undef KP
}

// workgroups of variant v resident on the device at once: the occupancy API's minimum over
// the instantiations the variant may launch (plain, bias, and -- variants 0..11 -- the BN
// backward apply), cached per variant
static long wg_slots(int v, const WGVar& w) {
  static int cache[WG_NVAR] = {};
  if (v < 0 || v >= WG_NVAR) return 2L * pdt_num_cus();
  if (cache[v] == 0) {
    int n = 1 << 20;
    const void* ks[3] = {wg_kernel<false, false>(w), wg_kernel<true, false>(w),
                         (w.NS <= 2 && w.NTH == NT) ? wg_kernel<false, true>(w) : nullptr};
    for (const void* k : ks) {
      int b = 0;
      if (k == nullptr) continue;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k, w.NTH, 0) != hipSuccess) b = 1;
      n = b < n ? b : n;
    }
    cache[v] = n < 1 ? 1 : n;
  }
  return (long)cache[v] * pdt_num_cus();
}

// Plan: splits s = ceil(target / tiles), at least 8 k-tiles per split so the pipeline
// amortises. Returns splits and writes ktiles_per_split.
// PDT_WG_PLAN=1: s <= ceil(target / tiles) minimising (dispatch waves) x (k-tiles per split)
// with wg_slots() workgroups resident -- the plan that took the fp8 weight gradient's
// one-workgroup-per-CU tiles from 3 dispatch waves to 1 (csrc/wgrad_f8.hip); on these
// multi-workgroup-per-CU tiles it picked grids of ~512 workgroups where ~2048 cycling through
// the resident slots hide latency better (ResNet-50: 290-650 vs 262-582 us per call,
// gpurun_out r4t vs r4w), so it is off by default here.
PDT_API int pdt_wgrad_plan(int M, int Mo, int No, int variant, int* ktiles_per_split) {
  const WGVar w = wg_variant(variant, Mo, No);
  const int BM = w.BM, BN = w.BN, target = w.target;
  int tiles = ((Mo + BM - 1) / BM) * ((No + BN - 1) / BN);
  int nk = (M + BK - 1) / BK;
  int smax = (target + tiles - 1) / tiles;
  if (smax > nk) smax = nk;
  if (smax < 1) smax = 1;
  static int mode = -1;  // PDT_WG_PLAN: 0 legacy for every tile, 1 wave plan for every tile, unset: by tile
  if (mode < 0) {
    const char* e = getenv("PDT_WG_PLAN");
    mode = (e && e[0] == '0') ? 0 : (e && e[0] == '1') ? 1 : 2;
  }
  int splits = smax;
  // the wave model fits one-workgroup-per-CU tiles (every resident workgroup runs at the same
  // rate): those take it by default; multi-workgroup tiles only with PDT_WG_PLAN=1
  const long slots = wg_slots(variant, w);
  if (mode == 0 || (mode == 2 && slots > pdt_num_cus())) {
    while (splits > 1 && (nk + splits - 1) / splits < 8) --splits;
  } else {
    long best_cost = -1;
    for (int s = 1; s <= smax; ++s) {
      const int kps = (nk + s - 1) / s;
      if (s > 1 && kps < 8) break;
      const int se = (nk + kps - 1) / kps;
      const long cost = (((long)tiles * se + slots - 1) / slots) * kps;
      if (best_cost < 0 || cost < best_cost) {
        best_cost = cost;
        splits = s;
      }
    }
  }
  int kps = (nk + splits - 1) / splits;
  splits = (nk + kps - 1) / kps;
  *ktiles_per_split = kps;
  return splits;
}

// Plan with the conv geometry (the halo variant's split depends on it): splits, and the
// per-split k-tiles (generic) or 224-pixel tiles (halo). -5: variant not applicable.
PDT_API int pdt_wgrad_plan2(int M, int Mo, int No, int Hs, int Ws, int C, int variant, int* per_split) {
  if (variant == WG_NVAR) {
    int splits = 0;
    const int rc = pdt_nt::halo_wgrad_plan(M, Mo, C, Hs, Ws, &splits, per_split);
    return rc ? rc : splits;
  }
  if (variant == WG_RING) {
    if (pdt_wgrad_ring_ok(Mo, No, C, 0) != 0) return -5;
    return wgrad_ring_plan(M, Mo, No, per_split);
  }
  return pdt_wgrad_plan(M, Mo, No, variant, per_split);
}

// stage-1 slab groups of the reduction: enough (column-block x group) blocks to stream the slabs
static int reduce_groups(int splits, int Mo, int No) {
  long n4 = (long)Mo * No / 4;
  int xb = (int)((n4 + 255) / 256);
  int G = splits < 2 ? 1 : (int)(1024 / xb);
  if (G > splits / 4) G = splits / 4;
  if (G < 1) G = 1;
  return G;
}

// floats of workspace pdt_conv_wgrad needs for `splits` slabs: slabs + stage-1
// partials + the [splits][Mo] bias-gradient slab
PDT_API long pdt_wgrad_workspace(int splits, int Mo, int No) {
  const long G = reduce_groups(splits, Mo, No);
  return (long)splits * Mo * No + (G > 1 ? G * Mo * No : 0) + (long)splits * Mo;
}

PDT_API int pdt_wgrad_reduce(float* slab, float* out, const float* bslab, float* bias_out, int splits, int Mo, int No,
                             float scale, int accumulate, hipStream_t stream);

// pdt_conv_wgrad2: the same with an optional BatchNorm backward apply on the dY operand
// (WGParams.bn_y / bn_c: `dy` is then dA); variants 0..11 only (NOT_APPLICABLE otherwise).
PDT_API int pdt_conv_wgrad2(const void* dy, const void* x, float* slab, float* out, int M, int Mo, int No,
                            int ldy, int Hs, int Ws, int C, int Hm, int Wm, int sh, int sw, int oh0, int ow0,
                            int dh, int dw, int ntw, int splits, int ktiles_per_split, float scale,
                            int accumulate, int variant, int pix, float* bias_out, const void* bn_y,
                            const float* bn_c, hipStream_t stream);

PDT_API int pdt_conv_wgrad(const void* dy, const void* x, float* slab, float* out, int M, int Mo, int No,
                           int ldy, int Hs, int Ws, int C, int Hm, int Wm, int sh, int sw, int oh0, int ow0,
                           int dh, int dw, int ntw, int splits, int ktiles_per_split, float scale,
                           int accumulate, int variant, int pix, float* bias_out, hipStream_t stream) {
  return pdt_conv_wgrad2(dy, x, slab, out, M, Mo, No, ldy, Hs, Ws, C, Hm, Wm, sh, sw, oh0, ow0, dh, dw, ntw, splits,
                         ktiles_per_split, scale, accumulate, variant, pix, bias_out, nullptr, nullptr, stream);
}

PDT_API int pdt_conv_wgrad2(const void* dy, const void* x, float* slab, float* out, int M, int Mo, int No,
                            int ldy, int Hs, int Ws, int C, int Hm, int Wm, int sh, int sw, int oh0, int ow0,
                            int dh, int dw, int ntw, int splits, int ktiles_per_split, float scale,
                            int accumulate, int variant, int pix, float* bias_out, const void* bn_y,
                            const float* bn_c, hipStream_t stream) {
  if (C % 8 != 0 || Mo % 8 != 0 || No % 8 != 0 || ldy % 8 != 0) return -1;
  const bool bna = bn_y != nullptr;
  if (bna && (bn_c == nullptr || variant < 0 || variant >= 12 || bias_out != nullptr)) return -5;
  if (pix != 0 && (pix % 4 != 0 || pix > C)) return -10;
  if (variant == WG_NVAR) {  // 3x3 / stride 1 / pad 1 halo-patch kernel
    if (ntw != 3 || No != 9 * C || sh != 1 || sw != 1 || oh0 != -1 || ow0 != -1 || dh != 1 || dw != 1 ||
        Hm != Hs || Wm != Ws || (pix != 0 && pix != C) || ldy != Mo || bias_out != nullptr || M % Wm != 0)
      return -5;
    const int rc = pdt_nt::run_halo_wgrad(dy, x, slab, M, Mo, C, Hs, Ws, splits, ktiles_per_split, stream);
    if (rc) return rc;
    return pdt_wgrad_reduce(slab, out, nullptr, nullptr, splits, Mo, No, scale, accumulate, stream);
  }
  if (variant == WG_RING) {  // the 256x256 ping-pong ring (plain dY, no bias)
    if (bna || bias_out != nullptr) return -5;
    const int rc = pdt_wgrad_ring_launch(dy, x, slab, M, Mo, No, ldy, Hs, Ws, C, Hm, Wm, sh, sw, oh0, ow0, dh, dw, ntw,
                                         splits, ktiles_per_split, pix, stream);
    if (rc) return rc;
    return pdt_wgrad_reduce(slab, out, nullptr, nullptr, splits, Mo, No, scale, accumulate, stream);
  }
  WGParams p;
  p.dy = (const u16*)dy;
  p.x = (const u16*)x;
  p.slab = slab;
  p.M = M; p.Mo = Mo; p.No = No; p.ldy = ldy;
  p.Hs = Hs; p.Ws = Ws; p.C = C; p.Hm = Hm; p.Wm = Wm;
  p.pix = pix > 0 ? pix : C;
  p.sh = sh; p.sw = sw; p.oh0 = oh0; p.ow0 = ow0; p.dh = dh; p.dw = dw; p.ntw = ntw;
  p.ktiles_per_split = ktiles_per_split; p.splits = splits;
  p.bn_y = (const u16*)bn_y;
  p.bn_c = bn_c;
  const int G = reduce_groups(splits, Mo, No);
  // bias_out (optional, fp32 [Mo]): also the column sums of dY, from the same pass
  p.bslab = bias_out ? slab + (long)splits * Mo * No + (G > 1 ? (long)G * Mo * No : 0) : nullptr;
  {
    static int xcd_env = -1;
    if (xcd_env < 0) {
      const char* e = getenv("PDT_WGRAD_XCD");
      xcd_env = (e && e[0] == '0') ? 0 : 1;
    }
    p.xcd = xcd_env;
  }
  p.div_Wm = make_fastdiv(Wm);
  p.div_HWm = make_fastdiv(Hm * Wm);
  p.div_C = make_fastdiv(C);
  p.div_ntw = make_fastdiv(ntw);
  {
    static const void* zc[PDT_MAX_DEV] = {};
    p.zero = pdt_symbol_addr(HIP_SYMBOL(wg_zero_chunk), zc);
    if (p.zero == nullptr) return PDT_ERR_SYMBOL;
  }
  const WGVar w = wg_variant(variant, Mo, No);
  int tiles = ((Mo + w.BM - 1) / w.BM) * ((No + w.BN - 1) / w.BN);
  dim3 grid(tiles * splits);
  if (bna) launch_wg_bna(w, grid, p, stream);
  else if (bias_out) launch_wg<true>(w, grid, p, stream);
  else launch_wg<false>(w, grid, p, stream);
  int e = (int)hipGetLastError();
  if (e) return e;
  return pdt_wgrad_reduce(slab, out, p.bslab, bias_out, splits, Mo, No, scale, accumulate, stream);
}

// Deterministic reduction of the split-K slabs [splits][Mo][No] (+ the optional bias slab
// [splits][Mo]) into out (= or += scale * sum); shared by the bf16 and fp8 weight gradients.
// row groups of the two-stage reduce of nrows partial rows (0: one stage)
static int reduce_rows_groups(int nrows) {
  if (nrows <= 32) return 0;
  int G = 1;
  while (G * G < nrows) ++G;
  return G > 64 ? 64 : G;
}

// floats of workspace pdt_wgrad_reduce_rows needs for nrows partial rows of n columns
PDT_API long pdt_reduce_rows_work(int nrows, int n) { return (long)reduce_rows_groups(nrows) * n; }

// out[n] (= or +=) scale * sum of nrows rows of [nrows][n] (n % 4 == 0): partial rows of a
// column sum (bias gradients). Many rows (an epilogue's per-tile rows, a LayerNorm backward's
// per-block rows) are summed in two stages through `work` (pdt_reduce_rows_work floats):
// the single-stage pass has only n / 1024 workgroups, each walking every row.
PDT_API int pdt_wgrad_reduce_rows(const float* rows, float* out, int nrows, int n, float scale, int accumulate,
                                  float* work, hipStream_t stream) {
  if (n % 4 != 0 || nrows < 1) return -1;
  const long n4 = n / 4;
  const int xb = (int)((n4 + 255) / 256);
  const int G = reduce_rows_groups(nrows);
  if (G > 1 && work != nullptr) {
    hipLaunchKernelGGL(wgrad_reduce1_kernel, dim3(xb, G), dim3(256), 0, stream, rows, work, n4, nrows, G, 1.f, 0, 0);
    hipLaunchKernelGGL(wgrad_reduce1_kernel, dim3(xb, 1), dim3(256), 0, stream, work, out, n4, G, 1, scale,
                       accumulate, 1);
  } else {
    hipLaunchKernelGGL(wgrad_reduce1_kernel, dim3(xb, 1), dim3(256), 0, stream, rows, out, n4, nrows, 1, scale,
                       accumulate, 1);
  }
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_wgrad_reduce(float* slab, float* out, const float* bslab, float* bias_out, int splits, int Mo, int No,
                             float scale, int accumulate, hipStream_t stream) {
  const int G = reduce_groups(splits, Mo, No);
  long n4 = (long)Mo * No / 4;
  int xb = (int)((n4 + 255) / 256);
  if (bias_out) {
    hipLaunchKernelGGL(wgrad_reduce1_kernel, dim3((Mo / 4 + 255) / 256, 1), dim3(256), 0, stream, bslab, bias_out,
                       (long)(Mo / 4), splits, 1, scale, accumulate, 1);
  }
  if (G == 1) {
    hipLaunchKernelGGL(wgrad_reduce1_kernel, dim3(xb, 1), dim3(256), 0, stream, slab, out, n4, splits, 1, scale,
                       accumulate, 1);
  } else {
    // stage-1 partials go to the workspace tail (pdt_wgrad_workspace), never into live slabs
    float* part = slab + (long)splits * Mo * No;
    hipLaunchKernelGGL(wgrad_reduce1_kernel, dim3(xb, G), dim3(256), 0, stream, slab, part, n4, splits, G, 1.f, 0,
                       0);
    hipLaunchKernelGGL(wgrad_reduce1_kernel, dim3(xb, 1), dim3(256), 0, stream, part, out, n4, G, 1, scale,
                       accumulate, 1);
  }
  PDT_RETURN_LAUNCH();
}
