// Weight-gradient GEMM on the 256x256 ping-pong ring (the schedule of csrc/gemm_ring.hip) for
// the K-outer operands of dW = dY^T X:
//
//   dW[co, tap*C + c] = sum_m dY[m, co] * X[n, oh*sh + oh0 + dh*th, ow*sw + ow0 + dw*tw, c]
//
// One 256 (co) x 256 (tap, c) output tile over a contiguous slice of the pixels m per
// 512-thread workgroup (8 waves as 2 x 4, 128 x 64 per wave), fp32 partial slabs reduced by
// pdt_wgrad_reduce (deterministic, no atomics) -- the contract of csrc/conv_wgrad.hip's tiles,
// so this is one more variant of pdt_conv_wgrad2 (id WG_RING).
//
// Both operands arrive pixel-major (channels contiguous), so a K-tile (64 pixels) is staged by
// LDS-DMA exactly as it sits in HBM and the MFMA fragments are read with the transposing
// ds_read_b64_tr_b16 (4 consecutive pixels of one channel per lane; two reads per 8-deep
// fragment). The stage is split into the ring's four quarters, each its own 16 KB LDS region
// of 64 pixel rows x 256 B: A rows of C-quadrant row 0 (co 0-63 and 128-191: the two wave rows'
// halves), B columns 0-127, B columns 128-255, A quadrant row 1. The 32-B segments of a region
// row are XOR-swizzled by the row (conflict-free transposed reads); the swizzle is applied to
// the DMA SOURCE, and each thread's physical slot maps to the same logical 8-channel chunk in
// every row it fills (the swizzle repeats every 8 rows, a thread's rows are 32 apart), so its
// B column -- tap and channel of the im2col gather -- is fixed: only the pixel decomposition
// runs per K-tile. Pixels past M, padding and out-of-image taps read a 16-byte zero page.
#include "pdt_common.h"

namespace {

constexpr int WBM = 256, WBN = 256, WBK = 64, WNTH = 512;
constexpr int RGN = WBK * 256;      // bytes per quarter region (64 rows x 256 B)
constexpr int WSTAGE = 4 * RGN;     // 64 KB
constexpr int WRB = 256;            // region row bytes

struct WRParams {
  const u16* dy;   // [M][ldy]
  const u16* x;    // NHWC source [N][Hs][Ws][pix]
  float* slab;     // [splits][Mo][No]
  const void* zero;
  int M, Mo, No, ldy;
  int Hs, Ws, C, pix, Hm, Wm;
  int sh, sw, oh0, ow0, dh, dw, ntw;
  int ktiles_per_split;
  FastDiv div_Wm, div_HWm, div_C, div_ntw;
};

// logical 32-B segment s of region row r sits at physical segment s ^ wr_swz(r)
__device__ __forceinline__ int wr_swz(int row) { return (row & 3) | ((row >> 1) & 4); }

// one transposed 8-byte LDS read (4 consecutive rows of one column per lane), issued as inline
// asm: hipcc's wait insertion treats the ds_read_tr builtin as possibly aliasing every LDS-DMA
// in flight and puts a vmcnt(0) -- the whole prefetch ring -- in front of each K-tile's reads.
// The asm result is consumed only after the section's explicit s_waitcnt lgkmcnt(0) (mma).
__device__ __forceinline__ bf16x4 tr_read(uint32_t addr) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

// 8-element bf16 fragment: rows krow0 + 8g + q (+4) (pixels), columns col0 + 4p .. +3 of a
// region at LDS byte address `base` (lane = 16 g + 4 q + p), as two transposed reads
__device__ __forceinline__ bf16x8 wr_frag(uint32_t base, int krow0, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int r1 = krow0 + 8 * g + q, r2 = r1 + 4;
  const int cb = (col0 + 4 * pp) * 2;
  const bf16x4 lo = tr_read(base + r1 * WRB + ((((cb >> 5) ^ wr_swz(r1))) << 5) + (cb & 31));
  const bf16x4 hi = tr_read(base + r2 * WRB + ((((cb >> 5) ^ wr_swz(r2))) << 5) + (cb & 31));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

__global__ void __launch_bounds__(WNTH, 1) wgrad_ring_kernel(WRParams p) {
  constexpr int WM = 2, WN = 4;
  constexpr int MI = WBM / WM / 16;  // 8
  constexpr int NI = WBN / WN / 16;  // 4
  constexpr int HM = MI / 2, HN = NI / 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * WSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntm = p.Mo / WBM, ntn = p.No / WBN;
  const int ntiles = ntm * ntn;
  const int bid = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tm = tile / ntn, tn = tile % ntn;
  const int co0 = tm * WBM, tc0 = tn * WBN;
  const int nk_total = (p.M + WBK - 1) / WBK;
  const int kt_begin = split * p.ktiles_per_split;
  const int kt_end = min(nk_total, kt_begin + p.ktiles_per_split);
  const int nk = kt_end - kt_begin;

  // ---- this thread's DMA slots: rows rr and rr + 32 of every region, physical 16-B chunk
  // pc = lane & 15 -> logical chunk lc (the same in both rows: the swizzle repeats every 8 rows)
  const int rr = 4 * wave + (lane >> 4);
  const int pc = lane & 15;
  const int lc = ((((pc >> 1) ^ wr_swz(rr))) << 1) | (pc & 1);
  // A (dY) regions: quadrant row r holds co {r*64 + [0,64)} U {128 + r*64 + [0,64)}
  const int a_co[2] = {co0 + (lc < 8 ? lc * 8 : 128 + (lc - 8) * 8), co0 + 64 + (lc < 8 ? lc * 8 : 128 + (lc - 8) * 8)};
  // B (X gather) halves: columns tc0 + h*128 + lc*8 -> (tap, c), fixed per thread
  int b_c[2], b_offh[2], b_offw[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int col = tc0 + h * 128 + lc * 8;
    const int tap = (int)fdiv((uint32_t)col, p.div_C);
    b_c[h] = col - tap * p.C;
    const int th = (int)fdiv((uint32_t)tap, p.div_ntw), tw = tap - th * p.ntw;
    b_offh[h] = p.oh0 + p.dh * th;
    b_offw[h] = p.ow0 + p.dw * tw;
  }
  // per K-tile: the source addresses of this thread's 2 rows in each of the 4 regions
  const void* src[4][2];
  auto prep = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = kt * WBK + rr + 32 * u;
      const bool ok = m < p.M;
      const uint32_t mm = ok ? m : 0;
      src[0][u] = ok ? (const void*)(p.dy + (size_t)mm * p.ldy + a_co[0]) : p.zero;
      src[3][u] = ok ? (const void*)(p.dy + (size_t)mm * p.ldy + a_co[1]) : p.zero;
      const uint32_t img = fdiv(mm, p.div_HWm);
      const uint32_t rem = mm - img * (uint32_t)(p.Hm * p.Wm);
      const uint32_t oh = fdiv(rem, p.div_Wm);
      const uint32_t ow = rem - oh * p.Wm;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ih = (int)(oh * p.sh) + b_offh[h], iw = (int)(ow * p.sw) + b_offw[h];
        const bool v = ok && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws;
        src[1 + h][u] = v ? (const void*)(p.x + ((size_t)(img * p.Hs + ih) * p.Ws + iw) * p.pix + b_c[h]) : p.zero;
      }
    }
  };
  // quarter q of a stage: region q (q0 = A row 0, q1 = B half 0, q2 = B half 1, q3 = A row 1)
  auto issue = [&](int q, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      __builtin_amdgcn_global_load_lds(src[q][u], (__attribute__((address_space(3))) void*)(
                                                      smem + buf * WSTAGE + q * RGN + (4 * wave + 32 * u) * WRB),
                                       16, 0, 0);
  };
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[HM][2], bq[HN][2];
  // A fragments of quadrant row r: region (r ? 3 : 0), local columns wm*64 + i*16
  const uint32_t lsm = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto read_a = [&](int cur, int r) __attribute__((always_inline)) {
    const uint32_t reg = lsm + cur * WSTAGE + (r ? 3 : 0) * RGN;
#pragma unroll
    for (int i = 0; i < HM; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = wr_frag(reg, kk * 32, wm * 64 + i * 16, lane);
  };
  // B fragments of column half c: region 1 + c, local columns wn*32 + j*16
  auto read_b = [&](int cur, int c) __attribute__((always_inline)) {
    const uint32_t reg = lsm + cur * WSTAGE + (1 + c) * RGN;
#pragma unroll
    for (int j = 0; j < HN; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bq[j][kk] = wr_frag(reg, kk * 32, wn * 32 + j * 16, lane);
  };
  auto pin = [&](int r, int c) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < HM; ++i)
#pragma unroll
      for (int j = 0; j < HN; ++j) asm volatile("" : "+v"(acc[r * HM + i][c * HN + j]));
  };
  auto mma = [&](int r, int c) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    pin(r, c);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < HM; ++i)
#pragma unroll
      for (int j = 0; j < HN; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          // swapped operands: lane holds 4 consecutive (tap, c) columns of one co row
          acc[r * HM + i][c * HN + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][kk], af[i][kk], acc[r * HM + i][c * HN + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    pin(r, c);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto bar = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mma_phase = [&](int r, int c) __attribute__((always_inline)) {
    bar();
    mma(r, c);
    bar();
  };
  if (nk > 0) {
    prep(kt_begin);
#pragma unroll
    for (int q = 0; q < 4; ++q) issue(q, 0);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // q0 q1 of the first K-tile
  }
  bar();
  if (wm == 1) bar();  // the stagger
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1, nxt = cur ^ 1;
    const bool more = t + 1 < nk;
    // M1: fragments of (0,0); retire q2 of this K-tile; the next K-tile's addresses and q0
    read_a(cur, 0);
    read_b(cur, 0);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    if (more) {
      prep(kt_begin + t + 1);
      issue(0, nxt);
    }
    mma_phase(0, 0);
    // M2: fragments of (0,1); retire q3; q1 of the next
    read_b(cur, 1);
    if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (more) issue(1, nxt);
    mma_phase(0, 1);
    // M3: fragments of (1,1); q2 of the next
    read_a(cur, 1);
    if (more) issue(2, nxt);
    mma_phase(1, 1);
    // M4: fragments of (1,0); retire q0 q1 of the next K-tile; q3 of the next
    read_b(cur, 0);
    if (more) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      issue(3, nxt);
    }
    mma_phase(1, 0);
  }
  if (wm == 0) bar();

  // ---- fp32 partial slab: co = co0 + wm*128 + i*16 + (lane & 15), tc = 4 consecutive
  float* out = p.slab + (size_t)split * p.Mo * p.No;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int co = co0 + wm * (WBM / WM) + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int tcl = j < NI / 2 ? wn * 32 + j * 16 : WBN / 2 + wn * 32 + (j - NI / 2) * 16;
      const int tc = tc0 + tcl + (lane >> 4) * 4;
      *reinterpret_cast<f32x4*>(out + (size_t)co * p.No + tc) = acc[i][j];
    }
  }
}

static __device__ __attribute__((aligned(64))) u32x4 wr_zero_chunk[4];

}  // namespace

// Applicability of the ring for a weight-gradient geometry (0 = applicable, -5 = not).
PDT_API int pdt_wgrad_ring_ok(int Mo, int No, int C, int pix) {
  if (Mo % WBM != 0 || No % WBN != 0 || C % 8 != 0 || (pix != 0 && pix != C)) return -5;
  return 0;
}

// The ring's launch; the caller (pdt_conv_wgrad2) plans the splits and reduces the slabs.
PDT_API int pdt_wgrad_ring_launch(const void* dy, const void* x, float* slab, int M, int Mo, int No, int ldy,
                                  int Hs, int Ws, int C, int Hm, int Wm, int sh, int sw, int oh0, int ow0, int dh,
                                  int dw, int ntw, int splits, int ktiles_per_split, int pix, hipStream_t st) {
  static const void* zcache[PDT_MAX_DEV] = {};
  if (pdt_wgrad_ring_ok(Mo, No, C, pix) != 0 || ldy % 8 != 0) return -5;
  if ((((uintptr_t)dy) | ((uintptr_t)x)) & 15) return -5;  // 16-B LDS-DMA chunks
  if (splits < 1 || ktiles_per_split < 1) return -1;
  WRParams p;
  p.dy = (const u16*)dy;
  p.x = (const u16*)x;
  p.slab = slab;
  p.zero = pdt_symbol_addr(HIP_SYMBOL(wr_zero_chunk), zcache);
  if (p.zero == nullptr) return PDT_ERR_SYMBOL;
  p.M = M; p.Mo = Mo; p.No = No; p.ldy = ldy;
  p.Hs = Hs; p.Ws = Ws; p.C = C; p.pix = pix > 0 ? pix : C; p.Hm = Hm; p.Wm = Wm;
  p.sh = sh; p.sw = sw; p.oh0 = oh0; p.ow0 = ow0; p.dh = dh; p.dw = dw; p.ntw = ntw;
  p.ktiles_per_split = ktiles_per_split;
  p.div_Wm = make_fastdiv(Wm);
  p.div_HWm = make_fastdiv(Hm * Wm);
  p.div_C = make_fastdiv(C);
  p.div_ntw = make_fastdiv(ntw);
  const int tiles = (Mo / WBM) * (No / WBN);
  hipLaunchKernelGGL(wgrad_ring_kernel, dim3(tiles * splits), dim3(WNTH), 0, st, p);
  PDT_RETURN_LAUNCH();
}
