// Stride-1, pad-1 3x3 convolution (forward, and the data gradient -- itself a
// stride-1 3x3 conv of dY with the flipped, transposed weight) as an implicit
// GEMM that stages each input pixel ONCE per 64-channel chunk for all 9 taps.
//
// Why: the generic implicit GEMM (conv_nt_kernel.h) gathers the A operand per
// tap, so a 3x3 conv re-reads its input 9x through L2: ~64 B per CU-cycle of
// operand traffic at the MFMA rate, over what L2 delivers (the 3x3
// shapes ran at 20-44 % of their MFMA floor). Here a workgroup owns an output
// tile of BM = 224 consecutive output pixels = k = BM / W whole image rows
// (W in {14, 28, 56}), and stages the (k + 2)-row halo patch of its input
// chunk -- [rows][rs][64 ch] bf16, rs = W + 2 rounded up to a power of two >= 16
// -- into LDS with LDS-DMA; the 9 taps' A fragments are then ds_reads of that
// one patch at pixel offsets a * rs + b (a, b in {-1, 0, 1}). Operand traffic
// per MAC drops ~3x (weights now dominate), and the weights stream per tap
// through a 3-slot LDS-DMA ring.
//
//   out[m, n] = sum_{tap, c} X[pix(m) + off(tap), c] * B[n, tap * Cin + c]
//   fwd   : X = input,  B = weight [Cout][3][3][Cin],       off = (th - 1, tw - 1)
//   dgrad : X = dY,     B = pdt_wt_dgrad [Cin][3][3][Cout], off = (1 - th, 1 - tw)
//
// Patch LDS image: pixel q of the patch (row q / rs, column q % rs; column c
// holds input column c - 1, zero outside the image) is 128 B with its 16-B
// chunks XOR-swizzled by (q & 7). (The generic kernel's (q >> 1) & 7 is
// conflict-free only for fragments starting at a multiple of 4 pixels; the column
// shifts b = +-1 start them anywhere: 2-way conflicts on 2 of 3 taps, measured 3.1
// conflict cycles per LDS instruction; with q & 7 a fragment of 16 consecutive
// pixels is conflict-free at any start -- rows that wrap inside a fragment, W = 14,
// still collide.) rs is a multiple of 16, so a row shift (a * rs) leaves the swizzle
// unchanged and every A-fragment address is a per-lane constant (precomputed
// per column shift b) plus a wave-uniform offset: ~1.5 VALU per ds_read.
// Rows above / below the image (the tile may straddle images: rows are counted
// globally over N*H) read a dedicated zero region instead.
//
// Schedule (persistent: a workgroup walks items = (tile, 64-channel chunk)):
// ONE raw barrier per tap. Tap t's weight slot was issued two taps earlier and
// the next item's patch during this item's tap 0, both by LDS-DMA with counted
// vmcnt waits (never vmcnt(0) inside an item); the ring slot / patch buffer an
// issue overwrites was last read before the barrier that precedes the issue.
// Loads are issued for every item slot even past the last item (a zero source),
// so the vmcnt counts are the same on every pass.
//
// Epilogues (straight from the accumulators, no LDS staging -- the LDS holds
// in-flight prefetches): bf16 store (+ per-wave BatchNorm statistics partials,
// the forward), or the fused BatchNorm-backward partials of the unit the data
// gradient feeds (BnbArgs, one partial row per (tile, wave row)).
#include "conv_nt_kernel.h"

namespace pdt_nt {
namespace {

constexpr int HBM = 224;           // output pixels per tile
constexpr int HWM = 2;             // waves along M (112 rows = 7 MFMA row blocks each)
constexpr int PMAX = 384;          // patch pixels per buffer
constexpr int PBYTES = PMAX * 128;
constexpr int ZBYTES = 1024;       // zero region (reads land at ZOFF +- 256 B)

// BNB: 0 plain output; the fused BN-backward partials with the ReLU gate 1 off, 2 recomputed
// from y, 3 from the unit's bit mask (compiled per gate: a run-time gate branched per element)
template <int BN, int NTH, int SGN, int BNB>
__global__ void __launch_bounds__(NTH, 1) conv3x3_halo_kernel(NTParams p, int rs_log2, int ntm, int ntn, int ncc) {
  constexpr int WN = NTH / 64 / HWM;
  constexpr int MI = HBM / (HWM * 16);  // 7
  constexpr int NI = BN / (WN * 16);
  constexpr int SB = BN * 128;          // weight slot bytes (BN rows x 64 k)
  constexpr int LB = BN * 8 / NTH;      // LDS-DMA instructions per thread per weight slot
  constexpr int GP = NTH / 8;           // patch pixels per block-wide LDS-DMA instruction
  constexpr int LP = PMAX / GP;         // LDS-DMA instructions per thread per patch
  constexpr int ZOFF = 2 * PBYTES + ZBYTES / 2;
  constexpr int SLOT0 = 2 * PBYTES + ZBYTES;
  static_assert(LB >= 1 && NI >= 1 && PMAX % GP == 0 && LB + LP <= 63, "halo tile shape");
  __shared__ __attribute__((aligned(16))) char smem[SLOT0 + 3 * SB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int W = p.Ws, H = p.Hs, Cin = p.Cs, K = p.K;
  const int rs = 1 << rs_log2;
  const int k = HBM / W;                 // output rows per tile
  const int P = (k + 2) * rs;            // patch pixels used
  const int NH = p.M / W;                // global input rows (N * H; source and output grids coincide)

  for (int z = tid; z < ZBYTES / 16; z += NTH)
    *reinterpret_cast<u32x4*>(smem + 2 * PBYTES + z * 16) = u32x4{0u, 0u, 0u, 0u};

  // ---- per-lane A-fragment addressing: output row r of the tile -> patch pixel
  int aoff[MI][3][2];  // byte offset in a patch buffer of (row block i, column shift b, k-half kk), row shift 0
  int lrow[MI];        // output row (within the tile) of this lane's fragment row
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int r = wm * (HBM / HWM) + i * 16 + (lane & 15);
    const int lr = r / W, w = r - (r / W) * W;
    lrow[i] = lr;
    const int pb = (lr + 1) * rs + w + 1;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int q = pb + b - 1;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) aoff[i][b][kk] = q * 128 + (((q & 7) ^ (kk * 4 + (lane >> 4))) << 4);
    }
  }
  // B fragments: slot row = this wave's column, 16-B chunk swizzled like the generic kernel
  int boff[NI][2];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int row = wn * (BN / WN) + j * 16 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) boff[j][kk] = row * 128 + (swz(row, kk * 4 + (lane >> 4)) << 4);
  }

  const int ntiles = ntm * ntn;
  const int my_tiles = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nitems = my_tiles * ncc;
  auto item_tile = [&](int it) -> int { return (int)blockIdx.x + (it / ncc) * (int)gridDim.x; };

  // ---- LDS-DMA issue of one weight slot: B[n0 + r][tap * Cin + cc * 64 + chunk]
  auto issue_b = [&](int it, int tap, int slot) __attribute__((always_inline)) {
    const bool live = it < nitems;
    const int tile = live ? item_tile(it) : 0;
    const int n0 = (tile % ntn) * BN;
    const int cc = live ? it % ncc : 0;
    char* sb = smem + SLOT0 + slot * SB;
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      const int r = (tid >> 3) + (NTH / 8) * j;
      const void* g = live ? (const void*)(p.b + (size_t)(n0 + r) * K + tap * Cin + cc * 64 + swz(r, tid & 7) * 8)
                           : p.zero;
      __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(sb + (8 * wave + (NTH / 8) * j) * 128),
                                       16, 0, 0);
    }
  };
  // ---- LDS-DMA issue of one patch: pixel q = (tid >> 3) + GP * l, physical chunk tid & 7
  auto issue_patch = [&](int it, int buf) __attribute__((always_inline)) {
    const bool live = it < nitems;
    const int tile = live ? item_tile(it) : 0;
    const int g0 = (tile / ntn) * k - 1;  // global input row of patch row 0
    const int cc = live ? it % ncc : 0;
    char* sp = smem + buf * PBYTES;
#pragma unroll
    for (int l = 0; l < LP; ++l) {
      const int q = (tid >> 3) + GP * l;
      const int g = g0 + (q >> rs_log2);
      const int w = (q & (rs - 1)) - 1;
      const bool ok = live && q < P && g >= 0 && g < NH && w >= 0 && w < W;
      const int ch = (tid & 7) ^ (q & 7);
      const void* src = ok ? (const void*)(p.src + ((size_t)g * W + w) * Cin + cc * 64 + ch * 8)
                           : p.zero;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sp + (8 * wave + GP * l) * 128),
                                       16, 0, 0);
    }
  };

  f32x4 acc[MI][NI];
  // BatchNorm statistics (forward) / BN-backward partials (data gradient) of this wave's rows
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  __syncthreads();  // zero region written

  if (nitems > 0) {
    issue_patch(0, 0);
    issue_b(0, 0, 0);
    issue_b(0, 1, 1);
  }
  bool after_epi = false;  // the first tap after an epilogue waits for everything (its stores count too)
  for (int it = 0; it < nitems; ++it) {
    const int tile = item_tile(it);
    const int tm = tile / ntn, tn = tile % ntn;
    const int cc = it % ncc;
    const int pbuf = it & 1;
    // per-item row validity: taps with row shift -1 / +1 read zeros at the image's top / bottom
    bool vtop[MI], vbot[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const uint32_t gr = (uint32_t)(tm * k + lrow[i]);
      const uint32_t h = gr - fdiv(gr, p.div_HWm) * (uint32_t)H;  // div_HWm holds H here
      vtop[i] = h != 0;
      vbot[i] = h != (uint32_t)(H - 1);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // retire this tap's weight slot (and at tap 0 this item's patch): the younger loads stay in flight
      if (t == 0) {
        if (after_epi) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LB) : "memory");
      } else if (t <= 2) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LB + LP) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LB) : "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // the slot two taps ahead (it held tap t - 1, whose readers all passed this barrier)
      {
        const int t2 = t + 2;
        issue_b(t2 < 9 ? it : it + 1, t2 < 9 ? t2 : t2 - 9, t2 % 3);
      }
      if (t == 0) issue_patch(it + 1, pbuf ^ 1);  // the other buffer: last read by item it - 1
      const int th = t / 3, tw = t % 3;
      const int a = SGN * (th - 1), b = SGN * (tw - 1);
      const char* sb = smem + SLOT0 + (t % 3) * SB;  // tap t of every item sits in slot t % 3
      const int rowoff = pbuf * PBYTES + a * rs * 128;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 bfr[NI], af[MI];
#pragma unroll
        for (int j = 0; j < NI; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + boff[j][kk]);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          int addr = aoff[i][b + 1][kk] + rowoff;
          if (a < 0 && !vtop[i]) addr = ZOFF;
          if (a > 0 && !vbot[i]) addr = ZOFF;
          af[i] = *reinterpret_cast<const bf16x8*>(smem + addr);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
    after_epi = false;
    if (cc != ncc - 1) continue;

    // ------------------------------------------------------------ epilogue of tile (tm, tn)
    after_epi = true;
    const int m0 = tm * HBM, n0 = tn * BN;
    const int lr16 = lane & 15, lc = (lane >> 4) * 4;
    if constexpr (!BNB) {
      if (p.stats != nullptr) {
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const int srow = tm * HWM + wm;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          f32x2 s01 = {0.f, 0.f}, s23 = s01, q01 = s01, q23 = s01;
#pragma unroll
          for (int i = 0; i < MI; ++i) {  // rows past M hold zeros (zero patch rows)
            const f32x2 v01 = {acc[i][j][0], acc[i][j][1]}, v23 = {acc[i][j][2], acc[i][j][3]};
            s01 += v01;
            s23 += v23;
            q01 = __builtin_elementwise_fma(v01, v01, q01);
            q23 = __builtin_elementwise_fma(v23, v23, q23);
          }
          float s[4] = {row16_sum(s01.x), row16_sum(s01.y), row16_sum(s23.x), row16_sum(s23.y)};
          float q[4] = {row16_sum(q01.x), row16_sum(q01.y), row16_sum(q23.x), row16_sum(q23.y)};
          if (lr16 < 8) {
            const int r = lr16 & 3;
            const float sv = (r & 2) ? ((r & 1) ? s[3] : s[2]) : ((r & 1) ? s[1] : s[0]);
            const float qv = (r & 2) ? ((r & 1) ? q[3] : q[2]) : ((r & 1) ? q[1] : q[0]);
            const int col = n0 + wn * (BN / WN) + j * 16 + lc + r;
            p.stats[(size_t)((lr16 < 4 ? 0 : p.nstat_rows) + srow) * p.Ncol + col] = lr16 < 4 ? sv : qv;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wm * (HBM / HWM) + i * 16 + lr16;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int col = n0 + wn * (BN / WN) + j * 16 + lc;
          typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<u32x2*>(p.out + (size_t)m * p.ldo + col) =
              u32x2{pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3])};
        }
      }
    } else {
      // fused BN-backward partials of the unit this gradient feeds: g = relu_gate(dA) on the
      // bf16-rounded stored dA (exactly what the separate reduce pass would read); a gated-off
      // element is cleared in its packed word, the sums run on the packed fp32 VALU
      typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = n0 + wn * (BN / WN) + j * 16 + lc;
        const f32x4 mu = *reinterpret_cast<const f32x4*>(p.bnb.mean + col);
        f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sh = sc;
        if constexpr (BNB == 2) {
          sc = *reinterpret_cast<const f32x4*>(p.bnb.scale + col);
          sh = *reinterpret_cast<const f32x4*>(p.bnb.shift + col);
        }
        f32x2 s01 = {0.f, 0.f}, s23 = s01, q01 = s01, q23 = s01;
        // every row's y (and mask byte) is loaded before the first is used: one wait, not MI
        uint2 yv[MI];
        uint32_t mv[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int m = m0 + wm * (HBM / HWM) + i * 16 + lr16;
          const size_t e = (size_t)(m < p.M ? m : 0) * p.ldo + col;
          yv[i] = *reinterpret_cast<const uint2*>(p.bnb.y + e);
          // (col is a multiple of 4: this lane's 4 mask bits are the byte's low or high nibble)
          mv[i] = BNB == 3 ? (uint32_t)(p.bnb.mask[e >> 3] >> (e & 7)) : 0xfu;
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int m = m0 + wm * (HBM / HWM) + i * 16 + lr16;
          const bool rok = m < p.M;
          const size_t e = (size_t)(rok ? m : 0) * p.ldo + col;
          const uint2 yy = yv[i];
          const uint32_t mk = mv[i];
          const uint32_t w0 = pack2bf(acc[i][j][0], acc[i][j][1]), w1 = pack2bf(acc[i][j][2], acc[i][j][3]);
          if (rok) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<u32x2*>(p.out + e) = u32x2{w0, w1};
          }
          const uint32_t kb = rok ? mk : 0u;
          const uint32_t g0w = w0 & pdt_bf16_pair_keep(kb, 0), g1w = w1 & pdt_bf16_pair_keep(kb, 1);
          f32x2 ga = {lo_bf(g0w), hi_bf(g0w)}, gb = {lo_bf(g1w), hi_bf(g1w)};
          const f32x2 ya = {lo_bf(yy.x), hi_bf(yy.x)}, yb = {lo_bf(yy.y), hi_bf(yy.y)};
          if constexpr (BNB == 2) {
            const f32x2 za = __builtin_elementwise_fma(ya, f32x2{sc[0], sc[1]}, f32x2{sh[0], sh[1]});
            const f32x2 zb = __builtin_elementwise_fma(yb, f32x2{sc[2], sc[3]}, f32x2{sh[2], sh[3]});
            ga.x = za.x > 0.f ? ga.x : 0.f;
            ga.y = za.y > 0.f ? ga.y : 0.f;
            gb.x = zb.x > 0.f ? gb.x : 0.f;
            gb.y = zb.y > 0.f ? gb.y : 0.f;
          }
          s01 += ga;
          s23 += gb;
          q01 = __builtin_elementwise_fma(ga, ya - f32x2{mu[0], mu[1]}, q01);
          q23 = __builtin_elementwise_fma(gb, yb - f32x2{mu[2], mu[3]}, q23);
        }
        float s[4] = {s01.x, s01.y, s23.x, s23.y}, q[4] = {q01.x, q01.y, q23.x, q23.y};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[r] = row16_sum(s[r]);
          q[r] = row16_sum(q[r]);
        }
        if (lr16 == 0) {
          const int prow = p.bnb.row0 + tm * HWM + wm;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p.bnb.part[(size_t)prow * p.Ncol + col + r] = s[r];
            p.bnb.part[(size_t)(p.bnb.R + prow) * p.Ncol + col + r] = q[r];
          }
        }
      }
    }
    zero_acc();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
}

template <int BN, int NTH>
int launch_halo(const NTParams& p, int sgn, int rs_log2, hipStream_t st) {
  const int ntm = (p.M + HBM - 1) / HBM, ntn = p.Ncol / BN, ncc = p.Cs / 64;
  int grid = ntm * ntn;
  if (grid > 256) grid = 256;  // persistent: one workgroup per CU (LDS-bound residency)
  const int bnb = p.bnb.part == nullptr ? 0 : !p.bnb.relu ? 1 : p.bnb.mask == nullptr ? 2 : 3;
  auto go = [&](auto sgn_c, auto bnb_c) {
    hipLaunchKernelGGL((conv3x3_halo_kernel<BN, NTH, decltype(sgn_c)::value, decltype(bnb_c)::value>), dim3(grid),
                       dim3(NTH), 0, st, p, rs_log2, ntm, ntn, ncc);
  };
  using std::integral_constant;
  if (sgn > 0) {
    if (bnb == 0) go(integral_constant<int, 1>{}, integral_constant<int, 0>{});
    else if (bnb == 1) go(integral_constant<int, 1>{}, integral_constant<int, 1>{});
    else if (bnb == 2) go(integral_constant<int, 1>{}, integral_constant<int, 2>{});
    else go(integral_constant<int, 1>{}, integral_constant<int, 3>{});
  } else {
    if (bnb == 0) go(integral_constant<int, -1>{}, integral_constant<int, 0>{});
    else if (bnb == 1) go(integral_constant<int, -1>{}, integral_constant<int, 1>{});
    else if (bnb == 2) go(integral_constant<int, -1>{}, integral_constant<int, 2>{});
    else go(integral_constant<int, -1>{}, integral_constant<int, 3>{});
  }
  PDT_RETURN_LAUNCH();
}

constexpr int HALO_BN[NVAR_HALO] = {64, 128, 128};

}  // namespace

// Applicability of the halo kernel to a conv_nt geometry (see the header comment): 0 = ok.
int halo_geometry(const NTParams& p, int hv, int* sgn, int* rs_log2) {
  if (hv < 0 || hv >= NVAR_HALO) return -3;
  if (p.nth != 3 || p.ntw != 3 || p.sh != 1 || p.sw != 1 || !p.ident_out) return -5;
  if (p.Hm != p.Hs || p.Wm != p.Ws || p.pix != p.Cs || p.Cs % 64 != 0 || p.K != 9 * p.Cs || p.ldb != p.K) return -5;
  if (p.bias != nullptr || p.act != 0 || p.aux != nullptr || p.addend != nullptr || p.ldo != p.Ncol) return -5;
  if (p.Ncol % HALO_BN[hv] != 0) return -5;
  if (p.dh == 1 && p.dw == 1 && p.oh0 == -1 && p.ow0 == -1) *sgn = 1;
  else if (p.dh == -1 && p.dw == -1 && p.oh0 == 1 && p.ow0 == 1) *sgn = -1;
  else return -5;
  const int W = p.Ws;
  if (W < 1 || HBM % W != 0) return -5;
  int rs = 16, l = 4;
  while (rs < W + 2) { rs <<= 1; ++l; }
  if ((HBM / W + 2) * rs > PMAX) return -5;
  if ((long long)p.M * p.Ncol >= (1LL << 31) || (long long)p.M * p.Cs >= (1LL << 31)) return -5;
  *rs_log2 = l;
  return 0;
}

int halo_rows(int M) { return ((M + HBM - 1) / HBM) * HWM; }

int run_halo(int hv, const NTParams& p_in, hipStream_t st) {
  if (p_in.bnb.part2 != nullptr) return -5;  // (no second-unit partials in the halo epilogue)
  int sgn = 0, rs_log2 = 0;
  const int rc = halo_geometry(p_in, hv, &sgn, &rs_log2);
  if (rc) return rc;
  NTParams p = p_in;
  p.div_HWm = make_fastdiv(p.Hs);  // the kernel divides global rows by H
  p.zero = zero_chunk_addr();
  if (p.zero == nullptr) return PDT_ERR_SYMBOL;
  switch (hv) {
    case 0: return launch_halo<64, 256>(p, sgn, rs_log2, st);
    case 1: return launch_halo<128, 512>(p, sgn, rs_log2, st);
    case 2: return launch_halo<128, 256>(p, sgn, rs_log2, st);
  }
  return -3;
}

// ============================================================================
// Weight gradient of the same stride-1 3x3 convs, on the same halo patch:
//
//   dW[co][tap][c] = sum_m dY[m][co] * X[pix(m) + off(tap)][c]
//
// A workgroup owns (64 output channels co) x (one 64-channel input chunk) x all
// 9 taps = 36 K of fp32 accumulators and walks a contiguous range of 224-pixel
// tiles (a split of the pixel reduction); per tile it stages the dY tile
// [224 px][64 co] and the X halo patch ONCE (LDS-DMA, double-buffered, one
// barrier per tile) and runs 7 pixel k-steps x 9 taps of MFMAs on them, where
// the generic weight-gradient kernel re-gathers X once per tap column. Both
// operands are pixel-major ("K-outer"), so fragments come through the CDNA4
// transposing LDS read ds_read_b64_tr_b16 with per-lane row addresses: the X
// rows of tap (a, b) are the patch pixels pix(m) + a * rs + b. 8 waves: co half
// (32) x 16-channel block; each wave holds all 9 taps of its 32 x 16 block.
// Each workgroup writes its [64][9 * 64] fp32 partial into the split's slab;
// pdt_wgrad_reduce sums the slabs (deterministic, no atomics).
namespace {

struct HWParams {
  const u16* dy;   // [M][Mo]
  const u16* x;    // [M][C] (the conv input; same pixel grid as dY)
  float* slab;     // [splits][Mo][9 * C]
  const void* zero;  // the LDS-DMA padding source (kernel argument: no per-issue GOT reload)
  int M, Mo, C, H, W, rs_log2, ntiles, tps, nco, ncc;
  FastDiv div_H;
};

constexpr int HW_DY = HBM * 128;                 // dY tile bytes (224 px x 64 co)
constexpr int HW_ZOFF = 2 * PBYTES + 2 * HW_DY;  // zero region
constexpr int HW_LDS = HW_ZOFF + ZBYTES;

// 8-byte transposed read: lane gets 4 k-consecutive bf16 of one column (see conv_wgrad.hip tr_frag)
__device__ __forceinline__ bf16x4 tr_read(const char* smem, int byte) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (bf16x4 __attribute__((address_space(3)))*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(
          uintptr_t)(smem + byte)));
}

__global__ void __launch_bounds__(512, 1) wgrad3x3_halo_kernel(HWParams p) {
  constexpr int NTH = 512, KS = HBM / 32;  // 7 pixel k-steps per tile
  constexpr int LP = PMAX / (NTH / 8);     // 6 patch LDS-DMA per thread
  __shared__ __attribute__((aligned(16))) char smem[HW_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave >> 2, wg = wave & 3;  // co half, 16-channel block
  const int W = p.W, H = p.H, C = p.C;
  const int rs = 1 << p.rs_log2;
  const int k = HBM / W;
  const int P = (k + 2) * rs;
  const int NH = p.M / W;

  const int bid = (int)blockIdx.x;
  const int ct = bid % p.nco, cc = (bid / p.nco) % p.ncc, split = bid / (p.nco * p.ncc);
  const int co0 = ct * 64;
  const int t_begin = split * p.tps;
  const int t_end = min(p.ntiles, t_begin + p.tps);

  for (int z = tid; z < ZBYTES / 16; z += NTH)
    *reinterpret_cast<u32x4*>(smem + HW_ZOFF + z * 16) = u32x4{0u, 0u, 0u, 0u};

  // transposed-read lane roles: lane = 16 g + 4 q + pp -> rows 8 g + q (+4), columns 4 pp .. 4 pp + 3
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  // X (patch) read offsets per (k-step, row half h, column shift b), row shift 0
  int xoff[KS][2][3];
  int lrow[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = ks * 32 + 8 * g + q + 4 * h;  // tile-local output pixel
      const int lr = r / W, w = r - lr * W;
      lrow[ks][h] = lr;
      const int pb = (lr + 1) * rs + w + 1;
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int px = pb + b - 1;
        xoff[ks][h][b] = px * 128 + ((((wg * 2 + (pp >> 1)) ^ ((px >> 1) & 7))) << 4) + (pp & 1) * 8;
      }
    }
  // dY read offsets per (k-step, half, co block mi): row r, co = wc * 32 + mi * 16 + 4 pp
  auto dyoff = [&](int ks, int h, int mi) -> int {
    const int r = ks * 32 + 8 * g + q + 4 * h;
    return r * 128 + (((wc * 4 + mi * 2 + (pp >> 1)) ^ ((r >> 1) & 7)) << 4) + (pp & 1) * 8;
  };

  auto issue = [&](int tj, int buf) __attribute__((always_inline)) {
    const bool live = tj < t_end;
    const int g0 = (live ? tj : 0) * k - 1;
    char* sp = smem + buf * PBYTES;
#pragma unroll
    for (int l = 0; l < LP; ++l) {
      const int qq = (tid >> 3) + (NTH / 8) * l;
      const int gr = g0 + (qq >> p.rs_log2);
      const int w = (qq & (rs - 1)) - 1;
      const bool ok = live && qq < P && gr >= 0 && gr < NH && w >= 0 && w < W;
      const int ch = (tid & 7) ^ ((qq >> 1) & 7);
      const void* src = ok ? (const void*)(p.x + ((size_t)gr * W + w) * C + cc * 64 + ch * 8)
                           : p.zero;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sp + (8 * wave + 64 * l) * 128),
                                       16, 0, 0);
    }
    char* sd = smem + 2 * PBYTES + buf * HW_DY;
    const int m0 = (live ? tj : 0) * HBM;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      if (l == 3 && wave >= 4) break;  // rows 224..255 do not exist (wave-uniform)
      const int r = (tid >> 3) + 64 * l;
      const int m = m0 + r;
      const int ch = (tid & 7) ^ ((r >> 1) & 7);
      const void* src = (live && m < p.M) ? (const void*)(p.dy + (size_t)m * p.Mo + co0 + ch * 8)
                                          : p.zero;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sd + (8 * wave + 64 * l) * 128),
                                       16, 0, 0);
    }
  };

  f32x4 acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // zero region

  if (t_begin < t_end) issue(t_begin, 0);
  for (int tj = t_begin; tj < t_end; ++tj) {
    const int buf = (tj - t_begin) & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this tile's patch + dY (this thread's share)
    __builtin_amdgcn_s_barrier();                       // ... everyone's; and tile tj-1's readers are done
    asm volatile("" ::: "memory");
    issue(tj + 1, buf ^ 1);
    // row validity of the shifted taps: the image's top / bottom row reads the zero region
    bool vt[KS][2], vb[KS][2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t gr = (uint32_t)(tj * k + lrow[ks][h]);
        const uint32_t hh = gr - fdiv(gr, p.div_H) * (uint32_t)H;
        vt[ks][h] = hh != 0;
        vb[ks][h] = hh != (uint32_t)(H - 1);
      }
    const int pbase = buf * PBYTES;
    const int dbase = 2 * PBYTES + buf * HW_DY;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 dyf[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const bf16x4 lo = tr_read(smem, dbase + dyoff(ks, 0, mi));
        const bf16x4 hi = tr_read(smem, dbase + dyoff(ks, 1, mi));
        dyf[mi] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int a = t / 3 - 1, b = t % 3 - 1;
        int o0 = xoff[ks][0][b + 1] + pbase + a * rs * 128;
        int o1 = xoff[ks][1][b + 1] + pbase + a * rs * 128;
        if (a < 0) {
          if (!vt[ks][0]) o0 = HW_ZOFF + 256;
          if (!vt[ks][1]) o1 = HW_ZOFF + 256;
        }
        if (a > 0) {
          if (!vb[ks][0]) o0 = HW_ZOFF + 256;
          if (!vb[ks][1]) o1 = HW_ZOFF + 256;
        }
        const bf16x4 lo = tr_read(smem, o0);
        const bf16x4 hi = tr_read(smem, o1);
        const bf16x8 xf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)  // D rows = channels c (4 consecutive per lane), columns = co
          acc[t][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, dyf[mi], acc[t][mi], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // partial slab of this split: [co][tap * C + c]
  float* out = p.slab + (size_t)split * p.Mo * (9 * C);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int co = co0 + wc * 32 + mi * 16 + (lane & 15);
      const int c = cc * 64 + wg * 16 + (lane >> 4) * 4;
      *reinterpret_cast<f32x4*>(out + (size_t)co * (9 * C) + t * C + c) = acc[t][mi];
    }
}

}  // namespace

// Halo weight gradient: applicability (0 = ok) and split plan.
int halo_wgrad_plan(int M, int Mo, int C, int Hs, int Ws, int* splits, int* tps) {
  if (C % 64 || Mo % 64 || Ws < 1 || HBM % Ws) return -5;
  int rs = 16;
  while (rs < Ws + 2) rs <<= 1;
  if ((HBM / Ws + 2) * rs > PMAX || (long long)M * C >= (1LL << 31) || (long long)M * Mo >= (1LL << 31)) return -5;
  const int ntiles = (M + HBM - 1) / HBM;
  const int blocks = (Mo / 64) * (C / 64);
  int s = (256 + blocks - 1) / blocks;
  if (s > ntiles) s = ntiles;
  if (s < 1) s = 1;
  const int per = (ntiles + s - 1) / s;
  *tps = per;
  *splits = (ntiles + per - 1) / per;
  return 0;
}

int run_halo_wgrad(const void* dy, const void* x, float* slab, int M, int Mo, int C, int Hs, int Ws, int splits,
                   int tps, hipStream_t st) {
  int s2 = 0, t2 = 0;
  const int rc = halo_wgrad_plan(M, Mo, C, Hs, Ws, &s2, &t2);
  if (rc) return rc;
  if (s2 != splits || t2 != tps) return -2;  // the workspace was sized for another plan
  HWParams p;
  p.dy = (const u16*)dy;
  p.x = (const u16*)x;
  p.slab = slab;
  p.zero = zero_chunk_addr();
  if (p.zero == nullptr) return PDT_ERR_SYMBOL;
  p.M = M; p.Mo = Mo; p.C = C; p.H = Hs; p.W = Ws;
  int l = 4, rs = 16;
  while (rs < Ws + 2) { rs <<= 1; ++l; }
  p.rs_log2 = l;
  p.ntiles = (M + HBM - 1) / HBM;
  p.tps = tps;
  p.nco = Mo / 64;
  p.ncc = C / 64;
  p.div_H = make_fastdiv(Hs);
  hipLaunchKernelGGL(wgrad3x3_halo_kernel, dim3(p.nco * p.ncc * splits), dim3(512), 0, st, p);
  PDT_RETURN_LAUNCH();
}

}  // namespace pdt_nt
