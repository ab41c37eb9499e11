// Implicit-GEMM convolution (forward and data-gradient) for NHWC bf16 on
// MI355X (gfx950) MFMA.  Also serves plain "NT" GEMMs (nn.Linear forward).
//
//   C[m, n] = sum_k A[m, k] * B[n, k]            (fp32 accumulate)
//   A[m, k] = src[n_img, ih, iw, c]  gathered on the fly (zero outside)
//   k = tap * Cs + c,  tap = (th, tw) on a (nth x ntw) tap grid
//   ih = oh * sh + oh0 + dh * th,  iw = ow * sw + ow0 + dw * tw
//
// forward conv : M-grid = output (Ho, Wo), taps = (kh, kw), oh0 = -pad, dh = 1,
//                B = weight [Cout][KH][KW][Cin]
// dgrad conv   : one launch per stride phase (ph, pw): M-grid = (H/s, W/s),
//                taps = {kh : (ph+pad-kh) % s == 0}, source = dY, dh = -1,
//                B = phase-sliced transposed weight [Cin][nth][ntw][Cout];
//                output row (n, ph + s*hh, pw + s*ww) of dX.
//
// Tile: BM x BN x 64, 256 threads = 4 wave64s in 2x2, each wave (BM/2)x(BN/2)
// built from 16x16x32 bf16 MFMAs.  Operands are register-staged
// (global_load_dwordx4 -> ds_write_b128) into a double-buffered LDS ring with
// one barrier per K-tile; the next tile's global loads are in flight while
// the current tile's MFMAs run.  LDS rows are 128 B; 16-B chunks are
// XOR-swizzled with ((row >> 1) & 7) so every ds_read_b128 lane group hits 16
// distinct bank slots.
//
// The MFMA is issued with operands swapped (D = B·Aᵀ) so each lane holds four
// *consecutive output channels* of one output row: the epilogue packs them to
// 8-byte bf16 words, stages the tile through LDS and writes 16-B coalesced rows.
// Epilogue options: per-channel BatchNorm partial statistics (sum, sum of
// squares over the tile's rows, from the fp32 accumulators), bias, ReLU.
#include "conv_nt_kernel.h"

using namespace pdt_nt;

namespace {

// ---------------------------------------------------------------------------
// Streaming skinny-K GEMM for 1x1 convolutions (K = Cin or Cout in {64, 128, 256}):
//   out[m, n] = sum_k A[row(m), k] * B[n, k]
// The LDS-tiled kernel above runs ONE K-tile per output tile when K <= 64, so
// load -> MFMA -> store never overlap inside a workgroup, and its 128-KB
// tiles leave one workgroup per CU. These shapes (the 1x1 expansions
// 64->256 / 128->512 / 256->1024 and their data gradients) are pure HBM
// streams (~4-8 FLOP/B), so this kernel drops LDS and barriers entirely:
//   * every wave owns NJ x 16 output columns; their B fragments (NJ x K/32 x
//     16 B per lane) are loaded ONCE into registers;
//   * the wave walks 16-row M tiles rg, rg + nrg, ... (all waves advance
//     through A together: one streaming pass), loading each tile's A
//     fragments straight from HBM into registers one tile ahead;
//   * epilogue per tile: (+ ReLU-masked addend) -> bf16 -> 8-B stores; the
//     BatchNorm partial sums stay in registers for the whole walk and are
//     reduced once at the end (nrg partial rows instead of M/BM).
// Waves of one workgroup take different column blocks of the same rows, so
// an A tile is fetched from HBM once and re-read from L1/L2 by the others.
struct SParams {
  const u16* a;
  const u16* b;
  u16* out;
  float* stats;                 // optional: [2][nrg][N]
  const u16* addend;            // optional: [M][ldo]
  const uint8_t* addend_mask;   // optional: 1 bit per addend element
  int N, ldo, ntiles, ncb, nrg;
  int Hs, Ws, Hm, Wm, sh, sw;   // strided 1x1 source geometry (STRIDED only)
  BnbArgs bnb;                  // BNB only: fused BatchNorm-backward partials (see BnbArgs)
  FastDiv div_Wm, div_HWm;
};

template <int KK, int NJ, bool STRIDED, bool BNB = false>
__global__ void __launch_bounds__(256) gemm_stream_kernel(SParams p) {
  constexpr int KS = KK / 32;
  const int lane = threadIdx.x & 63;
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int gw = (int)blk * 4 + (threadIdx.x >> 6);
  const int cb = gw % p.ncb, rg = gw / p.ncb;
  if (rg >= p.nrg) return;  // whole wave: the grid is rounded up to 4 waves
  const int n0 = cb * NJ * 16;
  const int lr = lane & 15, lk = (lane >> 4) * 8;

  bf16x8 bf[NJ][KS];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      bf[j][ks] = *reinterpret_cast<const bf16x8*>(p.b + (size_t)(n0 + j * 16 + lr) * KK + ks * 32 + lk);

  auto a_row = [&](int t) -> const u16* {
    const uint32_t m = (uint32_t)t * 16 + lr;
    if (!STRIDED) return p.a + (size_t)m * KK;
    const uint32_t img = fdiv(m, p.div_HWm);
    const uint32_t rem = m - img * (uint32_t)(p.Hm * p.Wm);
    const uint32_t oh = fdiv(rem, p.div_Wm);
    const uint32_t ow = rem - oh * p.Wm;
    return p.a + ((size_t)(img * p.Hs + oh * p.sh) * p.Ws + ow * p.sw) * KK;
  };

  float s[NJ][4], q[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) s[j][r] = q[j][r] = 0.f;
  // BNB: per-channel mean / ReLU-gate coefficients of this lane's 4 x NJ columns (and the
  // second unit's mean / partials when BnbArgs.part2 is set)
  const bool two = BNB && p.bnb.part2 != nullptr;
  float mu[BNB ? NJ : 1][4], gsc[BNB ? NJ : 1][4], gsh[BNB ? NJ : 1][4], mu2[BNB ? NJ : 1][4],
      q2[BNB ? NJ : 1][4];
  if constexpr (BNB) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = n0 + j * 16 + (lane >> 4) * 4 + r;
        mu[j][r] = p.bnb.mean[c];
        mu2[j][r] = two ? p.bnb.mean2[c] : 0.f;
        q2[j][r] = 0.f;
        const bool from_y = p.bnb.relu && p.bnb.mask == nullptr;
        gsc[j][r] = from_y ? p.bnb.scale[c] : 0.f;
        gsh[j][r] = from_y ? p.bnb.shift[c] : 0.f;
      }
  }

  bf16x8 a[KS];
  {
    const u16* ap = a_row(rg < p.ntiles ? rg : 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) a[ks] = *reinterpret_cast<const bf16x8*>(ap + ks * 32 + lk);
  }
  for (int t = rg; t < p.ntiles; t += p.nrg) {
    // next tile's A (clamped: the last trip re-reads a valid tile instead of branching)
    bf16x8 an[KS];
    {
      const int tn = t + p.nrg < p.ntiles ? t + p.nrg : t;
      const u16* ap = a_row(tn);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) an[ks] = *reinterpret_cast<const bf16x8*>(ap + ks * 32 + lk);
    }
    const size_t m = (size_t)t * 16 + lr;
    // epilogue operands of THIS tile issued before its MFMAs (latency hidden behind them)
    uint2 adv[BNB ? NJ : 1], yyv[BNB ? NJ : 1], yyb[BNB ? NJ : 1];
    if constexpr (BNB) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const size_t e = m * p.ldo + n0 + j * 16 + (lane >> 4) * 4;
        adv[j] = p.addend != nullptr ? *reinterpret_cast<const uint2*>(p.addend + e) : uint2{0u, 0u};
        yyv[j] = *reinterpret_cast<const uint2*>(p.bnb.y + e);
        yyb[j] = two ? *reinterpret_cast<const uint2*>(p.bnb.y2 + e) : uint2{0u, 0u};
      }
    }
    f32x4 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        // swapped operands: lane holds 4 consecutive output channels of row lr
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], a[ks], acc[j], 0, 0, 0);

#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = n0 + j * 16 + (lane >> 4) * 4;
      float v[4] = {acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
      if (!BNB && p.stats != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[j][r] += v[r];
          q[j][r] += v[r] * v[r];
        }
      }
      const size_t e = m * p.ldo + col;
      if (p.addend != nullptr) {
        uint2 ad = BNB ? adv[BNB ? j : 0] : *reinterpret_cast<const uint2*>(p.addend + e);
        if (p.addend_mask != nullptr) {
          const uint32_t mb = p.addend_mask[e >> 3] >> (e & 7);
          ad.x &= ((mb & 1u) ? 0xffffu : 0u) | ((mb & 2u) ? 0xffff0000u : 0u);
          ad.y &= ((mb & 4u) ? 0xffffu : 0u) | ((mb & 8u) ? 0xffff0000u : 0u);
        }
        v[0] += lo_bf(ad.x); v[1] += hi_bf(ad.x); v[2] += lo_bf(ad.y); v[3] += hi_bf(ad.y);
      }
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 packed = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      *reinterpret_cast<u32x2*>(p.out + e) = packed;
      if constexpr (BNB) {  // partials of the gated, bf16-rounded stored value
        const uint2 yy = yyv[BNB ? j : 0];
        const float yv[4] = {lo_bf(yy.x), hi_bf(yy.x), lo_bf(yy.y), hi_bf(yy.y)};
        const float g0[4] = {lo_bf(packed[0]), hi_bf(packed[0]), lo_bf(packed[1]), hi_bf(packed[1])};
        const uint32_t mk = p.bnb.mask != nullptr ? (uint32_t)(p.bnb.mask[e >> 3] >> (e & 7)) : 0xfu;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bool on = true;
          if (p.bnb.relu) on = p.bnb.mask != nullptr ? ((mk >> r) & 1u) != 0 : (yv[r] * gsc[j][r] + gsh[j][r]) > 0.f;
          const float g = on ? g0[r] : 0.f;
          s[j][r] += g;
          q[j][r] += g * (yv[r] - mu[j][r]);
          if (two) {
            const uint32_t w = r < 2 ? yyb[BNB ? j : 0].x : yyb[BNB ? j : 0].y;
            q2[BNB ? j : 0][r] += g * ((r & 1 ? hi_bf(w) : lo_bf(w)) - mu2[BNB ? j : 0][r]);
          }
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) a[ks] = an[ks];
  }

  if (BNB || p.stats != nullptr) {
    float* part = BNB ? p.bnb.part : p.stats;
    const int prow = BNB ? p.bnb.row0 + rg : rg;
    const int ptot = BNB ? p.bnb.R : p.nrg;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // DPP row = the 16 lanes sharing these columns
        s[j][r] = row16_sum(s[j][r]);
        q[j][r] = row16_sum(q[j][r]);
        if (two) q2[BNB ? j : 0][r] = row16_sum(q2[BNB ? j : 0][r]);
      }
      if (lr == 0) {
        const int col = n0 + j * 16 + (lane >> 4) * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          part[(size_t)prow * p.N + col + r] = s[j][r];
          part[(size_t)(ptot + prow) * p.N + col + r] = q[j][r];
          if (two) {
            p.bnb.part2[(size_t)prow * p.N + col + r] = s[j][r];
            p.bnb.part2[(size_t)(ptot + prow) * p.N + col + r] = q2[BNB ? j : 0][r];
          }
        }
      }
    }
  }
}

// stream variants (conv_nt variant ids NVAR..NVAR+3): NJ in {2, 4} x ~2048 / ~4096 waves
constexpr int NVAR_STREAM = 4;
constexpr int STREAM_NJ[NVAR_STREAM] = {2, 2, 4, 4};
constexpr int STREAM_WAVES[NVAR_STREAM] = {2048, 4096, 2048, 4096};

// partial-stat rows (= row groups) of stream variant s; 0 if the column split does not fit
int stream_rows(int s, int M, int Ncol) {
  const int cols = STREAM_NJ[s] * 16;
  if (Ncol % cols || M % 16) return 0;
  const int ncb = Ncol / cols, ntiles = M / 16;
  int nrg = STREAM_WAVES[s] / ncb;
  if (nrg > ntiles / 2) nrg = ntiles / 2;  // >= 2 tiles per wave (one in flight)
  return nrg < 1 ? 1 : nrg;
}

constexpr int NOT_APPLICABLE_S = -5;  // = NOT_APPLICABLE below

template <int KK, int NJ>
int launch_stream(const SParams& p, bool strided, hipStream_t st) {
  const int blocks = (p.ncb * p.nrg + 3) / 4;
  if (p.bnb.part != nullptr) {
    if (strided) return NOT_APPLICABLE_S;  // a strided 1x1 GEMM is never a data gradient
    hipLaunchKernelGGL((gemm_stream_kernel<KK, NJ, false, true>), dim3(blocks), dim3(256), 0, st, p);
  } else if (strided) {
    hipLaunchKernelGGL((gemm_stream_kernel<KK, NJ, true>), dim3(blocks), dim3(256), 0, st, p);
  } else {
    hipLaunchKernelGGL((gemm_stream_kernel<KK, NJ, false>), dim3(blocks), dim3(256), 0, st, p);
  }
  PDT_RETURN_LAUNCH();
}

constexpr int NOT_APPLICABLE = -5;  // variant cannot run this geometry (the tuner skips it)

int run_stream(int s, const NTParams& p, hipStream_t st) {
  const int NJ = STREAM_NJ[s];
  const int K = p.K;
  // 1x1, unpadded, dense [N][K] weights, output row == m, no bias / activation / aux
  if (p.nth != 1 || p.ntw != 1 || p.oh0 != 0 || p.ow0 != 0 || !p.ident_out || p.Cs != K || p.ldb != K ||
      p.bias != nullptr || p.act != 0 || p.aux != nullptr)
    return NOT_APPLICABLE;
  if (!(K == 64 || K == 128 || K == 256) || (K == 256 && NJ == 4)) return NOT_APPLICABLE;
  const int nrg = stream_rows(s, p.M, p.Ncol);
  if (nrg == 0) return NOT_APPLICABLE;
  const bool strided = !(p.sh == 1 && p.sw == 1 && p.Hs == p.Hm && p.Ws == p.Wm);
  if (strided && ((p.Hm - 1) * p.sh >= p.Hs || (p.Wm - 1) * p.sw >= p.Ws)) return NOT_APPLICABLE;
  SParams q;
  q.a = p.src; q.b = p.b; q.out = p.out; q.stats = p.stats;
  q.addend = p.addend; q.addend_mask = p.addend_mask;
  q.N = p.Ncol; q.ldo = p.ldo; q.ntiles = p.M / 16; q.ncb = p.Ncol / (NJ * 16); q.nrg = nrg;
  q.Hs = p.Hs; q.Ws = p.Ws; q.Hm = p.Hm; q.Wm = p.Wm; q.sh = p.sh; q.sw = p.sw;
  q.bnb = p.bnb;
  q.div_Wm = p.div_Wm; q.div_HWm = p.div_HWm;
  if (K == 64) return NJ == 2 ? launch_stream<64, 2>(q, strided, st) : launch_stream<64, 4>(q, strided, st);
  if (K == 128) return NJ == 2 ? launch_stream<128, 2>(q, strided, st) : launch_stream<128, 4>(q, strided, st);
  return launch_stream<256, 2>(q, strided, st);
}

}  // namespace

// variant ids: [0, NVAR) the LDS-tiled kernels, then NVAR_STREAM streaming 1x1 kernels,
// then NVAR_HALO 3x3 halo-patch kernels (conv3x3_halo.hip), then NVAR_PERS persistent
// ring tiles (conv_nt_kernel.h PERS_BASE: appended, so the ids of the shipped tune table hold)
constexpr int HALO0 = NVAR + NVAR_STREAM;
constexpr int PERS0 = HALO0 + NVAR_HALO;
constexpr int NVAR_ALL = PERS0 + NVAR_PERS;

PDT_API int pdt_conv_nt_num_variants() { return NVAR_ALL; }

// 0: LDS-tiled (persistent ones included), 1: streaming 1x1, 2: 3x3 halo-patch
// (conv3x3_halo.hip); -1: no such variant
PDT_API int pdt_conv_nt_variant_kind(int v) {
  if (v < 0 || v >= NVAR_ALL) return -1;
  if (v >= PERS0) return 0;
  return v >= HALO0 ? 2 : (v >= NVAR ? 1 : 0);
}

PDT_API int pdt_conv_nt_resolve_variant(int variant, int M, int Ncol, int K) {
  return (variant >= 0 && variant < NVAR_ALL) ? variant : heuristic_variant(M, Ncol, K);
}

// the LDS-tiled variant whose tile (BM, BN, WM) a variant id uses
static inline int tile_of_variant(int v) { return v >= PERS0 ? PERS_BASE[v - PERS0] : v; }

// Number of BN-statistics partial rows a launch of `variant` writes (sizes the stats buffer).
// Partial rows a fused BN-backward launch (pdt_conv_nt_bnb) of `variant` writes:
// one per M-tile (lanes and waves reduced in-block), or the stream kernel's row groups.
PDT_API int pdt_conv_nt_bnb_rows(int M, int Ncol, int K, int variant) {
  int v = pdt_conv_nt_resolve_variant(variant, M, Ncol, K);
  if (v >= HALO0 && v < PERS0) return halo_rows(M);
  if (v >= NVAR && v < PERS0) return stream_rows(v - NVAR, M, Ncol);
  v = tile_of_variant(v);
  return (M + VAR_BM[v] - 1) / VAR_BM[v];
}

// 1 when a variant's BN-backward epilogue compiles this configuration: the ring tiles (ids
// 34-37 and the persistent ones) carry only a block's inner unit (ReLU recomputed from y) and a
// block input (addend + ReLU bit mask), without a second unit; the halo tiles no second unit.
PDT_API int pdt_conv_nt_bnb_supports(int variant, int has_addend, int has_mask, int relu, int two) {
  const int v = variant;
  if ((v >= 34 && v < NVAR) || v >= PERS0) {
    const bool inner = !has_addend && !has_mask && relu;
    const bool input = has_addend && has_mask && relu;
    return !two && (inner || input);
  }
  if (v >= HALO0 && v < PERS0) return !two;
  return 1;
}

PDT_API int pdt_conv_nt_stat_rows(int M, int Ncol, int K, int variant) {
  int v = pdt_conv_nt_resolve_variant(variant, M, Ncol, K);
  if (v >= HALO0 && v < PERS0) return halo_rows(M);
  if (v >= NVAR && v < PERS0) return stream_rows(v - NVAR, M, Ncol);
  v = tile_of_variant(v);
  int BM = VAR_BM[v];
  return ((M + BM - 1) / BM) * VAR_WM[v];
}

// Generic launch: see header comment for the meaning of every argument.
static int conv_nt_impl(const void* src, const void* b, void* out, float* stats, const float* bias,
                        const void* addend, const void* addend_mask,
                        int Hs, int Ws, int Cs, int Nimg, int Hm, int Wm, int Ncol, int K, int ldb,
                        int sh, int sw, int oh0, int ow0, int dh, int dw, int nth, int ntw,
                        int Ho, int Wo, int osh, int osw, int oph, int opw, int ldo, int act,
                        void* aux, int variant, const BnbArgs& bnb, int pix, hipStream_t stream,
                        const AXArgs& ax = AXArgs{}) {
  if (Cs % 8 != 0 || K % 8 != 0 || Ncol % 8 != 0 || ldo % 8 != 0 || ldb % 8 != 0) return -1;
  if (pix != 0 && (pix % 4 != 0 || pix > Cs)) return -10;
  if (K != nth * ntw * Cs) return -2;
  if ((act == 3 || act == 5) && (addend == nullptr || addend_mask != nullptr || aux != nullptr || bias != nullptr))
    return -4;
  if (act == 4 && (aux == nullptr || addend != nullptr)) return -4;  // dual GELU: aux = gelu'(z)
  if (act < 0 || act > 5) return -4;
  NTParams p;
  p.src = (const u16*)src;
  p.b = (const u16*)b;
  p.out = (u16*)out;
  p.stats = stats;
  p.bias = bias;
  p.addend = (const u16*)addend;
  p.addend_mask = (const uint8_t*)addend_mask;
  if (addend_mask && (!addend || ldo != Ncol)) return -4;  // mask indexes the dense [M][Ncol] addend
  p.Hs = Hs; p.Ws = Ws; p.Cs = Cs;
  p.Hm = Hm; p.Wm = Wm;
  p.M = Nimg * Hm * Wm;
  p.Ncol = Ncol; p.K = K; p.ldb = ldb;
  p.sh = sh; p.sw = sw; p.oh0 = oh0; p.ow0 = ow0; p.dh = dh; p.dw = dw; p.nth = nth; p.ntw = ntw;
  p.Ho = Ho; p.Wo = Wo; p.osh = osh; p.osw = osw; p.oph = oph; p.opw = opw; p.ldo = ldo;
  p.act = act;
  p.pix = pix > 0 ? pix : Cs;
  p.aux = (u16*)aux;
  p.dq_a = p.dq_b = nullptr;
  p.q8 = nullptr; p.q8_meta = nullptr; p.q8_part = nullptr; p.q8_fmt = 0; p.q8_only = 0;
  p.bnb = bnb;
  p.ax = ax;
  if (bnb.part != nullptr && (stats != nullptr || bias != nullptr || act != 0 || aux != nullptr || ldo != Ncol))
    return -7;  // the fused BN-backward epilogue is for plain (dense-output) data gradients
  p.div_Wm = make_fastdiv(Wm);
  p.div_HWm = make_fastdiv(Hm * Wm);
  p.div_Cs8 = make_fastdiv(Cs / 8);
  p.div_ntw = make_fastdiv(ntw > 0 ? ntw : 1);
  p.ident_out = (Hm == Ho && Wm == Wo && osh == 1 && osw == 1 && oph == 0 && opw == 0) ? 1 : 0;
  {
    static int nt_env = -1;
    if (nt_env < 0) {
      const char* e = getenv("PDT_NT_STORE");
      nt_env = (e && e[0] == '1') ? 1 : 0;
    }
    p.nt_store = nt_env;
  }
  const int v = pdt_conv_nt_resolve_variant(variant, p.M, Ncol, K);
  p.nstat_rows = pdt_conv_nt_stat_rows(p.M, Ncol, K, v);
  if (ax.mode != 0) {
    // the A-staging BN apply: stride-1 source walk, 64-channel k-tiles, dense pixels, unsigned
    // 32-bit element offsets into the source (AX_NONE excluded)
    if (sh != 1 || sw != 1 || p.pix != Cs || Cs % 64 != 0 || bias != nullptr || aux != nullptr || act != 0 ||
        (addend != nullptr && bnb.part == nullptr) || ax.c1 == nullptr || ax.c2 == nullptr ||
        (ax.mode == 2 && (ax.y2 == nullptr || ax.c3 == nullptr || ax.mask_in == nullptr)) ||
        (ax.mode == 3 && (ax.y2 == nullptr || ax.c3 == nullptr || ax.rsc == nullptr || ax.rsh == nullptr)) ||
        (ax.mode == 1 && ax.y2 == nullptr && ax.rsc != nullptr) ||
        (long long)Nimg * Hs * Ws * Cs >= (1LL << 32) - 8 || v >= NVAR)
      return -5;
    p.ax.ctr = -1;
    if (ax.dst != nullptr || ax.mask_out != nullptr) {
      // written from the tap that maps each output row onto its own source pixel: needs the
      // output grid == the source grid
      for (int th = 0; th < nth; ++th)
        for (int tw = 0; tw < ntw; ++tw)
          if (oh0 + dh * th == 0 && ow0 + dw * tw == 0) p.ax.ctr = th * ntw + tw;
      if (p.ax.ctr < 0 || Hm != Hs || Wm != Ws) return -5;
    }
    return launch_variant_ax(v, p, stream);
  }
  // ring tiles: only the BN-backward walks they compile (conv_nt_tile.inc) -- a block's inner unit
  // (ReLU recomputed from y) or a block input (addend + ReLU bit mask); no second-unit partials
  if (bnb.part != nullptr && ((v >= 34 && v < NVAR) || v >= PERS0) &&
      !pdt_conv_nt_bnb_supports(v, addend != nullptr, bnb.mask != nullptr, bnb.relu, bnb.part2 != nullptr))
    return -5;
  const bool cs64 = (Cs % 64) == 0;
  if (v >= PERS0) {
    if (bnb.part != nullptr) return launch_variant_pers_bnb(v - PERS0, cs64, p, stream);
    return cs64 ? launch_variant_pers<true>(v - PERS0, p, stream) : launch_variant_pers<false>(v - PERS0, p, stream);
  }
  if (v >= HALO0) return run_halo(v - HALO0, p, stream);
  if (v >= NVAR) return run_stream(v - NVAR, p, stream);
  if (bnb.part != nullptr) return launch_variant_bnb(v, cs64, p, stream);
  return cs64 ? launch_variant<true>(v, p, stream) : launch_variant<false>(v, p, stream);
}

PDT_API int pdt_conv_nt(const void* src, const void* b, void* out, float* stats, const float* bias,
                        const void* addend, const void* addend_mask,
                        int Hs, int Ws, int Cs, int Nimg, int Hm, int Wm, int Ncol, int K, int ldb,
                        int sh, int sw, int oh0, int ow0, int dh, int dw, int nth, int ntw,
                        int Ho, int Wo, int osh, int osw, int oph, int opw, int ldo, int act,
                        void* aux, int variant, int pix, hipStream_t stream) {
  BnbArgs none{};
  return conv_nt_impl(src, b, out, stats, bias, addend, addend_mask, Hs, Ws, Cs, Nimg, Hm, Wm, Ncol, K, ldb, sh, sw,
                      oh0, ow0, dh, dw, nth, ntw, Ho, Wo, osh, osw, oph, opw, ldo, act, aux, variant, none, pix,
                      stream);
}

// Data gradient with the BatchNorm-backward reduction of the unit it feeds fused
// into the epilogue (see BnbArgs): writes partial rows [row0, row0 + rows) of
// the [2][R][Ncol] buffer `part`, rows = pdt_conv_nt_bnb_rows(M, Ncol, K, variant).
PDT_API int pdt_conv_nt_bnb(const void* src, const void* b, void* out, const void* addend, const void* addend_mask,
                            int Hs, int Ws, int Cs, int Nimg, int Hm, int Wm, int Ncol, int K, int ldb,
                            int sh, int sw, int oh0, int ow0, int dh, int dw, int nth, int ntw,
                            int Ho, int Wo, int osh, int osw, int oph, int opw, int ldo, int variant,
                            const void* bn_y, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                            const void* bn_mask, float* part, int relu, int row0, int R, hipStream_t stream) {
  if (part == nullptr || bn_y == nullptr || bn_mean == nullptr) return -8;
  if ((long long)Nimg * Ho * Wo * ldo >= (1LL << 32)) return -9;  // unsigned 32-bit offsets in the BN-backward epilogue
  if (relu && bn_mask == nullptr && (bn_scale == nullptr || bn_shift == nullptr)) return -8;
  BnbArgs bnb{(const u16*)bn_y, bn_mean, bn_scale, bn_shift, (const uint8_t*)bn_mask, part, relu, row0, R};
  return conv_nt_impl(src, b, out, nullptr, nullptr, addend, addend_mask, Hs, Ws, Cs, Nimg, Hm, Wm, Ncol, K, ldb, sh,
                      sw, oh0, ow0, dh, dw, nth, ntw, Ho, Wo, osh, osw, oph, opw, ldo, 0, nullptr, variant, bnb, 0,
                      stream);
}

// The same, also producing the partials of a second unit fed by the same gated gradient
// (BnbArgs.y2 / mean2 / part2: a downsample block's shortcut BN, gated by the block's ReLU
// mask like its bn3), part2 laid out like part. The 3x3 halo tiles return NOT_APPLICABLE.
PDT_API int pdt_conv_nt_bnb2(const void* src, const void* b, void* out, const void* addend, const void* addend_mask,
                             int Hs, int Ws, int Cs, int Nimg, int Hm, int Wm, int Ncol, int K, int ldb,
                             int sh, int sw, int oh0, int ow0, int dh, int dw, int nth, int ntw,
                             int Ho, int Wo, int osh, int osw, int oph, int opw, int ldo, int variant,
                             const void* bn_y, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                             const void* bn_mask, float* part, int relu, int row0, int R, const void* bn_y2,
                             const float* bn_mean2, float* part2, hipStream_t stream) {
  if (part == nullptr || bn_y == nullptr || bn_mean == nullptr || bn_y2 == nullptr || bn_mean2 == nullptr ||
      part2 == nullptr)
    return -8;
  if ((long long)Nimg * Ho * Wo * ldo >= (1LL << 32)) return -9;
  if (relu && bn_mask == nullptr && (bn_scale == nullptr || bn_shift == nullptr)) return -8;
  BnbArgs bnb{(const u16*)bn_y, bn_mean, bn_scale, bn_shift, (const uint8_t*)bn_mask, part, relu, row0, R,
              (const u16*)bn_y2, bn_mean2, part2};
  return conv_nt_impl(src, b, out, nullptr, nullptr, addend, addend_mask, Hs, Ws, Cs, Nimg, Hm, Wm, Ncol, K, ldb, sh,
                      sw, oh0, ow0, dh, dw, nth, ntw, Ho, Wo, osh, osw, oph, opw, ldo, 0, nullptr, variant, bnb, 0,
                      stream);
}

// GEMM with the BatchNorm apply folded into its A staging (AXArgs in conv_nt_kernel.h), any
// stride-1 geometry (full argument list as pdt_conv_nt_bnb): ax_mode 1 = forward (optional
// BN statistics of the output: stats), 2 / 3 = a BN-backward apply (with the fused bn
// partials of the unit the output feeds: part != 0). NOT_APPLICABLE (-5) for variants
// without an AX instantiation or geometries it does not cover.
// pdt_conv_nt_ax3: the same with an addend (+ its ReLU bit mask) added in the fused
// BN-backward epilogue (modes 2 / 3 only): a bottleneck's conv1 data gradient, whose
// output also carries the shortcut gradient, with bn1's backward apply in its A staging.
PDT_API int pdt_conv_nt_ax3(const void* src, const void* b, void* out, float* stats, const void* addend,
                            const void* addend_mask,
                            int Hs, int Ws, int Cs, int Nimg, int Hm, int Wm, int Ncol, int K, int ldb,
                            int sh, int sw, int oh0, int ow0, int dh, int dw, int nth, int ntw,
                            int Ho, int Wo, int osh, int osw, int oph, int opw, int ldo, int variant,
                            const void* bn_y, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                            const void* bn_mask, float* part, int relu, int row0, int R,
                            int ax_mode, const void* ax_y2, const float* ax_c1, const float* ax_c2,
                            const float* ax_c3, const float* ax_rsc, const float* ax_rsh, const void* ax_mask_in,
                            void* ax_mask_out, void* ax_dst, hipStream_t stream) {
  if (ax_mode < 1 || ax_mode > 3) return -8;
  if (addend != nullptr && (ax_mode == 1 || part == nullptr)) return -8;
  if (part != nullptr && (bn_y == nullptr || bn_mean == nullptr)) return -8;
  if (part != nullptr && relu && bn_mask == nullptr && (bn_scale == nullptr || bn_shift == nullptr)) return -8;
  if ((long long)Nimg * Ho * Wo * ldo >= (1LL << 32)) return -9;
  BnbArgs bnb{(const u16*)bn_y, bn_mean, bn_scale, bn_shift, (const uint8_t*)bn_mask, part, relu, row0, R};
  AXArgs ax{ax_mode, -1, (const u16*)ax_y2, ax_c1, ax_c2, ax_c3, ax_rsc, ax_rsh, (const uint8_t*)ax_mask_in,
            (uint8_t*)ax_mask_out, (u16*)ax_dst};
  return conv_nt_impl(src, b, out, stats, nullptr, addend, addend_mask, Hs, Ws, Cs, Nimg, Hm, Wm, Ncol, K, ldb, sh,
                      sw, oh0, ow0, dh, dw, nth, ntw, Ho, Wo, osh, osw, oph, opw, ldo, 0, nullptr, variant, bnb, 0,
                      stream, ax);
}

PDT_API int pdt_conv_nt_ax2(const void* src, const void* b, void* out, float* stats,
                            int Hs, int Ws, int Cs, int Nimg, int Hm, int Wm, int Ncol, int K, int ldb,
                            int sh, int sw, int oh0, int ow0, int dh, int dw, int nth, int ntw,
                            int Ho, int Wo, int osh, int osw, int oph, int opw, int ldo, int variant,
                            const void* bn_y, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                            const void* bn_mask, float* part, int relu, int row0, int R,
                            int ax_mode, const void* ax_y2, const float* ax_c1, const float* ax_c2,
                            const float* ax_c3, const float* ax_rsc, const float* ax_rsh, const void* ax_mask_in,
                            void* ax_mask_out, void* ax_dst, hipStream_t stream) {
  return pdt_conv_nt_ax3(src, b, out, stats, nullptr, nullptr, Hs, Ws, Cs, Nimg, Hm, Wm, Ncol, K, ldb, sh, sw, oh0,
                         ow0, dh, dw, nth, ntw, Ho, Wo, osh, osw, oph, opw, ldo, variant, bn_y, bn_mean, bn_scale,
                         bn_shift, bn_mask, part, relu, row0, R, ax_mode, ax_y2, ax_c1, ax_c2, ax_c3, ax_rsc, ax_rsh,
                         ax_mask_in, ax_mask_out, ax_dst, stream);
}

// the 1x1 form (stride 1, unpadded)
PDT_API int pdt_conv_nt_ax(const void* src, const void* b, void* out, float* stats,
                           int Hs, int Ws, int Cs, int Nimg, int Hm, int Wm, int Ncol, int K, int ldb,
                           int ldo, int variant,
                           const void* bn_y, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                           const void* bn_mask, float* part, int relu, int row0, int R,
                           int ax_mode, const void* ax_y2, const float* ax_c1, const float* ax_c2,
                           const float* ax_c3, const float* ax_rsc, const float* ax_rsh, const void* ax_mask_in,
                           void* ax_mask_out, void* ax_dst, hipStream_t stream) {
  return pdt_conv_nt_ax2(src, b, out, stats, Hs, Ws, Cs, Nimg, Hm, Wm, Ncol, K, ldb, 1, 1, 0, 0, 1, 1, 1, 1, Hm, Wm,
                         1, 1, 0, 0, ldo, variant, bn_y, bn_mean, bn_scale, bn_shift, bn_mask, part, relu, row0, R,
                         ax_mode, ax_y2, ax_c1, ax_c2, ax_c3, ax_rsc, ax_rsh, ax_mask_in, ax_mask_out, ax_dst, stream);
}

// ---------------------------------------------------------------------------
// fp8 GEMM  out[m, n] = dq_a * dq_b * sum_k A[m, k] B[n, k] (+ bias, act, aux)
// A: [M][lda] fp8 (e4m3 if fmt_a == 0, e5m2 if 1), B: [N][ldb] e4m3, out bf16 [M][ldo],
// optional bf16 addend [M][ldo] (residual add, or the GELU-backward operand with act 3 / the
// stored GELU derivative with act 5); act 4 = GELU with its derivative written to aux.
// K, lda, ldb in BYTES (= elements), multiples of 128 / 16 / 16.
PDT_API int pdt_fp8_meta_roll_partial(float* meta, const float* partial, int nblk, int fmt, float* dq_out,
                                      hipStream_t st);

namespace {
// id 11: the 256x256 tile on FOUR waves (2x2 of 128x128, 256 accumulators per lane, one wave
// per SIMD): per K-tile a CU's fragment reads fall from 192 KB (8 waves of 128x64) to 128 KB
// -- the fp8 MFMA consumes twice the bytes per cycle of the bf16 one, so the LDS read
// bandwidth, not the matrix core, bounds the 8-wave tile.
// ids 12 / 13: the dense 256x256 ping-pong ring (csrc/gemm_ring.hip, tile groupings GM 4 / 8),
// 14 / 15: the same ring persistent (one workgroup per CU walks the tiles, the next tile's first
// K-tile loading under the current tile's epilogue); the fused epilogue on 12 and 14
constexpr int NVAR_F8 = 16;
constexpr int F8_RING0 = 12;
constexpr int VAR_F8_BM[NVAR_F8] = {128, 128, 256, 128, 64, 128, 256, 128, 256, 128, 256, 256, 256, 256, 256, 256};
constexpr int VAR_F8_BN[NVAR_F8] = {128, 128, 128, 256, 128, 64, 64, 128, 128, 256, 256, 256, 256, 256, 256, 256};

template <int F8>
int launch_f8(int v, const NTParams& p, hipStream_t st) {
  switch (v) {
    case 0: return launch<128, 128, 2, true, false, false, 256, 2, F8>(p, st);
    case 1: return launch<128, 128, 2, true, false, true, 256, 2, F8>(p, st);
    case 2: return launch<256, 128, 2, true, false, true, 512, 4, F8>(p, st);
    case 3: return launch<128, 256, 2, true, false, true, 512, 2, F8>(p, st);
    case 4: return launch<64, 128, 2, true, false, true, 256, 2, F8>(p, st);
    case 5: return launch<128, 64, 2, true, false, true, 256, 2, F8>(p, st);
    case 6: return launch<256, 64, 2, true, false, true, 256, 2, F8>(p, st);
    case 7: return launch<128, 128, 2, true, true, true, 256, 2, F8>(p, st);
    case 8: return launch<256, 128, 3, true, false, true, 512, 4, F8, true>(p, st);
    case 9: return launch<128, 256, 3, true, false, true, 512, 2, F8, true>(p, st);
    case 10: return launch<256, 256, 2, true, false, true, 512, 2, F8, true>(p, st);
    case 11: return launch<256, 256, 2, true, false, true, 256, 2, F8, true>(p, st);
  }
  return -3;
}
}  // namespace

PDT_API int pdt_gemm_f8_num_variants() { return NVAR_F8; }

PDT_API int pdt_gemm_ring(const void* a, const void* b, void* c, const float* bias, const float* dq_a,
                          const float* dq_b, int M, int N, int K, int lda, int ldb, int ldc, int dt, int sub,
                          hipStream_t st);
PDT_API int pdt_gemm_ring_epi(const void* a, const void* b, void* c, const float* bias, const float* dq_a,
                              const float* dq_b, int M, int N, int K, int lda, int ldb, int ldc, int dt, int act,
                              void* aux, const void* addend, void* q8, const float* q8_meta, float* q8_part,
                              int q8_fmt, int q8_only, float* colsum, hipStream_t st);
PDT_API int pdt_gemm_ring_epi_pers(const void* a, const void* b, void* c, const float* bias, const float* dq_a,
                                   const float* dq_b, int M, int N, int K, int lda, int ldb, int ldc, int dt, int act,
                                   void* aux, const void* addend, void* q8, const float* q8_meta, float* q8_part,
                                   int q8_fmt, int q8_only, float* colsum, hipStream_t st);
PDT_API int pdt_gemm_ring_grid(int M, int N, int sub);

static int gemm_f8_impl(const void* a, const void* b, void* out, const float* bias, const float* dq_a,
                        const float* dq_b, int M, int N, int K, int lda, int ldb, int ldo, int fmt_a, int act,
                        void* aux, const void* addend, int variant, void* q8, float* q8_meta, float* q8_part,
                        int q8_fmt, int q8_only, float* q8_dq, hipStream_t stream, float* colsum = nullptr) {
  if (K % 128 != 0 || lda % 16 != 0 || ldb % 16 != 0 || N % 8 != 0 || ldo % 8 != 0) return -1;
  if (lda != K) return -2;  // rows of A are dense (the gather's source row stride is Cs)
  if (variant >= F8_RING0 && variant < NVAR_F8) {  // the dense ring (csrc/gemm_ring.hip)
    const int dt = fmt_a == 1 ? 2 : 1;
    int rc;
    const int sub = variant - F8_RING0;
    if (act != 0 || aux != nullptr || addend != nullptr || q8 != nullptr || colsum != nullptr) {
      if (sub != 0 && sub != 2) return -5;  // the fused epilogue: grouping GM 4 only
      rc = (sub == 2 ? pdt_gemm_ring_epi_pers : pdt_gemm_ring_epi)(a, b, out, bias, dq_a, dq_b, M, N, K, lda, ldb, ldo,
                                                                   dt, act, aux, addend, q8, q8_meta, q8_part, q8_fmt,
                                                                   q8_only, colsum, stream);
    } else {
      rc = pdt_gemm_ring(a, b, out, bias, dq_a, dq_b, M, N, K, lda, ldb, ldo, dt, sub, stream);
    }
    if (rc || q8 == nullptr) return rc;
    return pdt_fp8_meta_roll_partial(q8_meta, q8_part, pdt_gemm_ring_grid(M, N, sub), q8_fmt, q8_dq, stream);
  }
  NTParams p;
  p.src = (const u16*)a;
  p.b = (const u16*)b;
  p.out = (u16*)out;
  p.stats = nullptr;
  p.bias = bias;
  p.addend = (const u16*)addend;  // [M][ldo] bf16: out += addend (act 3: out *= gelu'(addend))
  p.addend_mask = nullptr;
  if ((act == 3 || act == 5) && (addend == nullptr || aux != nullptr || bias != nullptr)) return -4;
  if (act == 4 && (aux == nullptr || addend != nullptr)) return -4;
  if (act < 0 || act > 5) return -4;
  p.Hs = 1; p.Ws = 1; p.Cs = K / 2;
  p.Hm = 1; p.Wm = 1;
  p.M = M;
  p.Ncol = N; p.K = K / 2; p.ldb = ldb / 2;
  p.sh = 1; p.sw = 1; p.oh0 = 0; p.ow0 = 0; p.dh = 1; p.dw = 1; p.nth = 1; p.ntw = 1;
  p.Ho = 1; p.Wo = 1; p.osh = 1; p.osw = 1; p.oph = 0; p.opw = 0; p.ldo = ldo;
  p.act = act;
  p.pix = p.Cs;
  p.aux = (u16*)aux;
  p.nstat_rows = 0;
  p.nt_store = 0;
  p.ident_out = 1;
  p.dq_a = dq_a;
  p.dq_b = dq_b;
  p.bnb = BnbArgs{};
  p.ax = AXArgs{};
  p.div_Wm = make_fastdiv(1);
  p.div_HWm = make_fastdiv(1);
  p.div_Cs8 = make_fastdiv(K / 16);
  p.div_ntw = make_fastdiv(1);
  const int v = (variant >= 0 && variant < NVAR_F8) ? variant : 1;
  p.q8 = (uint8_t*)q8;
  p.q8_meta = q8_meta;
  p.q8_part = q8_part;
  p.q8_fmt = q8_fmt;
  p.q8_only = q8_only;
  if ((q8 != nullptr || colsum != nullptr) && v == 7) return -5;  // the direct-store epilogue has neither
  p.stats = colsum;  // fp8 instantiations: the column-sum output (conv_nt_kernel.h)
  const int rc = fmt_a == 1 ? launch_f8<2>(v, p, stream) : launch_f8<1>(v, p, stream);
  if (rc || q8 == nullptr) return rc;
  const int nblk = ((M + VAR_F8_BM[v] - 1) / VAR_F8_BM[v]) * ((N + VAR_F8_BN[v] - 1) / VAR_F8_BN[v]);
  return pdt_fp8_meta_roll_partial(q8_meta, q8_part, nblk, q8_fmt, q8_dq, stream);
}

PDT_API int pdt_gemm_f8(const void* a, const void* b, void* out, const float* bias, const float* dq_a,
                        const float* dq_b, int M, int N, int K, int lda, int ldb, int ldo, int fmt_a, int act,
                        void* aux, const void* addend, int variant, hipStream_t stream) {
  return gemm_f8_impl(a, b, out, bias, dq_a, dq_b, M, N, K, lda, ldb, ldo, fmt_a, act, aux, addend, variant, nullptr,
                      nullptr, nullptr, 0, 0, nullptr, stream);
}

// M-tile rows of variant v (the colsum partial rows of pdt_gemm_f8_q8_cs)
PDT_API int pdt_gemm_f8_bm(int variant) { return VAR_F8_BM[(variant >= 0 && variant < NVAR_F8) ? variant : 1]; }

// floats of amax workspace pdt_gemm_f8_q8 needs (any variant)
PDT_API long pdt_gemm_f8_q8_part(int M, int N) { return (long)((M + 63) / 64) * ((N + 63) / 64); }

// pdt_gemm_f8 that also emits the fp8 codes (format q8_fmt) of its bf16 output for the next
// fp8 GEMM with that GEMM's delayed scale (q8_meta[0]), rolls q8_meta's amax history and
// writes the codes' dequant factor to q8_dq; q8_only = 1 skips the bf16 output.
PDT_API int pdt_gemm_f8_q8(const void* a, const void* b, void* out, const float* bias, const float* dq_a,
                           const float* dq_b, int M, int N, int K, int lda, int ldb, int ldo, int fmt_a, int act,
                           void* aux, const void* addend, int variant, void* q8, float* q8_meta, float* q8_part,
                           int q8_fmt, int q8_only, float* q8_dq, hipStream_t stream) {
  if (!q8 || !q8_meta || !q8_part || ldo != N) return -1;
  return gemm_f8_impl(a, b, out, bias, dq_a, dq_b, M, N, K, lda, ldb, ldo, fmt_a, act, aux, addend, variant, q8,
                      q8_meta, q8_part, q8_fmt, q8_only, q8_dq, stream);
}

// pdt_gemm_f8_q8 that also writes the column sums of the final bf16 output (whether or not
// q8_only skips storing it) per M-tile: colsum[ceil(M / pdt_gemm_f8_bm(v))][N] -- the bias
// gradient of the layer whose output gradient this is, with no pass over that gradient
PDT_API int pdt_gemm_f8_q8_cs(const void* a, const void* b, void* out, const float* bias, const float* dq_a,
                              const float* dq_b, int M, int N, int K, int lda, int ldb, int ldo, int fmt_a, int act,
                              void* aux, const void* addend, int variant, void* q8, float* q8_meta, float* q8_part,
                              int q8_fmt, int q8_only, float* q8_dq, float* colsum, hipStream_t stream) {
  if (!q8 || !q8_meta || !q8_part || ldo != N || !colsum) return -1;
  return gemm_f8_impl(a, b, out, bias, dq_a, dq_b, M, N, K, lda, ldb, ldo, fmt_a, act, aux, addend, variant, q8,
                      q8_meta, q8_part, q8_fmt, q8_only, q8_dq, stream, colsum);
}
