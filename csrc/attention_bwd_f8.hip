// Fused fp8 attention backward for ViT (head dim 64, T <= 256): ONE kernel computes dQ,
// dK and dV of a (batch, head) -- the bf16 path (csrc/attention.hip) runs two kernels that
// each re-stage the head and recompute S / dP. Every GEMM runs on
// mfma_scale_f32_32x32x64_f8f6f4 (OCP e4m3 operands, K = 64 per instruction, 2x the bf16
// MFMA rate) with per-lane E8M0 block scales:
//
//   S    = Q K^T    A = Q rows, B = K rows          (per-head pow2 scales, K = head dim)
//   dP   = dO V^T   A = dO rows, B = V rows
//   P    = exp2(c S - lse),  dS = P (dP - delta)    fp32, in the S accumulator registers
//   dV^T = dO^T P   A = dO^T (ds_read_b64_tr_b8 from the dO rows), B = P (registers)
//   dK^T = Q^T dS   A = Q^T  (tr8 from the Q rows),                 B = dS (registers)
//   dQ^T = K^T dS^T A = K^T  (tr8 from the K rows),                 B = dS^T (LDS image)
//
// Operand k layout and its consequences: csrc/fp8_mfma.h (the first 16 bytes of BOTH lane
// halves form E8M0 scale block 0).
// Phase 1: wave w owns key tile w (32 keys) and walks the query tiles in pairs. An S / dP
// accumulator holds 16 queries x 1 key per lane; packed to fp8 as they are (tile 2qp in
// bytes 0..15, tile 2qp + 1 in bytes 16..31) they ARE the dV / dK B operand with scale
// block hh = query tile 2qp + hh, in the query order k -> 64 qp + 32 (k >> 5) + pi(k & 31),
// pi(p) = 8 ((p & 15) >> 2) + 4 (p >> 4) + (p & 3). The A operands (dO^T, Q^T) are read in
// that order: each tr8 read addresses its 8 rows through it.
// dS is also written, fp8 with one power-of-two scale per 32 x 32 tile, to a [key][query]
// LDS image. Phase 2: dQ^T = K^T dS^T from that image (tr8 reads, natural key order), the
// tile scales as the per-lane B block scales.
//
// Scales: Q, K, V, dO get per-head power-of-two scales at staging (exact dequantisation
// through the E8M0 operands); P uses the fixed 2^8 (P <= 1); dS a per-tile 2^e. All
// accumulation is fp32; dQ / dK / dV are written bf16 into the qkv-layout gradient as the
// bf16 kernels do. lse is the forward's (log2 domain), delta = rowsum(dO * O) is computed
// here from the bf16 O and dO.
#include "fp8_mfma.h"
#include <stdlib.h>

namespace {

constexpr int D = 64;
using namespace pdt_f8;

struct AttnBwdF8Params {
  const u16* qkv;    // [B, T, 3, H, 64] bf16
  const u16* out;    // forward output O [B, T, H*64]
  const u16* dout;   // [B, T, H*64]
  const float* lse;  // [B*H, T] (log2 domain)
  u16* dqkv;         // [B, T, 3, H, 64]
  int B, T, H;
  long ld, ldo;
  float c, scale;
  float* dbg;  // optional (tests): dS [B*H][ROWS][ROWS] fp32 as phase 1 computes it
  // Q8 instantiations (pdt_attn_bwd_f8_q8): the qkv projection's e5m2 output gradient and
  // its bias gradient come out of this kernel instead of a cast pass over bf16 d(qkv):
  uint8_t* q8;            // [B*T][3*H*64] e5m2 codes of bf16(d(qkv)) * q8_meta[0]
  const float* q8_meta;   // the projection's delayed-scaling state (scale in [0])
  float* q8_part;         // [gridDim.x] per-workgroup max |bf16(d(qkv))|
  float* colpart;         // [B][3*H*64] per-image column sums (the bias gradient's partial rows)
  int wbf;                // 1: also write the bf16 d(qkv) (0: nothing reads it)
};

// NQP query-tile pairs: images of ROWS = 64 NQP rows (zero beyond T); 8 waves
// DBG: the tests' fp32 dS dump (p.dbg) -- compiled only into the debug entry point: in the
// production kernel its address arithmetic held registers across phase 1 (NQP = 4 sits at 256)
//
// Q8 (the fused qkv-gradient epilogue): every dK / dV / dQ chunk a lane stores is also
// converted to e5m2 with the projection's delayed scale (amax over the bf16-rounded values,
// per workgroup), and the bias gradient's per-image column sums are formed from identities
// of the attention backward instead of a reduction over the written gradient:
//   sum_keys dV[key] = sum_q dO[q] (sum_keys P[q][key])         = sum_q dO[q]   (rows of P sum to 1)
//   sum_keys dK[key] = scale sum_q Q[q] (sum_keys dS[q][key])   = 0             (sum_k P (dP - delta) = 0)
//   sum_q dQ[q]      : reduced over the 32 query lanes of each dQ unit (DPP + permlane16)
// (exact in real arithmetic; the dV / dK sums of the fp8-rounded gradients differ from these
// by their quantisation noise only).
template <int NQP, bool DBG = false, bool Q8 = false>
__global__ void __launch_bounds__(512) attn_bwd_f8_kernel(AttnBwdF8Params p) {
  constexpr int NT2 = 2 * NQP;  // 32-row tiles (queries and keys)
  constexpr int ROWS = 32 * NT2;
  constexpr int IMG = ROWS * 64;
  constexpr int DSR = ROWS + 16;  // dS^T image row stride (bytes): 4 banks apart per row
  __shared__ __attribute__((aligned(16))) char smem[4 * IMG + ROWS * DSR];
  __shared__ float nlse_s[ROWS], dl_s[ROWS];
  __shared__ int tsc[NT2 * NT2];  // E8M0 dequant of each dS tile [q tile][key tile]
  __shared__ float red[8][4];
  // Q8: per head-parity buffers (the sums of head i are read after its closing barrier while
  // head i + 1 writes the other buffer): dO column sums per wave, dQ column sums per query tile
  __shared__ float vsum[Q8 ? 2 : 1][8][Q8 ? 64 : 1];
  __shared__ float qsum[Q8 ? 2 : 1][NT2][Q8 ? 64 : 1];
  float q8max = 0.f;
  const float q8s = Q8 ? p.q8_meta[0] : 0.f;
  // e5m2 codes (scale q8s) of 8 bf16 values -> dst; their |max| into q8max
  auto q8_put = [&](uint8_t* dst, const u32x4& w) __attribute__((always_inline)) {
    float f[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[2 * e] = lo_bf(w[e]);
      f[2 * e + 1] = hi_bf(w[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) q8max = fmaxf(q8max, fabsf(f[e]));
    uint2 c;
    c.x = pdt_cvt4_f8<1>(f[0] * q8s, f[1] * q8s, f[2] * q8s, f[3] * q8s);
    c.y = pdt_cvt4_f8<1>(f[4] * q8s, f[5] * q8s, f[6] * q8s, f[7] * q8s);
    *reinterpret_cast<uint2*>(dst) = c;
  };
  char* Qi = smem;
  char* Ki = smem + IMG;
  char* Vi = smem + 2 * IMG;
  char* Oi = smem + 3 * IMG;  // dO
  char* dSt = smem + 4 * IMG;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, hh = lane >> 5, g = lane >> 4, j = lane & 15;
  const int nbh = p.B * p.H;

  // ---------------------------------------------------------------- head loads
  // Persistent: a workgroup walks heads bh = blockIdx.x, + gridDim.x, ... (one 137-KB
  // workgroup per CU, so nothing else would overlap a head's HBM loads). The next head's
  // bf16 operands are fetched into registers while this head's dQ phase runs.
  // chunk q = tid + 512 it: row q >> 3, 16-B column ch = q & 7 (the 8 lanes of a row adjacent)
  u32x4 rq[NQP], rk[NQP], rv[NQP], rd[NQP], ro[NQP];
  float rl[NQP];
  // (always assigns every register -- zeros past the last head -- so no stale copy of the
  // previous head's operands stays live through a phase)
  auto load_head = [&](int bh) __attribute__((always_inline)) {
    const bool hok = bh < nbh;
    const int b = hok ? bh / p.H : 0, h = hok ? bh % p.H : 0;
    const u16* Qg = p.qkv + (long)b * p.T * p.ld + h * D;
    const u16* dOg = p.dout + (long)b * p.T * p.ldo + h * D;
    const u16* Og = p.out + (long)b * p.T * p.ldo + h * D;
#pragma unroll
    for (int it = 0; it < NQP; ++it) {
      const int q = tid + 512 * it, row = q >> 3, ch = q & 7;
      const u32x4 z = {0, 0, 0, 0};
      rq[it] = rk[it] = rv[it] = rd[it] = ro[it] = z;
      rl[it] = INFINITY;  // rows >= T: -lse = -inf -> P = 0
      if (hok && row < p.T) {
        rq[it] = *reinterpret_cast<const u32x4*>(Qg + (long)row * p.ld + ch * 8);
        rk[it] = *reinterpret_cast<const u32x4*>(Qg + p.H * D + (long)row * p.ld + ch * 8);
        rv[it] = *reinterpret_cast<const u32x4*>(Qg + 2 * p.H * D + (long)row * p.ld + ch * 8);
        rd[it] = *reinterpret_cast<const u32x4*>(dOg + (long)row * p.ldo + ch * 8);
        ro[it] = *reinterpret_cast<const u32x4*>(Og + (long)row * p.ldo + ch * 8);
        if (ch == 0) rl[it] = p.lse[(long)bh * p.T + row];
      }
    }
  };
  load_head(blockIdx.x);

  for (int bh = blockIdx.x; bh < nbh; bh += gridDim.x) {
  const int b = bh / p.H, h = bh % p.H;
  const int hb = Q8 ? ((bh - (int)blockIdx.x) / (int)gridDim.x) & 1 : 0;  // head-parity buffer

  if constexpr (Q8) {  // column sums of this head's dO (the V bias gradient, see above)
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < NQP; ++it)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cs[2 * e] += lo_bf(rd[it][e]);
        cs[2 * e + 1] += hi_bf(rd[it][e]);
      }
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // lanes of one 16-B column chunk: lane & 7 equal
      cs[e] += __shfl_xor(cs[e], 8, 64);
      cs[e] += __shfl_xor(cs[e], 16, 64);
      cs[e] += __shfl_xor(cs[e], 32, 64);
    }
    if (lane < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) vsum[hb][wave][lane * 8 + e] = cs[e];
    }
  }

  // ---------------------------------------------------------------- staging
  // |x|max on the packed bf16 bits (2 magnitudes per v_pk_max_u16), delta with v_dot2 on the
  // packed pairs: no unpacking in the staging pass
  uint32_t mxb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int it = 0; it < NQP; ++it) {
    const int q = tid + 512 * it, row = q >> 3, ch = q & 7;
    const u32x4 a = rq[it], k = rk[it], v = rv[it], d = rd[it], o = ro[it];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      mxb[0] = absmax_bf16x2(mxb[0], a[e]);
      mxb[1] = absmax_bf16x2(mxb[1], k[e]);
      mxb[2] = absmax_bf16x2(mxb[2], v[e]);
      mxb[3] = absmax_bf16x2(mxb[3], d[e]);
    }
    const float dl = row8_sum(dot8_bf16(d, o, 0.f));  // delta of this row: the 8 lanes of the row (DPP)
    if (ch == 0) {
      dl_s[row] = dl;
      nlse_s[row] = -rl[it];
    }
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const float w = warp_max(absmax_bf16x2_value(mxb[m]));
    if (lane == 0) red[wave][m] = w;
  }
  __syncthreads();
  int ex[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    float a = red[0][m];
#pragma unroll
    for (int w = 1; w < 8; ++w) a = fmaxf(a, red[w][m]);
    ex[m] = pow2_exp(a);
  }
  // quantisation divisors 2^-e (the scaled converts divide): codes of x * 2^e
  const float sq = ldexpf(1.f, -ex[0]), sk = ldexpf(1.f, -ex[1]), sv = ldexpf(1.f, -ex[2]), sd = ldexpf(1.f, -ex[3]);
#pragma unroll
  for (int it = 0; it < NQP; ++it) {
    const int q = tid + 512 * it, row = q >> 3, ch = q & 7;
    const int off = k8_off(row, ch >> 1) + (ch & 1) * 8;
    auto put = [&](char* img, const u32x4& x, float sdiv) __attribute__((always_inline)) {
      uint2 w;
      w.x = e4m3x4_bf16(x[0], x[1], sdiv);
      w.y = e4m3x4_bf16(x[2], x[3], sdiv);
      *reinterpret_cast<uint2*>(img + off) = w;
    };
    put(Qi, rq[it], sq);
    put(Ki, rk[it], sk);
    put(Vi, rv[it], sv);
    put(Oi, rd[it], sd);
  }
  __syncthreads();
  // E8M0 dequantisation operands of the staged tensors
  const int dq_q = 127 - ex[0], dq_k = 127 - ex[1], dq_v = 127 - ex[2], dq_d = 127 - ex[3];
  constexpr int P_EXP = 8;  // P in [0, 1] -> codes of 256 P

  // ---------------------------------------------------------------- phase 1: dK, dV
  // A key tile wholly past T (T = 197: keys 224..255) contributes nothing: its wave only
  // zeroes its rows of the dS^T image (phase 2 reads them, times zero K rows: stale LDS
  // bytes could hold e4m3 NaN codes) and sets its tiles' unit scales.
  if (wave < NT2 && 32 * wave >= p.T) {
    for (int i = lane; i < 32 * ROWS / 16; i += 64) {
      const int r = i / (ROWS / 16), c = i % (ROWS / 16);
      *reinterpret_cast<u32x4*>(dSt + (32 * wave + r) * DSR + 16 * c) = u32x4{0u, 0u, 0u, 0u};
    }
    if (lane < NT2) tsc[lane * NT2 + wave] = 127;
  } else if (wave < NT2) {
    const int kt = wave, k0 = 32 * kt;
    const int key = k0 + col;
    const bool kok = key < p.T;
    const i32x8 kf = row_frag(Ki, key, hh);
    const i32x8 vf = row_frag(Vi, key, hh);
    // Keys past T (lanes with !kok) are not masked per element: their K / V rows are zero, so
    // their P / dS only reach dV / dK columns that are never stored and the phase-2 products
    // with their zero K rows. What must hold: their dS codes are finite -- they are excluded
    // from the tile's |dS|max and converted with a 2^127 divisor (code 0).
    f32x16 dvT[2], dkT[2];
#pragma unroll
    for (int dn = 0; dn < 2; ++dn)
#pragma unroll
      for (int r = 0; r < 16; ++r) dvT[dn][r] = dkT[dn][r] = 0.f;
#pragma unroll 1  // (unrolled by 2 it spills at NQP 3 / 4)
    for (int qp = 0; qp < NQP; ++qp) {
      uint32_t pc[2][4], dc[2][4];
      int de[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * qp + u;
        if (32 * qt >= p.T) {  // a query tile wholly past T: P = dS = 0 (phase 2 never reads its dS^T columns)
#pragma unroll
          for (int w = 0; w < 4; ++w) pc[u][w] = dc[u][w] = 0u;
          de[u] = 0;
          continue;
        }
        const f32x16 z = {};
        // S[q = 32 qt + 8 (r >> 2) + 4 hh + (r & 3)][key]
        const f32x16 s = mfma8(row_frag(Qi, 32 * qt + col, hh), kf, z, dq_q, dq_k);
        const f32x16 dp = mfma8(row_frag(Oi, 32 * qt + col, hh), vf, z, dq_d, dq_v);
        float pv[16], ds[16], am = 0.f;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int q4 = 32 * qt + 8 * jj + 4 * hh;
          const f32x4 nl = *reinterpret_cast<const f32x4*>(nlse_s + q4);
          const f32x4 dl = *reinterpret_cast<const f32x4*>(dl_s + q4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * jj + e;
            const float pr = __builtin_amdgcn_exp2f(fmaf(s[r], p.c, nl[e]));
            pv[r] = pr;
            ds[r] = pr * (dp[r] - dl[e]);
            am = fmaxf(am, fabsf(ds[r]));
          }
        }
        if constexpr (DBG) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int q = 32 * qt + 8 * (r >> 2) + 4 * hh + (r & 3);
            p.dbg[((long)bh * ROWS + q) * ROWS + key] = ds[r];
          }
        }
        const int e = pow2_exp(warp_max(kok ? am : 0.f));  // one scale per 32 x 32 dS tile
        de[u] = e;
        // convert divisor: codes of dS * 2^e; 2^127 (codes 0) for the padded keys -- not inf: the
        // scaled convert takes the divisor's exponent as an E8M0 scale, and inf's is the NaN code
        const float sds = kok ? ldexpf(1.f, -e) : 0x1p127f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          pc[u][w] = e4m3x4_div(pv[4 * w], pv[4 * w + 1], pv[4 * w + 2], pv[4 * w + 3], 1.f / 256.f);
          dc[u][w] = e4m3x4_div(ds[4 * w], ds[4 * w + 1], ds[4 * w + 2], ds[4 * w + 3], sds);
          // dS^T image [key][q]: 4 consecutive queries 32 qt + 8 w + 4 hh of this key
          *reinterpret_cast<uint32_t*>(dSt + key * DSR + 32 * qt + 8 * w + 4 * hh) = dc[u][w];
        }
        if (lane == 0) tsc[qt * NT2 + kt] = 127 - e;
      }
      // B operands as packed: tile 2 qp in bytes 0..15, tile 2 qp + 1 in bytes 16..31, so
      // lane half hh's block scale is query tile 2 qp + hh's
      const i32x8 pf = {(int)pc[0][0], (int)pc[0][1], (int)pc[0][2], (int)pc[0][3],
                        (int)pc[1][0], (int)pc[1][1], (int)pc[1][2], (int)pc[1][3]};
      const i32x8 sf = {(int)dc[0][0], (int)dc[0][1], (int)dc[0][2], (int)dc[0][3],
                        (int)dc[1][0], (int)dc[1][1], (int)dc[1][2], (int)dc[1][3]};
      const int sb_ds = 127 - (hh ? de[1] : de[0]);
#pragma unroll
      for (int dn = 0; dn < 2; ++dn) {
        // A: rows d = 32 dn + 16 (g & 1) + j of dO^T / Q^T, k = the pair's queries (same order)
        const i32x8 oa = tr_frag<true>(Oi, 64 * qp, 2 * dn + (g & 1), j, hh);
        dvT[dn] = mfma8(oa, pf, dvT[dn], dq_d, 127 - P_EXP);
        const i32x8 qa = tr_frag<true>(Qi, 64 * qp, 2 * dn + (g & 1), j, hh);
        dkT[dn] = mfma8(qa, sf, dkT[dn], dq_q, sb_ds);
      }
    }
    // dK^T / dV^T[d = 32 dn + 8 jj + 4 hh + e][key]: lane (key, hh) holds 4 of each 8-d chunk,
    // lane ^ 32 the other 4; a v_permlane32_swap per dword of chunks jj (even), jj + 1 gives
    // lane hh chunk jj + hh whole: 16-B stores (the swaps run with the full EXEC; only the
    // stores of keys past T are predicated off)
    {
      u16* drow = p.dqkv + ((long)b * p.T + (kok ? key : 0)) * p.ld + h * D;
#pragma unroll
      for (int dn = 0; dn < 2; ++dn)
#pragma unroll
        for (int j2 = 0; j2 < 4; j2 += 2) {
          uint32_t wk[2][2], wv[2][2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int jj = j2 + u;
            wk[u][0] = pack2bf(dkT[dn][4 * jj] * p.scale, dkT[dn][4 * jj + 1] * p.scale);
            wk[u][1] = pack2bf(dkT[dn][4 * jj + 2] * p.scale, dkT[dn][4 * jj + 3] * p.scale);
            wv[u][0] = pack2bf(dvT[dn][4 * jj], dvT[dn][4 * jj + 1]);
            wv[u][1] = pack2bf(dvT[dn][4 * jj + 2], dvT[dn][4 * jj + 3]);
          }
          const auto k0 = __builtin_amdgcn_permlane32_swap(wk[0][0], wk[1][0], false, false);
          const auto k1 = __builtin_amdgcn_permlane32_swap(wk[0][1], wk[1][1], false, false);
          const auto v0 = __builtin_amdgcn_permlane32_swap(wv[0][0], wv[1][0], false, false);
          const auto v1 = __builtin_amdgcn_permlane32_swap(wv[0][1], wv[1][1], false, false);
          const int d0 = 32 * dn + 8 * (j2 + hh);
          if (kok) {
            const u32x4 kw = {k0[0], k1[0], k0[1], k1[1]}, vw = {v0[0], v1[0], v0[1], v1[1]};
            if (!Q8 || p.wbf) {
              *reinterpret_cast<u32x4*>(drow + p.H * D + d0) = kw;
              *reinterpret_cast<u32x4*>(drow + 2 * p.H * D + d0) = vw;
            }
            if constexpr (Q8) {
              uint8_t* crow = p.q8 + ((long)b * p.T + key) * p.ld + h * D;
              q8_put(crow + p.H * D + d0, kw);
              q8_put(crow + 2 * p.H * D + d0, vw);
            }
          }
        }
    }
  }
  __syncthreads();
  load_head(bh + gridDim.x);  // in flight across the dQ phase

  // ---------------------------------------------------------------- phase 2: dQ
  const int nqt = (p.T + 31) / 32;
  for (int unit = wave; unit < 2 * nqt; unit += 8) {
    const int qt = unit >> 1, dn = unit & 1;
    f32x16 acc = {};
#pragma unroll
    for (int kp = 0; kp < NQP; ++kp) {
      const int kt = 2 * kp + hh;  // this lane half's scale block = key tile kt
      // A: K^T rows d = 32 dn + 16 (g & 1) + j, k = keys 64 kp .. 64 kp + 63 (natural order)
      const i32x8 ka = tr_frag<false>(Ki, 64 * kp, 2 * dn + (g & 1), j, hh);
      // B: dS^T[key][q]: column q = 32 qt + 16 (g & 1) + j, the same keys
      i32x8 sb;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int krow = 64 * kp + kb_row<false>(r, j >> 1, hh);
        const i32x2 v = tr8(dSt + krow * DSR + 32 * qt + 16 * (g & 1) + 8 * (j & 1));
        sb[2 * r] = v[0];
        sb[2 * r + 1] = v[1];
      }
      acc = mfma8(ka, sb, acc, dq_k, tsc[qt * NT2 + kt]);
    }
    const int q = 32 * qt + col;
    {  // dQ^T[d = 32 dn + 8 jj + 4 hh + e][q]: the same lane-pair exchange, 16-B stores
      const bool qok = q < p.T;
      u16* drow = p.dqkv + ((long)b * p.T + (qok ? q : 0)) * p.ld + h * D;
#pragma unroll
      for (int j2 = 0; j2 < 4; j2 += 2) {
        uint32_t w[2][2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int jj = j2 + u;
          w[u][0] = pack2bf(acc[4 * jj] * p.scale, acc[4 * jj + 1] * p.scale);
          w[u][1] = pack2bf(acc[4 * jj + 2] * p.scale, acc[4 * jj + 3] * p.scale);
        }
        const auto r0 = __builtin_amdgcn_permlane32_swap(w[0][0], w[1][0], false, false);
        const auto r1 = __builtin_amdgcn_permlane32_swap(w[0][1], w[1][1], false, false);
        const u32x4 qw = {r0[0], r1[0], r0[1], r1[1]};
        const int d0 = 32 * dn + 8 * (j2 + hh);
        if (qok && (!Q8 || p.wbf)) *reinterpret_cast<u32x4*>(drow + d0) = qw;
        if constexpr (Q8) {
          if (qok) q8_put(p.q8 + ((long)b * p.T + q) * p.ld + h * D + d0, qw);
          // column sums over the tile's 32 queries (lanes of one half; queries past T hold 0)
          float cs[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            cs[2 * e] = lo_bf(qw[e]);
            cs[2 * e + 1] = hi_bf(qw[e]);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] = xor16_reduce(row16_sum(cs[e]), AddOp{});
          if (col == 0) {
#pragma unroll
            for (int e = 0; e < 8; ++e) qsum[hb][qt][d0 + e] = cs[e];
          }
        }
      }
    }
  }
  __syncthreads();  // every LDS image, scale and row statistic is restaged for the next head
  if constexpr (Q8) {  // this head's bias-gradient partials into image b's row: [q | k | v][h][d]
    if (tid < D) {
      float qs = 0.f, vs = 0.f;
      for (int t = 0; t < nqt; ++t) qs += qsum[hb][t][tid];
#pragma unroll
      for (int w = 0; w < 8; ++w) vs += vsum[hb][w][tid];
      float* cr = p.colpart + (long)b * p.ld + h * D + tid;
      cr[0] = qs;
      cr[p.H * D] = 0.f;
      cr[2 * p.H * D] = vs;
    }
  }
  }
  if constexpr (Q8) {  // workgroup max |bf16 d(qkv)| -> q8_part[blockIdx.x]
    q8max = warp_max(q8max);
    if (lane == 0) red[wave][0] = q8max;
    __syncthreads();
    if (tid == 0) {
      float m = red[0][0];
#pragma unroll
      for (int w = 1; w < 8; ++w) m = fmaxf(m, red[w][0]);
      p.q8_part[blockIdx.x] = m;
    }
  }
}

}  // namespace

// fused fp8 backward for T <= 256, head dim 64 (d(qkv) bf16); -1 when not covered
static int attn_bwd_f8(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv, int B,
                       int T, int H, float scale, float* dbg, const AttnBwdF8Params* q8, hipStream_t st);

PDT_API int pdt_fp8_meta_roll_partial(float* meta, const float* partial, int nblk, int fmt, float* dq_out,
                                      hipStream_t st);
PDT_API long pdt_reduce_rows_work(int nrows, int n);
PDT_API int pdt_wgrad_reduce_rows(const float* rows, float* out, int nrows, int n, float scale, int accumulate,
                                  float* work, hipStream_t st);

// Workgroups of the backward launch: the length of the q8_part the caller passes to
// pdt_attn_bwd_f8_q8.
static int attn_bwd_grid(int nbh);
PDT_API int pdt_attn_bwd_f8_grid(int B, int H) { return attn_bwd_grid(B * H); }

// pdt_attn_bwd_f8 with the qkv projection's gradient epilogue (Q8 above): the e5m2 codes of
// d(qkv) with the delayed scale q8_meta[0] -> q8 ([B*T][3*H*64]), the amax history rolled
// from the workgroups' partial maxima (q8_part: pdt_attn_bwd_f8_grid floats) with the new
// dequant factor -> q8_dq, and the bias gradient -> bias_out ([3*H*64] fp32, =) through the
// per-image partial rows colpart ([B][3*H*64] + pdt_reduce_rows_work(B, 3*H*64) floats).
// dqkv (bf16) is written only when it is not null.
PDT_API int pdt_attn_bwd_f8_q8(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                               int B, int T, int H, float scale, void* q8, const float* q8_meta, float* q8_part,
                               float* q8_dq, float* colpart, float* bias_out, hipStream_t st) {
  if (!q8 || !q8_meta || !q8_part || !q8_dq || !colpart || !bias_out) return -1;
  if (((uintptr_t)q8 & 7) != 0) return -5;  // 8-B code stores
  AttnBwdF8Params e{};
  e.q8 = (uint8_t*)q8;
  e.q8_meta = q8_meta;
  e.q8_part = q8_part;
  e.colpart = colpart;
  e.wbf = dqkv != nullptr;
  int rc = attn_bwd_f8(qkv, out, dout, lse, dqkv, B, T, H, scale, nullptr, &e, st);
  if (rc) return rc;
  rc = pdt_fp8_meta_roll_partial(const_cast<float*>(q8_meta), q8_part, attn_bwd_grid(B * H), 1, q8_dq, st);
  if (rc) return rc;
  const int n = 3 * H * D;
  return pdt_wgrad_reduce_rows(colpart, bias_out, B, n, 1.f, 0, colpart + (long)B * n, st);
}

PDT_API int pdt_attn_bwd_f8(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                            int B, int T, int H, float scale, hipStream_t st) {
  return attn_bwd_f8(qkv, out, dout, lse, dqkv, B, T, H, scale, nullptr, nullptr, st);
}

// the same, also writing phase 1's fp32 dS to dbg ([B*H][R][R], R = 64 ceil(T / 64)) for tests
PDT_API int pdt_attn_bwd_f8_debug(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                                  int B, int T, int H, float scale, float* dbg, hipStream_t st) {
  return attn_bwd_f8(qkv, out, dout, lse, dqkv, B, T, H, scale, dbg, nullptr, st);
}

// PDT_ATTN_BWD_PERSIST=0: one workgroup per head (the grid B*H, each running the head loop
// once) instead of one per CU -- an A/B switch
static int attn_bwd_grid(int nbh) {
  static int persist = -1;
  if (persist < 0) {
    const char* e = getenv("PDT_ATTN_BWD_PERSIST");
    persist = (e && e[0] == '0') ? 0 : 1;
  }
  const int g = persist ? pdt_num_cus() : nbh;
  return nbh < g ? nbh : g;
}

static int attn_bwd_f8(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv, int B,
                       int T, int H, float scale, float* dbg, const AttnBwdF8Params* q8, hipStream_t st) {
  if (T < 1 || T > 256) return -1;
  AttnBwdF8Params p = q8 ? *q8 : AttnBwdF8Params{};
  p.qkv = (const u16*)qkv;
  p.out = (const u16*)out;
  p.dout = (const u16*)dout;
  p.lse = lse;
  p.dqkv = (u16*)dqkv;
  p.B = B; p.T = T; p.H = H;
  p.ld = 3L * H * D;
  p.ldo = (long)H * D;
  p.c = scale * 1.4426950408889634f;
  p.scale = scale;
  p.dbg = dbg;
  const int nqp = (T + 63) / 64;
  // one workgroup per CU (the LDS images hold 137 KB), each walking B*H / grid heads
  dim3 g(attn_bwd_grid(B * H));
#define BWD(N)                                                                                  \
  if (dbg != nullptr) hipLaunchKernelGGL((attn_bwd_f8_kernel<N, true>), g, dim3(512), 0, st, p);            \
  else if (q8 != nullptr) hipLaunchKernelGGL((attn_bwd_f8_kernel<N, false, true>), g, dim3(512), 0, st, p); \
  else hipLaunchKernelGGL((attn_bwd_f8_kernel<N>), g, dim3(512), 0, st, p)
  switch (nqp) {
    case 1: BWD(1); break;
    case 2: BWD(2); break;
    case 3: BWD(3); break;
    default: BWD(4); break;
  }
#undef BWD
  PDT_RETURN_LAUNCH();
}
