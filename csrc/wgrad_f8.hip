// fp8 weight gradient of nn.Linear (ViT fp8 path) on the CDNA4 block-scaled MFMA:
//
//   dW[co][c] = dq_dy * dq_x * sum_m dY8[m][co] * X8[m][c]      (+ bias grad = sum_m dY[m][co])
//
// dY8 = the e5m2 codes the data-gradient GEMM already consumes, X8 = the e4m3 codes the
// forward GEMM consumed (saved for backward): no extra quantisation pass and no
// transposed copies. Both operands are K-outer (token rows, features contiguous), so
// tiles are staged into LDS as they come from HBM -- [128 token rows][BM | BN bytes] --
// and MFMA fragments are read with the byte-transposing LDS read ds_read_b64_tr_b8:
// per 16-lane group the lanes address an 8-row x 16-byte block (lane j: row j/2,
// bytes 8*(j%2)..+7) and lane j receives column j of it, i.e. 8 consecutive k of ONE
// feature (probe: scripts/probes/tr8_probe.hip). Four such reads give the 32-byte
// operand of mfma_scale_f32_16x16x128_f8f6f4; lane group g holds k rows 32g..32g+31
// of the 128-row k-step in both operands (the same k order on both sides, so the
// contraction is exact). 16-B chunks of an LDS row are XOR-swizzled by a function of
// the row so the 8 rows a group reads fall on distinct bank groups.
//
// Split over the token dimension (K of the GEMM) exactly like the bf16 weight gradient
// (csrc/conv_wgrad.hip): fp32 partial slabs, dequant scales applied in the epilogue,
// deterministic two-stage reduction (pdt_wgrad_reduce). The BIAS instantiation also
// sums the bf16 dY columns of its split in the tn == 0 blocks.
#include "pdt_common.h"
#include <stdlib.h>

PDT_API int pdt_wgrad_reduce(float* slab, float* out, const float* bslab, float* bias_out, int splits, int Mo, int No,
                             float scale, int accumulate, hipStream_t stream);
PDT_API int pdt_wgrad_reduce_rows(const float* rows, float* out, int nrows, int n, float scale, int accumulate,
                                  float* work, hipStream_t stream);

namespace {

typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int BK1 = 128;  // token rows per MFMA k-step (a k-tile holds KS of them)

struct WG8Params {
  const uint8_t* dy;    // [M][ldy] e5m2 codes (co contiguous)
  const uint8_t* x;     // [M][ldx] e4m3 codes (c contiguous)
  const u16* dy16;      // bf16 dY (BIAS only): [M][ldy]
  const float* dq_dy;   // dequant scales (device scalars)
  const float* dq_x;
  float* slab;          // [splits][Mo][No]
  float* bslab;         // [splits][Mo] (BIAS)
  int M, Mo, No, ldy, ldx;
  int ktiles_per_split;
  int xcd;
  const void* zero;     // wg8_zero_chunk's address (kernel argument: no per-issue GOT reload)
};

// physical 16-B chunk of logical chunk c in row r of a RB-byte LDS row
// The 8 rows one 16-lane group reads get distinct bank groups from (r / WRAP); lane
// groups g and g+1 (k rows 32 apart, serviced together) are moved to the other half of
// the row's chunks by bit HB (the counter profile showed ~1.7 conflict cycles per LDS
// instruction without it).
template <int RB>
__device__ __forceinline__ int chunk_swz(int r, int c) {
  constexpr int WRAP = RB >= 256 ? 1 : 256 / RB;  // rows per 256-B bank period
  constexpr int NCH = RB / 16;
  constexpr int MSK = (NCH < 8 ? NCH : 8) - 1;
  constexpr int HB = 8 / WRAP;                      // first chunk bit one group's rows do not use
  static_assert(HB < NCH, "swizzle bits");
  return c ^ ((r / WRAP) & MSK) ^ (((r >> 5) & 1) * HB);
}

template <int RB>
__device__ __forceinline__ i32x8 frag8(const char* base, int col0, int lane, int krow0) {
  // lane group g = lane/16 -> k rows krow0 + 32g .. +31; lane j -> row j/2, bytes 8*(j%2) of column block col0
  const int g = lane >> 4, j = lane & 15;
  const int c = col0 >> 4;
  i32x8 out;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = krow0 + 32 * g + 8 * r + (j >> 1);
    const char* a = base + row * RB + (chunk_swz<RB>(row, c) << 4) + 8 * (j & 1);
    i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
        (i32x2 __attribute__((address_space(3)))*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(
            uintptr_t)a));
    out[2 * r] = v[0];
    out[2 * r + 1] = v[1];
  }
  return out;
}

// rows one pass of all waves covers when every lane moves 16 B of RB-byte rows
constexpr int NW_ROWS(int nth, int rb) { return nth * 16 / rb; }

// zero bytes: the LDS-DMA source for rows past M / columns past Mo, No
static __device__ __attribute__((aligned(64))) u32x4 wg8_zero_chunk[4];

// GL: tiles go global -> LDS by global_load_lds_dwordx4 (no VGPR staging) on an
// NSTAGE-deep ring with ONE barrier per k-tile: tile t+NSTAGE-1 is issued right after
// the barrier that proves every wave finished reading its buffer (tile t-1's), and the
// counted vmcnt before the barrier retires only tile t's DMA (later tiles stay in
// flight across it). A wave instruction writes 1 KB of LDS lane-linearly, so the chunk
// swizzle moves to the source address (the XOR is an involution).
//
// SP (software-pipelined fragment reads): within a k-step the B fragments and the first A
// fragment are read, then every A row block's MFMAs run while the NEXT row block's fragment
// reads are in flight (two A fragment registers sets; scheduling barriers keep hipcc from
// regrouping them). Without it hipcc reads a row block's fragment and waits for it right
// before its 4 MFMAs, so the matrix pipe idles for an LDS round trip per 4 MFMAs (the
// counter pass measured it busy 37 % of the kernel: profiles/vit_b16_fp8_pmc_round5_r6p.txt).
template <int BM, int BN, int NSTAGE, int NTH, int WM, bool BIAS, int KS = 1, bool GL = false, bool SP = false>
__global__ void __launch_bounds__(NTH, NTH == 256 && !GL && BM * BN < 65536 ? 2 : 1) wgrad_f8_kernel(WG8Params p) {
  constexpr int BK = BK1 * KS;
  constexpr int WN = NTH / 64 / WM;
  constexpr int RBA = BM, RBB = BN;  // bytes per LDS row
  constexpr int A_BYTES = BK * RBA, B_BYTES = BK * RBB, STAGE = A_BYTES + B_BYTES;
  constexpr int ACH = BM / 16, BCH = BN / 16;         // 16-B chunks per row
  constexpr int AROWS = NTH / ACH, BROWS = NTH / BCH;  // rows per staging pass
  constexpr int NA = BK / AROWS, NB = BK / BROWS;
  constexpr int MI = BM / (WM * 16), NI = BN / (WN * 16);
  static_assert(NA >= 1 && NB >= 1 && MI >= 1 && NI >= 1 && WM * WN * 64 == NTH, "wgrad_f8 tile shape");
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntm = (p.Mo + BM - 1) / BM, ntn = (p.No + BN - 1) / BN;
  const int ntiles = ntm * ntn;
  const int bid = p.xcd ? (int)xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tm = tile / ntn, tn = tile % ntn;
  const int co0 = tm * BM, tc0 = tn * BN;
  const int nk_total = (p.M + BK - 1) / BK;
  const int kt_begin = split * p.ktiles_per_split;
  const int kt_end = min(nk_total, kt_begin + p.ktiles_per_split);

  const int cA = tid % ACH, rA0 = tid / ACH;
  const int coA = co0 + cA * 16;
  const bool okA = coA < p.Mo;
  const int cB = tid % BCH, rB0 = tid / BCH;
  const int tcB = tc0 + cB * 16;
  const bool okB = tcB < p.No;

  u32x4 ra[NA], rb[NB];
  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = k0 + rA0 + AROWS * i;
      // every load is issued (padding from the zero page): hipcc branches around a load under a
      // per-chunk condition and waits for it alone
      ra[i] = *reinterpret_cast<const u32x4*>((okA && m < p.M) ? (const void*)(p.dy + (size_t)m * p.ldy + coA) : p.zero);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int m = k0 + rB0 + BROWS * i;
      rb[i] = *reinterpret_cast<const u32x4*>((okB && m < p.M) ? (const void*)(p.x + (size_t)m * p.ldx + tcB) : p.zero);
    }
  };
  auto store_tile = [&](int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int r = rA0 + AROWS * i;
      *reinterpret_cast<u32x4*>(sa + r * RBA + (chunk_swz<RBA>(r, cA) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int r = rB0 + BROWS * i;
      *reinterpret_cast<u32x4*>(sb + r * RBB + (chunk_swz<RBB>(r, cB) << 4)) = rb[i];
    }
  };

  // GL source mapping: pass i of a wave instruction covers rows i*AROWS + wave*(1024/RB) + lane/(RB/16)
  auto gl_tile = [&](int kt, int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int r = i * AROWS + wave * (1024 / RBA) + lane / ACH;
      const int c = chunk_swz<RBA>(r, lane % ACH);  // logical chunk stored at this physical slot
      const int m = k0 + r, co = co0 + c * 16;
      const void* g = (co < p.Mo && m < p.M) ? (const void*)(p.dy + (size_t)m * p.ldy + co) : p.zero;
      __builtin_amdgcn_global_load_lds(
          g, (__attribute__((address_space(3))) void*)(sa + (i * AROWS + wave * (1024 / RBA)) * RBA), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int r = i * BROWS + wave * (1024 / RBB) + lane / BCH;
      const int c = chunk_swz<RBB>(r, lane % BCH);
      const int m = k0 + r, tc = tc0 + c * 16;
      const void* g = (tc < p.No && m < p.M) ? (const void*)(p.x + (size_t)m * p.ldx + tc) : p.zero;
      __builtin_amdgcn_global_load_lds(
          g, (__attribute__((address_space(3))) void*)(sb + (i * BROWS + wave * (1024 / RBB)) * RBB), 16, 0, 0);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const char* sa) {
    const char* sb = sa + A_BYTES;
    if constexpr (SP) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        i32x8 bfr[NI], af[2];
#pragma unroll
        for (int j = 0; j < NI; ++j) bfr[j] = frag8<RBB>(sb, wn * (BN / WN) + j * 16, lane, ks * BK1);
        af[0] = frag8<RBA>(sa, wm * (BM / WM), lane, ks * BK1);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          if (i + 1 < MI) af[(i + 1) & 1] = frag8<RBA>(sa, wm * (BM / WM) + (i + 1) * 16, lane, ks * BK1);
          __builtin_amdgcn_sched_barrier(0);
          // retire row block i's fragment (and, at i = 0, the B fragments); the next row
          // block's 4 reads stay in flight across the MFMAs
          if (i + 1 < MI) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
          else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i & 1], acc[i][j], 0, 1, 0, 127,
                                                                           0, 127);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      i32x8 bfr[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = frag8<RBB>(sb, wn * (BN / WN) + j * 16, lane, ks * BK1);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const i32x8 af = frag8<RBA>(sa, wm * (BM / WM) + i * 16, lane, ks * BK1);
#pragma unroll
        for (int j = 0; j < NI; ++j)  // X (e4m3) x dY (e5m2): lane holds 4 consecutive c of one co
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af, acc[i][j], 0, 1, 0, 127, 0, 127);
      }
    }
  };

  if constexpr (GL) {
    static_assert(NSTAGE >= 2 && NSTAGE <= 4 && AROWS == NW_ROWS(NTH, RBA) && BROWS == NW_ROWS(NTH, RBB),
                  "GL ring shape");
    const int n = kt_end - kt_begin;
    for (int t = 0; t < NSTAGE - 1; ++t)
      if (t < n) gl_tile(kt_begin + t, t);
    for (int t = 0; t < n; ++t) {
      if (t + NSTAGE - 2 < n) {  // tiles t+1 .. t+NSTAGE-2 were issued after tile t: leave them in flight
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSTAGE - 2) * (NA + NB)) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (t + NSTAGE - 1 < n) gl_tile(kt_begin + t + NSTAGE - 1, (t + NSTAGE - 1) % NSTAGE);
      compute(smem + (t % NSTAGE) * STAGE);
    }
    __syncthreads();  // before the bias tail reuses LDS
  } else {
  if (kt_begin < kt_end) {
    load_tile(kt_begin);
    store_tile(0);
  }
  __syncthreads();
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int cur = NSTAGE == 2 ? ((kt - kt_begin) & 1) : 0;
    if (kt + 1 < kt_end) load_tile(kt + 1);
    compute(smem + cur * STAGE);
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

  if constexpr (BIAS) {
    {  // bias gradient: column sums of the bf16 dY rows of this split (L2-resident), the rows
       // shared out among the split's ntn tile columns (one workgroup summing all of them
       // was the critical path once splits grew long): partial row split * ntn + tn
      constexpr int CPR = BM / 8, RPP = NTH / CPR;
      const int cc = tid % CPR, rr = tid / CPR;
      const int co = co0 + cc * 8;
      float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const int sm0 = kt_begin * BK, sm1 = min(p.M, kt_end * BK);
      const int share = ((sm1 - sm0 + ntn - 1) / ntn + RPP - 1) / RPP * RPP;
      if (co < p.Mo) {
        const int m1 = min(sm1, sm0 + (tn + 1) * share);
        int m = sm0 + tn * share + rr;
        for (; m + 3 * RPP < m1; m += 4 * RPP) {
          u32x4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const u32x4*>(p.dy16 + (size_t)(m + u * RPP) * p.ldy + co);
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bs[2 * e] += lo_bf(v[u][e]);
              bs[2 * e + 1] += hi_bf(v[u][e]);
            }
        }
        for (; m < m1; m += RPP) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(p.dy16 + (size_t)m * p.ldy + co);
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
        float* bo = p.bslab + ((size_t)split * ntn + tn) * p.Mo + co;
        *reinterpret_cast<f32x4*>(bo) = f32x4{t8[0], t8[1], t8[2], t8[3]};
        *reinterpret_cast<f32x4*>(bo + 4) = f32x4{t8[4], t8[5], t8[6], t8[7]};
      }
    }
  }

  const float dq = p.dq_dy[0] * p.dq_x[0];
  float* out = p.slab + (size_t)split * p.Mo * p.No;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int co = co0 + wm * (BM / WM) + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int tc = tc0 + wn * (BN / WN) + j * 16 + (lane >> 4) * 4;
      if (co < p.Mo && tc < p.No) *reinterpret_cast<f32x4*>(out + (size_t)co * p.No + tc) = acc[i][j] * dq;
    }
  }
}

struct WG8Var {
  int BM, BN, NS, NTH, target, KS, GL, SP;
};
// 4-wave tiles (2x2 waves, two workgroups per CU) and 8-wave tiles; target = workgroups,
// KS = MFMA k-steps (128 token rows each) per k-tile / barrier
// GL = LDS-DMA ring (NS stages, one workgroup per CU)
// ids 21-24: 256x256 on FOUR waves (2x2 of 128x128, one wave per SIMD, accumulators in
// AGPRs): a CU's fragment reads per k-step fall from 192 KB (8 waves of 128x64) to 128 KB
// ids 25-28: the software-pipelined fragment reads (SP) on the 256x256 8-wave tiles (1 / 2
// register-staged stages, the 2-stage LDS-DMA ring) and the 128x128 2-stage tile
constexpr int WG8_NVAR = 29;
constexpr WG8Var WG8_VARS[WG8_NVAR] = {
    {128, 128, 2, 256, 1024, 1, 0}, {128, 128, 1, 256, 1024, 1, 0}, {128, 128, 2, 256, 512, 1, 0},
    {128, 128, 1, 256, 2048, 1, 0}, {256, 128, 2, 512, 512, 1, 0},  {128, 256, 2, 512, 512, 1, 0},
    {256, 128, 2, 512, 1024, 1, 0}, {64, 128, 2, 256, 1024, 1, 0},  {128, 128, 1, 256, 1024, 2, 0},
    {128, 128, 1, 256, 512, 2, 0},  {256, 256, 1, 512, 256, 1, 0},  {256, 256, 2, 512, 256, 1, 0},
    {256, 256, 1, 512, 512, 1, 0},  {128, 128, 3, 256, 1024, 1, 1}, {128, 128, 4, 256, 1024, 1, 1},
    {256, 128, 3, 512, 512, 1, 1},  {128, 256, 3, 512, 512, 1, 1},  {256, 128, 3, 512, 1024, 1, 1},
    {128, 128, 2, 256, 1024, 1, 1}, {256, 256, 2, 512, 256, 1, 1},  {256, 256, 2, 512, 512, 1, 1},
    {256, 256, 2, 256, 512, 1, 0},  {256, 256, 2, 256, 256, 1, 0},  {256, 256, 2, 256, 256, 1, 1},
    {256, 256, 2, 256, 512, 1, 1},
    {256, 256, 1, 512, 256, 1, 0, 1}, {256, 256, 2, 512, 256, 1, 0, 1}, {256, 256, 2, 512, 256, 1, 1, 1},
    {128, 128, 2, 256, 1024, 1, 0, 1},
};

WG8Var wg8_variant(int v) { return (v < 0 || v >= WG8_NVAR) ? WG8_VARS[0] : WG8_VARS[v]; }

template <bool BIAS>
int launch8(const WG8Var& w, dim3 grid, const WG8Params& p_in, hipStream_t st) {
  static const void* cache[PDT_MAX_DEV] = {};
  WG8Params p = p_in;
  p.zero = pdt_symbol_addr(HIP_SYMBOL(wg8_zero_chunk), cache);
  if (p.zero == nullptr) return PDT_ERR_SYMBOL;
#define L8(a, b, ns, t, wm) hipLaunchKernelGGL((wgrad_f8_kernel<a, b, ns, t, wm, BIAS>), grid, dim3(t), 0, st, p)
#define G8(a, b, ns, t, wm) hipLaunchKernelGGL((wgrad_f8_kernel<a, b, ns, t, wm, BIAS, 1, true>), grid, dim3(t), 0, st, p)
#define S8(a, b, ns, t, wm, gl) \
  hipLaunchKernelGGL((wgrad_f8_kernel<a, b, ns, t, wm, BIAS, 1, gl, true>), grid, dim3(t), 0, st, p)
  if (w.SP) {
    if (w.BM == 128) S8(128, 128, 2, 256, 2, false);
    else if (w.GL) S8(256, 256, 2, 512, 2, true);
    else if (w.NS == 2) S8(256, 256, 2, 512, 2, false);
    else S8(256, 256, 1, 512, 2, false);
  } else if (w.GL) {
    if (w.BM == 256 && w.BN == 256) {
      if (w.NTH == 256) G8(256, 256, 2, 256, 2);
      else G8(256, 256, 2, 512, 2);
    } else if (w.NTH == 512) {
      if (w.BM == 256) G8(256, 128, 3, 512, 4);
      else G8(128, 256, 3, 512, 2);
    } else if (w.NS == 4) {
      G8(128, 128, 4, 256, 2);
    } else if (w.NS == 3) {
      G8(128, 128, 3, 256, 2);
    } else {
      G8(128, 128, 2, 256, 2);
    }
  } else if (w.KS == 2) {
    hipLaunchKernelGGL((wgrad_f8_kernel<128, 128, 1, 256, 2, BIAS, 2>), grid, dim3(256), 0, st, p);
  } else if (w.BM == 256 && w.BN == 256 && w.NTH == 256) {
    L8(256, 256, 2, 256, 2);  // (single-stage: 620 B/lane of scratch, not built)
  } else if (w.BM == 256 && w.BN == 256) {
    if (w.NS == 2) L8(256, 256, 2, 512, 2);
    else L8(256, 256, 1, 512, 2);
  } else if (w.NTH == 512) {
    if (w.BM == 256) L8(256, 128, 2, 512, 4);
    else L8(128, 256, 2, 512, 2);
  } else if (w.BM == 64) {
    L8(64, 128, 2, 256, 2);
  } else if (w.NS == 2) {
    L8(128, 128, 2, 256, 2);
  } else {
    L8(128, 128, 1, 256, 2);
  }
#undef L8
#undef G8
#undef S8
  return 0;
}

// the kernel a variant launches (launch8's dispatch), for the occupancy query
template <bool BIAS>
const void* kernel8(const WG8Var& w) {
#define K8(a, b, ns, t, wm) return reinterpret_cast<const void*>(&wgrad_f8_kernel<a, b, ns, t, wm, BIAS>)
#define KG8(a, b, ns, t, wm) return reinterpret_cast<const void*>(&wgrad_f8_kernel<a, b, ns, t, wm, BIAS, 1, true>)
#define KS8(a, b, ns, t, wm, gl) \
  return reinterpret_cast<const void*>(&wgrad_f8_kernel<a, b, ns, t, wm, BIAS, 1, gl, true>)
  if (w.SP) {
    if (w.BM == 128) KS8(128, 128, 2, 256, 2, false);
    if (w.GL) KS8(256, 256, 2, 512, 2, true);
    if (w.NS == 2) KS8(256, 256, 2, 512, 2, false);
    KS8(256, 256, 1, 512, 2, false);
  }
  if (w.GL) {
    if (w.BM == 256 && w.BN == 256) {
      if (w.NTH == 256) KG8(256, 256, 2, 256, 2);
      KG8(256, 256, 2, 512, 2);
    }
    if (w.NTH == 512) {
      if (w.BM == 256) KG8(256, 128, 3, 512, 4);
      KG8(128, 256, 3, 512, 2);
    }
    if (w.NS == 4) KG8(128, 128, 4, 256, 2);
    if (w.NS == 3) KG8(128, 128, 3, 256, 2);
    KG8(128, 128, 2, 256, 2);
  }
  if (w.KS == 2) return reinterpret_cast<const void*>(&wgrad_f8_kernel<128, 128, 1, 256, 2, BIAS, 2>);
  if (w.BM == 256 && w.BN == 256 && w.NTH == 256) K8(256, 256, 2, 256, 2);
  if (w.BM == 256 && w.BN == 256) {
    if (w.NS == 2) K8(256, 256, 2, 512, 2);
    K8(256, 256, 1, 512, 2);
  }
  if (w.NTH == 512) {
    if (w.BM == 256) K8(256, 128, 2, 512, 4);
    K8(128, 256, 2, 512, 2);
  }
  if (w.BM == 64) K8(64, 128, 2, 256, 2);
  if (w.NS == 2) K8(128, 128, 2, 256, 2);
  K8(128, 128, 1, 256, 2);
#undef K8
#undef KG8
#undef KS8
}

// workgroups of variant v resident on the whole device at once (occupancy API, the smaller of
// the bias / no-bias instantiations; cached per variant)
int slots8(int v) {
  static int cache[WG8_NVAR] = {};
  const int vi = (v < 0 || v >= WG8_NVAR) ? 0 : v;
  if (cache[vi] == 0) {
    const WG8Var w = wg8_variant(vi);
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, kernel8<true>(w), w.NTH, 0) != hipSuccess) a = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel8<false>(w), w.NTH, 0) != hipSuccess) b = 1;
    int n = a < b ? a : b;
    cache[vi] = (n < 1 ? 1 : n) * pdt_num_cus();
  }
  return cache[vi];
}

int reduce_groups8(int splits, int Mo, int No) {
  long n4 = (long)Mo * No / 4;
  int xb = (int)((n4 + 255) / 256);
  int G = splits < 2 ? 1 : (int)(1024 / xb);
  if (G > splits / 4) G = splits / 4;
  if (G < 1) G = 1;
  return G;
}

}  // namespace

PDT_API int pdt_wgrad_f8_num_variants() { return WG8_NVAR; }

PDT_API int pdt_wgrad_f8_plan(int M, int Mo, int No, int variant, int* ktiles_per_split) {
  const WG8Var w = wg8_variant(variant);
  const int tiles = ((Mo + w.BM - 1) / w.BM) * ((No + w.BN - 1) / w.BN);
  const int BK = BK1 * w.KS;
  const int nk = (M + BK - 1) / BK;
  // Splits s <= ceil(target / tiles) minimising (dispatch waves) x (k-tiles per split): the
  // device holds slots8(v) workgroups at once, and a grid one workgroup past a multiple of it
  // runs a whole extra wave for that straggler (tiles = 27 at target 512: 513 workgroups, 3
  // waves of 83 k-tiles; s = 9: 243 workgroups, 1 wave of 176). Ties keep fewer splits (less
  // slab traffic). >= 512 token rows per split.
  int smax = (w.target + tiles - 1) / tiles;
  if (smax > nk) smax = nk;
  if (smax < 1) smax = 1;
  static int legacy = -1;  // PDT_WG8_PLAN=0: the previous plan, s = ceil(target / tiles) (A/B switch)
  if (legacy < 0) {
    const char* e = getenv("PDT_WG8_PLAN");
    legacy = (e && e[0] == '0') ? 1 : 0;
  }
  if (legacy) {
    int s = smax;
    while (s > 1 && (nk + s - 1) / s * BK < 512) --s;
    const int kps = (nk + s - 1) / s;
    *ktiles_per_split = kps;
    return (nk + kps - 1) / kps;
  }
  const long slots = slots8(variant);
  int best_s = 1;
  long best_cost = -1;
  for (int s = 1; s <= smax; ++s) {
    const int kps = (nk + s - 1) / s;
    if (s > 1 && kps * BK < 512) break;
    const int se = (nk + kps - 1) / kps;
    const long waves = ((long)tiles * se + slots - 1) / slots;
    const long cost = waves * kps;
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best_s = s;
    }
  }
  const int kps = (nk + best_s - 1) / best_s;
  *ktiles_per_split = kps;
  return (nk + kps - 1) / kps;
}

// floats of workspace: slabs + stage-1 partials (same layout as pdt_wgrad_workspace) + the
// bias partial rows ([splits][tile columns][Mo]; tile columns <= ceil(No / 128) for every variant)
PDT_API long pdt_wgrad_f8_workspace(int splits, int Mo, int No) {
  const long G = reduce_groups8(splits, Mo, No);
  return (long)splits * Mo * No + (G > 1 ? G * Mo * No : 0) + (long)splits * ((No + 127) / 128) * Mo;
}

// dW[Mo][No] (fp32, = or +=) from e5m2 dY codes [M][ldy] and e4m3 X codes [M][ldx];
// bias_out (optional) = column sums of the bf16 dY (dy16, same layout as the codes).
PDT_API int pdt_linear_wgrad_f8(const void* dy8, const void* x8, const float* dq_dy, const float* dq_x,
                                const void* dy16, float* slab, float* out, float* bias_out, int M, int Mo, int No,
                                int ldy, int ldx, int splits, int ktiles_per_split, int accumulate, int variant,
                                hipStream_t stream) {
  if (Mo % 16 || No % 16 || ldy % 16 || ldx % 16) return -1;
  if (bias_out && !dy16) return -2;
  const WG8Var w = wg8_variant(variant);
  WG8Params p;
  p.dy = (const uint8_t*)dy8;
  p.x = (const uint8_t*)x8;
  p.dy16 = (const u16*)dy16;
  p.dq_dy = dq_dy;
  p.dq_x = dq_x;
  p.slab = slab;
  p.M = M; p.Mo = Mo; p.No = No; p.ldy = ldy; p.ldx = ldx;
  p.ktiles_per_split = ktiles_per_split;
  const int G = reduce_groups8(splits, Mo, No);
  p.bslab = bias_out ? slab + (long)splits * Mo * No + (G > 1 ? (long)G * Mo * No : 0) : nullptr;
  {
    static int xcd_env = -1;
    if (xcd_env < 0) {
      const char* e = getenv("PDT_WGRAD_XCD");
      xcd_env = (e && e[0] == '0') ? 0 : 1;
    }
    p.xcd = xcd_env;
  }
  const int tiles = ((Mo + w.BM - 1) / w.BM) * ((No + w.BN - 1) / w.BN);
  dim3 grid(tiles * splits);
  const int lrc = bias_out ? launch8<true>(w, grid, p, stream) : launch8<false>(w, grid, p, stream);
  if (lrc) return lrc;
  int e = (int)hipGetLastError();
  if (e) return e;
  if (bias_out) {
    const int rc = pdt_wgrad_reduce_rows(p.bslab, bias_out, splits * ((No + w.BN - 1) / w.BN), Mo, 1.f, accumulate,
                                         nullptr, stream);
    if (rc) return rc;
  }
  return pdt_wgrad_reduce(slab, out, nullptr, nullptr, splits, Mo, No, 1.f, accumulate, stream);
}
