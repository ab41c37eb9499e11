// Implicit-GEMM kernel template shared by conv_igemm.hip (plain epilogues) and
// conv_igemm_bnb.hip (the fused BatchNorm-backward epilogue instantiations).
// See conv_igemm.hip for the algorithm.
#pragma once
#include "pdt_common.h"
#include <stdlib.h>

namespace pdt_nt {

// BatchNorm-backward reduction fused into a data-gradient epilogue. The GEMM
// output (+ addend) is dA, the gradient arriving at a BN(+ReLU) unit's output;
// instead of a separate pass that re-reads dA and y, the epilogue computes
// per-channel partials of g = relu_gate(dA) over its rows:
//   part[row0 + r][c] = sum g,   part[R + row0 + r][c] = sum g * (y - mean)
// (the layout pdt_bn_bwd_finalize reduces). dA is stored UNGATED (it stays the
// true gradient of the unit's output); g uses the bf16-rounded stored value,
// exactly what the reduce pass would have read.
struct BnbArgs {
  const u16* y;          // the unit's pre-BN conv output, same layout as the GEMM output
  const float* mean;     // [Ncol]
  const float* scale;    // [Ncol] (ReLU gate recomputed from y when mask == nullptr)
  const float* shift;
  const uint8_t* mask;   // optional ReLU bit mask of the unit's output
  float* part;           // nullptr = disabled
  int relu, row0, R;
  // optional second unit fed by the SAME gated gradient (a downsample block's shortcut BN,
  // gated by the block's ReLU mask like bn3): its partials [sum g | sum g * (y2 - mean2)]
  // go to part2 with part's row layout (sum g is shared, written to both)
  const u16* y2 = nullptr;
  const float* mean2 = nullptr;
  float* part2 = nullptr;
};

// BatchNorm apply folded into the A-operand staging of a 1x1 GEMM (register-staged
// variants only), so the BN'd tensor is produced by its consumer instead of by a
// separate element pass that writes it and a GEMM that re-reads it. The A loads read
// `src` (and `y2`), the staging pass applies the BN, feeds the MFMAs and -- in the
// tn == 0 workgroups, which stage every A row exactly once -- writes the result to
// `dst` (and the ReLU bit mask), equal to the element pass (csrc/bn_act.hip) up to FMA
// contraction (one bf16 rounding).
//   mode 1 (forward, the next conv1):  A = relu(src*c1 + c2 + y2)       (src = y3, y2 = residual)
//                                      y2 term = y2*rsc + rsh when rsc (raw downsample output)
//                                      dst = the block output, mask_out = its ReLU bit mask
//          (forward, conv2 / conv3):   y2 = nullptr: A = relu(src*c1 + c2) (src = the raw conv
//                                      output of bn1 / bn2), dst = the input the weight gradient reads
//   mode 3 (backward, conv2's dgrad):  A = c1*gate + c2*y2 + c3, gate = src where y2*rsc + rsh > 0
//                                      (the ReLU recomputed from the BN input), dst = dy2
// Any stride-1 geometry with 64-channel k-tiles (3x3 included): dst / mask_out are written
// from the k-tiles of tap `ctr`, the one that maps every output row onto its own source pixel.
//   mode 2 (backward, conv3's dgrad):  A = c1*gate(src) + c2*y2 + c3   (src = dout, y2 = y3,
//                                      gate = mask_in bit), dst = dy3 (the wgrad operand)
struct AXArgs {
  int mode;
  int ctr;  // the tap whose A chunks are the source pixels themselves (dst / mask_out written there)
  const u16* y2;
  const float* c1;
  const float* c2;
  const float* c3;
  const float* rsc;
  const float* rsh;
  const uint8_t* mask_in;
  uint8_t* mask_out;
  u16* dst;
};

struct NTParams {
  const u16* src;
  const u16* b;
  u16* out;
  float* stats;        // optional: [2][nstat_rows][Ncol] partial sums (sum, sumsq)
  const float* bias;   // optional: [Ncol]
  const u16* addend;   // optional: out = conv + addend (same layout as out)
  int Hs, Ws, Cs;      // source geometry (NHWC, batch implied by M-grid)
  int Hm, Wm;          // M-grid per image
  int M, Ncol, K, ldb;
  int sh, sw, oh0, ow0, dh, dw, nth, ntw;
  int Ho, Wo, osh, osw, oph, opw, ldo;
  int act;             // 0 none, 1 relu, 2 gelu(tanh), 3 GELU backward: out = C * gelu'(addend)
                       //   (addend = the saved pre-activation z; fuses the activation backward
                       //   into the data-gradient GEMM that produces dL/dgelu(z))
  int pix;             // elements per source pixel in memory (= Cs, or Cs/2 for the space-to-depth stem
                       // whose 16-B chunk spans two adjacent 4-channel pixels)
  u16* aux;            // optional: pre-activation copy of the output (same layout)
  int nstat_rows;
  int nt_store;        // 1: non-temporal (streaming) output stores
  int ident_out;       // 1: output row == m (no stride-phase remap) -> skip the index math
  const uint8_t* addend_mask;  // optional: addend is masked by this ReLU bit mask (1 bit / element)
  const float* dq_a;   // fp8 only: dequant scale of the A (src) operand (device scalar)
  const float* dq_b;   // fp8 only: dequant scale of the B operand
  BnbArgs bnb;         // optional: BatchNorm-backward partial sums of the unit this output feeds
  AXArgs ax;           // optional (AX instantiations): BN apply in the A staging
  FastDiv div_Wm, div_HWm, div_Cs8, div_ntw;
  // optional fp8 copy of the final output for the NEXT fp8 GEMM (staged epilogue only):
  // codes of the bf16-rounded values times q8_meta[0] (its delayed scale), same layout
  // as out (1 byte / element), and each workgroup's max |value| in q8_part[blockIdx.x]
  // (pdt_fp8_meta_roll_partial folds those into the amax history afterwards)
  uint8_t* q8;
  const float* q8_meta;
  float* q8_part;
  int q8_fmt;          // 0 e4m3, 1 e5m2
  int q8_only;         // 1: the bf16 output itself is not written
  const void* zero;    // 16 zero bytes in device memory (set by launch(): the LDS-DMA padding source)
};

constexpr int BK = 64;
constexpr int NT = 256;

// d gelu_tanh(z) / dz
__device__ __forceinline__ float gelu_grad(float z) {
  const float u = 0.7978845608f * (z + 0.044715f * z * z * z);
  const float t = pdt_tanh(u);
  const float du = 0.7978845608f * (1.f + 3.f * 0.044715f * z * z);
  return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * du;
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ i32x8 cat8(const bf16x8& lo, const bf16x8& hi) {
  const u32x4 a = __builtin_bit_cast(u32x4, lo), b = __builtin_bit_cast(u32x4, hi);
  return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}

// 16 zero bytes: the global_load_lds source for padding / out-of-range rows
static __device__ __attribute__((aligned(64))) u32x4 pdt_zero_chunk[4];
// its device address on the current device (host side, cached per device; nullptr on failure)
static inline const void* zero_chunk_addr() {
  static const void* cache[PDT_MAX_DEV] = {};
  return pdt_symbol_addr(HIP_SYMBOL(pdt_zero_chunk), cache);
}

// F8 = 0: bf16 operands. F8 = 1 / 2: fp8 operands (B = OCP e4m3; src = e4m3 / e5m2)
// handled as byte PAIRS -- every index below is in 2-byte units, so staging,
// swizzle and gather are unchanged -- and one block-scaled
// mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate, unit block scales)
// consumes a whole 128-byte LDS k-row: the two bf16 k-step fragments of a lane
// ARE its 32-byte fp8 fragment (a k permutation shared by both operands).
// The per-tensor dequant scales multiply the accumulators in the epilogue.
// PIPE 1: NSTAGE-deep LDS-DMA ring, one barrier per K-tile. PIPE 2 (256x256, 8 waves): a
// 4-phase ring -- each K-tile's MFMAs run as four C-quadrant phases, and the next K-tile
// is fetched one quarter per phase with counted vmcnt (never 0 in the loop), so three
// quarters stay in flight across every barrier (the schedule of the guide's 256^2 8-phase
// template, 4 phases per K-tile).
// PERS: persistent -- a grid of one workgroup per CU walks the output tiles (tile t, t + grid,
// ...) in the XCD-grouped order of the one-tile-per-workgroup launch, so the tiles one XCD has
// in flight stay neighbours in its L2; the workgroup's first wave of tiles starts at once and the
// ring's next tile needs no new dispatch (short-K shapes: 5-18 % in scripts/gemm_lab, v7 vs v4).
// Every tile runs the whole body (operand prologue .. epilogue); one barrier between tiles frees
// the LDS the previous epilogue staged through.
template <int BM, int BN, int NSTAGE, bool CS64, bool DIRECT, bool GLDS, int NTH = 256, int WM = 2, int F8 = 0,
          int PIPE = 0, bool BNB = false, int AX = 0, bool PERS = false>
__global__ void __launch_bounds__(NTH, PIPE ? 1 : 2) conv_nt_kernel(NTParams p) {
  static_assert(AX == 0 || (!PIPE && F8 == 0 && CS64), "the A-staging BN apply: bf16, 64-channel chunks, no ring");
  static_assert(!PERS || (PIPE && AX == 0), "persistent: the 1-workgroup-per-CU ring tiles");
  constexpr int WN = NTH / 64 / WM;       // waves along N
  constexpr int MI = BM / (WM * 16);      // 16-row MFMA tiles per wave
  constexpr int NI = BN / (WN * 16);
  constexpr int LA = BM * 8 / NTH;        // 16-B A chunks each thread stages per K-tile
  constexpr int LB = BN * 8 / NTH;
  constexpr int RS = NTH / 8;             // rows covered by one staging pass
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int C_STRIDE = BN * 2 + 16;  // bytes per staged output row
  constexpr int CST = (DIRECT && !BNB) ? 0 : BM * C_STRIDE;  // epilogue staging bytes (BNB always stages)
  constexpr int SMEM = (NSTAGE * STAGE > CST) ? NSTAGE * STAGE : CST;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // the zero page's address comes in the kernel arguments (SGPRs for the whole kernel):
  // referenced as a symbol, every LDS-DMA issue reloads it through the GOT (s_load +
  // s_waitcnt lgkmcnt(0)), and that wait also drains the fragment ds_reads the memory
  // section just issued
  const void* zchunk = p.zero;
  // tile column of this wave's j-th 16-column block. PIPE 2 gives each wave one 32-column
  // block in each HALF of the tile, so a K-tile's B operand arrives as two contiguous
  // 128-row halves (one per phase pair).
  auto wcol = [&](int j) -> int {
    if constexpr (PIPE == 2)
      return j < NI / 2 ? wn * (BN / 2 / WN) + j * 16 : BN / 2 + wn * (BN / 2 / WN) + (j - NI / 2) * 16;
    else
      return wn * (BN / WN) + j * 16;
  };

  const int ntm = (p.M + BM - 1) / BM;
  const int ntn = (p.Ncol + BN - 1) / BN;
  const int ntiles = ntm * ntn;
  for (int tile = blockIdx.x; tile < ntiles; tile += PERS ? (int)gridDim.x : ntiles) {
  if (PERS && tile != (int)blockIdx.x) __syncthreads();  // the previous tile's epilogue LDS reads are done
  const uint32_t logical = xcd_remap(tile, ntiles);
  const int tm = logical / ntn, tn = logical % ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-thread A rows: r = tid/8 + 32*i, chunk column ca = tid%8
  const int ca = tid & 7;
  int a_base[LA], a_ih[LA], a_iw[LA];
  bool a_ok[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    int m = m0 + (tid >> 3) + RS * i;
    a_ok[i] = m < p.M;
    uint32_t mm = a_ok[i] ? m : 0;
    uint32_t img = fdiv(mm, p.div_HWm);
    uint32_t rem = mm - img * (uint32_t)(p.Hm * p.Wm);
    uint32_t oh = fdiv(rem, p.div_Wm);
    uint32_t ow = rem - oh * p.Wm;
    a_base[i] = img * p.Hs * p.Ws;
    a_ih[i] = oh * p.sh + p.oh0;
    a_iw[i] = ow * p.sw + p.ow0;
  }
  // ---- per-thread B rows
  int b_row[LB];
  bool b_ok[LB];
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    int n = n0 + (tid >> 3) + RS * j;
    b_ok[j] = n < p.Ncol;
    b_row[j] = b_ok[j] ? n : 0;
  }

  u32x4 ra[LA], rb[LB];
  const int nk = (p.K + BK - 1) / BK;
  // AX: the second A operand, the mask bytes, the element offset of each staged chunk
  // (-1: padding / out of range) and this thread's 8 channels' coefficients for the k-tile
  u32x4 ry[AX ? LA : 1];
  uint32_t rmk[AX ? LA : 1];
  int roff[AX ? LA : 1];
  constexpr bool AXC3 = AX == 2 || AX == 3, AXRS = AX == 1 || AX == 3;
  float cf1[AX ? 8 : 1], cf2[AX ? 8 : 1], cf3[AXC3 ? 8 : 1], cfs[AXRS ? 8 : 1], cfh[AXRS ? 8 : 1];
  const bool ax_write = AX != 0 && p.ax.dst != nullptr && tn == 0;
  bool ax_wr = false;  // ax_write AND the staged k-tile is the centre tap (set with its fetch)

  // AX: this thread's 8 channels' BN coefficients (channel c0..c0+7 of the k-tile)
  auto ax_coef = [&](int c0) __attribute__((always_inline)) {
    if constexpr (AX != 0) {
#pragma unroll
      for (int e = 0; e < 8; e += 4) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(p.ax.c1 + c0 + e);
        const f32x4 b = *reinterpret_cast<const f32x4*>(p.ax.c2 + c0 + e);
#pragma unroll
        for (int q = 0; q < 4; ++q) { cf1[e + q] = a[q]; cf2[e + q] = b[q]; }
        if constexpr (AXC3) {
          const f32x4 c = *reinterpret_cast<const f32x4*>(p.ax.c3 + c0 + e);
#pragma unroll
          for (int q = 0; q < 4; ++q) cf3[e + q] = c[q];
        }
        if constexpr (AXRS) {
          const bool raff = p.ax.rsc != nullptr;
          const f32x4 c = raff ? *reinterpret_cast<const f32x4*>(p.ax.rsc + c0 + e) : f32x4{1.f, 1.f, 1.f, 1.f};
          const f32x4 d = raff ? *reinterpret_cast<const f32x4*>(p.ax.rsh + c0 + e) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int q = 0; q < 4; ++q) { cfs[e + q] = c[q]; cfh[e + q] = d[q]; }
        }
      }
    }
  };

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    if (CS64) {
      const int tap = k0 / p.Cs;
      const int c0 = k0 - tap * p.Cs + ca * 8;
      const int th = fdiv(tap, p.div_ntw);
      const int tw = tap - th * p.ntw;
      const int dho = p.dh * th, dwo = p.dw * tw;
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        int ih = a_ih[i] + dho, iw = a_iw[i] + dwo;
        bool ok = a_ok[i] && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws;
        const size_t off = (size_t)(a_base[i] + ih * p.Ws + iw) * p.pix + c0;
        if (ok) {
          ra[i] = *reinterpret_cast<const u32x4*>(p.src + off);
        } else {
          ra[i] = u32x4{0, 0, 0, 0};
        }
        if constexpr (AX != 0) {
          roff[i] = ok ? (int)off : -1;  // host guarantees 32-bit element offsets
          // mode 1 without a residual (y2 == nullptr): r = 0, f + 0 == f exactly
          ry[i] = (ok && p.ax.y2 != nullptr) ? *reinterpret_cast<const u32x4*>(p.ax.y2 + off) : u32x4{0, 0, 0, 0};
          rmk[i] = (AX == 2 && ok) ? (uint32_t)p.ax.mask_in[off >> 3] : 0u;
        }
      }
      if constexpr (AX != 0) {
        ax_coef(c0);
        ax_wr = ax_write && tap == p.ax.ctr;
      }
    } else {
      const int kc = k0 / 8 + ca;  // global 8-channel chunk index
      const bool kin = kc * 8 < p.K;
      const int tap = fdiv(kc, p.div_Cs8);
      const int c0 = (kc - tap * (p.Cs / 8)) * 8;
      const int th = fdiv(tap, p.div_ntw);
      const int tw = tap - th * p.ntw;
      const int dho = p.dh * th, dwo = p.dw * tw;
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        int ih = a_ih[i] + dho, iw = a_iw[i] + dwo;
        bool ok = kin && a_ok[i] && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws;
        if (ok) {
          ra[i] = *reinterpret_cast<const u32x4*>(p.src + (size_t)(a_base[i] + ih * p.Ws + iw) * p.pix + c0);
        } else {
          ra[i] = u32x4{0, 0, 0, 0};
        }
      }
    }
    const int kb = k0 + ca * 8;
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      if (b_ok[j] && kb < p.K) {
        rb[j] = *reinterpret_cast<const u32x4*>(p.b + (size_t)b_row[j] * p.ldb + kb);
      } else {
        rb[j] = u32x4{0, 0, 0, 0};
      }
    }
  };

  // AX: apply the BN to the staged A chunk (same arithmetic as csrc/bn_act.hip's element
  // passes), write it (+ mask) once from the tn == 0 workgroups
  auto ax_apply = [&](int i) __attribute__((always_inline)) {
    if constexpr (AX != 0) {
      if (roff[i] < 0) return;  // padding / out-of-range rows stay zero (never written)
      float f[8], r[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[2 * e] = lo_bf(ra[i][e]); f[2 * e + 1] = hi_bf(ra[i][e]);
        r[2 * e] = lo_bf(ry[i][e]); r[2 * e + 1] = hi_bf(ry[i][e]);
      }
      u32x4 o;
      if constexpr (AX == 1) {
        const bool raff = p.ax.rsc != nullptr;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          f[k] = f[k] * cf1[k] + cf2[k];
          f[k] += raff ? r[k] * cfs[k] + cfh[k] : r[k];
          f[k] = fmaxf(f[k], 0.f);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = pack2bf(f[2 * e], f[2 * e + 1]);
        if (ax_wr && p.ax.mask_out != nullptr) {
          uint32_t m = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {  // mask of the ROUNDED output, as bn_apply_kernel
            m |= ((o[e] & 0x7fffu) != 0 && !(o[e] & 0x8000u)) ? (1u << (2 * e)) : 0u;
            m |= ((o[e] & 0x7fff0000u) != 0 && !(o[e] & 0x80000000u)) ? (1u << (2 * e + 1)) : 0u;
          }
          p.ax.mask_out[roff[i] >> 3] = (uint8_t)m;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // mode 2: ReLU gate from the bit mask; mode 3: recomputed as bn_bwd_apply does (y s + b > 0)
          const bool on = AX == 2 ? ((rmk[i] >> k) & 1u) != 0 : r[k] * cfs[k] + cfh[k] > 0.f;
          const float g = on ? f[k] : 0.f;
          f[k] = cf1[k] * g + cf2[k] * r[k] + cf3[k];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = pack2bf(f[2 * e], f[2 * e + 1]);
      }
      if (ax_wr) *reinterpret_cast<u32x4*>(p.ax.dst + roff[i]) = o;
      ra[i] = o;
    }
  };

  auto store_tile = [&](int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      ax_apply(i);
      int r = (tid >> 3) + RS * i;
      *reinterpret_cast<u32x4*>(sa + r * 128 + swz(r, ca) * 16) = ra[i];
    }
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      int r = (tid >> 3) + RS * j;
      *reinterpret_cast<u32x4*>(sb + r * 128 + swz(r, ca) * 16) = rb[j];
    }
  };

  // GLDS + AX: the A tile lands in LDS untouched; the thread that DMA'd a chunk (row r,
  // physical chunk ca = logical chunk swz(r, ca) -- the same logical chunk for all its
  // rows, RS being a multiple of 16) fetches that chunk's second operand / mask /
  // coefficients into registers alongside the DMA (ax_fetch), then, once the tile is in
  // LDS, rewrites the chunk in place with the applied values (ax_lds) before the MFMAs
  // read it. 64-channel k-tiles (CS64): each k-tile lies within one tap.
  auto ax_fetch = [&](int kt) __attribute__((always_inline)) {
    if constexpr (AX != 0 && GLDS) {
      static_assert(RS % 16 == 0, "one logical chunk per thread");
      const int k0 = kt * BK;
      const int tap = k0 / p.Cs;
      const int c0 = k0 - tap * p.Cs + swz(tid >> 3, ca) * 8;
      const int th = fdiv(tap, p.div_ntw);
      const int tw = tap - th * p.ntw;
      const int dho = p.dh * th, dwo = p.dw * tw;
      ax_wr = ax_write && tap == p.ax.ctr;
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        const int ih = a_ih[i] + dho, iw = a_iw[i] + dwo;
        const bool ok = a_ok[i] && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws;
        const size_t off = (size_t)(a_base[i] + ih * p.Ws + iw) * p.pix + c0;
        roff[i] = ok ? (int)off : -1;
        ry[i] = (ok && p.ax.y2 != nullptr) ? *reinterpret_cast<const u32x4*>(p.ax.y2 + off) : u32x4{0, 0, 0, 0};
        rmk[i] = (AX == 2 && ok) ? (uint32_t)p.ax.mask_in[off >> 3] : 0u;
      }
      ax_coef(c0);
    }
  };
  auto ax_lds = [&](int buf) __attribute__((always_inline)) {
    if constexpr (AX != 0 && GLDS) {
      char* sa = smem + buf * STAGE;
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        u32x4* q = reinterpret_cast<u32x4*>(sa + ((tid >> 3) + RS * i) * 128 + ca * 16);
        ra[i] = *q;
        ax_apply(i);
        *q = ra[i];
      }
    }
  };

  // GLDS: global_load_lds_dwordx4 straight into LDS (no VGPR staging). The
  // LDS image stays lane-linear per wave instruction (8 rows x 128 B), so the
  // XOR swizzle moves to the SOURCE: lane (row r, physical chunk ca) fetches
  // logical chunk ca ^ swz(r). Padding / out-of-range rows read a zero page.
  auto glds_a = [&](int kt, int buf, int i) __attribute__((always_inline)) {
    char* sa = smem + buf * STAGE;
    const int k0 = kt * BK;
    const int r = (tid >> 3) + RS * i;
    const int c = swz(r, ca);  // logical chunk for this lane's LDS slot
    const void* g = zchunk;
    if constexpr (F8 != 0) {  // the fp8 GEMM's A is a dense [M][K] matrix (pdt_gemm_f8): no gather math
      if (m0 + r < p.M) g = p.src + (size_t)(m0 + r) * p.Cs + k0 + c * 8;
    } else if (CS64) {
      const int tap = k0 / p.Cs;
      const int c0 = k0 - tap * p.Cs + c * 8;
      const int th = fdiv(tap, p.div_ntw);
      const int tw = tap - th * p.ntw;
      const int ih = a_ih[i] + p.dh * th, iw = a_iw[i] + p.dw * tw;
      if (a_ok[i] && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws)
        g = p.src + (size_t)(a_base[i] + ih * p.Ws + iw) * p.pix + c0;
    } else {
      const int kc = k0 / 8 + c;
      const int tap = fdiv(kc, p.div_Cs8);
      const int c0 = (kc - tap * (p.Cs / 8)) * 8;
      const int th = fdiv(tap, p.div_ntw);
      const int tw = tap - th * p.ntw;
      const int ih = a_ih[i] + p.dh * th, iw = a_iw[i] + p.dw * tw;
      if (kc * 8 < p.K && a_ok[i] && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws)
        g = p.src + (size_t)(a_base[i] + ih * p.Ws + iw) * p.pix + c0;
    }
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(sa + (8 * wave + RS * i) * 128),
                                     16, 0, 0);
  };
  auto glds_b = [&](int kt, int buf, int j) __attribute__((always_inline)) {
    char* sb = smem + buf * STAGE + A_BYTES;
    const int r = (tid >> 3) + RS * j;
    const int kb = kt * BK + swz(r, ca) * 8;
    const void* g = (b_ok[j] && kb < p.K) ? (const void*)(p.b + (size_t)b_row[j] * p.ldb + kb)
                                          : zchunk;
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(sb + (8 * wave + RS * j) * 128),
                                     16, 0, 0);
  };
  // GLDS: global_load_lds_dwordx4 straight into LDS (no VGPR staging). The
  // LDS image stays lane-linear per wave instruction (8 rows x 128 B), so the
  // XOR swizzle moves to the SOURCE: lane (row r, physical chunk ca) fetches
  // logical chunk ca ^ swz(r). Padding / out-of-range rows read a zero page.
  auto glds_tile = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < LA; ++i) glds_a(kt, buf, i);
#pragma unroll
    for (int j = 0; j < LB; ++j) glds_b(kt, buf, j);
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one K-tile of MFMA work on the LDS stage at sa / sb
  auto compute_tile = [&](const char* sa, const char* sb) {
    if constexpr (F8 != 0) {
      bf16x8 af[2][MI], bfr[2][NI];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int kch = kk * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          int r = wm * (BM / WM) + i * 16 + (lane & 15);
          af[kk][i] = *reinterpret_cast<const bf16x8*>(sa + r * 128 + swz(r, kch) * 16);
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          int r = wcol(j) + (lane & 15);
          bfr[kk][j] = *reinterpret_cast<const bf16x8*>(sb + r * 128 + swz(r, kch) * 16);
        }
      }
      if (PIPE) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              cat8(bfr[0][j], bfr[1][j]), cat8(af[0][i], af[1][i]), acc[i][j], 0, F8 == 2 ? 1 : 0, 0, 127, 0, 127);
      if (PIPE) __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int kch = kk * 4 + (lane >> 4);
        bf16x8 af[MI], bfr[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          int r = wm * (BM / WM) + i * 16 + (lane & 15);
          af[i] = *reinterpret_cast<const bf16x8*>(sa + r * 128 + swz(r, kch) * 16);
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          int r = wcol(j) + (lane & 15);
          bfr[j] = *reinterpret_cast<const bf16x8*>(sb + r * 128 + swz(r, kch) * 16);
        }
        if (PIPE) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            // swapped operands: lane holds 4 consecutive output channels of one row
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        if (PIPE) __builtin_amdgcn_s_setprio(0);
      }
    }
  };

  if constexpr (PIPE == 2) {
    // 4-phase ring (see the template comment). Quarter loads of a K-tile: q0 = A rows of
    // quadrant row r = 0 (chunks i = 0, 2), q1 = B half 0 (j = 0, 1), q2 = B half 1 (j = 2, 3),
    // q3 = A rows r = 1 (i = 1, 3); 2 LDS-DMA instructions each per thread. Phases of K-tile t
    // (C-quadrant (r, c)): 1 = (0,0) needs q0 q1, 2 = (0,1) needs q2, 3 = (1,1) needs q3, 4 =
    // (1,0) needs nothing new; phase p issues quarter p-1 of K-tile t+1 into the other buffer,
    // whose last reads (K-tile t-1) all precede phase 1's barrier.
    // RAW: each wave retires its own DMA of a quarter with a counted vmcnt, then the barrier
    // makes every wave's copy visible; reads of a quarter never precede that barrier.
    static_assert(GLDS && NSTAGE == 2 && LA == 4 && LB == 4 && MI % 2 == 0 && NI % 2 == 0, "4-phase ring shape");
    auto issue = [&](int q, int kt, int buf) __attribute__((always_inline)) {
      if (q == 0) { glds_a(kt, buf, 0); glds_a(kt, buf, 2); }
      else if (q == 1) { glds_b(kt, buf, 0); glds_b(kt, buf, 1); }
      else if (q == 2) { glds_b(kt, buf, 2); glds_b(kt, buf, 3); }
      else { glds_a(kt, buf, 1); glds_a(kt, buf, 3); }
    };
    constexpr int HM = MI / 2, HN = NI / 2;
    // bf16: two k-step fragments per 16-row block; fp8: the same 32 bytes as ONE operand
    // (the k permutation of the F8 note above), assembled at read time
    bf16x8 af[F8 ? 1 : HM][2], bq[F8 ? 1 : HN][2];
    i32x8 af8[F8 ? HM : 1], bq8[F8 ? HN : 1];
    auto read_a = [&](const char* sa, int r) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < HM; ++i) {
        const int row = wm * (BM / WM) + (r * HM + i) * 16 + (lane & 15);
        const bf16x8 f0 = *reinterpret_cast<const bf16x8*>(sa + row * 128 + swz(row, lane >> 4) * 16);
        const bf16x8 f1 = *reinterpret_cast<const bf16x8*>(sa + row * 128 + swz(row, 4 + (lane >> 4)) * 16);
        if constexpr (F8 != 0) {
          af8[i] = cat8(f0, f1);
        } else {
          af[i][0] = f0;
          af[i][1] = f1;
        }
      }
    };
    auto read_b = [&](const char* sb, int c) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < HN; ++j) {
        const int row = wcol(c * HN + j) + (lane & 15);
        const bf16x8 f0 = *reinterpret_cast<const bf16x8*>(sb + row * 128 + swz(row, lane >> 4) * 16);
        const bf16x8 f1 = *reinterpret_cast<const bf16x8*>(sb + row * 128 + swz(row, 4 + (lane >> 4)) * 16);
        if constexpr (F8 != 0) {
          bq8[j] = cat8(f0, f1);
        } else {
          bq[j][0] = f0;
          bq[j][1] = f1;
        }
      }
    };
    auto mma = [&](int r, int c) __attribute__((always_inline)) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < HM; ++i)
#pragma unroll
        for (int j = 0; j < HN; ++j) {
          if constexpr (F8 != 0) {
            acc[r * HM + i][c * HN + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                bq8[j], af8[i], acc[r * HM + i][c * HN + j], 0, F8 == 2 ? 1 : 0, 0, 127, 0, 127);
          } else {
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
              acc[r * HM + i][c * HN + j] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][kk], af[i][kk], acc[r * HM + i][c * HN + j], 0, 0, 0);
          }
        }
      __builtin_amdgcn_s_setprio(0);
    };
    // Two wave groups (wm = 0 / 1) run one barrier apart (ping-pong): each phase is a
    // memory section (wait, LDS-DMA issue, fragment ds_reads, lgkmcnt(0)), a barrier, the
    // 16-MFMA section, a barrier -- so one group's MFMAs overlap the other group's memory
    // section. A quarter is waited (vmcnt) in the memory section BEFORE the phase that
    // reads it: every wave has retired its copy before the barrier that ends that section,
    // which every reader has passed. A buffer is restaged only after the barrier that
    // follows both groups' last reads of it (their lgkmcnt(0) precedes it).
    auto bar = [&]() __attribute__((always_inline)) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    auto mma_phase = [&](int r, int c) __attribute__((always_inline)) {
      bar();
      mma(r, c);
      bar();
    };
    if (nk > 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) issue(q, 0, 0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // q0 q1 of K-tile 0
    }
    bar();
    if (wm == 1) bar();  // the stagger
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1, nxt = cur ^ 1;
      const bool more = kt + 1 < nk;
      const char* sa = smem + cur * STAGE;
      const char* sb = sa + A_BYTES;
      // Memory sections: fragment ds_reads first (their data was retired one section
      // earlier), then the counted wait for the quarter the NEXT section reads, then the
      // prefetch of the next K-tile's quarter. The reads are retired by the lgkmcnt(0) after
      // the section's barrier (inside mma): every restage comes >= 2 phases after the last
      // read of its region, so no wait is needed before that barrier.
      // M1: reads (0,0); retire q2 of this K-tile (read in phase 2); prefetch q0 of the next
      read_a(sa, 0);
      read_b(sb, 0);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      if (more) issue(0, kt + 1, nxt);
      mma_phase(0, 0);
      // M2: reads (0,1); retire q3 (read in phase 3)
      read_b(sb, 1);
      if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (more) issue(1, kt + 1, nxt);
      mma_phase(0, 1);
      // M3: reads (1,1)
      read_a(sa, 1);
      if (more) issue(2, kt + 1, nxt);
      mma_phase(1, 1);
      // M4: reads (1,0); retire q0 q1 of the next K-tile (read in its phase 1)
      read_b(sb, 0);
      if (more) {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        issue(3, kt + 1, nxt);
      }
      mma_phase(1, 0);
    }
    if (wm == 0) bar();  // close the stagger: equal barrier counts on every wave
    if (!DIRECT) __syncthreads();  // before the epilogue reuses LDS
  } else if constexpr (PIPE) {
    // NSTAGE-deep LDS-DMA ring, ONE raw barrier per K-tile: tile kt+NSTAGE-1
    // is issued right after the barrier that proves every wave finished
    // reading its buffer (tile kt-1's); the counted vmcnt before the barrier
    // retires only this thread's tile-kt DMA (with 3 stages tile kt+1's stays
    // in flight across it). No __syncthreads (vmcnt(0) lgkmcnt(0)) in the loop.
    static_assert(GLDS && (NSTAGE == 2 || NSTAGE == 3), "the ring is the LDS-DMA pipeline");
    for (int t = 0; t < NSTAGE - 1; ++t)
      if (t < nk) glds_tile(t, t);
    for (int kt = 0; kt < nk; ++kt) {
      if (NSTAGE == 3 && kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LA + LB) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + NSTAGE - 1 < nk) glds_tile(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
      const char* sa = smem + (kt % NSTAGE) * STAGE;
      compute_tile(sa, sa + A_BYTES);
    }
    if (!DIRECT) __syncthreads();  // before the epilogue reuses LDS
  } else {
  if (GLDS) {
    if (nk > 0) {
      glds_tile(0, 0);
      ax_fetch(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (nk > 0) ax_lds(0);  // a lane's DMA fills its own LDS slot: no barrier before the rewrite
  } else if (nk > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = NSTAGE == 2 ? (kt & 1) : 0;
    if (GLDS) {
      if (NSTAGE == 2 && kt + 1 < nk) {
        glds_tile(kt + 1, cur ^ 1);
        ax_fetch(kt + 1);
      }
    } else if (kt + 1 < nk) {
      load_tile(kt + 1);
    }
    const char* sa = smem + cur * STAGE;
    compute_tile(sa, sa + A_BYTES);
    if (GLDS) {
      if (NSTAGE == 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my DMA into the other buffer landed
        if (kt + 1 < nk) ax_lds(cur ^ 1);                  // (AX) rewrite my chunks of it in place
        __syncthreads();                                   // ... and everyone's; buffer cur is free
      } else if (kt + 1 < nk) {
        __syncthreads();
        glds_tile(kt + 1, 0);
        ax_fetch(kt + 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ax_lds(0);
        __syncthreads();
      }
    } else if (NSTAGE == 2) {
      if (kt + 1 < nk) store_tile(cur ^ 1);
      __syncthreads();
    } else if (kt + 1 < nk) {
      __syncthreads();  // everyone is done reading the single buffer
      store_tile(0);
      __syncthreads();
    }
  }
  if (NSTAGE == 1 && !DIRECT) __syncthreads();  // before the epilogue reuses LDS
  }

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][r] = C[row = wm*BM/2 + i*16 + (lane&15)][col = wn*BN/2 + j*16 + (lane>>4)*4 + r]
  const int lrow = lane & 15;
  const int lcol = (lane >> 4) * 4;
  if constexpr (F8 != 0) {
    const float alpha = p.dq_a[0] * p.dq_b[0];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] *= alpha;
  }
  if (p.bias != nullptr) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int col = n0 + wcol(j) + lcol + r;
        float bv = col < p.Ncol ? p.bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < MI; ++i) acc[i][j][r] += bv;
      }
    }
  }

  if constexpr (BNB) {
    // Fused BatchNorm-backward partials (BnbArgs). The bf16 tile is staged
    // through LDS as in the plain epilogue; each thread then owns one 16-B
    // chunk column (8 channels) and walks rows, so y / addend are read -- and
    // dA written -- as coalesced 16-B row chunks, exactly the bytes the
    // separate reduce pass would have read. Loads of IB rows are issued before
    // any is consumed. Output = bf16(bf16(acc) + masked addend): bit-identical
    // to the plain data gradient; the partials see that stored value.
    // Partial rows: one per M-tile (lanes, then waves, reduced in-block).
    constexpr int CPR = BN / 8;
    constexpr int RPI = NTH / CPR;        // rows covered per pass
    constexpr int NIT = BM / RPI;         // passes
    constexpr int IB = NIT < 4 ? NIT : 4;  // rows in flight per thread
    static_assert(NTH % CPR == 0 && BM % RPI == 0, "chunk-column ownership");
    __syncthreads();  // all waves are done with the operand stages
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int r = wm * (BM / WM) + i * 16 + lrow;
        int c = wcol(j) + lcol;
        uint2 w;
        w.x = pack2bf(acc[i][j][0], acc[i][j][1]);
        w.y = pack2bf(acc[i][j][2], acc[i][j][3]);
        *reinterpret_cast<uint2*>(smem + r * C_STRIDE + c * 2) = w;
      }
    __syncthreads();
    const int cc = tid % CPR, r0 = tid / CPR;
    const int col = n0 + cc * 8;
    const bool cok = col < p.Ncol;
    const int colc = cok ? col : 0;
    const bool has_add = p.addend != nullptr, has_amask = p.addend_mask != nullptr;
    const bool has_mask = p.bnb.mask != nullptr, gate_y = p.bnb.relu && !has_mask;
    // (not in the ring tiles: their 256-VGPR budget spills; the host refuses part2 there)
    const bool two = PIPE == 0 && p.bnb.part2 != nullptr;
    float mu[8], sc[8], sh[8], s[8], q[8], mu2[8], q2[8];
    {
      const f32x4 m0v = *reinterpret_cast<const f32x4*>(p.bnb.mean + colc);
      const f32x4 m1v = *reinterpret_cast<const f32x4*>(p.bnb.mean + colc + 4);
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, h0 = s0, h1 = s0;
      if (gate_y) {
        s0 = *reinterpret_cast<const f32x4*>(p.bnb.scale + colc);
        s1 = *reinterpret_cast<const f32x4*>(p.bnb.scale + colc + 4);
        h0 = *reinterpret_cast<const f32x4*>(p.bnb.shift + colc);
        h1 = *reinterpret_cast<const f32x4*>(p.bnb.shift + colc + 4);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        mu[k] = m0v[k]; mu[k + 4] = m1v[k];
        sc[k] = s0[k]; sc[k + 4] = s1[k];
        sh[k] = h0[k]; sh[k + 4] = h1[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] = q[k] = q2[k] = mu2[k] = 0.f;
      if (two) {
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(p.bnb.mean2 + colc);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(p.bnb.mean2 + colc + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) { mu2[k] = a0[k]; mu2[k + 4] = a1[k]; }
      }
    }
#pragma unroll
    for (int it0 = 0; it0 < NIT; it0 += IB) {
      uint32_t eo[IB];
      bool rok[IB];
      u32x4 yv4[IB], ad4[IB], yb4[IB];
      uint32_t amb[IB], mkb[IB];
#pragma unroll
      for (int b = 0; b < IB; ++b) {
        const int m = m0 + r0 + (it0 + b) * RPI;
        rok[b] = cok && m < p.M;
        const uint32_t mm = m < p.M ? m : 0;
        uint32_t orow = mm;
        if (!p.ident_out) {
          uint32_t img = fdiv(mm, p.div_HWm);
          uint32_t rem = mm - img * (uint32_t)(p.Hm * p.Wm);
          uint32_t oh = fdiv(rem, p.div_Wm);
          uint32_t ow = rem - oh * p.Wm;
          orow = (img * p.Ho + oh * p.osh + p.oph) * p.Wo + ow * p.osw + p.opw;
        }
        eo[b] = orow * (uint32_t)p.ldo + colc;  // host guarantees rows * ldo < 2^31
        yv4[b] = *reinterpret_cast<const u32x4*>(p.bnb.y + eo[b]);
        yb4[b] = two ? *reinterpret_cast<const u32x4*>(p.bnb.y2 + eo[b]) : u32x4{0u, 0u, 0u, 0u};
        ad4[b] = has_add ? *reinterpret_cast<const u32x4*>(p.addend + eo[b]) : u32x4{0u, 0u, 0u, 0u};
        amb[b] = has_amask ? (uint32_t)p.addend_mask[eo[b] >> 3] : 0xffu;
        mkb[b] = has_mask ? (uint32_t)p.bnb.mask[eo[b] >> 3] : 0xffu;
      }
#pragma unroll
      for (int b = 0; b < IB; ++b) {
        const int r = r0 + (it0 + b) * RPI;
        u32x4 v = *reinterpret_cast<const u32x4*>(smem + r * C_STRIDE + cc * 16);
        if (has_add) {
          u32x4 a = ad4[b];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] &= ((amb[b] >> (2 * e)) & 1u ? 0xffffu : 0u) | ((amb[b] >> (2 * e + 1)) & 1u ? 0xffff0000u : 0u);
            v[e] = pack2bf(lo_bf(v[e]) + lo_bf(a[e]), hi_bf(v[e]) + hi_bf(a[e]));
          }
        }
        if (rok[b]) *reinterpret_cast<u32x4*>(p.out + eo[b]) = v;
        float g[8], yf[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          g[2 * e] = lo_bf(v[e]); g[2 * e + 1] = hi_bf(v[e]);
          yf[2 * e] = lo_bf(yv4[b][e]); yf[2 * e + 1] = hi_bf(yv4[b][e]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          bool on = rok[b];
          if (p.bnb.relu) on = on && (has_mask ? ((mkb[b] >> k) & 1u) != 0 : (yf[k] * sc[k] + sh[k]) > 0.f);
          const float gg = on ? g[k] : 0.f;
          s[k] += gg;
          q[k] += gg * (yf[k] - mu[k]);
          if (two) q2[k] += gg * ((k & 1 ? hi_bf(yb4[b][k >> 1]) : lo_bf(yb4[b][k >> 1])) - mu2[k]);
        }
      }
    }
    // lanes sharing a chunk column: lane, lane ^ CPR, ... (CPR < 64); the xor-16 / xor-32
    // steps on the permlane swaps (VALU), smaller strides on ds_bpermute
#pragma unroll
    for (int o = CPR; o < 16; o <<= 1)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += __shfl_xor(s[k], o, 64);
        q[k] += __shfl_xor(q[k], o, 64);
        if (two) q2[k] += __shfl_xor(q2[k], o, 64);
      }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (CPR <= 16) {
        s[k] = xor16_reduce(s[k], AddOp{});
        q[k] = xor16_reduce(q[k], AddOp{});
        if (two) q2[k] = xor16_reduce(q2[k], AddOp{});
      }
      s[k] = xor32_reduce(s[k], AddOp{});
      q[k] = xor32_reduce(q[k], AddOp{});
      if (two) q2[k] = xor32_reduce(q2[k], AddOp{});
    }
    constexpr int NW = NTH / 64;
    constexpr int RW = PIPE == 0 ? 24 : 16;  // floats per (wave, chunk column): s[8] q[8] (q2[8])
    float* red = reinterpret_cast<float*>(smem);  // [NW][CPR][RW], staging reads are done after the barrier
    __syncthreads();
    if (lane < CPR) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[(wave * CPR + lane) * RW + k] = s[k];
        red[(wave * CPR + lane) * RW + 8 + k] = q[k];
        if (two) red[(wave * CPR + lane) * RW + 16 + k] = q2[k];
      }
    }
    __syncthreads();
    const int srow = p.bnb.row0 + tm;
    const int nred = two ? 24 : 16;
    for (int t = tid; t < CPR * nred; t += NTH) {
      const int c8 = t / nred, k = t % nred;
      float acc_w = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) acc_w += red[(w * CPR + c8) * RW + k];
      const int cl = n0 + c8 * 8 + (k & 7);
      if (cl < p.Ncol) {
        if (k < 8) {
          p.bnb.part[(size_t)srow * p.Ncol + cl] = acc_w;
          if (two) p.bnb.part2[(size_t)srow * p.Ncol + cl] = acc_w;
        } else {
          float* dst = k < 16 ? p.bnb.part : p.bnb.part2;
          dst[(size_t)(p.bnb.R + srow) * p.Ncol + cl] = acc_w;
        }
      }
    }
    continue;  // (next tile of a persistent workgroup; the loop ends otherwise)
  }

  if (p.stats != nullptr) {
    // per-wave column partials over its BM/2 rows (invalid rows hold zeros)
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const int srow = tm * WM + wm;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      // column sums over this lane's MI rows on packed fp32 (v_pk_add / v_pk_fma: 2 columns
      // each) in the bf16 instantiations; scalar in the fp8 ones (the packed temporaries push
      // the 256x256 fp8 ring into more scratch, and no fp8 GEMM feeds a BatchNorm)
      f32x2 s01 = {0.f, 0.f}, s23 = s01, q01 = s01, q23 = s01;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if constexpr (F8 == 0) {
          const f32x2 v01 = {acc[i][j][0], acc[i][j][1]}, v23 = {acc[i][j][2], acc[i][j][3]};
          s01 += v01;
          s23 += v23;
          q01 = __builtin_elementwise_fma(v01, v01, q01);
          q23 = __builtin_elementwise_fma(v23, v23, q23);
        } else {
          s01.x += acc[i][j][0]; s01.y += acc[i][j][1]; s23.x += acc[i][j][2]; s23.y += acc[i][j][3];
          q01.x += acc[i][j][0] * acc[i][j][0]; q01.y += acc[i][j][1] * acc[i][j][1];
          q23.x += acc[i][j][2] * acc[i][j][2]; q23.y += acc[i][j][3] * acc[i][j][3];
        }
      }
      // the 16 lanes of a DPP row hold the 16 rows of this column group
      float s[4] = {row16_sum(s01.x), row16_sum(s01.y), row16_sum(s23.x), row16_sum(s23.y)};
      float q[4] = {row16_sum(q01.x), row16_sum(q01.y), row16_sum(q23.x), row16_sum(q23.y)};
      // every lane of the row now has all 8 sums: lanes 0-3 store sum[r], lanes 4-7 sumsq[r]
      // (one store per lane instead of eight from one lane)
      if (lrow < 8) {
        const int r = lrow & 3;
        const float sv = (r & 2) ? ((r & 1) ? s[3] : s[2]) : ((r & 1) ? s[1] : s[0]);
        const float qv = (r & 2) ? ((r & 1) ? q[3] : q[2]) : ((r & 1) ? q[1] : q[0]);
        const int col = n0 + wcol(j) + lcol + r;
        if (col < p.Ncol)
          p.stats[(size_t)((lrow < 4 ? 0 : p.nstat_rows) + srow) * p.Ncol + col] = lrow < 4 ? sv : qv;
      }
    }
  }

  // stage the bf16 tile through LDS (row-major [BM][BN], 16-B row pad) and
  // write 16-B coalesced rows; `pre` = pre-activation copy (aux output)
  constexpr int CPR = BN / 8;  // 16-B chunks per row
  // DIRECT: each lane stores its 4 consecutive channels (8 B) straight to HBM
  // (no LDS round trip / barrier); L2 merges the 32-B row pieces into lines.
  auto direct_store = [&](u16* dst, const u16* addend) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      int m = m0 + wm * (BM / WM) + i * 16 + lrow;
      if (m >= p.M) continue;
      size_t orow = m;
      if (!p.ident_out) {
        uint32_t img = fdiv(m, p.div_HWm);
        uint32_t rem = m - img * (uint32_t)(p.Hm * p.Wm);
        uint32_t oh = fdiv(rem, p.div_Wm);
        uint32_t ow = rem - oh * p.Wm;
        orow = ((size_t)img * p.Ho + oh * p.osh + p.oph) * p.Wo + ow * p.osw + p.opw;
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int col = n0 + wcol(j) + lcol;
        if (col >= p.Ncol) continue;
        float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        if (addend != nullptr) {
          uint2 a = *reinterpret_cast<const uint2*>(addend + orow * p.ldo + col);
          if (p.addend_mask != nullptr) {
            const size_t e = orow * p.ldo + col;
            const uint32_t mb = p.addend_mask[e >> 3] >> (e & 7);
            a.x &= ((mb & 1u) ? 0xffffu : 0u) | ((mb & 2u) ? 0xffff0000u : 0u);
            a.y &= ((mb & 4u) ? 0xffffu : 0u) | ((mb & 8u) ? 0xffff0000u : 0u);
          }
          if (p.act == 3) {
            v0 *= gelu_grad(lo_bf(a.x)); v1 *= gelu_grad(hi_bf(a.x));
            v2 *= gelu_grad(lo_bf(a.y)); v3 *= gelu_grad(hi_bf(a.y));
          } else {
            v0 += lo_bf(a.x); v1 += hi_bf(a.x); v2 += lo_bf(a.y); v3 += hi_bf(a.y);
          }
        }
        uint2 w;
        w.x = pack2bf(v0, v1);
        w.y = pack2bf(v2, v3);
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        u32x2 w2 = {w.x, w.y};
        u32x2* dp = reinterpret_cast<u32x2*>(dst + orow * p.ldo + col);
        if (p.nt_store) __builtin_nontemporal_store(w2, dp);
        else *dp = w2;
      }
    }
  };

  auto stage_store = [&](u16* dst, const u16* addend, bool q8) __attribute__((always_inline)) {
    if (DIRECT) {
      direct_store(dst, addend);
      return;
    }
    const float q8s = q8 ? p.q8_meta[0] : 0.f;
    float q8max = 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int r = wm * (BM / WM) + i * 16 + lrow;
        int c = wcol(j) + lcol;
        uint2 w;
        w.x = pack2bf(acc[i][j][0], acc[i][j][1]);
        w.y = pack2bf(acc[i][j][2], acc[i][j][3]);
        *reinterpret_cast<uint2*>(smem + r * C_STRIDE + c * 2) = w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < (BM * CPR) / NTH; ++it) {
      int q = tid + it * NTH;
      int r = q / CPR, cc = q % CPR;
      int m = m0 + r;
      int col = n0 + cc * 8;
      if (m < p.M && col < p.Ncol) {
        u32x4 v = *reinterpret_cast<const u32x4*>(smem + r * C_STRIDE + cc * 16);
        size_t orow = m;
        if (!p.ident_out) {
          uint32_t img = fdiv(m, p.div_HWm);
          uint32_t rem = m - img * (uint32_t)(p.Hm * p.Wm);
          uint32_t oh = fdiv(rem, p.div_Wm);
          uint32_t ow = rem - oh * p.Wm;
          orow = ((size_t)img * p.Ho + oh * p.osh + p.oph) * p.Wo + ow * p.osw + p.opw;
        }
        if (addend != nullptr) {
          u32x4 a = *reinterpret_cast<const u32x4*>(addend + orow * p.ldo + col);
          if (p.addend_mask != nullptr) {
            const uint32_t mb = p.addend_mask[(orow * p.ldo + col) >> 3];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              a[e] &= ((mb >> (2 * e)) & 1u ? 0xffffu : 0u) | ((mb >> (2 * e + 1)) & 1u ? 0xffff0000u : 0u);
          }
          if (p.act == 3) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              v[e] = pack2bf(lo_bf(v[e]) * gelu_grad(lo_bf(a[e])), hi_bf(v[e]) * gelu_grad(hi_bf(a[e])));
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = pack2bf(lo_bf(v[e]) + lo_bf(a[e]), hi_bf(v[e]) + hi_bf(a[e]));
          }
        }
        if (q8) {
          float f[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            f[2 * e] = lo_bf(v[e]);
            f[2 * e + 1] = hi_bf(v[e]);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) q8max = fmaxf(q8max, fabsf(f[e]));
          uint2 c8;
          if (p.q8_fmt == 0) {
            c8.x = pdt_cvt4_f8<0>(f[0] * q8s, f[1] * q8s, f[2] * q8s, f[3] * q8s);
            c8.y = pdt_cvt4_f8<0>(f[4] * q8s, f[5] * q8s, f[6] * q8s, f[7] * q8s);
          } else {
            c8.x = pdt_cvt4_f8<1>(f[0] * q8s, f[1] * q8s, f[2] * q8s, f[3] * q8s);
            c8.y = pdt_cvt4_f8<1>(f[4] * q8s, f[5] * q8s, f[6] * q8s, f[7] * q8s);
          }
          *reinterpret_cast<uint2*>(p.q8 + orow * p.ldo + col) = c8;
          if (p.q8_only) continue;
        }
        u32x4* dp = reinterpret_cast<u32x4*>(dst + orow * p.ldo + col);
        if (p.nt_store) __builtin_nontemporal_store(v, dp);
        else *dp = v;
      }
    }
    if (q8) {  // workgroup max |value| -> q8_part[blockIdx.x]
      __shared__ float q8red[NTH / 64];
      q8max = warp_max(q8max);
      if ((tid & 63) == 0) q8red[tid >> 6] = q8max;
      __syncthreads();
      if (tid == 0) {
        float m = q8red[0];
#pragma unroll
        for (int w = 1; w < NTH / 64; ++w) m = fmaxf(m, q8red[w]);
        p.q8_part[blockIdx.x] = m;
      }
    }
  };

  if (p.aux != nullptr) {
    stage_store(p.aux, nullptr, false);
    if (!DIRECT) __syncthreads();
  }
  if (p.act == 1 || p.act == 2) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = acc[i][j][r];
          if (p.act == 1) {
            x = fmaxf(x, 0.f);
          } else {
            float u = 0.7978845608f * (x + 0.044715f * x * x * x);
            x = 0.5f * x * (1.f + pdt_tanh(u));
          }
          acc[i][j][r] = x;
        }
  }
  stage_store(p.out, p.addend, !DIRECT && p.q8 != nullptr);
  }  // tile loop
}

template <int BM, int BN, int NS, bool CS64, bool DIRECT, bool GLDS = false, int NTH = 256, int WM = 2, int F8 = 0,
          int PIPE = 0, bool BNB = false, int AX = 0, bool PERS = false>
int launch(const NTParams& p, hipStream_t st) {
  int ntm = (p.M + BM - 1) / BM, ntn = (p.Ncol + BN - 1) / BN;
  if (PERS && p.q8 != nullptr) return -5;  // the fp8 side output keeps one max per workgroup AND tile
  NTParams q = p;
  q.zero = zero_chunk_addr();
  if (q.zero == nullptr) return PDT_ERR_SYMBOL;
  // persistent: one workgroup per CU (the ring tiles hold >= 128 KB of LDS), all 256 CUs
  const int grid = PERS ? (ntm * ntn < 256 ? ntm * ntn : 256) : ntm * ntn;
  hipLaunchKernelGGL((conv_nt_kernel<BM, BN, NS, CS64, DIRECT, GLDS, NTH, WM, F8, PIPE, BNB, AX, PERS>),
                     dim3(grid), dim3(NTH), 0, st, q);
  PDT_RETURN_LAUNCH();
}

// Tile variants (autotuned per shape from Python; -1 = built-in heuristic).
//   id : BM x BN, LDS stages
//   ids 10..19 : the same tiles with the direct (no LDS staging) epilogue
//   ids 20..29 : the same tiles loaded by global_load_lds (LDS-DMA)
//   ids 30..33 : 512-thread (8-wave) tiles, 2 stages, 64x64 per wave:
//                256x128 (4x2 waves) and 128x256 (2x4 waves), each LDS-DMA
//                and register-staged
//   ids 34..35 : the 8-wave tiles on the 3-stage LDS-DMA ring (1 barrier per
//                K-tile, counted vmcnt, s_setprio around the MFMA bursts;
//                144 KB LDS -> one workgroup of 8 waves per CU)
//   id 36      : 256x256 (2x4 waves of 128x64), 2-stage ring (128 KB LDS): the
//                per-wave tile that lifts the LDS-bytes-per-MFMA ratio above the
//                64x64 tiles' (LDS read bandwidth, not MFMA, bounds those)
//   id 37      : the same tile on the 4-phase ping-pong ring (PIPE 2): bit-identical to id 36,
//                within +-5 % of it on the ViT / ResNet GEMM shapes (scripts/ab_variant.py;
//                the fp8 instantiation spilled and ran 1.7x slower, so it is not built)
constexpr int NVAR = 38;
constexpr int VAR_BM[NVAR] = {128, 256, 64, 128, 64, 128, 256, 64, 128, 64,
                              128, 256, 64, 128, 64, 128, 256, 64, 128, 64,
                              128, 256, 64, 128, 64, 128, 256, 64, 128, 64,
                              256, 128, 256, 128, 256, 128, 256, 256};
constexpr int VAR_BN[NVAR] = {128, 64, 128, 64, 64, 128, 64, 128, 64, 64,
                              128, 64, 128, 64, 64, 128, 64, 128, 64, 64,
                              128, 64, 128, 64, 64, 128, 64, 128, 64, 64,
                              128, 256, 128, 256, 128, 256, 256, 256};
constexpr int VAR_WM[NVAR] = {2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2,
                              2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 4, 2, 4, 2, 4, 2, 2, 2};

inline int heuristic_variant(int M, int Ncol, int K) {
  (void)M;
  if (Ncol <= 64) return K <= 64 ? 6 : 1;
  return K <= 64 ? 5 : 0;
}

template <bool CS64, bool BNB = false>
int launch_variant(int v, const NTParams& p, hipStream_t st) {
  switch (v) {
    case 0: return launch<128, 128, 2, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 1: return launch<256, 64, 2, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 2: return launch<64, 128, 2, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 3: return launch<128, 64, 2, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 4: return launch<64, 64, 2, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 5: return launch<128, 128, 1, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 6: return launch<256, 64, 1, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 7: return launch<64, 128, 1, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 8: return launch<128, 64, 1, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 9: return launch<64, 64, 1, CS64, false, false, 256, 2, 0, false, BNB>(p, st);
    case 10: return launch<128, 128, 2, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 11: return launch<256, 64, 2, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 12: return launch<64, 128, 2, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 13: return launch<128, 64, 2, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 14: return launch<64, 64, 2, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 15: return launch<128, 128, 1, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 16: return launch<256, 64, 1, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 17: return launch<64, 128, 1, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 18: return launch<128, 64, 1, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 19: return launch<64, 64, 1, CS64, true, false, 256, 2, 0, false, BNB>(p, st);
    case 20: return launch<128, 128, 2, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 21: return launch<256, 64, 2, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 22: return launch<64, 128, 2, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 23: return launch<128, 64, 2, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 24: return launch<64, 64, 2, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 25: return launch<128, 128, 1, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 26: return launch<256, 64, 1, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 27: return launch<64, 128, 1, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 28: return launch<128, 64, 1, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 29: return launch<64, 64, 1, CS64, false, true, 256, 2, 0, false, BNB>(p, st);
    case 30: return launch<256, 128, 2, CS64, false, true, 512, 4, 0, false, BNB>(p, st);
    case 31: return launch<128, 256, 2, CS64, false, true, 512, 2, 0, false, BNB>(p, st);
    case 32: return launch<256, 128, 2, CS64, false, false, 512, 4, 0, false, BNB>(p, st);
    case 33: return launch<128, 256, 2, CS64, false, false, 512, 2, 0, false, BNB>(p, st);
    case 34: return launch<256, 128, 3, CS64, false, true, 512, 4, 0, true, BNB>(p, st);
    case 35: return launch<128, 256, 3, CS64, false, true, 512, 2, 0, true, BNB>(p, st);
    case 36: return launch<256, 256, 2, CS64, false, true, 512, 2, 0, true, BNB>(p, st);
    case 37: return launch<256, 256, 2, CS64, false, true, 512, 2, 0, 2, BNB>(p, st);
  }
  return -3;
}

// persistent ring tiles (variant ids PERS0 + i in conv_igemm.hip): the tiles of ids
// PERS_BASE[i], one workgroup per CU walking the output tiles (see PERS above)
constexpr int NVAR_PERS = 4;
constexpr int PERS_BASE[NVAR_PERS] = {37, 36, 34, 35};

template <bool CS64, bool BNB = false>
int launch_variant_pers(int i, const NTParams& p, hipStream_t st) {
  switch (i) {
    case 0: return launch<256, 256, 2, CS64, false, true, 512, 2, 0, 2, BNB, 0, true>(p, st);
    case 1: return launch<256, 256, 2, CS64, false, true, 512, 2, 0, true, BNB, 0, true>(p, st);
    case 2: return launch<256, 128, 3, CS64, false, true, 512, 4, 0, true, BNB, 0, true>(p, st);
    case 3: return launch<128, 256, 3, CS64, false, true, 512, 2, 0, true, BNB, 0, true>(p, st);
  }
  return -3;
}


// the fused BatchNorm-backward instantiations (defined in conv_igemm_bnb.hip)
int launch_variant_bnb(int v, bool cs64, const NTParams& p, hipStream_t st);
int launch_variant_pers_bnb(int i, bool cs64, const NTParams& p, hipStream_t st);

// The A-staging BN apply (AXArgs) is instantiated for some register-staged tiles
// (conv_igemm_ax.hip: mode 1 plain epilogue, mode 2 with the BN-backward epilogue);
// other variant ids return NOT_APPLICABLE (-5).
int launch_variant_ax(int v, const NTParams& p, hipStream_t st);

// stride-1 pad-1 3x3 halo-patch kernels (conv3x3_halo.hip): variant hv in [0, NVAR_HALO)
//   0: BN 64, 4 waves; 1: BN 128, 8 waves; 2: BN 128, 4 waves (112 x 64 per wave)
constexpr int NVAR_HALO = 3;
int run_halo(int hv, const NTParams& p, hipStream_t st);  // -5: geometry not supported
int halo_rows(int M);                                     // stats / BN-backward partial rows
// the halo weight gradient (conv3x3_halo.hip): plan (0 = applicable) and launch of the slab kernel
int halo_wgrad_plan(int M, int Mo, int C, int Hs, int Ws, int* splits, int* tps);
int run_halo_wgrad(const void* dy, const void* x, float* slab, int M, int Mo, int C, int Hs, int Ws, int splits,
                   int tps, hipStream_t st);

}  // namespace pdt_nt
