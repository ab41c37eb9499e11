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
// staged-chunk sentinel of the AX path (padding / rows past M); valid element offsets of the
// source are < 2^32 - 8 (conv_nt_impl refuses larger sources for AX)
constexpr uint32_t AX_NONE = 0xffffffffu;

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
// fp8 instantiations (no BatchNorm consumes an fp8 GEMM, so they never form BN statistics):
// `stats` instead receives the column sums of the final bf16 output per M-tile,
// stats[tm][Ncol] -- the bias gradient of the layer this output is the gradient of
// (kept in the existing field: a new one perturbed the register allocation of the bf16 rings)

constexpr int BK = 64;
constexpr int NT = 256;

// d gelu_tanh(z) / dz
__device__ __forceinline__ float gelu_grad(float z) {
  const float u = 0.7978845608f * (z + 0.044715f * z * z * z);
  const float t = pdt_tanh(u);
  const float du = 0.7978845608f * (1.f + 3.f * 0.044715f * z * z);
  return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * du;
}

// act 4 (the MLP's fc1): gelu_tanh(z) AND its derivative from one tanh -- the derivative is
// stored as the aux output so the fc2 data gradient's epilogue is a plain multiply (act 5)
__device__ __forceinline__ void gelu_dual(float z, float& g, float& d) { pdt_gelu_dual(z, g, d); }

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
template <int BM, int BN, int NSTAGE, bool CS64, bool DIRECT, bool GLDS, int NTH = 256, int WM = 2, int F8 = 0,
          int PIPE = 0, bool BNB = false, int AX = 0>
__global__ void __launch_bounds__(NTH, PIPE ? 1 : 2) conv_nt_kernel(NTParams p) {
  static_assert(AX == 0 || (!PIPE && F8 == 0 && CS64), "the A-staging BN apply: bf16, 64-channel chunks, no ring");
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
#define PDT_TILE_DONE return
#define PDT_TILE_ID blockIdx.x
#include "conv_nt_tile.inc"
#undef PDT_TILE_ID
#undef PDT_TILE_DONE
}

// PERS: the persistent ring tiles. One workgroup per CU walks the output tiles t, t + grid, ...
// in the XCD-grouped order of the one-tile launch (the tiles an XCD has in flight stay
// neighbours in its L2), so a new tile needs no new dispatch (short-K shapes: 5-18 % in
// scripts/gemm_lab, v7 vs v4). The kernel arguments are re-read from the kernarg segment per
// tile (an opaque pointer): held across the tile loop they spilled ~70 VGPRs.
template <int BM, int BN, int NSTAGE, bool CS64, bool DIRECT, bool GLDS, int NTH = 256, int WM = 2, int F8 = 0,
          int PIPE = 0, bool BNB = false, int AX = 0>
__global__ void __launch_bounds__(NTH, 1) conv_nt_kernel_pers(NTParams p_arg) {
  static_assert(PIPE && AX == 0 && F8 == 0, "persistent: the bf16 1-workgroup-per-CU ring tiles");
  // (the same prologue as conv_nt_kernel)
  constexpr int WN = NTH / 64 / WM;
  constexpr int MI = BM / (WM * 16);
  constexpr int NI = BN / (WN * 16);
  constexpr int LA = BM * 8 / NTH;
  constexpr int LB = BN * 8 / NTH;
  constexpr int RS = NTH / 8;
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int C_STRIDE = BN * 2 + 16;
  constexpr int CST = (DIRECT && !BNB) ? 0 : BM * C_STRIDE;
  constexpr int SMEM = (NSTAGE * STAGE > CST) ? NSTAGE * STAGE : CST;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  auto wcol = [&](int j) -> int {
    if constexpr (PIPE == 2)
      return j < NI / 2 ? wn * (BN / 2 / WN) + j * 16 : BN / 2 + wn * (BN / 2 / WN) + (j - NI / 2) * 16;
    else
      return wn * (BN / WN) + j * 16;
  };
  const int ntm = (p_arg.M + BM - 1) / BM;
  const int ntn = (p_arg.Ncol + BN - 1) / BN;
  const int ntiles = ntm * ntn;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    if (tile != (int)blockIdx.x) __syncthreads();  // the previous tile's epilogue LDS reads are done
    const NTParams& p = p_arg;
    const void* zchunk = p.zero;
#define PDT_TILE_DONE continue
#define PDT_TILE_ID tile
#include "conv_nt_tile.inc"
#undef PDT_TILE_ID
#undef PDT_TILE_DONE
  }
}

template <int BM, int BN, int NS, bool CS64, bool DIRECT, bool GLDS = false, int NTH = 256, int WM = 2, int F8 = 0,
          int PIPE = 0, bool BNB = false, int AX = 0, bool PERS = false>
int launch(const NTParams& p, hipStream_t st) {
  int ntm = (p.M + BM - 1) / BM, ntn = (p.Ncol + BN - 1) / BN;
  NTParams q = p;
  q.zero = zero_chunk_addr();
  if (q.zero == nullptr) return PDT_ERR_SYMBOL;
  if constexpr (PERS) {
    if (p.q8 != nullptr) return -5;  // the fp8 side output keeps one max per workgroup AND tile
    // one workgroup per CU (the ring tiles hold >= 128 KB of LDS), all 256 CUs
    const int grid = ntm * ntn < 256 ? ntm * ntn : 256;
    hipLaunchKernelGGL((conv_nt_kernel_pers<BM, BN, NS, CS64, DIRECT, GLDS, NTH, WM, F8, PIPE, BNB, AX>),
                       dim3(grid), dim3(NTH), 0, st, q);
  } else {
    hipLaunchKernelGGL((conv_nt_kernel<BM, BN, NS, CS64, DIRECT, GLDS, NTH, WM, F8, PIPE, BNB, AX>),
                       dim3(ntm * ntn), dim3(NTH), 0, st, q);
  }
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
// PERS_BASE[i], one workgroup per CU walking the output tiles (conv_nt_kernel_pers).
// The 256x128 / 128x256 rings, and the 256x256 one (id 36) with the BN-backward epilogue only:
// its plain-store instantiation sits at 256 VGPRs one tile per workgroup and spilled 236 B
// around the tile loop, while the compiled BN-backward walks fit in 255 without spilling.
constexpr int NVAR_PERS = 3;
constexpr int PERS_BASE[NVAR_PERS] = {34, 35, 36};

template <bool CS64, bool BNB = false>
int launch_variant_pers(int i, const NTParams& p, hipStream_t st) {
  switch (i) {
    case 0: return launch<256, 128, 3, CS64, false, true, 512, 4, 0, true, BNB, 0, true>(p, st);
    case 1: return launch<128, 256, 3, CS64, false, true, 512, 2, 0, true, BNB, 0, true>(p, st);
    case 2:
      if constexpr (BNB) return launch<256, 256, 2, CS64, false, true, 512, 2, 0, true, BNB, 0, true>(p, st);
      else return -5;
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
