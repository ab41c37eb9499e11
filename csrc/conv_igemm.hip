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
#include "pdt_common.h"
#include <stdlib.h>

namespace {

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
  int act;             // 0 none, 1 relu, 2 gelu(tanh)
  u16* aux;            // optional: pre-activation copy of the output (same layout)
  int nstat_rows;
  int nt_store;        // 1: non-temporal (streaming) output stores
  int ident_out;       // 1: output row == m (no stride-phase remap) -> skip the index math
  const uint8_t* addend_mask;  // optional: addend is masked by this ReLU bit mask (1 bit / element)
  const float* dq_a;   // fp8 only: dequant scale of the A (src) operand (device scalar)
  const float* dq_b;   // fp8 only: dequant scale of the B operand
  FastDiv div_Wm, div_HWm, div_Cs8, div_ntw;
};

constexpr int BK = 64;
constexpr int NT = 256;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ i32x8 cat8(const bf16x8& lo, const bf16x8& hi) {
  const u32x4 a = __builtin_bit_cast(u32x4, lo), b = __builtin_bit_cast(u32x4, hi);
  return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}

// 16 zero bytes: the global_load_lds source for padding / out-of-range rows
__device__ __attribute__((aligned(64))) u32x4 pdt_zero_chunk[4];

// F8 = 0: bf16 operands. F8 = 1 / 2: fp8 operands (B = OCP e4m3; src = e4m3 / e5m2)
// handled as byte PAIRS -- every index below is in 2-byte units, so staging,
// swizzle and gather are unchanged -- and one block-scaled
// mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate, unit block scales)
// consumes a whole 128-byte LDS k-row: the two bf16 k-step fragments of a lane
// ARE its 32-byte fp8 fragment (a k permutation shared by both operands).
// The per-tensor dequant scales multiply the accumulators in the epilogue.
template <int BM, int BN, int NSTAGE, bool CS64, bool DIRECT, bool GLDS, int NTH = 256, int WM = 2, int F8 = 0,
          bool PIPE = false>
__global__ void __launch_bounds__(NTH, PIPE ? 1 : 2) conv_nt_kernel(NTParams p) {
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
  constexpr int CST = DIRECT ? 0 : BM * C_STRIDE;  // epilogue staging bytes
  constexpr int SMEM = (NSTAGE * STAGE > CST) ? NSTAGE * STAGE : CST;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int ntm = (p.M + BM - 1) / BM;
  const int ntn = (p.Ncol + BN - 1) / BN;
  const uint32_t logical = xcd_remap(blockIdx.x, ntm * ntn);
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
        if (ok) {
          ra[i] = *reinterpret_cast<const u32x4*>(p.src + (size_t)(a_base[i] + ih * p.Ws + iw) * p.Cs + c0);
        } else {
          ra[i] = u32x4{0, 0, 0, 0};
        }
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
          ra[i] = *reinterpret_cast<const u32x4*>(p.src + (size_t)(a_base[i] + ih * p.Ws + iw) * p.Cs + c0);
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

  auto store_tile = [&](int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      int r = (tid >> 3) + RS * i;
      *reinterpret_cast<u32x4*>(sa + r * 128 + swz(r, ca) * 16) = ra[i];
    }
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      int r = (tid >> 3) + RS * j;
      *reinterpret_cast<u32x4*>(sb + r * 128 + swz(r, ca) * 16) = rb[j];
    }
  };

  // GLDS: global_load_lds_dwordx4 straight into LDS (no VGPR staging). The
  // LDS image stays lane-linear per wave instruction (8 rows x 128 B), so the
  // XOR swizzle moves to the SOURCE: lane (row r, physical chunk ca) fetches
  // logical chunk ca ^ swz(r). Padding / out-of-range rows read a zero page.
  auto glds_tile = [&](int kt, int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int r = (tid >> 3) + RS * i;
      const int c = swz(r, ca);  // logical chunk for this lane's LDS slot
      const void* g = pdt_zero_chunk;
      if (CS64) {
        const int tap = k0 / p.Cs;
        const int c0 = k0 - tap * p.Cs + c * 8;
        const int th = fdiv(tap, p.div_ntw);
        const int tw = tap - th * p.ntw;
        const int ih = a_ih[i] + p.dh * th, iw = a_iw[i] + p.dw * tw;
        if (a_ok[i] && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws)
          g = p.src + (size_t)(a_base[i] + ih * p.Ws + iw) * p.Cs + c0;
      } else {
        const int kc = k0 / 8 + c;
        const int tap = fdiv(kc, p.div_Cs8);
        const int c0 = (kc - tap * (p.Cs / 8)) * 8;
        const int th = fdiv(tap, p.div_ntw);
        const int tw = tap - th * p.ntw;
        const int ih = a_ih[i] + p.dh * th, iw = a_iw[i] + p.dw * tw;
        if (kc * 8 < p.K && a_ok[i] && (unsigned)ih < (unsigned)p.Hs && (unsigned)iw < (unsigned)p.Ws)
          g = p.src + (size_t)(a_base[i] + ih * p.Ws + iw) * p.Cs + c0;
      }
      __builtin_amdgcn_global_load_lds(
          g, (__attribute__((address_space(3))) void*)(sa + (8 * wave + RS * i) * 128), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      const int r = (tid >> 3) + RS * j;
      const int kb = k0 + swz(r, ca) * 8;
      const void* g = (b_ok[j] && kb < p.K) ? (const void*)(p.b + (size_t)b_row[j] * p.ldb + kb)
                                            : (const void*)pdt_zero_chunk;
      __builtin_amdgcn_global_load_lds(
          g, (__attribute__((address_space(3))) void*)(sb + (8 * wave + RS * j) * 128), 16, 0, 0);
    }
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
          int r = wn * (BN / WN) + j * 16 + (lane & 15);
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
          int r = wn * (BN / WN) + j * 16 + (lane & 15);
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

  if constexpr (PIPE) {
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
    if (nk > 0) glds_tile(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (nk > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = NSTAGE == 2 ? (kt & 1) : 0;
    if (GLDS) {
      if (NSTAGE == 2 && kt + 1 < nk) glds_tile(kt + 1, cur ^ 1);
    } else if (kt + 1 < nk) {
      load_tile(kt + 1);
    }
    const char* sa = smem + cur * STAGE;
    compute_tile(sa, sa + A_BYTES);
    if (GLDS) {
      if (NSTAGE == 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my DMA into the other buffer landed
        __syncthreads();                                   // ... and everyone's; buffer cur is free
      } else if (kt + 1 < nk) {
        __syncthreads();
        glds_tile(kt + 1, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
        int col = n0 + wn * (BN / WN) + j * 16 + lcol + r;
        float bv = col < p.Ncol ? p.bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < MI; ++i) acc[i][j][r] += bv;
      }
    }
  }

  if (p.stats != nullptr) {
    // per-wave column partials over its BM/2 rows (invalid rows hold zeros)
    const int srow = tm * WM + wm;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      float s[4], q[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          float v = acc[i][j][r];
          a += v;
          b += v * v;
        }
        s[r] = a;
        q[r] = b;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[r] += __shfl_xor(s[r], o, 64);
          q[r] += __shfl_xor(q[r], o, 64);
        }
      }
      if (lrow == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int col = n0 + wn * (BN / WN) + j * 16 + lcol + r;
          if (col < p.Ncol) {
            p.stats[(size_t)srow * p.Ncol + col] = s[r];
            p.stats[(size_t)(p.nstat_rows + srow) * p.Ncol + col] = q[r];
          }
        }
      }
    }
  }

  // stage the bf16 tile through LDS (row-major [BM][BN], 16-B row pad) and
  // write 16-B coalesced rows; `pre` = pre-activation copy (aux output)
  constexpr int CPR = BN / 8;  // 16-B chunks per row
  // DIRECT: each lane stores its 4 consecutive channels (8 B) straight to HBM
  // (no LDS round trip / barrier); L2 merges the 32-B row pieces into lines.
  auto direct_store = [&](u16* dst, const u16* addend) {
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
        int col = n0 + wn * (BN / WN) + j * 16 + lcol;
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
          v0 += lo_bf(a.x); v1 += hi_bf(a.x); v2 += lo_bf(a.y); v3 += hi_bf(a.y);
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

  auto stage_store = [&](u16* dst, const u16* addend) {
    if (DIRECT) {
      direct_store(dst, addend);
      return;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int r = wm * (BM / WM) + i * 16 + lrow;
        int c = wn * (BN / WN) + j * 16 + lcol;
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
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = pack2bf(lo_bf(v[e]) + lo_bf(a[e]), hi_bf(v[e]) + hi_bf(a[e]));
        }
        u32x4* dp = reinterpret_cast<u32x4*>(dst + orow * p.ldo + col);
        if (p.nt_store) __builtin_nontemporal_store(v, dp);
        else *dp = v;
      }
    }
  };

  if (p.aux != nullptr) {
    stage_store(p.aux, nullptr);
    if (!DIRECT) __syncthreads();
  }
  if (p.act != 0) {
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
            x = 0.5f * x * (1.f + tanhf(u));
          }
          acc[i][j][r] = x;
        }
  }
  stage_store(p.out, p.addend);
}

template <int BM, int BN, int NS, bool CS64, bool DIRECT, bool GLDS = false, int NTH = 256, int WM = 2, int F8 = 0,
          bool PIPE = false>
int launch(const NTParams& p, hipStream_t st) {
  int ntm = (p.M + BM - 1) / BM, ntn = (p.Ncol + BN - 1) / BN;
  hipLaunchKernelGGL((conv_nt_kernel<BM, BN, NS, CS64, DIRECT, GLDS, NTH, WM, F8, PIPE>), dim3(ntm * ntn), dim3(NTH),
                     0, st, p);
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
constexpr int NVAR = 37;
constexpr int VAR_BM[NVAR] = {128, 256, 64, 128, 64, 128, 256, 64, 128, 64,
                              128, 256, 64, 128, 64, 128, 256, 64, 128, 64,
                              128, 256, 64, 128, 64, 128, 256, 64, 128, 64,
                              256, 128, 256, 128, 256, 128, 256};
constexpr int VAR_BN[NVAR] = {128, 64, 128, 64, 64, 128, 64, 128, 64, 64,
                              128, 64, 128, 64, 64, 128, 64, 128, 64, 64,
                              128, 64, 128, 64, 64, 128, 64, 128, 64, 64,
                              128, 256, 128, 256, 128, 256, 256};
constexpr int VAR_WM[NVAR] = {2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2,
                              2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 4, 2, 4, 2, 4, 2, 2};

int heuristic_variant(int M, int Ncol, int K) {
  (void)M;
  if (Ncol <= 64) return K <= 64 ? 6 : 1;
  return K <= 64 ? 5 : 0;
}

template <bool CS64>
int launch_variant(int v, const NTParams& p, hipStream_t st) {
  switch (v) {
    case 0: return launch<128, 128, 2, CS64, false>(p, st);
    case 1: return launch<256, 64, 2, CS64, false>(p, st);
    case 2: return launch<64, 128, 2, CS64, false>(p, st);
    case 3: return launch<128, 64, 2, CS64, false>(p, st);
    case 4: return launch<64, 64, 2, CS64, false>(p, st);
    case 5: return launch<128, 128, 1, CS64, false>(p, st);
    case 6: return launch<256, 64, 1, CS64, false>(p, st);
    case 7: return launch<64, 128, 1, CS64, false>(p, st);
    case 8: return launch<128, 64, 1, CS64, false>(p, st);
    case 9: return launch<64, 64, 1, CS64, false>(p, st);
    case 10: return launch<128, 128, 2, CS64, true>(p, st);
    case 11: return launch<256, 64, 2, CS64, true>(p, st);
    case 12: return launch<64, 128, 2, CS64, true>(p, st);
    case 13: return launch<128, 64, 2, CS64, true>(p, st);
    case 14: return launch<64, 64, 2, CS64, true>(p, st);
    case 15: return launch<128, 128, 1, CS64, true>(p, st);
    case 16: return launch<256, 64, 1, CS64, true>(p, st);
    case 17: return launch<64, 128, 1, CS64, true>(p, st);
    case 18: return launch<128, 64, 1, CS64, true>(p, st);
    case 19: return launch<64, 64, 1, CS64, true>(p, st);
    case 20: return launch<128, 128, 2, CS64, false, true>(p, st);
    case 21: return launch<256, 64, 2, CS64, false, true>(p, st);
    case 22: return launch<64, 128, 2, CS64, false, true>(p, st);
    case 23: return launch<128, 64, 2, CS64, false, true>(p, st);
    case 24: return launch<64, 64, 2, CS64, false, true>(p, st);
    case 25: return launch<128, 128, 1, CS64, false, true>(p, st);
    case 26: return launch<256, 64, 1, CS64, false, true>(p, st);
    case 27: return launch<64, 128, 1, CS64, false, true>(p, st);
    case 28: return launch<128, 64, 1, CS64, false, true>(p, st);
    case 29: return launch<64, 64, 1, CS64, false, true>(p, st);
    case 30: return launch<256, 128, 2, CS64, false, true, 512, 4>(p, st);
    case 31: return launch<128, 256, 2, CS64, false, true, 512, 2>(p, st);
    case 32: return launch<256, 128, 2, CS64, false, false, 512, 4>(p, st);
    case 33: return launch<128, 256, 2, CS64, false, false, 512, 2>(p, st);
    case 34: return launch<256, 128, 3, CS64, false, true, 512, 4, 0, true>(p, st);
    case 35: return launch<128, 256, 3, CS64, false, true, 512, 2, 0, true>(p, st);
    case 36: return launch<256, 256, 2, CS64, false, true, 512, 2, 0, true>(p, st);
  }
  return -3;
}

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
  FastDiv div_Wm, div_HWm;
};

template <int KK, int NJ, bool STRIDED>
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
    f32x4 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        // swapped operands: lane holds 4 consecutive output channels of row lr
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], a[ks], acc[j], 0, 0, 0);

    const size_t m = (size_t)t * 16 + lr;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = n0 + j * 16 + (lane >> 4) * 4;
      float v[4] = {acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
      if (p.stats != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[j][r] += v[r];
          q[j][r] += v[r] * v[r];
        }
      }
      const size_t e = m * p.ldo + col;
      if (p.addend != nullptr) {
        uint2 ad = *reinterpret_cast<const uint2*>(p.addend + e);
        if (p.addend_mask != nullptr) {
          const uint32_t mb = p.addend_mask[e >> 3] >> (e & 7);
          ad.x &= ((mb & 1u) ? 0xffffu : 0u) | ((mb & 2u) ? 0xffff0000u : 0u);
          ad.y &= ((mb & 4u) ? 0xffffu : 0u) | ((mb & 8u) ? 0xffff0000u : 0u);
        }
        v[0] += lo_bf(ad.x); v[1] += hi_bf(ad.x); v[2] += lo_bf(ad.y); v[3] += hi_bf(ad.y);
      }
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2*>(p.out + e) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) a[ks] = an[ks];
  }

  if (p.stats != nullptr) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[j][r] += __shfl_xor(s[j][r], o, 64);
          q[j][r] += __shfl_xor(q[j][r], o, 64);
        }
      }
      if (lr == 0) {
        const int col = n0 + j * 16 + (lane >> 4) * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p.stats[(size_t)rg * p.N + col + r] = s[j][r];
          p.stats[(size_t)(p.nrg + rg) * p.N + col + r] = q[j][r];
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

template <int KK, int NJ>
int launch_stream(const SParams& p, bool strided, hipStream_t st) {
  const int blocks = (p.ncb * p.nrg + 3) / 4;
  if (strided)
    hipLaunchKernelGGL((gemm_stream_kernel<KK, NJ, true>), dim3(blocks), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_stream_kernel<KK, NJ, false>), dim3(blocks), dim3(256), 0, st, p);
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
  q.div_Wm = p.div_Wm; q.div_HWm = p.div_HWm;
  if (K == 64) return NJ == 2 ? launch_stream<64, 2>(q, strided, st) : launch_stream<64, 4>(q, strided, st);
  if (K == 128) return NJ == 2 ? launch_stream<128, 2>(q, strided, st) : launch_stream<128, 4>(q, strided, st);
  return launch_stream<256, 2>(q, strided, st);
}

}  // namespace

PDT_API int pdt_conv_nt_num_variants() { return NVAR + NVAR_STREAM; }

PDT_API int pdt_conv_nt_resolve_variant(int variant, int M, int Ncol, int K) {
  return (variant >= 0 && variant < NVAR + NVAR_STREAM) ? variant : heuristic_variant(M, Ncol, K);
}

// Number of BN-statistics partial rows a launch of `variant` writes (sizes the stats buffer).
PDT_API int pdt_conv_nt_stat_rows(int M, int Ncol, int K, int variant) {
  int v = pdt_conv_nt_resolve_variant(variant, M, Ncol, K);
  if (v >= NVAR) return stream_rows(v - NVAR, M, Ncol);
  int BM = VAR_BM[v];
  return ((M + BM - 1) / BM) * VAR_WM[v];
}

// Generic launch: see header comment for the meaning of every argument.
PDT_API int pdt_conv_nt(const void* src, const void* b, void* out, float* stats, const float* bias,
                        const void* addend, const void* addend_mask,
                        int Hs, int Ws, int Cs, int Nimg, int Hm, int Wm, int Ncol, int K, int ldb,
                        int sh, int sw, int oh0, int ow0, int dh, int dw, int nth, int ntw,
                        int Ho, int Wo, int osh, int osw, int oph, int opw, int ldo, int act,
                        void* aux, int variant, hipStream_t stream) {
  if (Cs % 8 != 0 || K % 8 != 0 || Ncol % 8 != 0 || ldo % 8 != 0 || ldb % 8 != 0) return -1;
  if (K != nth * ntw * Cs) return -2;
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
  p.aux = (u16*)aux;
  p.dq_a = p.dq_b = nullptr;
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
  if (v >= NVAR) return run_stream(v - NVAR, p, stream);
  const bool cs64 = (Cs % 64) == 0;
  return cs64 ? launch_variant<true>(v, p, stream) : launch_variant<false>(v, p, stream);
}

// ---------------------------------------------------------------------------
// fp8 GEMM  out[m, n] = dq_a * dq_b * sum_k A[m, k] B[n, k] (+ bias, act, aux)
// A: [M][lda] fp8 (e4m3 if fmt_a == 0, e5m2 if 1), B: [N][ldb] e4m3, out bf16 [M][ldo].
// K, lda, ldb in BYTES (= elements), multiples of 128 / 16 / 16.
namespace {
constexpr int NVAR_F8 = 11;
constexpr int VAR_F8_BM[NVAR_F8] = {128, 128, 256, 128, 64, 128, 256, 128, 256, 128, 256};
constexpr int VAR_F8_BN[NVAR_F8] = {128, 128, 128, 256, 128, 64, 64, 128, 128, 256, 256};

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
  }
  return -3;
}
}  // namespace

PDT_API int pdt_gemm_f8_num_variants() { return NVAR_F8; }

PDT_API int pdt_gemm_f8(const void* a, const void* b, void* out, const float* bias, const float* dq_a,
                        const float* dq_b, int M, int N, int K, int lda, int ldb, int ldo, int fmt_a, int act,
                        void* aux, int variant, hipStream_t stream) {
  if (K % 128 != 0 || lda % 16 != 0 || ldb % 16 != 0 || N % 8 != 0 || ldo % 8 != 0) return -1;
  if (lda != K) return -2;  // rows of A are dense (the gather's source row stride is Cs)
  NTParams p;
  p.src = (const u16*)a;
  p.b = (const u16*)b;
  p.out = (u16*)out;
  p.stats = nullptr;
  p.bias = bias;
  p.addend = nullptr;
  p.addend_mask = nullptr;
  p.Hs = 1; p.Ws = 1; p.Cs = K / 2;
  p.Hm = 1; p.Wm = 1;
  p.M = M;
  p.Ncol = N; p.K = K / 2; p.ldb = ldb / 2;
  p.sh = 1; p.sw = 1; p.oh0 = 0; p.ow0 = 0; p.dh = 1; p.dw = 1; p.nth = 1; p.ntw = 1;
  p.Ho = 1; p.Wo = 1; p.osh = 1; p.osw = 1; p.oph = 0; p.opw = 0; p.ldo = ldo;
  p.act = act;
  p.aux = (u16*)aux;
  p.nstat_rows = 0;
  p.nt_store = 0;
  p.ident_out = 1;
  p.dq_a = dq_a;
  p.dq_b = dq_b;
  p.div_Wm = make_fastdiv(1);
  p.div_HWm = make_fastdiv(1);
  p.div_Cs8 = make_fastdiv(K / 16);
  p.div_ntw = make_fastdiv(1);
  const int v = (variant >= 0 && variant < NVAR_F8) ? variant : 1;
  return fmt_a == 1 ? launch_f8<2>(v, p, stream) : launch_f8<1>(v, p, stream);
}
