// Dense GEMM ring for MI355X: C[M][N] (bf16) = alpha * A[M][K] . B[N][K]^T (+ bias[N]),
// A and B row-major with K contiguous (the nn.Linear forward / data-gradient layout).
//
// One 256x256 output tile per 512-thread workgroup (8 waves as 2 along M x 4 along N, a
// 128x64 tile per wave), one workgroup per CU (128 KB of LDS). Operand staging is LDS-DMA
// (global_load_lds_dwordx4, 16 B per lane) into a 2-stage ring of 128-byte K rows: a K-tile
// is 64 bf16 or 128 fp8 elements per row, i.e. one 16x16x32 bf16 MFMA pair or ONE block-scaled
// 16x16x128 fp8 MFMA per 16x16 output block -- the same 256 matrix-core cycles per quadrant
// phase for both element types, so one schedule serves both.
//
// Schedule (the 4-phase ping-pong of the 256^2 template): the two wave groups (wm = 0 / 1)
// run one barrier apart, so on every SIMD one wave is in its 256-cycle MFMA section while its
// partner is in its memory section. A K-tile is four C-quadrant phases (0,0) (0,1) (1,1) (1,0);
// the next K-tile is fetched one quarter per phase into the other stage with counted vmcnt
// (never 0 inside the loop), so DMA stays in flight across every barrier. Quarter q of a stage
// (2 DMA instructions per thread): q0 = A rows of quadrant row 0 (both wave groups), q1 = B
// columns of the first half, q2 = B second half, q3 = A quadrant row 1. RAW: a quarter is
// retired by each wave's own vmcnt in the memory section BEFORE the phase that reads it and
// made visible by the following barrier; WAR: a stage is restaged only after the barrier that
// follows both groups' last fragment reads of that region (their lgkmcnt(0) precedes it).
//
// Tile order: consecutive logical ids on one XCD (blocks b, b+8, ... share an XCD's L2) and
// grouped GM tile rows x all tile columns, so the tiles one XCD has in flight share A and B
// panels in its L2. Epilogue straight from the accumulators: v_permlane16_swap pairs two
// lanes' 4-column quads into one 16-byte store per lane (no LDS round trip).
//
// LDS image: 128-B rows, 16-B chunk c of row r at physical chunk c ^ ((r >> 1) & 7) (the
// swizzle is applied to the DMA SOURCE address: the DMA image itself is lane-linear), which
// makes the ds_read_b128 fragment reads (16 rows x one logical chunk per 16-lane group)
// conflict-free.
//
// Developed in scripts/gemm_lab/gemm_lab.hip (v4: 1.28-1.33 PF/s bf16 at 4096^3).
#include "pdt_common.h"
#include <type_traits>

namespace {

constexpr int RBM = 256, RBN = 256, RKB = 128, RNTH = 512;  // RKB: bytes of K per tile row
constexpr int RA_BYTES = RBM * RKB, RB_BYTES = RBN * RKB, RSTAGE = RA_BYTES + RB_BYTES;

struct RingParams {
  const char* A;      // [M][lda] bytes per row = lda
  const char* B;      // [N][ldb]
  u16* C;             // [M][ldc] bf16
  const float* bias;  // [N] or nullptr
  const float* dq_a;  // device scalars (fp8: dequant factors); nullptr = 1
  const float* dq_b;
  const void* zero;   // 16 zero bytes (DMA source of rows past M)
  int M, N, nk;       // nk = K-tiles (K bytes / 128)
  int lda, ldb, ldc;  // lda / ldb in bytes, ldc in elements
  // fused epilogue (EPI instantiations; conv_nt_kernel.h's staged-epilogue semantics, on the
  // bf16-rounded values): act 0 out = z (+ addend); act 3 out = z * gelu'(addend);
  // act 4 out = gelu(z), aux = gelu'(z); act 5 out = z * addend -- z = bf16(alpha acc + bias)
  int act;
  u16* aux;             // [M][ldc]
  const u16* addend;    // [M][ldc]
  uint8_t* q8;          // [M][ldc] fp8 codes of out (x q8_meta[0]); nullptr = none
  const float* q8_meta;
  float* q8_part;       // [grid]: the workgroup's max |out|
  int q8_fmt, q8_only;  // 0 e4m3 / 1 e5m2; 1: out itself is not stored
  float* colsum;        // [ceil(M / 256)][N]: column sums of out per 256-row tile; nullptr = none
};

__device__ __forceinline__ float ring_gelu_grad(float z) {  // d gelu_tanh(z) / dz
  const float u = 0.7978845608f * (z + 0.044715f * z * z * z);
  const float t = pdt_tanh(u);
  const float du = 0.7978845608f * (1.f + 3.f * 0.044715f * z * z);
  return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * du;
}

__device__ __forceinline__ int rswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ i32x8 rcat8(const u32x4& lo, const u32x4& hi) {
  return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

template <int GM>
__device__ __forceinline__ void ring_tile_of(uint32_t bid, int ntm, int ntn, int& tm, int& tn) {
  const uint32_t nwg = ntm * ntn;
  uint32_t l = bid;
  if (nwg >= 8) {  // bijective XCD remap (q, r split), then GM-row groups
    const uint32_t q = nwg / 8, r = nwg % 8, x = bid % 8, k = bid / 8;
    l = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  }
  const int per = GM * ntn;
  const int g = l / per, in = l % per;
  const int rows = (ntm - g * GM) < GM ? (ntm - g * GM) : GM;
  tm = g * GM + in % rows;
  tn = in / rows;
}

// DT 0: bf16 x bf16; 1: e4m3 A x e4m3 B; 2: e5m2 A x e4m3 B (OCP fp8, unit block scales)
//
// PERS (persistent): one workgroup per CU walks the tiles t = blockIdx.x, + gridDim.x, ... in the
// one-tile launch's order (gridDim.x is a multiple of 8, so a workgroup's tiles keep its XCD).
// Right after a tile's mainloop -- both LDS stages free, before the epilogue -- it issues the
// LDS-DMA of the NEXT tile's first K-tile, so that load's HBM round trip runs under this tile's
// epilogue (VALU, stores) instead of after a new workgroup's dispatch. Per-tile math and the
// output bytes are those of the one-tile launch; the fp8 side output's max |out| is one
// partial per workgroup (q8_part[blockIdx.x], the host rolls gridDim.x partials).
template <int DT, bool BIAS, int GM, bool EPI, bool PERS = false>
__global__ void __launch_bounds__(RNTH, 1) gemm_ring_kernel(RingParams p) {
  constexpr int WM = 2, WN = 4;
  constexpr int MI = RBM / WM / 16;  // 8 row blocks per wave
  constexpr int NI = RBN / WN / 16;  // 4 column blocks per wave
  constexpr int HM = MI / 2, HN = NI / 2;
  constexpr int RS = RNTH / 8;       // 64 rows per DMA round (8 lanes x 16 B per row)
  __shared__ __attribute__((aligned(16))) char smem[2 * RSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntm = (p.M + RBM - 1) / RBM, ntn = p.N / RBN;
  const int ntiles = ntm * ntn;
  float q8all = 0.f;  // (EPI persistent: this workgroup's max |out| over all its tiles)
  // one output tile (a lambda so the one-tile launch compiles to the straight-line kernel)
  auto run_tile = [&](const int tile) __attribute__((always_inline)) {
  // (persistent fused epilogue: the lane-dependent values are re-derived per tile from an
  // opaque copy of the thread id -- hoisted out of the tile loop they stayed live across the
  // mainloop and spilled 120-192 B; the plain persistent walk keeps them hoisted, 245 VGPRs, no
  // scratch, and measured faster so on the long-K shapes: profiles/ring_persistent_ab_round6.txt)
  int tid = (int)threadIdx.x;
  if constexpr (PERS && EPI) asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int tm, tn;
  ring_tile_of<GM>(PERS ? (uint32_t)tile : blockIdx.x, ntm, ntn, tm, tn);
  const int m0 = tm * RBM, n0 = tn * RBN;
  const int ca = tid & 7;
  const int nk = p.nk;
  // the wave's j-th 16-column block: one 32-column pair in each half of the tile, so a K-tile's
  // B operand arrives as two 128-row halves (quarters q1 / q2)
  auto wcol = [&](int j) -> int {
    return j < NI / 2 ? wn * (RBN / 2 / WN) + j * 16 : RBN / 2 + wn * (RBN / 2 / WN) + (j - NI / 2) * 16;
  };
  const char* Ab = p.A + (size_t)m0 * p.lda;
  const char* Bb = p.B + (size_t)n0 * p.ldb;
  const int mrem = p.M - m0;  // rows of A that exist in this tile
  auto glds_a = [&](int kt, int buf, int i) __attribute__((always_inline)) {
    const int r = (tid >> 3) + RS * i;
    const void* g = r < mrem ? (const void*)(Ab + (size_t)r * p.lda + kt * RKB + rswz(r, ca) * 16) : p.zero;
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + buf * RSTAGE +
                                                                                  (8 * wave + RS * i) * RKB),
                                     16, 0, 0);
  };
  auto glds_b = [&](int kt, int buf, int j) __attribute__((always_inline)) {
    const int r = (tid >> 3) + RS * j;
    const char* g = Bb + (size_t)r * p.ldb + kt * RKB + rswz(r, ca) * 16;
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + buf * RSTAGE + RA_BYTES +
                                                                                  (8 * wave + RS * j) * RKB),
                                     16, 0, 0);
  };
  auto issue = [&](int q, int kt, int buf) __attribute__((always_inline)) {
    if (q == 0) { glds_a(kt, buf, 0); glds_a(kt, buf, 2); }
    else if (q == 1) { glds_b(kt, buf, 0); glds_b(kt, buf, 1); }
    else if (q == 2) { glds_b(kt, buf, 2); glds_b(kt, buf, 3); }
    else { glds_a(kt, buf, 1); glds_a(kt, buf, 3); }
  };
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // a lane's two 16-B chunks of a fragment row: logical chunks (lane >> 4) and 4 + (lane >> 4)
  // (bf16: the two 32-deep k-steps; fp8: ONE 32-byte operand -- the same k permutation for A
  // and B, so the dot products are unchanged)
  // (held as one 8-dword vector per fragment: the fp8 MFMA takes it as one contiguous operand)
  i32x8 af[HM], bq[HN];
  auto frag = [&](const char* base, int row) __attribute__((always_inline)) -> i32x8 {
    const u32x4 lo = *reinterpret_cast<const u32x4*>(base + row * RKB + rswz(row, lane >> 4) * 16);
    const u32x4 hi = *reinterpret_cast<const u32x4*>(base + row * RKB + rswz(row, 4 + (lane >> 4)) * 16);
    return rcat8(lo, hi);
  };
  auto read_a = [&](const char* sa, int r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < HM; ++i) af[i] = frag(sa, wm * (RBM / WM) + (r * HM + i) * 16 + (lane & 15));
  };
  auto read_b = [&](const char* sb, int c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < HN; ++j) bq[j] = frag(sb, wcol(c * HN + j) + (lane & 15));
  };
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  auto half = [](const i32x8& v, int h) __attribute__((always_inline)) -> bf16x8 {
    const i32x4 q = h ? __builtin_shufflevector(v, v, 4, 5, 6, 7) : __builtin_shufflevector(v, v, 0, 1, 2, 3);
    return __builtin_bit_cast(bf16x8, q);
  };
  // sched_barrier(0) pins the program order at the section boundaries: MFMAs have no memory
  // side effects, so without it the scheduler moves them across s_barrier / s_setprio and
  // merges phases (which also raised the fp8 instantiation past 256 VGPRs into scratch)
  // The empty asm statements with the phase's accumulators as in/out operands fence the MFMAs
  // into their section at the IR level too (hipcc otherwise sinks the block-scaled fp8 MFMAs
  // of one phase into the next, keeping two phases' fragments live at once).
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
      for (int j = 0; j < HN; ++j) {
        f32x4& d = acc[r * HM + i][c * HN + j];
        if constexpr (DT == 0) {
          // swapped operands: a lane's 4 accumulators are 4 consecutive output columns of one row
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(half(bq[j], kk), half(af[i], kk), d, 0, 0, 0);
        } else {
          d = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bq[j], af[i], d, 0, DT == 2 ? 1 : 0, 0, 127, 0, 127);
        }
      }
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
    if (!PERS || tile == (int)blockIdx.x) {
#pragma unroll
      for (int q = 0; q < 4; ++q) issue(q, 0, 0);
    }
    // q0 q1 of K-tile 0 (a persistent walk issued them before the previous tile's epilogue:
    // loads retire in order, so <= 4 outstanding -- stores included -- proves q0 and q1 landed)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  bar();
  if (wm == 1) bar();  // the stagger: group 1 runs one barrier behind group 0
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1, nxt = cur ^ 1;
    const bool more = kt + 1 < nk;
    const char* sa = smem + cur * RSTAGE;
    const char* sb = sa + RA_BYTES;
    // M1: fragments of (0,0); retire q2 of this K-tile (read in M2); q0 of the next
    read_a(sa, 0);
    read_b(sb, 0);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    if (more) issue(0, kt + 1, nxt);
    mma_phase(0, 0);
    // M2: fragments of (0,1); retire q3 (read in M3); q1 of the next
    read_b(sb, 1);
    if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (more) issue(1, kt + 1, nxt);
    mma_phase(0, 1);
    // M3: fragments of (1,1); q2 of the next
    read_a(sa, 1);
    if (more) issue(2, kt + 1, nxt);
    mma_phase(1, 1);
    // M4: fragments of (1,0); retire q0 q1 of the next K-tile (read in its M1); q3 of the next
    read_b(sb, 0);
    if (more) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      issue(3, kt + 1, nxt);
    }
    mma_phase(1, 0);
  }
  if (wm == 0) bar();  // close the stagger: equal barrier counts on every wave

  // ---- epilogue: alpha, bias, bf16, 16-B stores
  const float alpha = (p.dq_a ? p.dq_a[0] : 1.f) * (p.dq_b ? p.dq_b[0] : 1.f);
  const int lrow = lane & 15, lcol = (lane >> 4) * 4;
  float bv[NI][4];
#pragma unroll
  for (int j = 0; j < NI; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = BIAS ? p.bias[n0 + wcol(j) + lcol + e] : 0.f;
  if constexpr (PERS) {
    // the next tile's K-tile 0 into stage 0 (every wave is past its last fragment read: the
    // closing barrier above), in flight under this epilogue
    const int nt = tile + (int)gridDim.x;
    if (nt < ntiles && nk > 0) {
      int tm2, tn2;
      ring_tile_of<GM>((uint32_t)nt, ntm, ntn, tm2, tn2);
      const char* An = p.A + (size_t)(tm2 * RBM) * p.lda;
      const char* Bn = p.B + (size_t)(tn2 * RBN) * p.ldb;
      const int mremn = p.M - tm2 * RBM;
      auto na = [&](int i) __attribute__((always_inline)) {
        const int r = (tid >> 3) + RS * i;
        const void* g = r < mremn ? (const void*)(An + (size_t)r * p.lda + rswz(r, ca) * 16) : p.zero;
        __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + (8 * wave + RS * i) * RKB),
                                         16, 0, 0);
      };
      auto nb = [&](int j) __attribute__((always_inline)) {
        const int r = (tid >> 3) + RS * j;
        const char* g = Bn + (size_t)r * p.ldb + rswz(r, ca) * 16;
        __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + RA_BYTES +
                                                                                      (8 * wave + RS * j) * RKB),
                                         16, 0, 0);
      };
      // quarter order q0 (A 0, 2), q1 (B 0, 1), q2 (B 2, 3), q3 (A 1, 3): the next tile's
      // vmcnt(4) then covers q0 q1 exactly as the one-tile prologue's
      na(0); na(2); nb(0); nb(1); nb(2); nb(3); na(1); na(3);
    }
  }
  const bool odd = (lane >> 4) & 1;
  // EPI: this lane's 8 columns of each column pair are fixed (colsum partials), its max |out|
  float csum[EPI ? 2 : 1][EPI ? 8 : 1];
  float q8max = 0.f;
  const float q8s = (EPI && p.q8 != nullptr) ? p.q8_meta[0] : 0.f;
  if constexpr (EPI) {
#pragma unroll
    for (int jp = 0; jp < 2; ++jp)
#pragma unroll
      for (int e = 0; e < 8; ++e) csum[jp][e] = 0.f;
  }
  // EPI addend: every chunk of the tile is loaded (from clamped rows: no branch) before the first
  // store. Loaded next to its use, each row block's wait was a vmcnt(0): with loads and stores both
  // in flight hipcc treats vmcnt as out of order and waits for zero, which drained the previous
  // row block's stores as well (16 serialised round trips per tile; a one-ahead prefetch hit the
  // same drain). The MFMA fragments are dead here, so the 64 registers fit.
  const bool has_add = EPI && p.addend != nullptr;
  // The EPI loop nest is compiled per configuration (compile-time act / fp8 code format): the
  // ViT MLP runs two -- fc1 forward (GELU + GELU', e4m3 codes, no addend) and fc2's data gradient
  // (x gelu' addend, e5m2 codes) -- and with run-time fields every element group branched on
  // act, q8 and the format (~450 branches and ~320 exec moves per tile); anything else takes the
  // run-time path.
  auto run = [&](auto act_c, auto q8_c, auto cs_c) __attribute__((always_inline)) {
    constexpr int CA = decltype(act_c)::value;  // -1: p.act at run time
    constexpr int CQ = decltype(q8_c)::value;   // -1: p.q8 / p.q8_fmt at run time; 1 e4m3, 2 e5m2
    constexpr int CC = decltype(cs_c)::value;   // column sums: -1 run time (summed, used if p.colsum), 0 no, 1 yes
    const int act = CA >= 0 ? CA : p.act;
    const bool q8on = CQ > 0 ? true : (EPI && p.q8 != nullptr);
    const int fmt = CQ > 0 ? CQ - 1 : p.q8_fmt;
    const bool hadd = CA == 4 ? false : (CA == 5 ? true : has_add);
    const bool cstore = !(q8on && p.q8_only);
    (void)act; (void)fmt; (void)hadd; (void)cstore;
    // EPI addend: every chunk of the tile is loaded (from clamped rows: no branch) before the first
    // store. Loaded next to its use, each row block's wait was a vmcnt(0): with loads and stores
    // both in flight hipcc treats vmcnt as out of order and waits for zero, which drained the
    // previous row block's stores as well (16 serialised round trips per tile; a one-ahead
    // prefetch hit the same drain). The MFMA fragments are dead here, so the 64 registers fit.
    u32x4 adv[EPI ? MI : 1][EPI ? 2 : 1];
    if constexpr (EPI) {
      if (hadd) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int mc = min(m0 + wm * (RBM / WM) + i * 16 + lrow, p.M - 1);
#pragma unroll
          for (int jp = 0; jp < 2; ++jp) {
            const int col = n0 + wcol(odd ? 2 * jp + 1 : 2 * jp) + ((lane >> 5) * 8);
            adv[i][jp] = *reinterpret_cast<const u32x4*>(p.addend + (size_t)mc * p.ldc + col);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * (RBM / WM) + i * 16 + lrow;
#pragma unroll
      for (int j = 0; j < NI; j += 2) {
        const f32x4 x = acc[i][j], y = acc[i][j + 1];
        const uint32_t a0 = pack2bf(x[0] * alpha + bv[j][0], x[1] * alpha + bv[j][1]);
        const uint32_t a1 = pack2bf(x[2] * alpha + bv[j][2], x[3] * alpha + bv[j][3]);
        const uint32_t b0 = pack2bf(y[0] * alpha + bv[j + 1][0], y[1] * alpha + bv[j + 1][1]);
        const uint32_t b1 = pack2bf(y[2] * alpha + bv[j + 1][2], y[3] * alpha + bv[j + 1][3]);
        // lanes l (group g = l >> 4 even) and l + 16 (g odd) hold the low / high 4 columns of
        // one 8-column half of blocks j and j + 1: one swap per dword gives the even lane block
        // j's 8 columns and the odd lane block j + 1's
        const auto r0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
        u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
        const int col = n0 + wcol(odd ? j + 1 : j) + ((lane >> 5) * 8);
        if constexpr (!EPI) {
          if (m < p.M) *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.ldc + col) = v;
        } else {
          if (m < p.M) {
            const size_t e0 = (size_t)m * p.ldc + col;
            if (hadd) {
              const u32x4 ad = adv[EPI ? i : 0][EPI ? (j >> 1) : 0];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                if (act == 3)
                  v[e] = pack2bf(lo_bf(v[e]) * ring_gelu_grad(lo_bf(ad[e])), hi_bf(v[e]) * ring_gelu_grad(hi_bf(ad[e])));
                else if (act == 5)
                  v[e] = pack2bf(lo_bf(v[e]) * lo_bf(ad[e]), hi_bf(v[e]) * hi_bf(ad[e]));
                else
                  v[e] = pack2bf(lo_bf(v[e]) + lo_bf(ad[e]), hi_bf(v[e]) + hi_bf(ad[e]));
              }
            }
            if (act == 4) {
              u32x4 gd;
#pragma unroll
              for (int e = 0; e < 4; ++e) {  // (the pair on the packed VALU)
                pdt_f32x2 g, d;
                pdt_gelu_dual2(pdt_f32x2{lo_bf(v[e]), hi_bf(v[e])}, g, d);
                v[e] = pack2bf(g.x, g.y);
                gd[e] = pack2bf(d.x, d.y);
              }
              *reinterpret_cast<u32x4*>(p.aux + e0) = gd;
            }
            float f[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              f[2 * e] = lo_bf(v[e]);
              f[2 * e + 1] = hi_bf(v[e]);
            }
            if constexpr (CC != 0) {
#pragma unroll
              for (int e = 0; e < 8; ++e) csum[j >> 1][e] += f[e];
            }
            if (q8on) {
#pragma unroll
              for (int e = 0; e < 8; ++e) q8max = fmaxf(q8max, fabsf(f[e]));
              uint2 c8;
              if (fmt == 0) {
                c8.x = pdt_cvt4_f8<0>(f[0] * q8s, f[1] * q8s, f[2] * q8s, f[3] * q8s);
                c8.y = pdt_cvt4_f8<0>(f[4] * q8s, f[5] * q8s, f[6] * q8s, f[7] * q8s);
              } else {
                c8.x = pdt_cvt4_f8<1>(f[0] * q8s, f[1] * q8s, f[2] * q8s, f[3] * q8s);
                c8.y = pdt_cvt4_f8<1>(f[4] * q8s, f[5] * q8s, f[6] * q8s, f[7] * q8s);
              }
              *reinterpret_cast<uint2*>(p.q8 + e0) = c8;
            }
            if (cstore) *reinterpret_cast<u32x4*>(p.C + e0) = v;
          }
        }
      }
    }
  };
  if constexpr (EPI) {
    // fc1 forward (no column sums) and fc2's data gradient (with them: fc1's bias gradient)
    if (p.act == 4 && p.q8 != nullptr && p.q8_fmt == 0 && !has_add && p.colsum == nullptr)
      run(std::integral_constant<int, 4>{}, std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
    else if (p.act == 5 && p.q8 != nullptr && p.q8_fmt == 1 && has_add && p.colsum != nullptr)
      run(std::integral_constant<int, 5>{}, std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
    else
      run(std::integral_constant<int, -1>{}, std::integral_constant<int, -1>{}, std::integral_constant<int, -1>{});
  } else {
    run(std::integral_constant<int, -1>{}, std::integral_constant<int, -1>{}, std::integral_constant<int, -1>{});
  }
  if constexpr (EPI) {
    // every LDS fragment read finished before the loop's last barrier: smem is free here
    // (a persistent walk prefetches into stage 0: the reductions use stage 1)
    float* red = reinterpret_cast<float*>(smem + (PERS ? RSTAGE : 0));
    if (p.colsum != nullptr) {
      // lanes of one 16-lane row hold 16 rows of the same 8 columns: DPP row sums, then the
      // two wave rows (wm) with the same columns through LDS: [wm][wn][jp][g][8]
#pragma unroll
      for (int jp = 0; jp < 2; ++jp)
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[jp][e] = row16_sum(csum[jp][e]);
      if (lrow == 0) {
#pragma unroll
        for (int jp = 0; jp < 2; ++jp)
#pragma unroll
          for (int e = 0; e < 8; ++e) red[((wm * WN + wn) * 2 + jp) * 32 + (lane >> 4) * 8 + e] = csum[jp][e];
      }
    }
    if (p.q8 != nullptr) {
      if constexpr (PERS) {
        q8all = fmaxf(q8all, q8max);
      } else {
        q8max = warp_max(q8max);
        if (lane == 0) red[2 * WN * 2 * 32 + wave] = q8max;
      }
    }
    __syncthreads();
    if (p.colsum != nullptr && wm == 0 && lrow == 0) {
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int base = ((wn)*2 + jp) * 32 + (lane >> 4) * 8;
        const int cl = wcol(2 * jp + (odd ? 1 : 0)) + ((lane >> 5) * 8);
        f32x4 s0, s1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s0[e] = red[base + e] + red[WN * 2 * 32 + base + e];
          s1[e] = red[base + 4 + e] + red[WN * 2 * 32 + base + 4 + e];
        }
        float* dst = p.colsum + (size_t)tm * p.N + n0 + cl;
        *reinterpret_cast<f32x4*>(dst) = s0;
        *reinterpret_cast<f32x4*>(dst + 4) = s1;
      }
    }
    if (p.q8 != nullptr && tid == 0 && !PERS) {
      float mx = 0.f;
#pragma unroll
      for (int w = 0; w < RNTH / 64; ++w) mx = fmaxf(mx, red[2 * WN * 2 * 32 + w]);
      p.q8_part[blockIdx.x] = mx;
    }
  }
  };
  if constexpr (PERS) {
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) run_tile(tile);
  } else {
    run_tile(blockIdx.x);
  }
  if constexpr (EPI && PERS) {  // the workgroup's max |out| over its tiles -> q8_part[blockIdx.x]
    if (p.q8 != nullptr) {
      __syncthreads();  // (the last tile's reductions read stage 1)
      float* red = reinterpret_cast<float*>(smem + RSTAGE);
      const float w = warp_max(q8all);
      if (lane == 0) red[wave] = w;
      __syncthreads();
      if (tid == 0) {
        float mx = 0.f;
#pragma unroll
        for (int i = 0; i < RNTH / 64; ++i) mx = fmaxf(mx, red[i]);
        p.q8_part[blockIdx.x] = mx;
      }
    }
  }
}

static __device__ __attribute__((aligned(64))) u32x4 ring_zero_chunk[4];

// workgroups of a launch: one per tile, or (persistent sub-variants 2 / 3) one per CU -- a
// multiple of 8 (whole XCD rounds) -- when there are more tiles than that
int ring_grid(int M, int N, int sub) {
  const int ntiles = ((M + RBM - 1) / RBM) * (N / RBN);
  if (sub < 2) return ntiles;
  const int g = pdt_num_cus() / 8 * 8;
  return ntiles < g ? ntiles : g;
}

template <int DT, bool BIAS, int GM, bool EPI, bool PERS>
int ring_launch(const RingParams& p, hipStream_t st) {
  hipLaunchKernelGGL((gemm_ring_kernel<DT, BIAS, GM, EPI, PERS>), dim3(ring_grid(p.M, p.N, PERS ? 2 : 0)),
                     dim3(RNTH), 0, st, p);
  PDT_RETURN_LAUNCH();
}

// sub: 0 / 1 tile groupings GM 4 / 8, one tile per workgroup; 2 / 3 the same, persistent
template <int DT>
int ring_dispatch(int sub, bool bias, bool epi, const RingParams& p, hipStream_t st) {
  if constexpr (DT != 0) {
    if (epi) {
      if (sub == 0) return bias ? ring_launch<DT, true, 4, true, false>(p, st) : ring_launch<DT, false, 4, true, false>(p, st);
      if (sub == 2) return bias ? ring_launch<DT, true, 4, true, true>(p, st) : ring_launch<DT, false, 4, true, true>(p, st);
      return -5;  // (the fused epilogue: grouping GM 4 only)
    }
  } else if (epi) {
    return -5;  // (the fused epilogue is built for the fp8 GEMMs only)
  }
  switch (sub) {
    case 0: return bias ? ring_launch<DT, true, 4, false, false>(p, st) : ring_launch<DT, false, 4, false, false>(p, st);
    case 1: return bias ? ring_launch<DT, true, 8, false, false>(p, st) : ring_launch<DT, false, 8, false, false>(p, st);
    case 2: return bias ? ring_launch<DT, true, 4, false, true>(p, st) : ring_launch<DT, false, 4, false, true>(p, st);
    default: return bias ? ring_launch<DT, true, 8, false, true>(p, st) : ring_launch<DT, false, 8, false, true>(p, st);
  }
}

int ring_run(const void* a, const void* b, void* c, const float* bias, const float* dq_a, const float* dq_b, int M,
             int N, int K, int lda, int ldb, int ldc, int dt, int sub, int act, void* aux, const void* addend,
             void* q8, const float* q8_meta, float* q8_part, int q8_fmt, int q8_only, float* colsum,
             hipStream_t st) {
  static const void* zcache[PDT_MAX_DEV] = {};
  const int esz = dt == 0 ? 2 : 1;
  const long kbytes = (long)K * esz;
  if (M <= 0 || N <= 0 || K <= 0) return -1;
  if (N % RBN != 0 || kbytes % RKB != 0 || (lda * esz) % 16 != 0 || (ldb * esz) % 16 != 0 || ldc % 8 != 0 ||
      lda < K || ldb < K || ldc < N)
    return -5;
  if ((long)M * lda * esz >= (1L << 40)) return -1;
  // 16-B LDS-DMA / global loads and 16-B / 8-B epilogue stores go through these pointers: a
  // view with an offset is "not applicable" (-5) here, not a fault
  if ((((uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)addend | (uintptr_t)aux) & 15) != 0 ||
      ((uintptr_t)q8 & 7) != 0)
    return -5;
  if (!(act == 0 || act == 3 || act == 4 || act == 5)) return -5;
  if ((act == 3 || act == 5) && addend == nullptr) return -4;
  if (act == 4 && (aux == nullptr || addend != nullptr)) return -4;
  if (q8 != nullptr && (q8_meta == nullptr || q8_part == nullptr || ldc != N)) return -4;
  RingParams p;
  p.A = (const char*)a;
  p.B = (const char*)b;
  p.C = (u16*)c;
  p.bias = bias;
  p.dq_a = dq_a;
  p.dq_b = dq_b;
  p.zero = pdt_symbol_addr(HIP_SYMBOL(ring_zero_chunk), zcache);
  if (p.zero == nullptr) return PDT_ERR_SYMBOL;
  p.M = M;
  p.N = N;
  p.nk = (int)(kbytes / RKB);
  p.lda = lda * esz;
  p.ldb = ldb * esz;
  p.ldc = ldc;
  p.act = act;
  p.aux = (u16*)aux;
  p.addend = (const u16*)addend;
  p.q8 = (uint8_t*)q8;
  p.q8_meta = q8_meta;
  p.q8_part = q8_part;
  p.q8_fmt = q8_fmt;
  p.q8_only = q8_only;
  p.colsum = colsum;
  const bool epi = act != 0 || aux != nullptr || addend != nullptr || q8 != nullptr || colsum != nullptr;
  if (sub < 0 || sub > 3) sub = 0;
  switch (dt) {
    case 0: return ring_dispatch<0>(sub, bias != nullptr, epi, p, st);
    case 1: return ring_dispatch<1>(sub, bias != nullptr, epi, p, st);
    case 2: return ring_dispatch<2>(sub, bias != nullptr, epi, p, st);
  }
  return -1;
}

}  // namespace

// Number of ring sub-variants (tile-order groupings GM = 4, 8; one-tile / persistent).
PDT_API int pdt_gemm_ring_num_variants() { return 4; }

// Workgroups a launch of sub-variant `sub` runs (the fp8 side output's partial-max count).
PDT_API int pdt_gemm_ring_grid(int M, int N, int sub) { return ring_grid(M, N, sub); }

// Rows of the ring's M tile (the colsum partial rows).
PDT_API int pdt_gemm_ring_bm() { return RBM; }

// C[M][N] = dq_a*dq_b * A[M][K] . B[N][K]^T (+ bias), bf16 out. dt: 0 bf16 operands (K in
// elements, a multiple of 64), 1 / 2 e4m3 / e5m2 A with e4m3 B (K a multiple of 128).
// Returns -5 (not applicable) for N not a multiple of 256 or unaligned strides.
PDT_API int pdt_gemm_ring(const void* a, const void* b, void* c, const float* bias, const float* dq_a,
                          const float* dq_b, int M, int N, int K, int lda, int ldb, int ldc, int dt, int sub,
                          hipStream_t st) {
  return ring_run(a, b, c, bias, dq_a, dq_b, M, N, K, lda, ldb, ldc, dt, sub, 0, nullptr, nullptr, nullptr, nullptr,
                  nullptr, 0, 0, nullptr, st);
}

// The same with the fused fp8 epilogue (RingParams: act / aux / addend, the fp8 codes of the
// output with the next GEMM's delayed scale and the workgroup amax partials, per-tile column
// sums); dt 1 / 2 only (the fused instantiation is grouping GM = 4).
PDT_API int pdt_gemm_ring_epi(const void* a, const void* b, void* c, const float* bias, const float* dq_a,
                              const float* dq_b, int M, int N, int K, int lda, int ldb, int ldc, int dt, int act,
                              void* aux, const void* addend, void* q8, const float* q8_meta, float* q8_part,
                              int q8_fmt, int q8_only, float* colsum, hipStream_t st) {
  if (dt == 0) return -5;
  return ring_run(a, b, c, bias, dq_a, dq_b, M, N, K, lda, ldb, ldc, dt, 0, act, aux, addend, q8, q8_meta, q8_part,
                  q8_fmt, q8_only, colsum, st);
}

// pdt_gemm_ring_epi on the persistent walk (sub-variant 2): q8_part receives
// pdt_gemm_ring_grid(M, N, 2) partial maxima
PDT_API int pdt_gemm_ring_epi_pers(const void* a, const void* b, void* c, const float* bias, const float* dq_a,
                                   const float* dq_b, int M, int N, int K, int lda, int ldb, int ldc, int dt, int act,
                                   void* aux, const void* addend, void* q8, const float* q8_meta, float* q8_part,
                                   int q8_fmt, int q8_only, float* colsum, hipStream_t st) {
  if (dt == 0) return -5;
  return ring_run(a, b, c, bias, dq_a, dq_b, M, N, K, lda, ldb, ldc, dt, 2, act, aux, addend, q8, q8_meta, q8_part,
                  q8_fmt, q8_only, colsum, st);
}
