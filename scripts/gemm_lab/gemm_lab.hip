// GEMM mainloop lab: a standalone bf16 C[M][N] = A[M][K] . B[N][K]^T benchmark (no torch),
// used to develop the 256x256 8-wave mainloop before it goes into csrc/conv_nt_kernel.h.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/gemm_lab/gemm_lab.hip -o build/gemm_lab
//   build/gemm_lab M N K [iters] [variant ...]
//
// Every variant is checked against an fp32 dot product on sampled output elements, then
// timed over `iters` back-to-back launches on uniform random [-1, 1) bf16 operands.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

typedef unsigned short u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  const __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (uint32_t)__builtin_bit_cast(u16, a) | ((uint32_t)__builtin_bit_cast(u16, b) << 16);
}

struct GP {
  const u16* A;
  const u16* B;
  u16* C;
  int M, N, K;
};

constexpr int BM = 256, BN = 256, BK = 64, NTH = 512;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;

// 16-B chunk swizzle of a 128-B LDS row: conflict-free ds_read_b128 for the 16x16x32 operand
// reads (rows lane&15, chunk 4kk + lane>>4), applied to the DMA SOURCE (the DMA image is
// lane-linear) and to the read address.
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Tile order: XCD-aware (consecutive logical ids on one XCD) and grouped GM row-tiles x all
// column tiles, so the tiles one XCD runs at a time share A and B panels in its L2.
template <int GM>
__device__ __forceinline__ void tile_of(uint32_t bid, int ntm, int ntn, int& tm, int& tn) {
  const uint32_t nwg = ntm * ntn;
  uint32_t l = bid;
  if (nwg >= 8) {
    const uint32_t q = nwg / 8, r = nwg % 8, x = bid % 8, k = bid / 8;
    l = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
  }
  if (GM <= 1) {
    tm = l / ntn;
    tn = l % ntn;
    return;
  }
  const int per = GM * ntn;
  const int g = l / per, in = l % per;
  const int rows = (ntm - g * GM) < GM ? (ntm - g * GM) : GM;
  tm = g * GM + in % rows;
  tn = in / rows;
}

// V0: the 4-phase ping-pong ring (two wave groups one barrier apart; each K-tile = four
// C-quadrant phases; the next K-tile's quarters are issued one per phase with counted vmcnt).
// GM: tile grouping; PRIO: s_setprio around the MFMA bursts.
template <int GM, bool PRIO, int EPI = 0, bool SPRIO = false, bool PERSIST = false>
__global__ void __launch_bounds__(NTH, 1) gemm_v0(GP p) {
  constexpr int WM = 2, WN = 4;
  constexpr int MI = BM / WM / 16;  // 8
  constexpr int NI = BN / WN / 16;  // 4
  constexpr int HM = MI / 2, HN = NI / 2;
  constexpr int RS = NTH / 8;  // 64 rows per DMA round
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntm = p.M / BM, ntn = p.N / BN;
  const int ntiles = ntm * ntn;
  for (int tile = blockIdx.x; tile < ntiles; tile += PERSIST ? gridDim.x : ntiles) {
  if (PERSIST && tile != (int)blockIdx.x) __syncthreads();  // LDS of the previous tile fully read
  int tm, tn;
  tile_of<GM>(tile, ntm, ntn, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int ca = tid & 7;
  const int nk = p.K / BK;
  // wave's j-th 16-column block: one 32-column block in each half of the tile
  auto wcol = [&](int j) -> int {
    return j < NI / 2 ? wn * (BN / 2 / WN) + j * 16 : BN / 2 + wn * (BN / 2 / WN) + (j - NI / 2) * 16;
  };
  const u16* Ab = p.A + (size_t)m0 * p.K;
  const u16* Bb = p.B + (size_t)n0 * p.K;
  auto glds_a = [&](int kt, int buf, int i) __attribute__((always_inline)) {
    const int r = (tid >> 3) + RS * i;
    const u16* g = Ab + (size_t)r * p.K + kt * BK + swz(r, ca) * 8;
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + buf * STAGE +
                                                                                  (8 * wave + RS * i) * 128),
                                     16, 0, 0);
  };
  auto glds_b = [&](int kt, int buf, int j) __attribute__((always_inline)) {
    const int r = (tid >> 3) + RS * j;
    const u16* g = Bb + (size_t)r * p.K + kt * BK + swz(r, ca) * 8;
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + buf * STAGE + A_BYTES +
                                                                                  (8 * wave + RS * j) * 128),
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
  bf16x8 af[HM][2], bq[HN][2];
  auto read_a = [&](const char* sa, int r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < HM; ++i) {
      const int row = wm * (BM / WM) + (r * HM + i) * 16 + (lane & 15);
      af[i][0] = *reinterpret_cast<const bf16x8*>(sa + row * 128 + swz(row, lane >> 4) * 16);
      af[i][1] = *reinterpret_cast<const bf16x8*>(sa + row * 128 + swz(row, 4 + (lane >> 4)) * 16);
    }
  };
  auto read_b = [&](const char* sb, int c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < HN; ++j) {
      const int row = wcol(c * HN + j) + (lane & 15);
      bq[j][0] = *reinterpret_cast<const bf16x8*>(sb + row * 128 + swz(row, lane >> 4) * 16);
      bq[j][1] = *reinterpret_cast<const bf16x8*>(sb + row * 128 + swz(row, 4 + (lane >> 4)) * 16);
    }
  };
  auto mma = [&](int r, int c) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < HM; ++i)
#pragma unroll
      for (int j = 0; j < HN; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          acc[r * HM + i][c * HN + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][kk], af[i][kk], acc[r * HM + i][c * HN + j], 0, 0, 0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  auto bar = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto mma_phase = [&](int r, int c) __attribute__((always_inline)) {
    bar();
    mma(r, c);
    bar();
  };
#pragma unroll
  for (int q = 0; q < 4; ++q) issue(q, 0, 0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  bar();
  if (wm == 1) bar();
  if (SPRIO && __builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1, nxt = cur ^ 1;
    const bool more = kt + 1 < nk;
    const char* sa = smem + cur * STAGE;
    const char* sb = sa + A_BYTES;
    read_a(sa, 0);
    read_b(sb, 0);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    if (more) issue(0, kt + 1, nxt);
    mma_phase(0, 0);
    read_b(sb, 1);
    if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (more) issue(1, kt + 1, nxt);
    mma_phase(0, 1);
    read_a(sa, 1);
    if (more) issue(2, kt + 1, nxt);
    mma_phase(1, 1);
    read_b(sb, 0);
    if (more) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      issue(3, kt + 1, nxt);
    }
    mma_phase(1, 0);
  }
  if (wm == 0) bar();
  const int lrow = lane & 15, lcol = (lane >> 4) * 4;
  if constexpr (EPI == 0) {
    // direct epilogue: each lane stores its 4 consecutive channels (8 B)
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * (BM / WM) + i * 16 + lrow;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = n0 + wcol(j) + lcol;
        u32x2 w = {pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3])};
        *reinterpret_cast<u32x2*>(p.C + (size_t)m * p.N + col) = w;
      }
    }
  } else {
    // 16-B stores: lanes l and l ^ 16 hold columns 0-3 / 4-7 of the same row in the same
    // 16-column block; one v_permlane16_swap per dword pairs block j's upper quad with block
    // j+1's lower quad, so lane l (l & 16 == 0) gets cols 0-7 of block j and lane l|16 cols 0-7
    // of block j+1 ... per pair of blocks (j, j+1) with the same row.
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * (BM / WM) + i * 16 + lrow;
#pragma unroll
      for (int j = 0; j < NI; j += 2) {
        uint32_t a0 = pack2bf(acc[i][j][0], acc[i][j][1]), a1 = pack2bf(acc[i][j][2], acc[i][j][3]);
        uint32_t b0 = pack2bf(acc[i][j + 1][0], acc[i][j + 1][1]), b1 = pack2bf(acc[i][j + 1][2], acc[i][j + 1][3]);
        // lane groups g = lane >> 4: g even holds cols 8k..8k+3 (k = g/2), g odd cols 8k+4..8k+7.
        // swap between lane l (g even) and l+16 (g odd): even lanes take the odd lanes' block-j
        // quad, odd lanes take the even lanes' block-(j+1) quad.
        const auto r0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
        const bool odd = (lane >> 4) & 1;
        // after the swap: even lanes: r[0] = own a (block j, cols lo) , r[1] = partner's a (block j, cols hi)
        //                 odd lanes:  r[0] = partner's b (block j+1, cols lo), r[1] = own b (block j+1, cols hi)
        u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
        const int blk = odd ? j + 1 : j;
        const int col = n0 + wcol(blk) + ((lane >> 5) * 8);
        *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.N + col) = v;
      }
    }
  }
  }  // tile loop
}

// V2: 2-phase ping-pong. Each K-tile = two row-half phases of the 128x64 wave tile (32 MFMAs,
// 512 MFMA cycles each), so the partner group's memory section has twice the MFMA time to hide
// in. Regions of a stage: QA0 = the A rows of half 0 of both wave groups (i = 0, 2), QA1 = half 1
// (i = 1, 3), QB = all of B. Sections per group: M1 (read QA0 + QB fragments), X1, M2 (read QA1
// fragments), X2; group 1 runs one barrier behind group 0. With G0's section s in barrier slot
// [s-1, s] and G1's in [s, s+1], tile t's QA0/QB are free after barrier 4t+3 and QA1 after 4t+5:
// QA0/QB(t+2) are issued in M1(t+1), QA1(t+2) in M2(t+1); each section first retires (vmcnt 0)
// what the other group reads next (QA1(t+1) in M1(t+1), QA0/QB(t+2) in M2(t+1)).
template <int GM>
__global__ void __launch_bounds__(NTH, 1) gemm_v2(GP p) {
  constexpr int WM = 2, WN = 4;
  constexpr int MI = BM / WM / 16;  // 8
  constexpr int NI = BN / WN / 16;  // 4
  constexpr int HM = MI / 2;        // 4 row blocks per phase
  constexpr int RS = NTH / 8;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntm = p.M / BM, ntn = p.N / BN;
  int tm, tn;
  tile_of<GM>(blockIdx.x, ntm, ntn, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int ca = tid & 7;
  const int nk = p.K / BK;
  const u16* Ab = p.A + (size_t)m0 * p.K;
  const u16* Bb = p.B + (size_t)n0 * p.K;
  auto glds_a = [&](int kt, int buf, int i) __attribute__((always_inline)) {
    const int r = (tid >> 3) + RS * i;
    const u16* g = Ab + (size_t)r * p.K + kt * BK + swz(r, ca) * 8;
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + buf * STAGE +
                                                                                  (8 * wave + RS * i) * 128),
                                     16, 0, 0);
  };
  auto glds_b = [&](int kt, int buf, int j) __attribute__((always_inline)) {
    const int r = (tid >> 3) + RS * j;
    const u16* g = Bb + (size_t)r * p.K + kt * BK + swz(r, ca) * 8;
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + buf * STAGE + A_BYTES +
                                                                                  (8 * wave + RS * j) * 128),
                                     16, 0, 0);
  };
  auto issue_a0b = [&](int kt, int buf) __attribute__((always_inline)) {
    glds_a(kt, buf, 0); glds_a(kt, buf, 2);
    glds_b(kt, buf, 0); glds_b(kt, buf, 1); glds_b(kt, buf, 2); glds_b(kt, buf, 3);
  };
  auto issue_a1 = [&](int kt, int buf) __attribute__((always_inline)) {
    glds_a(kt, buf, 1); glds_a(kt, buf, 3);
  };
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[HM][2], bq[NI][2];
  // half h of the wave's rows: A rows wm*64 + h*128 + 16i (so half h lies in region QAh)
  auto read_a = [&](const char* sa, int h) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < HM; ++i) {
      const int row = h * 64 + wm * 128 + i * 16 + (lane & 15);
      af[i][0] = *reinterpret_cast<const bf16x8*>(sa + row * 128 + swz(row, lane >> 4) * 16);
      af[i][1] = *reinterpret_cast<const bf16x8*>(sa + row * 128 + swz(row, 4 + (lane >> 4)) * 16);
    }
  };
  auto read_b = [&](const char* sb) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wn * 64 + j * 16 + (lane & 15);
      bq[j][0] = *reinterpret_cast<const bf16x8*>(sb + row * 128 + swz(row, lane >> 4) * 16);
      bq[j][1] = *reinterpret_cast<const bf16x8*>(sb + row * 128 + swz(row, 4 + (lane >> 4)) * 16);
    }
  };
  auto mma = [&](int h) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < HM; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          acc[h * HM + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][kk], af[i][kk], acc[h * HM + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // prologue: tile 0 landed and visible
  issue_a0b(0, 0);
  issue_a1(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  if (wm == 1) bar();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* sa = smem + cur * STAGE;
    const char* sb = sa + A_BYTES;
    const bool more = kt + 1 < nk;
    // M1: fragments of half 0; retire QA1(kt) (read in M2); QA0/QB(kt+1) into the other stage
    read_a(sa, 0);
    read_b(sb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (more) issue_a0b(kt + 1, cur ^ 1);
    bar();
    mma(0);
    bar();
    // M2: fragments of half 1; retire QA0/QB(kt+1) (read in the next M1); QA1(kt+1)
    read_a(sa, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (more) issue_a1(kt + 1, cur ^ 1);
    bar();
    mma(1);
    bar();
  }
  if (wm == 0) bar();
  const int lrow = lane & 15, lcol = (lane >> 4) * 4;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < HM; ++i) {
      const int m = m0 + h * 64 + wm * 128 + i * 16 + lrow;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = n0 + wn * 64 + j * 16 + lcol;
        const f32x4 a = acc[h * HM + i][j];
        u32x2 w = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3])};
        *reinterpret_cast<u32x2*>(p.C + (size_t)m * p.N + col) = w;
      }
    }
}

// V6: narrow-N tile (BN = 64: ResNet's 64-channel convs). Each wave owns 64 (or 128) rows x all
// 64 columns, so an A row is read by exactly one wave: A goes global -> VGPRs in the MFMA fragment
// layout (lane: row lane & 15 of a 16-row block, 16 B at k = 8 * (lane >> 4) + 32 kk), double-
// buffered one K-tile ahead, never through LDS. B (64 x BK, shared by every wave) goes through a
// 2-stage LDS-DMA ring. LDS traffic is B's fragments only.
template <int NW, int RW>
__global__ void __launch_bounds__(NW * 64, 2) gemm_v6(GP p) {
  constexpr int BNn = 64, MIw = RW / 16, NIw = 4;
  constexpr int BMn = NW * RW;
  constexpr int BSTAGE = BNn * BK * 2;  // 8 KB
  constexpr int NT = NW * 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * BSTAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (no waterfall loops)
  const int ntm = p.M / BMn, ntn = p.N / BNn;
  int tm, tn;
  tile_of<1>(blockIdx.x, ntm, ntn, tm, tn);
  const int m0 = tm * BMn + wave * RW, n0 = tn * BNn;
  const int nk = p.K / BK;
  const u16* Bb = p.B + (size_t)n0 * p.K;
  // B DMA: 64 rows x 128 B = 8 KB = NT * 16 B * (8 KB / (NT * 16))
  constexpr int LBn = BSTAGE / (NT * 16);
  auto glds_b = [&](int kt, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < LBn; ++j) {
      const int r = (tid >> 3) + (NT / 8) * j;
      const u16* g = Bb + (size_t)r * p.K + kt * BK + swz(r, tid & 7) * 8;
      __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + buf * BSTAGE +
                                                                                    (8 * wave + (NT / 8) * j) * 128),
                                       16, 0, 0);
    }
  };
  bf16x8 a0[MIw][2], a1[MIw][2];
  // buffer loads: one 32-bit lane offset, the rest in the scalar offset (few VGPRs)
  const u16* Aw = p.A + (size_t)m0 * p.K;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<u16*>(Aw), (short)0, RW * p.K * 2, 0x00020000);
  const int voff = ((lane & 15) * p.K + (lane >> 4) * 8) * 2;
  auto load_a = [&](bf16x8 (&a)[MIw][2], int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MIw; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        a[i][kk] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                  ra, voff, (i * 16 * p.K + kt * BK + kk * 32) * 2, 0));
  };
  f32x4 acc[MIw][NIw];
#pragma unroll
  for (int i = 0; i < MIw; ++i)
#pragma unroll
    for (int j = 0; j < NIw; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const bf16x8 (&a)[MIw][2], int buf) __attribute__((always_inline)) {
    const char* sb = smem + buf * BSTAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bq[NIw];
#pragma unroll
      for (int j = 0; j < NIw; ++j) {
        const int row = j * 16 + (lane & 15);
        bq[j] = *reinterpret_cast<const bf16x8*>(sb + row * 128 + swz(row, kk * 4 + (lane >> 4)) * 16);
      }
#pragma unroll
      for (int i = 0; i < MIw; ++i)
#pragma unroll
        for (int j = 0; j < NIw; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j], a[i][kk], acc[i][j], 0, 0, 0);
    }
  };
  // B register-staged (plain loads + ds_write after the barrier), so every VMEM load is an
  // ordinary VGPR load and the compiler's counted vmcnt keeps A(kt+1) in flight across the
  // K-tile (an LDS-DMA beside VGPR loads makes hipcc wait vmcnt(0) at each A use).
  u32x4 rb[LBn];
  auto load_b = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < LBn; ++j) {
      const int r = (tid >> 3) + (NT / 8) * j;
      rb[j] = *reinterpret_cast<const u32x4*>(Bb + (size_t)r * p.K + kt * BK + (tid & 7) * 8);
    }
  };
  auto store_b = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < LBn; ++j) {
      const int r = (tid >> 3) + (NT / 8) * j;
      *reinterpret_cast<u32x4*>(smem + buf * BSTAGE + r * 128 + swz(r, tid & 7) * 16) = rb[j];
    }
  };
  (void)glds_b;
  load_b(0);
  load_a(a0, 0);
  store_b(0);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    if (kt + 1 < nk) { load_b(kt + 1); load_a(a1, kt + 1); }
    compute(a0, 0);
    if (kt + 1 >= nk) break;
    store_b(1);
    __syncthreads();
    if (kt + 2 < nk) { load_b(kt + 2); load_a(a0, kt + 2); }
    compute(a1, 1);
    if (kt + 2 < nk) store_b(0);
    __syncthreads();
  }
  const int lrow = lane & 15, lcol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < MIw; ++i) {
    const int m = m0 + i * 16 + lrow;
#pragma unroll
    for (int j = 0; j < NIw; ++j) {
      const int col = n0 + j * 16 + lcol;
      u32x2 w = {pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3])};
      *reinterpret_cast<u32x2*>(p.C + (size_t)m * p.N + col) = w;
    }
  }
}

// V8: two workgroups per CU. 256 threads = 2 x 2 waves, wave tile (TBM/2) x (TBN/2) (128 x 64
// for 256 x 128), BK = 32 (64-B LDS rows), 3-stage LDS-DMA ring (24 KB per stage at 256 x 128,
// 72 KB per workgroup), ONE raw barrier per K-tile with a counted vmcnt that keeps the next
// K-tile's DMA in flight across it. The second workgroup on the CU runs its MFMAs while the first
// waits or stores its epilogue: on short-K shapes the output stores of one tile overlap the other
// workgroup's mainloop instead of idling the CU.
// LDS row r (64 B = 4 16-B chunks) holds logical chunk c at physical chunk c ^ ((r >> 2) & 3):
// a ds_read_b128 16-lane group (rows 16b .. 16b+15, one logical chunk) covers all 16 slots of a
// 256-B bank row.
template <int TBM, int TBN, int NS = 3>
__global__ void __launch_bounds__(256, 2) gemm_v8(GP p) {
  constexpr int BKs = 32, ROWB = 64;
  constexpr int MI = TBM / 2 / 16, NI = TBN / 2 / 16;
  constexpr int AB = TBM * ROWB, BB = TBN * ROWB, ST = AB + BB;
  constexpr int LA = TBM / 64, LB = TBN / 64;  // DMA instructions per thread per K-tile
  __shared__ __attribute__((aligned(16))) char smem[NS * ST];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntm = p.M / TBM, ntn = p.N / TBN;
  int tm, tn;
  tile_of<4>(blockIdx.x, ntm, ntn, tm, tn);
  const int m0 = tm * TBM, n0 = tn * TBN;
  const int nk = p.K / BKs;
  const int rr = tid >> 2, pc = tid & 3;  // DMA: row within a 64-row pass, physical chunk
  const u16* Ab = p.A + (size_t)m0 * p.K;
  const u16* Bb = p.B + (size_t)n0 * p.K;
  auto issue = [&](int kt, int buf) __attribute__((always_inline)) {
    char* sa = smem + buf * ST;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int r = rr + 64 * i;
      const u16* g = Ab + (size_t)r * p.K + kt * BKs + ((pc ^ ((r >> 2) & 3)) * 8);
      __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(sa + (64 * i + 16 * wave) * ROWB),
                                       16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      const int r = rr + 64 * j;
      const u16* g = Bb + (size_t)r * p.K + kt * BKs + ((pc ^ ((r >> 2) & 3)) * 8);
      __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(sa + AB + (64 * j + 16 * wave) * ROWB),
                                       16, 0, 0);
    }
  };
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lr = lane & 15, lc = lane >> 4;
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t, t);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NS - 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (LA + LB)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NS - 1 < nk) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const char* sa = smem + (kt % NS) * ST;
    const char* sb = sa + AB;
    bf16x8 af[MI], bq[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wn * (TBN / 2) + j * 16 + lr;
      bq[j] = *reinterpret_cast<const bf16x8*>(sb + row * ROWB + ((lc ^ ((row >> 2) & 3)) << 4));
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * (TBM / 2) + i * 16 + lr;
      af[i] = *reinterpret_cast<const bf16x8*>(sa + row * ROWB + ((lc ^ ((row >> 2) & 3)) << 4));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  // 16-B stores (the v0 epi16 lane exchange)
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wm * (TBM / 2) + i * 16 + lr;
#pragma unroll
    for (int j = 0; j < NI; j += 2) {
      uint32_t a0 = pack2bf(acc[i][j][0], acc[i][j][1]), a1 = pack2bf(acc[i][j][2], acc[i][j][3]);
      uint32_t b0 = pack2bf(acc[i][j + 1][0], acc[i][j + 1][1]), b1 = pack2bf(acc[i][j + 1][2], acc[i][j + 1][3]);
      const auto r0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
      const bool odd = (lane >> 4) & 1;
      u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
      const int blk = odd ? j + 1 : j;
      const int col = n0 + wn * (TBN / 2) + blk * 16 + ((lane >> 5) * 8);
      *reinterpret_cast<u32x4*>(p.C + (size_t)m * p.N + col) = v;
    }
  }
}

// ------------------------------------------------------------------------------ harness
__global__ void fill_kernel(u16* x, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float f = (float)(h >> 8) * (2.f / 16777216.f) - 1.f;
    const __bf16 b = (__bf16)f;
    x[i] = __builtin_bit_cast(u16, b);
  }
}

__global__ void ref_kernel(const u16* A, const u16* B, const int* rows, const int* cols, int ns, int K, float* out) {
  const int s = blockIdx.x;
  if (s >= ns) return;
  const u16* a = A + (size_t)rows[s] * K;
  const u16* b = B + (size_t)cols[s] * K;
  float acc = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    acc += __uint_as_float((uint32_t)a[k] << 16) * __uint_as_float((uint32_t)b[k] << 16);
  __shared__ float red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[s] = red[0];
}

typedef void (*Kern)(GP);
struct Var {
  const char* name;
  Kern k;
  int persist = 0;  // 1: grid = min(tiles, 256 CUs) and the kernel loops over tiles
  int bm = 256, bn = 256, nth = 512;
};
static const Var VARS[] = {
    {"v0 4phase gm1", gemm_v0<1, true>},
    {"v0 4phase gm4", gemm_v0<4, true>},
    {"v0 4phase gm8", gemm_v0<8, true>},
    {"v0 4phase gm4 noprio", gemm_v0<4, false>},
    {"v0 epi16 gm4", gemm_v0<4, true, 1>},
    {"v0 epi16 gm4 static-prio", gemm_v0<4, true, 1, true>},
    {"v0 epi16 gm4 static-prio only", gemm_v0<4, false, 1, true>},
    {"v0 epi16 gm4 persistent", gemm_v0<4, true, 1, false, true>, 1},
    {"v2 2phase gm1", gemm_v2<1>},
    {"v2 2phase gm4", gemm_v2<4>},
    {"v6 narrowN 4w x 64r", gemm_v6<4, 64>, 0, 256, 64, 256},
    {"v6 narrowN 4w x 128r", gemm_v6<4, 128>, 0, 512, 64, 256},
    {"v6 narrowN 8w x 64r", gemm_v6<8, 64>, 0, 512, 64, 512},
    {"v8 2wg 256x128 bk32 3st", gemm_v8<256, 128>, 0, 256, 128, 256},
    {"v8 2wg 128x256 bk32 3st", gemm_v8<128, 256>, 0, 128, 256, 256},
    {"v8 2wg 256x128 bk32 2st", gemm_v8<256, 128, 2>, 0, 256, 128, 256},
    {"v8 2wg 128x128 bk32 3st", gemm_v8<128, 128>, 0, 128, 128, 256},
};
constexpr int NVARS = sizeof(VARS) / sizeof(VARS[0]);

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 8192;
  const int N = argc > 2 ? atoi(argv[2]) : 8192;
  const int K = argc > 3 ? atoi(argv[3]) : 8192;
  const int iters = argc > 4 ? atoi(argv[4]) : 20;
  std::vector<int> sel;
  for (int i = 5; i < argc; ++i) sel.push_back(atoi(argv[i]));
  if (sel.empty())
    for (int i = 0; i < NVARS; ++i) sel.push_back(i);
  if (M % 64 || N % 64 || K % BK) {  // (BK = 64 covers the BK = 32 variants too)
    fprintf(stderr, "M, N must be multiples of 64 and K of 64\n");
    return 2;
  }
  u16 *A, *B, *C;
  CHECK(hipMalloc(&A, (size_t)M * K * 2));
  CHECK(hipMalloc(&B, (size_t)N * K * 2));
  CHECK(hipMalloc(&C, (size_t)M * N * 2));
  fill_kernel<<<4096, 256>>>(A, (size_t)M * K, 1234u);
  fill_kernel<<<4096, 256>>>(B, (size_t)N * K, 987u);
  const int NS = 512;
  std::vector<int> hr(NS), hc(NS);
  srand(7);
  for (int s = 0; s < NS; ++s) {
    hr[s] = (s < 8) ? s * (M / 8) + (s % 3) : rand() % M;
    hc[s] = (s < 8) ? s * (N / 8) + (N / 8 > 8 ? N / 8 - 1 - s : 0) : rand() % N;  // last columns of each 1/8
  }
  int *dr, *dc;
  float* dref;
  CHECK(hipMalloc(&dr, NS * 4));
  CHECK(hipMalloc(&dc, NS * 4));
  CHECK(hipMalloc(&dref, NS * 4));
  CHECK(hipMemcpy(dr, hr.data(), NS * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dc, hc.data(), NS * 4, hipMemcpyHostToDevice));
  ref_kernel<<<NS, 256>>>(A, B, dr, dc, NS, K, dref);
  std::vector<float> ref(NS);
  CHECK(hipMemcpy(ref.data(), dref, NS * 4, hipMemcpyDeviceToHost));
  const double flop = 2.0 * M * N * (double)K;
  GP p{A, B, C, M, N, K};

  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<u16> hC((size_t)M * N);
  for (int v : sel) {
    if (v < 0 || v >= NVARS) continue;
    if (M % VARS[v].bm || N % VARS[v].bn) continue;
    const int ntiles = (M / VARS[v].bm) * (N / VARS[v].bn);
    const dim3 grid(VARS[v].persist ? (ntiles < 256 ? ntiles : 256) : ntiles);
    CHECK(hipMemset(C, 0xff, (size_t)M * N * 2));
    hipLaunchKernelGGL(VARS[v].k, grid, dim3(VARS[v].nth), 0, 0, p);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(hC.data(), C, (size_t)M * N * 2, hipMemcpyDeviceToHost));
    double maxerr = 0.0;
    for (int s = 0; s < NS; ++s) {
      const float got = __builtin_bit_cast(float, (uint32_t)hC[(size_t)hr[s] * N + hc[s]] << 16);
      const double err = fabs((double)got - ref[s]) / (1.0 + fabs((double)ref[s]));
      if (!(err <= maxerr)) maxerr = err;  // NaN-propagating
    }
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(VARS[v].k, grid, dim3(VARS[v].nth), 0, 0, p);
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(VARS[v].k, grid, dim3(VARS[v].nth), 0, 0, p);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("M=%d N=%d K=%d  v%-2d %-28s %9.1f us  %7.1f TF/s  maxrelerr %.2e %s\n", M, N, K, v, VARS[v].name,
           ms * 1e3, flop / (ms * 1e-3) / 1e12, maxerr, maxerr < 2e-2 ? "ok" : "WRONG");
    fflush(stdout);
  }
  return 0;
}
