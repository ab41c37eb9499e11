// Common definitions for the MI355X (gfx950 / CDNA4) kernel library.
//
// All kernels are plain HIP C++ written for wave64 + MFMA; the library exposes
// a C ABI (PDT_API) that the Python layer calls through ctypes with raw device
// pointers and the current HIP stream (no torch headers, no hipify).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// tanh for activation epilogues: 1 - 2 / (1 + e^{2x}) on the hardware exp / reciprocal
// (v_exp_f32, v_rcp_f32: a few instructions instead of libm's tanhf, which costs ~2x a
// bf16 GEMM's epilogue time in a fused GELU). Saturates correctly (exp -> inf / 0);
// abs error ~1e-7, far below bf16 output rounding.
__device__ __forceinline__ float pdt_tanh(float x) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x));
}

// gelu_tanh(z) and its derivative from one tanh (the MLP's act-4 epilogue and its library-GEMM
// twin in csrc/fp8.hip)
// h = 0.5 (1 + tanh(u)) = sigmoid(2u), u = sqrt(2/pi) (z + 0.044715 z^3), with the constants
// folded by hand (no fast-math reassociation): 9 VALU ops + exp2 + rcp per element instead of ~20
// -- the fc1 epilogue that runs it is VALU-bound
__device__ __forceinline__ void pdt_gelu_dual(float z, float& g, float& d) {
  constexpr float K1 = -2.f * 0.7978845608f * 1.4426950409f;  // exp2 argument -2u log2(e) = z (K1 + K3 z^2)
  constexpr float K3 = K1 * 0.044715f;
  constexpr float C1 = 2.f * 0.7978845608f;  // 2 du/dz = C1 + C3 z^2
  constexpr float C3 = C1 * 3.f * 0.044715f;
  const float z2 = z * z;
  const float h = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z * fmaf(K3, z2, K1)));
  g = z * h;
  d = fmaf(g * (1.f - h), fmaf(C3, z2, C1), h);  // h + 0.5 z (1 - t^2) 2du, t = 2h - 1
}

// pdt_gelu_dual of two values on the packed fp32 VALU (v_pk_mul / v_pk_fma / v_pk_add: one
// instruction per pair; exp2 / rcp stay scalar) -- the same operations in the same order, so
// the results are those of two pdt_gelu_dual calls
typedef float pdt_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void pdt_gelu_dual2(pdt_f32x2 z, pdt_f32x2& g, pdt_f32x2& d) {
  constexpr float K1 = -2.f * 0.7978845608f * 1.4426950409f;
  constexpr float K3 = K1 * 0.044715f;
  constexpr float C1 = 2.f * 0.7978845608f;
  constexpr float C3 = C1 * 3.f * 0.044715f;
  const pdt_f32x2 z2 = z * z;
  const pdt_f32x2 a = z * __builtin_elementwise_fma(pdt_f32x2{K3, K3}, z2, pdt_f32x2{K1, K1});
  pdt_f32x2 h;
  h.x = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(a.x));
  h.y = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(a.y));
  g = z * h;
  d = __builtin_elementwise_fma(g * (pdt_f32x2{1.f, 1.f} - h),
                                __builtin_elementwise_fma(pdt_f32x2{C3, C3}, z2, pdt_f32x2{C1, C1}), h);
}

// four floats already within +-448 -> four packed e4m3fn codes, no clamp (8 VALU ops fewer
// than pdt_cvt4_f8<0>): values scaled by a power of two from their own |max| (attention's
// per-head / per-tile scales) or bounded by construction (256 P, P <= 1)
__device__ __forceinline__ uint32_t pdt_cvt4_e4m3_inrange(float a, float b, float c, float d) {
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return (uint32_t)r;
}

// four floats -> four packed OCP fp8 codes (FMT 0 = e4m3fn, 1 = e5m2) with the gfx950
// packed converts (round to nearest even); clamped to the finite range first
template <int FMT>
__device__ __forceinline__ uint32_t pdt_cvt4_f8(float a, float b, float c, float d) {
  constexpr float FMAX = FMT == 0 ? 448.f : 57344.f;
  a = fminf(fmaxf(a, -FMAX), FMAX);
  b = fminf(fmaxf(b, -FMAX), FMAX);
  c = fminf(fmaxf(c, -FMAX), FMAX);
  d = fminf(fmaxf(d, -FMAX), FMAX);
  int r;
  if (FMT == 0) {
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  } else {
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, r, true);
  }
  return (uint32_t)r;
}

#define PDT_API extern "C" __attribute__((visibility("default")))
#define LDS_PTR(T) T __attribute__((address_space(3)))*

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ u16 f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  return __builtin_bit_cast(u16, b);
}

__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// low / high bf16 of a packed 32-bit word
__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// keep mask of packed bf16 word e from a bit mask: bit 2e keeps its low half, bit 2e + 1 its
// high half (0 / 0xffff / 0xffff0000 / ~0: a gated-off element becomes +0 under AND)
__device__ __forceinline__ uint32_t pdt_bf16_pair_keep(uint32_t bits, int e) {
  const uint32_t lo = (uint32_t)((int)(bits << (31 - 2 * e)) >> 31);
  const uint32_t hi = (uint32_t)((int)(bits << (30 - 2 * e)) >> 31);
  return (lo & 0x0000ffffu) | (hi & 0xffff0000u);
}

// DPP row reductions: a DPP "row" is 16 lanes; the operand permutes ride on the
// VALU add (no LDS round trip, unlike __shfl_xor's ds_bpermute).
//   quad_perm [1,0,3,2] (0xB1) = lane ^ 1, quad_perm [2,3,0,1] (0x4E) = lane ^ 2,
//   row_half_mirror (0x141) = 7 - lane within 8, row_mirror (0x140) = 15 - lane.
// bound_ctrl set (every source lane is in range anyway) lets the compiler fold the
// move into the add: one v_add_f32_dpp per step.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// sum over the 8 lanes (lane & ~7 group); every lane of the group gets it
__device__ __forceinline__ float row8_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  return v + dpp_f<0x141>(v);
}
// sum over the 16 lanes of a DPP row (same set as xor 1, 2, 4, 8); every lane gets it
__device__ __forceinline__ float row16_sum(float v) {
  v = row8_sum(v);
  return v + dpp_f<0x140>(v);
}

template <typename Op>
__device__ __forceinline__ float row16_reduce(float v, Op op) {
  v = op(v, dpp_f<0xB1>(v));
  v = op(v, dpp_f<0x4E>(v));
  v = op(v, dpp_f<0x141>(v));
  return op(v, dpp_f<0x140>(v));
}

// Cross-row lane exchanges on gfx950's v_permlane{16,32}_swap (VALU, no LDS): swapping a
// register with itself leaves {x[l], x[l ^ 32]} (resp. x[l ^ 16]) in the two results, so
// op(r0, r1) equals op(v, __shfl_xor(v, 32)) bit for bit (op commutative).
template <typename Op>
__device__ __forceinline__ float xor32_reduce(float v, Op op) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return op(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
template <typename Op>
__device__ __forceinline__ float xor16_reduce(float v, Op op) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return op(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
struct AddOp {
  __device__ float operator()(float a, float b) const { return a + b; }
};
struct MaxOp {
  __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
};

// whole-wave reductions (every lane gets the result): 2 permlane swaps + 4 DPP steps
__device__ __forceinline__ float warp_sum(float v) {
  return row16_reduce(xor16_reduce(xor32_reduce(v, AddOp{}), AddOp{}), AddOp{});
}
__device__ __forceinline__ float warp_max(float v) {
  return row16_reduce(xor16_reduce(xor32_reduce(v, MaxOp{}), MaxOp{}), MaxOp{});
}

// Fast unsigned division by a runtime-constant divisor (Granlund-Montgomery).
struct FastDiv {
  uint32_t d, m, s;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d == 1) { f.m = 0; f.s = 0; return f; }
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  if (f.d == 1) return n;
  uint32_t t = __umulhi(n, f.m);
  return (t + ((n - t) >> 1)) >> (f.s - 1);
}

// Bijective XCD-aware remap of a 1-D block id: consecutive *logical* ids land
// on the same XCD (blocks b, b+8, b+16.. share one XCD under round-robin
// dispatch), so tiles that share an operand panel share that XCD's L2.
// Speed only -- never relied on for correctness.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
  const uint32_t NX = 8;
  if (nwg < NX) return bid;
  uint32_t q = nwg / NX, r = nwg % NX, x = bid % NX, k = bid / NX;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

#define PDT_RETURN_LAUNCH() return (int)hipGetLastError()

// Launcher error code: a __device__ symbol's address could not be resolved (the kernel is
// not launched -- a null LDS-DMA source would fault on the GPU).
#define PDT_ERR_SYMBOL (-7)
#define PDT_MAX_DEV 64

// Device address of a __device__ symbol, cached per device id (each device the code object
// is loaded on has its own copy of the symbol). nullptr if the lookup fails.
static inline const void* pdt_symbol_addr(const void* sym, const void** cache) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= PDT_MAX_DEV) return nullptr;
  if (cache[dev] == nullptr) {
    void* d = nullptr;
    if (hipGetSymbolAddress(&d, sym) == hipSuccess) cache[dev] = d;
  }
  return cache[dev];
}

// compute units of the current device (cached per device id; 256 if the query fails) --
// the grid of a persistent kernel
static inline int pdt_num_cus() {
  static int cache[PDT_MAX_DEV] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= PDT_MAX_DEV) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    cache[dev] = (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) ? n
                                                                                                               : 256;
  }
  return cache[dev];
}
