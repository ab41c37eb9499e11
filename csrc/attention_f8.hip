// FP8 attention forward for ViT (head dim 64, T <= 256), the "CDNA4 fp8 MFMA
// attention path" of BASELINE config #5.
//
//   S^T = K Q^T   on mfma_scale_f32_32x32x64_f8f6f4 (OCP e4m3 operands, K = 64 =
//                 the head dim: ONE instruction per 32 keys x 32 queries, 2x the
//                 bf16 MFMA rate); fp32 accumulate, unit block scales.
//   softmax       fp32, online over 32-key tiles (running max / sum per query,
//                 O rescaled when the max moves), exp2 with the scale folded in.
//   O^T = V^T P^T on mfma_scale_f32_32x32x64_f8f6f4 as well (64 keys = two key tiles per
//                 instruction, softmax max / rescale per tile pair): P^T comes straight from
//                 the S^T accumulator registers as e4m3 codes of 256 P (P <= 1), packed
//                 tile 2tp in bytes 0..15 / 2tp + 1 in 16..31 -- the operand k layout of
//                 csrc/fp8_mfma.h -- and V^T from an e4m3 row image of V (per-head power-of-
//                 two scale) through ds_read_b64_tr_b8 in that same key order. The row sums
//                 l are of the fp32 P. The bf16 instantiation (F8 = false) keeps the bf16
//                 PV on mfma_f32_32x32x16_bf16 with V^T via ds_read_b64_tr_b16.
//
// Quantization (no extra pass over HBM, no host sync): each workgroup owns one
// (batch, head); it stages the head's K from the bf16 qkv buffer, reduces |K|max
// over the head and quantizes K with a power-of-two scale into an fp8 LDS image
// (16 KB instead of 32 KB of bf16). Each wave quantizes its 32-query Q tile the
// same way (wave-wide |Q|max). Power-of-two scales make the dequantisation an
// exact exponent shift, applied once to the fp32 scores.
//
// Output layout and the saved log-sum-exp follow csrc/attention.hip exactly, so
// the bf16 recomputing backward consumes them unchanged (it recomputes P from the
// bf16 Q and K: the fp8 forward's probabilities differ from it by the fp8 score
// error only).
#include "fp8_mfma.h"

namespace {

constexpr int D = 64;

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// fp8 K / V images: [rows][64 B], 16-B chunk c of row r at chunk c ^ ((r >> 2) & 3)
// (pdt_f8::k8_off): a 16-lane ds_read_b128 group (16 consecutive rows, one chunk) hits 16
// distinct slots
using pdt_f8::k8_off;

// bf16 V image for transposed reads (same swizzle as csrc/attention.hip): [rows][128 B]
__device__ __forceinline__ int vt_off(int row, int byte_in_row) {
  const int seg = byte_in_row >> 5;
  const int sw = ((row >> 1) & 1) | ((row >> 2) & 2);
  return row * 128 + ((seg ^ sw) << 5) + (byte_in_row & 31);
}

__device__ __forceinline__ uint32_t cvt4_e4m3(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f);
  d = fminf(fmaxf(d, -448.f), 448.f);
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return (uint32_t)r;
}

// power-of-two quantization scale for |x|max = amax: largest 2^e with amax * 2^e <= 448
__device__ __forceinline__ float pow2_scale(float amax) {
  if (!(amax > 0.f)) return 1.f;
  int e = max(min((int)floorf(__log2f(448.f / amax)), 100), -100);
  if (ldexpf(amax, e) > 448.f) --e;  // (the fast log2 may round up at an exact power of two)
  return ldexpf(1.f, e);
}

struct AttnF8Params {
  const u16* qkv;   // [B, T, 3, H, 64] bf16
  u16* out;         // [B, T, H*64]
  float* lse;       // [B*H, T]
  int B, T, H;
  long ld, ldo;
  float c;          // softmax scale * log2(e)
  // optional: e4m3 codes of the (bf16-rounded) output for the next fp8 GEMM (the attention
  // projection) with its delayed scale q8_meta[0]; per-workgroup max |O| -> q8_part[bh]
  uint8_t* q8;
  const float* q8_meta;
  float* q8_part;
};

// bf16 K row image: [rows][128 B], chunk c of row r at c ^ ((r >> 1) & 7)
__device__ __forceinline__ int k16_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// NKT = number of 32-key tiles (ceil(T/32) <= 8). F8 = false: the same kernel with the
// score GEMM in bf16 (4 x mfma_f32_32x32x16_bf16 per 32 x 32 tile, K kept as bf16) -- the
// bf16 forward of ViT (126 VGPRs, 3 workgroups per CU, vs 248 VGPRs / 1 wave per SIMD
// for the whole-sequence kernel in csrc/attention.hip)
// Q8: the e4m3 codes of O for the projection GEMM -- -1 decided by p.q8 at run time, 0 / 1
// compiled out / in (the 8-wave launches: no per-chunk branches in the epilogue)
template <int NKT, bool F8, bool PV8 = false, int NW = 4, int Q8 = -1>
__global__ void __launch_bounds__(64 * NW) attn_fwd_f8_kernel(AttnF8Params p) {
  const bool q8on = Q8 >= 0 ? Q8 == 1 : p.q8 != nullptr;
  constexpr int NTH = 64 * NW;
  static_assert(F8 || !PV8, "the fp8 PV rides on the fp8 score kernel");
  constexpr int ROWS = NKT * 32;
  constexpr int VROWS = PV8 ? 64 * ((NKT + 1) / 2) : ROWS;         // fp8 V: whole key-tile pairs
  __shared__ __attribute__((aligned(16))) char Ks[ROWS * (F8 ? 64 : 128)];  // fp8 or bf16 K
  __shared__ __attribute__((aligned(16))) char Vs[VROWS * (PV8 ? 64 : 128)];  // fp8 rows / bf16 tr image
  __shared__ float red[NW], vred[NW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const u16* base = p.qkv + (long)b * p.T * p.ld + h * D;
  const u16* Kg = base + p.H * D;
  const u16* Vg = base + 2 * p.H * D;

  // ---- stage V (bf16 transposed-read image, or e4m3 rows) and K (registers first: |K|max)
  constexpr int CH = ROWS * 8;  // 16-B chunks of one [ROWS][64] bf16 matrix
  constexpr int VCH = VROWS * 8;
  constexpr int NIT = (VCH + NTH - 1) / NTH;
  u32x4 kv[NIT], vv[NIT];
  // Every staging load is issued before any is consumed, from a clamped (always valid) row:
  // with the bounds test around the loads, hipcc waited for each iteration's pair before the
  // next one's issue (vmcnt(1) between pairs), serialising ~NIT + 1 HBM latencies per head.
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int q = tid + it * NTH;
    const int rr = min(q >> 3, p.T - 1), ch = q & 7;
    vv[it] = *reinterpret_cast<const u32x4*>(Vg + (long)rr * p.ld + ch * 8);
    kv[it] = *reinterpret_cast<const u32x4*>(Kg + (long)rr * p.ld + ch * 8);
  }
  // fp8: this wave's first query tile is loaded here too, so its latency overlaps the staging
  // loads' instead of following the staging barrier (with 8 waves and T <= 256 it is the wave's
  // only tile). Same lane layout as the in-loop load below.
  u32x4 qpre[F8 ? 4 : 1];
  if constexpr (F8) {
    const int q = wave * 32 + (lane & 31);
    const int qr = min(q, p.T - 1);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u32x4 t = *reinterpret_cast<const u32x4*>(base + (long)qr * p.ld + 32 * (lane >> 5) + 8 * c);
      qpre[c] = q < p.T ? t : u32x4{0, 0, 0, 0};
    }
  }
  // |K|max / |V|max on the packed bf16 bits (pdt_f8::absmax_bf16x2: two magnitudes per u16 max)
  uint32_t kmb = 0u, vmb = 0u;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int q = tid + it * NTH;
    const int row = q >> 3, ch = q & 7;
    const bool ok = q < VCH && row < p.T;
    const u32x4 v = ok ? vv[it] : u32x4{0, 0, 0, 0};
    const u32x4 k = ok ? kv[it] : u32x4{0, 0, 0, 0};
    if constexpr (PV8) {
      vv[it] = v;
#pragma unroll
      for (int e = 0; e < 4; ++e) vmb = pdt_f8::absmax_bf16x2(vmb, v[e]);
    } else if (q < CH) {
      *reinterpret_cast<u32x4*>(Vs + vt_off(row, ch * 16)) = v;
    }
    kv[it] = k;
#pragma unroll
    for (int e = 0; e < 4; ++e) kmb = pdt_f8::absmax_bf16x2(kmb, k[e]);
  }
  float kmax = pdt_f8::absmax_bf16x2_value(kmb), vmax = pdt_f8::absmax_bf16x2_value(vmb);
  float sk = 1.f, sv = 1.f;
  int ev = 0;
  if constexpr (F8) {
    kmax = warp_max(kmax);
    vmax = warp_max(vmax);
    if (lane == 0) {
      red[wave] = kmax;
      vred[wave] = vmax;
    }
    __syncthreads();
    kmax = red[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) kmax = fmaxf(kmax, red[w]);
    sk = pow2_scale(kmax);
  }
  if constexpr (PV8) {
    float vm = vred[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) vm = fmaxf(vm, vred[w]);
    ev = pdt_f8::pow2_exp(vm);
    sv = ldexpf(1.f, ev);
    const float vdiv = ldexpf(1.f, -ev);  // the scaled converts divide: codes of V * 2^ev
#pragma unroll
    for (int it = 0; it < NIT; ++it) {  // e4m3 V rows (zero rows up to the tile pair)
      const int q = tid + it * NTH;
      if (q < VCH) {
        const int row = q >> 3, ch = q & 7;
        const u32x4 v = vv[it];
        uint2 w;
        w.x = pdt_f8::e4m3x4_bf16(v[0], v[1], vdiv);
        w.y = pdt_f8::e4m3x4_bf16(v[2], v[3], vdiv);
        *reinterpret_cast<uint2*>(Vs + k8_off(row, ch >> 1) + (ch & 1) * 8) = w;
      }
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int q = tid + it * NTH;
    if (!F8 && q < CH) {
      const int row = q >> 3, ch = q & 7;
      *reinterpret_cast<u32x4*>(Ks + k16_off(row, ch)) = kv[it];
    } else if (q < CH) {
      const int row = q >> 3, ch = q & 7;  // 8 bf16 -> 8 fp8 bytes: half of a 16-B fp8 chunk
      const u32x4 k = kv[it];
      uint2 w;
      w.x = pdt_f8::e4m3x4_bf16(k[0], k[1], 1.f / sk);  // (sk a power of two: exact divisor)
      w.y = pdt_f8::e4m3x4_bf16(k[2], k[3], 1.f / sk);
      *reinterpret_cast<uint2*>(Ks + k8_off(row, ch >> 1) + (ch & 1) * 8) = w;
    }
  }
  __syncthreads();

  // lane roles in the 32x32 tiles: query / d column = lane & 31, half hh = lane >> 5
  const int col = lane & 31, hh = lane >> 5;
  const int grp = lane >> 4, i16 = lane & 15;  // 16-lane group of the transposed V reads
  const int nqt = (p.T + 31) / 32;
  float q8max = 0.f;
  for (int qt = wave; qt < nqt; qt += NW) {
    // ---- Q tile -> e4m3 B fragment: lane (q = col, hh) holds Q[q][32 hh .. 32 hh + 31]
    const int q = qt * 32 + col;
    // fp8: qv[c] = Q[q][32 hh + 8 c .. +7] (one 32-B fp8 fragment); bf16: qb[kk] = Q[q][16 kk + 8 hh .. +7]
    u32x4 qv[4], qb[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      qv[c] = u32x4{0, 0, 0, 0};
      qb[c] = u32x4{0, 0, 0, 0};
      if (F8 && qt == wave) {
        qv[c] = qpre[F8 ? c : 0];
      } else if (q < p.T) {
        if (F8) qv[c] = *reinterpret_cast<const u32x4*>(base + (long)q * p.ld + 32 * hh + 8 * c);
        else qb[c] = *reinterpret_cast<const u32x4*>(base + (long)q * p.ld + 16 * c + 8 * hh);
      }
    }
    float sq = 1.f;
    if constexpr (F8) {
      uint32_t qmb = 0u;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) qmb = pdt_f8::absmax_bf16x2(qmb, qv[c][e]);
      const float qm = warp_max(pdt_f8::absmax_bf16x2_value(qmb));
      sq = pow2_scale(qm);
    }
    i32x8 qf;
#pragma unroll
    for (int c = 0; c < (F8 ? 4 : 0); ++c) {
      qf[2 * c] = (int)pdt_f8::e4m3x4_bf16(qv[c][0], qv[c][1], 1.f / sq);
      qf[2 * c + 1] = (int)pdt_f8::e4m3x4_bf16(qv[c][2], qv[c][3], 1.f / sq);
    }
    // scores in the log2 domain: c * S = (c / (sk sq)) * S_fp8
    const float cs = p.c / (sk * sq);

    float m = -INFINITY, l = 0.f;
    f32x16 o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;

    if constexpr (PV8) {
      // key tiles in pairs: S^T of tiles 2tp, 2tp + 1 (e4m3), one softmax update, then
      // O^T += V^T P^T on ONE 64-key fp8 MFMA per 32-d half
#pragma unroll 1
      for (int tp = 0; tp < (NKT + 1) / 2; ++tp) {
        f32x16 s2[2];
        float mt = -INFINITY;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int t = 2 * tp + u;
          f32x16 s = {};
          if (t < NKT) {
            const int krow = 32 * t + col;
            const u32x4 a0 = *reinterpret_cast<const u32x4*>(Ks + k8_off(krow, 2 * hh));
            const u32x4 a1 = *reinterpret_cast<const u32x4*>(Ks + k8_off(krow, 2 * hh + 1));
            const i32x8 kf = {(int)a0[0], (int)a0[1], (int)a0[2], (int)a0[3],
                              (int)a1[0], (int)a1[1], (int)a1[2], (int)a1[3]};
            s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qf, s, 0, 0, 0, 127, 0, 127);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const float v = (t < NKT && (t < NKT - 1 || key < p.T)) ? s[r] * cs : -INFINITY;
            s[r] = v;
            mt = fmaxf(mt, v);
          }
          s2[u] = s;
        }
        mt = xor32_reduce(mt, MaxOp{});
        const float mn = fmaxf(m, mt);
        const float alpha = exp2f(m - mn);
        float ls = 0.f;
        uint32_t pc[2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float e = __builtin_amdgcn_exp2f(s2[u][r] - mn);
            s2[u][r] = e;
            ls += e;
          }
#pragma unroll
          for (int w = 0; w < 4; ++w)
            pc[u][w] = pdt_f8::e4m3x4_div(s2[u][4 * w], s2[u][4 * w + 1], s2[u][4 * w + 2], s2[u][4 * w + 3],
                                          1.f / 256.f);
        }
        ls = xor32_reduce(ls, AddOp{});
        l = l * alpha + ls;
        m = mn;
        const i32x8 pf = {(int)pc[0][0], (int)pc[0][1], (int)pc[0][2], (int)pc[0][3],
                          (int)pc[1][0], (int)pc[1][1], (int)pc[1][2], (int)pc[1][3]};
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          o[dt] *= alpha;
          // A: V^T rows d = 32 dt + 16 (grp & 1) + i16, k = keys of the pair (P's order)
          const i32x8 va = pdt_f8::tr_frag<true>(Vs, 64 * tp, 2 * dt + (grp & 1), i16, hh);
          o[dt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(va, pf, o[dt], 0, 0, 0, 127 - ev, 0, 127 - 8);
        }
      }
    }
    // not unrolled: a fully unrolled key loop hoists every tile's K fragment (214 VGPRs
    // at 7 tiles, 2 waves/SIMD); rolled it stays near 100 (more workgroups per CU)
#pragma unroll 1
    for (int t = 0; t < (PV8 ? 0 : NKT); ++t) {
      const int krow = 32 * t + col;
      f32x16 s = {};
      if constexpr (F8) {
        // A fragment: K[key = 32t + col][d = 32 hh .. +31] (two swizzled 16-B chunks)
        const u32x4 a0 = *reinterpret_cast<const u32x4*>(Ks + k8_off(krow, 2 * hh));
        const u32x4 a1 = *reinterpret_cast<const u32x4*>(Ks + k8_off(krow, 2 * hh + 1));
        const i32x8 kf = {(int)a0[0], (int)a0[1], (int)a0[2], (int)a0[3], (int)a1[0], (int)a1[1], (int)a1[2], (int)a1[3]};
        s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qf, s, 0, 0, 0, 127, 0, 127);
      } else {
        // k-step kk covers d = 16 kk .. +15: lane half hh holds d = 16 kk + 8 hh .. +7
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + k16_off(krow, 2 * kk + hh));
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, __builtin_bit_cast(bf16x8, qb[kk]), s, 0, 0, 0);
        }
      }
      // s[r] = S[key = 32t + (r & 3) + 8 (r >> 2) + 4 hh][query q], raw (scaled) fp8 product
      float mt = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const float v = (t < NKT - 1 || key < p.T) ? s[r] * cs : -INFINITY;
        s[r] = v;
        mt = fmaxf(mt, v);
      }
      mt = xor32_reduce(mt, MaxOp{});  // the other 16 keys of this query
      const float mn = fmaxf(m, mt);
      const float alpha = exp2f(m - mn);  // m = -inf first: 0
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[r] - mn);
        s[r] = e;
        ls += e;
      }
      ls = xor32_reduce(ls, AddOp{});
      l = l * alpha + ls;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) o[dt] *= alpha;
      // O^T[d][q] += V^T[d][key] P^T[key][q], two 16-key steps. B = registers 8s..8s+7 of s
      // (element j of half hh = key 16s + 8(j>>2) + 4hh + (j&3)); A = the same keys of V^T
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (__bf16)s[8 * st + j];
        const int kb = 32 * t + 16 * st + 4 * (grp >> 1);  // this 16-lane group's 4 keys (j = 0..3)
        const int rq = i16 >> 2, cp = i16 & 3;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int d0 = 32 * dt + 16 * (grp & 1);
          const char* a_lo = Vs + vt_off(kb + rq, (d0 + 4 * cp) * 2);
          const char* a_hi = Vs + vt_off(kb + 8 + rq, (d0 + 4 * cp) * 2);
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)a_lo));
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)((__attribute__((address_space(3))) char*)(uintptr_t)(uint32_t)(uintptr_t)a_hi));
          const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[dt], 0, 0, 0);
        }
      }
    }
    // o[dt][r] = O^T[d = 32 dt + (r & 3) + 8 (r >> 2) + 4 hh][query q]: lane (q, hh) holds 4 of
    // each 8-column chunk, lane (q, 1 - hh) = lane ^ 32 the other 4. One v_permlane32_swap per
    // dword of two chunks g4 (even), g4 + 1 gives lane hh = 0 chunk g4's 8 columns and lane
    // hh = 1 chunk g4 + 1's: 16-B O stores and 8-B code stores instead of 8-B / 4-B ones (a
    // row-per-lane epilogue is store-issue-bound). The swaps run with the full EXEC (lanes
    // q >= T hold finite values: their Q rows are zero); only the stores are predicated.
    {
      const bool qok = q < p.T;
      const float inv = 1.f / l;
      const long orow_off = ((long)b * p.T + (qok ? q : 0)) * p.ldo + h * D;
      u16* orow = p.out + orow_off;
      const float s8 = q8on ? p.q8_meta[0] : 0.f;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g2 = 0; g2 < 4; g2 += 2) {
          uint32_t w[2][2], c8[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int g4 = g2 + u;
            w[u][0] = pack2bf(o[dt][4 * g4] * inv, o[dt][4 * g4 + 1] * inv);
            w[u][1] = pack2bf(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
            if (q8on) {
              const float f0 = lo_bf(w[u][0]), f1 = hi_bf(w[u][0]), f2 = lo_bf(w[u][1]), f3 = hi_bf(w[u][1]);
              if (qok) q8max = fmaxf(q8max, fmaxf(fmaxf(fabsf(f0), fabsf(f1)), fmaxf(fabsf(f2), fabsf(f3))));
              c8[u] = cvt4_e4m3(f0 * s8, f1 * s8, f2 * s8, f3 * s8);
            }
          }
          const auto r0 = __builtin_amdgcn_permlane32_swap(w[0][0], w[1][0], false, false);
          const auto r1 = __builtin_amdgcn_permlane32_swap(w[0][1], w[1][1], false, false);
          const int col0 = 32 * dt + 8 * (g2 + hh);
          if (qok) *reinterpret_cast<u32x4*>(orow + col0) = u32x4{r0[0], r1[0], r0[1], r1[1]};
          if (q8on) {
            const auto rc = __builtin_amdgcn_permlane32_swap(c8[0], c8[1], false, false);
            if (qok) *reinterpret_cast<uint2*>(p.q8 + orow_off + col0) = uint2{rc[0], rc[1]};
          }
        }
      if (qok && hh == 0) p.lse[(long)bh * p.T + q] = m + log2f(l);
    }
  }
  if (q8on) {  // workgroup max |O| (all waves reach this after their query tiles)
    q8max = warp_max(q8max);
    __syncthreads();
    if (lane == 0) red[wave] = q8max;
    __syncthreads();
    if (tid == 0) {
      float m8 = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) m8 = fmaxf(m8, red[w]);
      p.q8_part[bh] = m8;
    }
  }
}

}  // namespace

// PDT_FP8_ATTN_PV=1 (or pdt_attn_set_pv8(1)): the PV GEMM on e4m3 as well. Off by default:
// measured slower at ViT-B/16 bs 1024 (6.66 vs 5.27 ms per step over 12 layers: the
// per-pair softmax and the tr8 V reads lengthen the serial chain more than the 2x MFMA
// rate saves) and it adds ~1.5 % logits error (profiles/vit_b16_fp8_bs1024_step_round3_*).
static int g_attn_pv8 = -1;
static int attn_pv8() {
  if (g_attn_pv8 < 0) {
    const char* e = getenv("PDT_FP8_ATTN_PV");
    g_attn_pv8 = (e && e[0] == '1') ? 1 : 0;
  }
  return g_attn_pv8;
}
// PDT_ATTN_FWD_NW8=0: the 4-wave forward for T > 128 as well (A/B switch; 8 waves give each of
// the 7 query tiles of T = 197 its own wave instead of 2 rounds with one wave idle)
static int attn_fwd_nw8() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PDT_ATTN_FWD_NW8");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v;
}

PDT_API int pdt_attn_set_pv8(int on) {
  g_attn_pv8 = on ? 1 : 0;
  return 0;
}

// fp8 forward for T <= 256, head dim 64; -1 when the geometry is not covered
PDT_API int pdt_attn_fwd_f8(const void* qkv, void* out, float* lse, int B, int T, int H, float scale,
                            hipStream_t st) {
  if (T < 1 || T > 256) return -1;
  AttnF8Params p;
  p.qkv = (const u16*)qkv;
  p.out = (u16*)out;
  p.lse = lse;
  p.B = B; p.T = T; p.H = H;
  p.ld = 3L * H * D;
  p.ldo = (long)H * D;
  p.c = scale * 1.4426950408889634f;
  p.q8 = nullptr; p.q8_meta = nullptr; p.q8_part = nullptr;
  const int nkt = (T + 31) / 32;
  dim3 g(B * H);
  if (nkt >= 5 && !attn_pv8() && attn_fwd_nw8()) {  // 8 waves: one 32-query tile each (T = 197: 7)
    switch (nkt) {
      case 5: hipLaunchKernelGGL((attn_fwd_f8_kernel<5, true, false, 8, 0>), g, dim3(512), 0, st, p); break;
      case 6: hipLaunchKernelGGL((attn_fwd_f8_kernel<6, true, false, 8, 0>), g, dim3(512), 0, st, p); break;
      case 7: hipLaunchKernelGGL((attn_fwd_f8_kernel<7, true, false, 8, 0>), g, dim3(512), 0, st, p); break;
      default: hipLaunchKernelGGL((attn_fwd_f8_kernel<8, true, false, 8, 0>), g, dim3(512), 0, st, p); break;
    }
    PDT_RETURN_LAUNCH();
  }
#define F8(N)                                                                         \
  if (attn_pv8()) hipLaunchKernelGGL((attn_fwd_f8_kernel<N, true, true>), g, dim3(256), 0, st, p); \
  else hipLaunchKernelGGL((attn_fwd_f8_kernel<N, true, false>), g, dim3(256), 0, st, p)
  switch (nkt) {
    case 1: F8(1); break;
    case 2: F8(2); break;
    case 3: F8(3); break;
    case 4: F8(4); break;
    case 5: F8(5); break;
    case 6: F8(6); break;
    case 7: F8(7); break;
    default: F8(8); break;
  }
#undef F8
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_fp8_meta_roll_partial(float* meta, const float* partial, int nblk, int fmt, float* dq_out,
                                      hipStream_t st);

// pdt_attn_fwd_f8 that also writes the e4m3 codes of O for the projection GEMM (delayed scale
// q8_meta[0]), rolls that GEMM's amax history (q8_part: B*H floats) and writes the codes'
// dequant factor to q8_dq
PDT_API int pdt_attn_fwd_f8_q8(const void* qkv, void* out, float* lse, int B, int T, int H, float scale, void* q8,
                               float* q8_meta, float* q8_part, float* q8_dq, hipStream_t st) {
  if (T < 1 || T > 256 || !q8 || !q8_meta || !q8_part) return -1;
  AttnF8Params p;
  p.qkv = (const u16*)qkv;
  p.out = (u16*)out;
  p.lse = lse;
  p.B = B; p.T = T; p.H = H;
  p.ld = 3L * H * D;
  p.ldo = (long)H * D;
  p.c = scale * 1.4426950408889634f;
  p.q8 = (uint8_t*)q8; p.q8_meta = q8_meta; p.q8_part = q8_part;
  const int nkt = (T + 31) / 32;
  dim3 g(B * H);
  if (nkt >= 5 && !attn_pv8() && attn_fwd_nw8()) {  // 8 waves, as in pdt_attn_fwd_f8
    switch (nkt) {
      case 5: hipLaunchKernelGGL((attn_fwd_f8_kernel<5, true, false, 8, 1>), g, dim3(512), 0, st, p); break;
      case 6: hipLaunchKernelGGL((attn_fwd_f8_kernel<6, true, false, 8, 1>), g, dim3(512), 0, st, p); break;
      case 7: hipLaunchKernelGGL((attn_fwd_f8_kernel<7, true, false, 8, 1>), g, dim3(512), 0, st, p); break;
      default: hipLaunchKernelGGL((attn_fwd_f8_kernel<8, true, false, 8, 1>), g, dim3(512), 0, st, p); break;
    }
  } else {
#define F8(N)                                                                         \
  if (attn_pv8()) hipLaunchKernelGGL((attn_fwd_f8_kernel<N, true, true>), g, dim3(256), 0, st, p); \
  else hipLaunchKernelGGL((attn_fwd_f8_kernel<N, true, false>), g, dim3(256), 0, st, p)
    switch (nkt) {
      case 1: F8(1); break;
      case 2: F8(2); break;
      case 3: F8(3); break;
      case 4: F8(4); break;
      case 5: F8(5); break;
      case 6: F8(6); break;
      case 7: F8(7); break;
      default: F8(8); break;
    }
#undef F8
  }
  int e = (int)hipGetLastError();
  if (e) return e;
  return pdt_fp8_meta_roll_partial(q8_meta, q8_part, B * H, 0, q8_dq, st);
}

// the same kernel with a bf16 score GEMM (ViT bf16 forward); -1 when not covered
PDT_API int pdt_attn_fwd_tiles(const void* qkv, void* out, float* lse, int B, int T, int H, float scale,
                               hipStream_t st) {
  if (T < 1 || T > 256) return -1;
  AttnF8Params p;
  p.qkv = (const u16*)qkv;
  p.out = (u16*)out;
  p.lse = lse;
  p.B = B; p.T = T; p.H = H;
  p.ld = 3L * H * D;
  p.ldo = (long)H * D;
  p.c = scale * 1.4426950408889634f;
  p.q8 = nullptr; p.q8_meta = nullptr; p.q8_part = nullptr;
  const int nkt = (T + 31) / 32;
  dim3 g(B * H);
#define BF(N) hipLaunchKernelGGL((attn_fwd_f8_kernel<N, false>), g, dim3(256), 0, st, p)
  switch (nkt) {
    case 1: BF(1); break;
    case 2: BF(2); break;
    case 3: BF(3); break;
    case 4: BF(4); break;
    case 5: BF(5); break;
    case 6: BF(6); break;
    case 7: BF(7); break;
    default: BF(8); break;
  }
#undef BF
  PDT_RETURN_LAUNCH();
}
