// Small utility kernels: on-device synthetic data, fp32->bf16 casts, the
// cast+transpose that produces the data-gradient weight operand, bf16 adds.
#include "pdt_common.h"

namespace {
constexpr int NT = 256;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU;
  x ^= x >> 15; x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// uniform [-1, 1) bf16, 8 per thread, counter-based (same seed -> same data)
__global__ void fill_uniform_kernel(u16* __restrict__ out, long n8, uint32_t seed) {
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t h = hash32((uint32_t)(i * 8 + j) * 0x9E3779B9u ^ seed);
      f[j] = (float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f;
    }
    reinterpret_cast<u32x4*>(out)[i] =
        u32x4{pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7])};
  }
}

// Index-addressable synthetic images (data/synthetic.py SyntheticImageNet): sample i
// of the dataset is a pure function of (seed, i), so a DistributedSampler's index
// batch is materialised on the device in one launch. out: [B][HW][Cp] bf16 (NHWC,
// channel dim padded to Cp in storage, pad channels 0); labels[b] in [0, classes).
// One thread per (image, pixel, 4-channel group): one 8-byte store.
__global__ void synth_images_kernel(u16* __restrict__ out, const int64_t* __restrict__ idx, long B, int HW, int C,
                                    int Cp, uint32_t seed, int64_t* __restrict__ labels, int classes) {
  const int G = Cp / 4;
  const long total = B * HW * G;
  for (long t = (long)blockIdx.x * NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    const long pix = t / G;
    const int g = (int)(t - pix * G);
    const long b = pix / HW;
    const int p = (int)(pix - b * HW);
    const uint32_t s = hash32((uint32_t)idx[b] * 0x9E3779B9u ^ seed);
    float f[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = g * 4 + j;
      const uint32_t h = hash32((uint32_t)(p * C + c) * 0x85EBCA6Bu ^ s);
      f[j] = c < C ? (float)(h >> 8) * (2.0f / 16777216.0f) - 1.0f : 0.f;
    }
    reinterpret_cast<uint2*>(out)[t] = uint2{pack2bf(f[0], f[1]), pack2bf(f[2], f[3])};
    if (t < B) labels[t] = (int64_t)(hash32((uint32_t)idx[t] * 0xC2B2AE35u ^ seed ^ 0x5bd1e995u) % (uint32_t)classes);
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, u16* __restrict__ y, long n) {
  long n4 = n / 4;
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
    f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    uint2 w;
    w.x = pack2bf(v[0], v[1]);
    w.y = pack2bf(v[2], v[3]);
    reinterpret_cast<uint2*>(y)[i] = w;
  }
  for (long i = n4 * 4 + (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) y[i] = f2bf(x[i]);
}

// out[ci][th][tw][co] = W[co][kh0 + s*th][kw0 + s*tw][ci]   (W fp32 [Cout][KH][KW][Cin])
__global__ void wt_dgrad_kernel(const float* __restrict__ w, u16* __restrict__ out, int Cout, int KH, int KW,
                                int Cin, int kh0, int kw0, int s, int nth, int ntw) {
  long total = (long)Cin * nth * ntw * Cout;
  for (long t = (long)blockIdx.x * NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    int co = t % Cout;
    long r = t / Cout;
    int tw = r % ntw; r /= ntw;
    int th = r % nth;
    int ci = r / nth;
    int kh = kh0 + s * th, kw = kw0 + s * tw;
    out[t] = f2bf(w[(((long)co * KH + kh) * KW + kw) * Cin + ci]);
  }
}

// Many wt_dgrad jobs in one launch (all conv weights of a model after an
// optimizer step): job j covers elements [start_j, start_{j+1}) of the flat
// index space; a thread finds its job by binary search over the starts.
struct WtJob {
  const float* w;
  u16* out;
  long start;
  int Cout, KH, KW, Cin, kh0, kw0, s, nth, ntw, pad;
};

__global__ void wt_dgrad_multi_kernel(const WtJob* __restrict__ jobs, int njobs, long total) {
  __shared__ long starts[512];  // job starts staged once per block (njobs <= 512 checked on the host)
  for (int i = threadIdx.x; i < njobs; i += NT) starts[i] = jobs[i].start;
  __syncthreads();
  for (long t = (long)blockIdx.x * NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (starts[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const WtJob& J = jobs[lo];
    long e = t - J.start;
    const int co = e % J.Cout;
    long r = e / J.Cout;
    const int tw = r % J.ntw;
    r /= J.ntw;
    const int th = r % J.nth;
    const int ci = r / J.nth;
    const int kh = J.kh0 + J.s * th, kw = J.kw0 + J.s * tw;
    J.out[e] = f2bf(J.w[(((long)co * J.KH + kh) * J.KW + kw) * J.Cin + ci]);
  }
}

// out[r][c] = W[c][r] for a [R][C] fp32 matrix -> bf16 [C][R]
__global__ void transpose_cast_kernel(const float* __restrict__ w, u16* __restrict__ out, int R, int C) {
  __shared__ float tile[32][33];
  int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int j = ty; j < 32; j += 8) {
    int r = by + j, c = bx + tx;
    tile[j][tx] = (r < R && c < C) ? w[(long)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    int c = bx + j, r = by + tx;
    if (c < C && r < R) out[(long)c * R + r] = f2bf(tile[tx][j]);
  }
}

// y = a + b (bf16, n % 8 == 0)
__global__ void add_bf16_kernel(const u16* __restrict__ a, const u16* __restrict__ b, u16* __restrict__ y, long n8) {
  for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    u32x4 va = reinterpret_cast<const u32x4*>(a)[i], vb = reinterpret_cast<const u32x4*>(b)[i];
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = pack2bf(lo_bf(va[k]) + lo_bf(vb[k]), hi_bf(va[k]) + hi_bf(vb[k]));
    reinterpret_cast<u32x4*>(y)[i] = o;
  }
}

int grid_for(long n) {
  long b = (n + NT - 1) / NT;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}
}  // namespace

PDT_API int pdt_fill_uniform_bf16(void* out, long n, unsigned seed, hipStream_t st) {
  if (n % 8) return -1;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3(grid_for(n / 8)), dim3(NT), 0, st, (u16*)out, n / 8, seed);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_synth_images_bf16(void* out, const int64_t* idx, long B, int HW, int C, int Cp, unsigned seed,
                                  int64_t* labels, int classes, hipStream_t st) {
  if (B <= 0 || HW <= 0 || C <= 0 || Cp % 4 || C > Cp || classes <= 0 || (long)HW * Cp * B >= (1L << 40)) return -1;
  const long n = B * HW * (Cp / 4);
  if (n < B) return -1;  // the label writes ride on the first B threads
  hipLaunchKernelGGL(synth_images_kernel, dim3(grid_for(n)), dim3(NT), 0, st, (u16*)out, idx, B, HW, C, Cp, seed,
                     labels, classes);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_cast_f32_bf16(const float* x, void* y, long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n / 4 + 1)), dim3(NT), 0, st, x, (u16*)y, n);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_wt_dgrad(const float* w, void* out, int Cout, int KH, int KW, int Cin, int kh0, int kw0, int s,
                         int nth, int ntw, hipStream_t st) {
  long total = (long)Cin * nth * ntw * Cout;
  if (total == 0) return 0;
  hipLaunchKernelGGL(wt_dgrad_kernel, dim3(grid_for(total)), dim3(NT), 0, st, w, (u16*)out, Cout, KH, KW, Cin, kh0,
                     kw0, s, nth, ntw);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_wt_job_size() { return (int)sizeof(WtJob); }

// jobs: device array of WtJob (host-packed, see native_ops._DgradWeights)
PDT_API int pdt_wt_dgrad_multi(const void* jobs, int njobs, long total, hipStream_t st) {
  if (njobs <= 0 || total <= 0) return 0;
  if (njobs > 512) return -1;
  long g = (total + NT - 1) / NT;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(wt_dgrad_multi_kernel, dim3((unsigned)g), dim3(NT), 0, st, (const WtJob*)jobs, njobs, total);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_transpose_cast(const float* w, void* out, int R, int C, hipStream_t st) {
  dim3 g((C + 31) / 32, (R + 31) / 32);
  hipLaunchKernelGGL(transpose_cast_kernel, g, dim3(256), 0, st, w, (u16*)out, R, C);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_add_bf16(const void* a, const void* b, void* y, long n, hipStream_t st) {
  if (n % 8) return -1;
  hipLaunchKernelGGL(add_bf16_kernel, dim3(grid_for(n / 8)), dim3(NT), 0, st, (const u16*)a, (const u16*)b, (u16*)y,
                     n / 8);
  PDT_RETURN_LAUNCH();
}

// Probe of the cross-lane reduction primitives (pdt_common.h) for the unit tests: one
// wave per 64 inputs; out[6][n] = row16_sum, row8_sum, xor16+xor32 sum (4 lanes l^16k),
// xor32 max, warp_sum, warp_max of each lane's value.
__global__ void __launch_bounds__(64) lane_reduce_probe_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                               int n) {
  const int i = blockIdx.x * 64 + threadIdx.x;  // n is a multiple of 64 (host check)
  const float v = x[i];
  out[i] = row16_sum(v);
  out[n + i] = row8_sum(v);
  out[2 * n + i] = xor32_reduce(xor16_reduce(v, AddOp{}), AddOp{});
  out[3 * n + i] = xor32_reduce(v, MaxOp{});
  out[4 * n + i] = warp_sum(v);
  out[5 * n + i] = warp_max(v);
}

PDT_API int pdt_lane_reduce_probe(const float* x, float* out, int n, hipStream_t st) {
  if (n <= 0 || n % 64) return -1;
  hipLaunchKernelGGL(lane_reduce_probe_kernel, dim3(n / 64), dim3(64), 0, st, x, out, n);
  PDT_RETURN_LAUNCH();
}
