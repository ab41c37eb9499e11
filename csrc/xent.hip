// Fused softmax cross-entropy (mean reduction, optional label smoothing),
// plus a column-sum kernel (bias gradients of nn.Linear).
// Reference op: log_softmax + nll_loss (/root/reference/model/model.py:22,
// /root/reference/model/loss.py:5) -- here a single online-softmax pass per row.
//
// forward : one wave per row: running max / sum-exp over V (16-B bf16 loads),
//           lse[row], loss[row] = lse - (1-eps)*x[t] - eps*mean(x)
//           then a one-block deterministic mean over rows.
// backward: dlogits = g/B * (softmax - (1-eps)*onehot - eps/V), bf16 out.
#include "pdt_common.h"

namespace {

__device__ __forceinline__ float ldx(const u16* p, long i) { return bf2f(p[i]); }

template <bool BF16>
__device__ __forceinline__ float ldv(const void* p, long i) {
  if (BF16) return bf2f(reinterpret_cast<const u16*>(p)[i]);
  return reinterpret_cast<const float*>(p)[i];
}

template <bool BF16>
__global__ void xent_fwd_kernel(const void* __restrict__ logits, const long* __restrict__ target,
                                float* __restrict__ lse, float* __restrict__ loss, int B, int V, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= B) return;
  const long base = (long)row * V;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  for (int j = lane; j < V; j += 64) {
    float v = ldv<BF16>(logits, base + j);
    sx += v;
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  }
  // combine (m, s) across lanes
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    float mm = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
    m = mm;
  }
  sx = warp_sum(sx);
  if (lane == 0) {
    float l = m + __logf(s);
    lse[row] = l;
    long t = target[row];
    float xt = (t >= 0 && t < V) ? ldv<BF16>(logits, base + t) : 0.f;
    loss[row] = (t >= 0 && t < V) ? (l - (1.f - eps) * xt - eps * (sx / V)) : 0.f;
  }
}

__global__ void mean_kernel(const float* __restrict__ x, float* __restrict__ out, int n, float scale) {
  __shared__ float red[256];
  float a = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) a += x[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0] * scale;
}

template <bool BF16>
__global__ void xent_bwd_kernel(const void* __restrict__ logits, const long* __restrict__ target,
                                const float* __restrict__ lse, const float* __restrict__ gout, u16* __restrict__ dlogits,
                                int B, int V, float eps) {
  const int row = blockIdx.y;
  const float g = gout[0] / B;
  const float l = lse[row];
  const long t = target[row];
  const long base = (long)row * V;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < V; j += gridDim.x * blockDim.x) {
    float p = __expf(ldv<BF16>(logits, base + j) - l);
    float d = p - eps / V - (j == t ? (1.f - eps) : 0.f);
    dlogits[base + j] = f2bf(t >= 0 && t < V ? g * d : 0.f);
  }
}

// Column sums of a bf16 [R][C] matrix into fp32 (bias gradients):
// stage 1: grid (ceil(C/64), G) blocks of 256 threads = 64 columns x 4 row
//          lanes; block (x, g) sums rows g*rpb .. (g+1)*rpb -> part[g][C]
// stage 2: out[c] = (acc ? out[c] : 0) + sum_g part[g][c]
__global__ void __launch_bounds__(256) colsum1_kernel(const u16* __restrict__ x, float* __restrict__ part, int R,
                                                      int C, int rpb) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * rpb, r1 = min(R, r0 + rpb);
  float s = 0.f;
  if (c < C)
    for (int r = r0 + rg; r < r1; r += 4) s += bf2f(x[(long)r * C + c]);
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < C) part[(long)blockIdx.y * C + c] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

// vectorised stage 1 for C % 8 == 0: thread = one 16-B chunk (8 columns) of a
// row; a block covers rp rows per pass of up to 256 chunks (blockIdx.y picks
// the chunk range) and strides over rows; rows combine in LDS -> part[g][C]
__global__ void __launch_bounds__(256) colsum1v_kernel(const u16* __restrict__ x, float* __restrict__ part, int R,
                                                       int C, int cpb) {
  __shared__ float red[256][9];
  const int t = threadIdx.x;
  const int cpr = C / 8;
  const int rp = 256 / cpb;
  const int ch = blockIdx.y * cpb + t % cpb, rr = t / cpb;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rr < rp && ch < cpr) {
    for (long r = (long)blockIdx.x * rp + rr; r < R; r += (long)gridDim.x * rp) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(x + r * C + ch * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[2 * e] += lo_bf(v[e]);
        s[2 * e + 1] += hi_bf(v[e]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[t][k] = s[k];
  __syncthreads();
  if (t < cpb && blockIdx.y * cpb + t < cpr) {
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < rp; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += red[j * cpb + t][k];
#pragma unroll
    for (int k = 0; k < 8; ++k) part[(long)blockIdx.x * C + (blockIdx.y * cpb + t) * 8 + k] = a[k];
  }
}

// stage 2: 256 threads = 64 columns x 4 row groups (fixed order -> deterministic)
__global__ void __launch_bounds__(256) colsum2_kernel(const float* __restrict__ part, float* __restrict__ out, int G,
                                                      int C, int acc) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < C)
    for (int g = rg; g < G; g += 4) s += part[(long)g * C + c];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < C) {
    const float t = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
    out[c] = acc ? out[c] + t : t;
  }
}

}  // namespace

PDT_API int pdt_xent_fwd(const void* logits, int bf16, const long* target, float* lse, float* loss_rows,
                         float* loss_out, int B, int V, float eps, hipStream_t st) {
  dim3 blk(256), grd((B + 3) / 4);
  if (bf16)
    hipLaunchKernelGGL(xent_fwd_kernel<true>, grd, blk, 0, st, logits, target, lse, loss_rows, B, V, eps);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<false>, grd, blk, 0, st, logits, target, lse, loss_rows, B, V, eps);
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, st, loss_rows, loss_out, B, 1.f / B);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_xent_bwd(const void* logits, int bf16, const long* target, const float* lse, const float* gout,
                         void* dlogits, int B, int V, float eps, hipStream_t st) {
  dim3 blk(256), grd((V + 255) / 256, B);
  if (bf16)
    hipLaunchKernelGGL(xent_bwd_kernel<true>, grd, blk, 0, st, logits, target, lse, gout, (u16*)dlogits, B, V, eps);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<false>, grd, blk, 0, st, logits, target, lse, gout, (u16*)dlogits, B, V,
                       eps);
  PDT_RETURN_LAUNCH();
}

// workspace floats pdt_colsum needs
// row groups of stage 1: enough blocks to fill 256 CUs several times over
static int colsum_groups(int R, int C) {
  int G = (R + 31) / 32;
  const int cap = C % 8 == 0 ? 512 : 128;
  if (G > cap) G = cap;
  if (G < 1) G = 1;
  return G;
}

PDT_API long pdt_colsum_workspace(int R, int C) { return (long)colsum_groups(R, C) * C; }

PDT_API int pdt_colsum(const void* x, float* out, float* work, int R, int C, int acc, hipStream_t st) {
  const int G = colsum_groups(R, C);
  int rpb = (R + G - 1) / G;
  if (C % 8 == 0) {
    const int cpr = C / 8;
    const int cpb = cpr < 256 ? cpr : 256;
    hipLaunchKernelGGL(colsum1v_kernel, dim3(G, (cpr + cpb - 1) / cpb), dim3(256), 0, st, (const u16*)x, work, R, C,
                       cpb);
  } else {
    hipLaunchKernelGGL(colsum1_kernel, dim3((C + 63) / 64, G), dim3(256), 0, st, (const u16*)x, work, R, C, rpb);
  }
  hipLaunchKernelGGL(colsum2_kernel, dim3((C + 63) / 64), dim3(256), 0, st, work, out, G, C, acc);
  PDT_RETURN_LAUNCH();
}
