// The reference's demo model, MnistModel (/root/reference/model/model.py:6-22), as
// two whole-network kernels plus the NLL loss (/root/reference/model/loss.py:4-5).
//
//   conv1 1->10 k5 -> max_pool 2 -> relu -> conv2 10->20 k5 -> Dropout2d -> max_pool 2
//   -> relu -> flatten(320, NCHW order) -> fc1 320->50 -> relu -> dropout -> fc2 50->NC
//   -> log_softmax
//
// At MNIST sizes (28x28, 21,840 parameters, ~0.5 MFLOP per image) every layer is a
// few microseconds of work, so a layer-per-launch design is launch-latency bound
// (~15 launches forward, ~30 backward). Here ONE workgroup owns ONE image and runs
// the whole network out of LDS: lenet_fwd writes only the log-probabilities;
// lenet_bwd recomputes the forward in LDS (cheaper than saving and re-reading the
// activations) and writes one row of per-image parameter-gradient partials, which
// lenet_grad_reduce sums over the batch in a fixed order (deterministic, no atomics).
// Everything stays fp32, like the reference model.
//
// Dropout masks come from a counter-based hash of (seed, image, unit), so the
// backward regenerates exactly the forward's mask without storing it; kept units
// are scaled by 1 / (1 - p) (torch's inverted dropout).
#include "pdt_common.h"

namespace {

constexpr int NT = 256;
constexpr int IH = 28, K5 = 5;
constexpr int C1 = 10, H1 = 24, P1 = 12;  // conv1 output 24x24, pooled 12x12
constexpr int C2 = 20, H2 = 8, P2 = 4;    // conv2 output 8x8, pooled 4x4
constexpr int F0 = C2 * P2 * P2;          // 320
constexpr int F1 = 50;
constexpr int MAXNC = 64;

// offsets of each parameter's gradient in one per-image partial row
constexpr int O_W1 = 0, O_B1 = O_W1 + C1 * K5 * K5, O_W2 = O_B1 + C1, O_B2 = O_W2 + C2 * C1 * K5 * K5,
              O_WF1 = O_B2 + C2, O_BF1 = O_WF1 + F1 * F0, O_WF2 = O_BF1 + F1;
__host__ __device__ constexpr int grad_row(int nc) { return O_WF2 + F1 * nc + nc; }

struct LeNetArgs {
  const float* x;  // [B][1][28][28]
  const float *w1, *b1, *w2, *b2, *wf1, *bf1, *wf2, *bf2;
  int B, NC, training;
  float p2, p1;  // Dropout2d / dropout probabilities
  uint32_t seed;
};

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x7feb352du;
  h ^= h >> 15; h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

// inverted-dropout multiplier of unit u of image b (0 or 1/(1-p))
__device__ __forceinline__ float keep_mult(uint32_t seed, int b, int u, float p) {
  if (p <= 0.f) return 1.f;
  if (p >= 1.f) return 0.f;
  const uint32_t h = mix32(seed ^ mix32((uint32_t)b * 0x9E3779B9u + (uint32_t)u * 0x85EBCA6Bu + 0x632BE5ABu));
  const float r = (float)(h >> 8) * (1.f / 16777216.f);
  return r >= p ? 1.f / (1.f - p) : 0.f;
}

struct FwdSmem {
  float x[IH * IH];
  float w1[C1 * K5 * K5], b1[C1];
  float h1[C1 * P1 * P1];  // pooled + relu conv1
  uint8_t a1[C1 * P1 * P1];  // argmax (dy*2+dx) in each 2x2 window
  float w2[C2 * C1 * K5 * K5], b2[C2];
  float c2[C2 * H2 * H2];  // conv2 output (pre-dropout)
  float h2[F0];            // pooled + relu(dropout2d(conv2)) -- the flattened fc1 input
  uint8_t a2[F0];
  float keep2[C2], keep1[MAXNC];
  float z1[MAXNC], f1[MAXNC];  // fc1 pre-activation, post relu+dropout
  float z2[MAXNC], lp[MAXNC];  // logits, log-probabilities
};

// Forward of image b into LDS (all threads participate; ends with a barrier). The conv
// weights are staged only when `weights` (a workgroup looping over images keeps them).
__device__ void lenet_forward(const LeNetArgs& a, int b, FwdSmem& s, bool weights = true) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* xb = a.x + (size_t)b * IH * IH;
  for (int i = tid; i < IH * IH; i += NT) s.x[i] = xb[i];
  if (weights) {
    for (int i = tid; i < C1 * K5 * K5; i += NT) s.w1[i] = a.w1[i];
    for (int i = tid; i < C2 * C1 * K5 * K5; i += NT) s.w2[i] = a.w2[i];
    if (tid < C1) s.b1[tid] = a.b1[tid];
    if (tid < C2) s.b2[tid] = a.b2[tid];
  }
  if (tid < C2) s.keep2[tid] = a.training ? keep_mult(a.seed, b, tid, a.p2) : 1.f;
  if (tid < F1) s.keep1[tid] = a.training ? keep_mult(a.seed, b, 64 + tid, a.p1) : 1.f;
  __syncthreads();

  // conv1 + 2x2 max-pool + relu, one pooled cell per thread-iteration
  for (int i = tid; i < C1 * P1 * P1; i += NT) {
    const int c = i / (P1 * P1), py = (i / P1) % P1, px = i % P1;
    const float* w = s.w1 + c * K5 * K5;
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int oy = 2 * py + (d >> 1), ox = 2 * px + (d & 1);
      float acc = s.b1[c];
#pragma unroll
      for (int kh = 0; kh < K5; ++kh)
#pragma unroll
        for (int kw = 0; kw < K5; ++kw) acc = fmaf(w[kh * K5 + kw], s.x[(oy + kh) * IH + ox + kw], acc);
      if (acc > best) { best = acc; arg = d; }
    }
    s.h1[i] = fmaxf(best, 0.f);
    s.a1[i] = (uint8_t)arg;
  }
  __syncthreads();

  // conv2 (every output position; pooled afterwards)
  for (int i = tid; i < C2 * H2 * H2; i += NT) {
    const int c = i / (H2 * H2), oy = (i / H2) % H2, ox = i % H2;
    float acc = s.b2[c];
    for (int ci = 0; ci < C1; ++ci) {
      const float* w = s.w2 + (c * C1 + ci) * K5 * K5;
      const float* h = s.h1 + ci * P1 * P1;
#pragma unroll
      for (int kh = 0; kh < K5; ++kh)
#pragma unroll
        for (int kw = 0; kw < K5; ++kw) acc = fmaf(w[kh * K5 + kw], h[(oy + kh) * P1 + ox + kw], acc);
    }
    s.c2[i] = acc;
  }
  __syncthreads();

  // Dropout2d (channel multiplier) -> 2x2 max-pool -> relu
  for (int i = tid; i < F0; i += NT) {
    const int c = i / (P2 * P2), py = (i / P2) % P2, px = i % P2;
    const float k = s.keep2[c];
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const float v = k * s.c2[(c * H2 + 2 * py + (d >> 1)) * H2 + 2 * px + (d & 1)];
      if (v > best) { best = v; arg = d; }
    }
    s.h2[i] = fmaxf(best, 0.f);
    s.a2[i] = (uint8_t)arg;
  }
  __syncthreads();

  // fc1 + relu + dropout: one wave per output row, lanes split K
  for (int j = wave; j < F1; j += NT / 64) {
    const float* w = a.wf1 + (size_t)j * F0;
    float acc = 0.f;
    for (int k = lane; k < F0; k += 64) acc = fmaf(w[k], s.h2[k], acc);
    acc = warp_sum(acc) + a.bf1[j];
    if (lane == 0) {
      s.z1[j] = acc;
      s.f1[j] = fmaxf(acc, 0.f) * s.keep1[j];
    }
  }
  __syncthreads();

  // fc2
  for (int c = wave; c < a.NC; c += NT / 64) {
    float v = lane < F1 ? a.wf2[(size_t)c * F1 + lane] * s.f1[lane] : 0.f;
    v = warp_sum(v) + a.bf2[c];
    if (lane == 0) s.z2[c] = v;
  }
  __syncthreads();

  // log_softmax over the NC logits (one wave)
  if (wave == 0) {
    const float z = lane < a.NC ? s.z2[lane] : -INFINITY;
    const float m = warp_max(z);
    const float e = lane < a.NC ? __expf(z - m) : 0.f;
    const float lse = m + __logf(warp_sum(e));
    if (lane < a.NC) s.lp[lane] = z - lse;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(NT) lenet_fwd_kernel(LeNetArgs a, float* __restrict__ logp,
                                                       uint8_t* __restrict__ mask2, uint8_t* __restrict__ mask1) {
  __shared__ FwdSmem s;
  const int b = blockIdx.x;
  lenet_forward(a, b, s);
  const int tid = threadIdx.x;
  if (tid < a.NC) logp[(size_t)b * a.NC + tid] = s.lp[tid];
  if (mask2 && tid < C2) mask2[b * C2 + tid] = s.keep2[tid] != 0.f;
  if (mask1 && tid < F1) mask1[b * F1 + tid] = s.keep1[tid] != 0.f;
}

struct BwdSmem {
  float g[MAXNC], dz2[MAXNC], dz1[MAXNC];
  float dh2[F0];
  float dc2[C2 * H2 * H2];
  float dh1[C1 * P1 * P1];
  float dp1[C1 * P1 * P1];  // pooled-cell gradient of conv1's output (at the argmax position)
};

// One workgroup per `per` consecutive images: each image's parameter gradient is added into
// an LDS row (24.6 K floats), written once per workgroup -- at batch 1024 the per-image rows
// were 89 MB of partials (the fc1 outer products) and the kernel fell behind the stock ops.
__global__ void __launch_bounds__(NT) lenet_bwd_kernel(LeNetArgs a, const float* __restrict__ dlogp,
                                                       float* __restrict__ part, int per) {
  __shared__ FwdSmem s;
  __shared__ BwdSmem t;
  __shared__ float pr[grad_row(MAXNC)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = grad_row(a.NC);
  for (int i = tid; i < row; i += NT) pr[i] = 0.f;
  for (int img = 0; img < per; ++img) {
  const int b = blockIdx.x * per + img;
  if (b >= a.B) break;  // uniform over the workgroup
  lenet_forward(a, b, s, img == 0);

  // log_softmax backward: dz = g - softmax * sum(g)
  if (wave == 0) {
    const float g = lane < a.NC ? dlogp[(size_t)b * a.NC + lane] : 0.f;
    const float sg = warp_sum(g);
    if (lane < a.NC) t.dz2[lane] = g - __expf(s.lp[lane]) * sg;
  }
  __syncthreads();

  // fc2: dW = dz2 (x) f1, db = dz2, df1 = W^T dz2 -> through dropout + relu -> dz1
  for (int e = tid; e < a.NC * F1; e += NT) pr[O_WF2 + e] += t.dz2[e / F1] * s.f1[e % F1];
  if (tid < a.NC) pr[O_WF2 + a.NC * F1 + tid] += t.dz2[tid];
  if (tid < F1) {
    float d = 0.f;
    for (int c = 0; c < a.NC; ++c) d = fmaf(a.wf2[(size_t)c * F1 + tid], t.dz2[c], d);
    t.dz1[tid] = s.z1[tid] > 0.f ? d * s.keep1[tid] : 0.f;
  }
  __syncthreads();

  // fc1: dW = dz1 (x) h2, db = dz1, dh2 = W^T dz1 (coalesced over k for each row j)
  for (int e = tid; e < F1 * F0; e += NT) pr[O_WF1 + e] += t.dz1[e / F0] * s.h2[e % F0];
  if (tid < F1) pr[O_BF1 + tid] += t.dz1[tid];
  for (int k = tid; k < F0; k += NT) {
    float d = 0.f;
    for (int j = 0; j < F1; ++j) d = fmaf(a.wf1[(size_t)j * F0 + k], t.dz1[j], d);
    t.dh2[k] = d;
  }
  for (int i = tid; i < C2 * H2 * H2; i += NT) t.dc2[i] = 0.f;
  __syncthreads();

  // relu -> max-pool -> Dropout2d backward: the gradient lands on each window's argmax
  for (int i = tid; i < F0; i += NT) {
    const int c = i / (P2 * P2), py = (i / P2) % P2, px = i % P2, d = s.a2[i];
    const float g = s.h2[i] > 0.f ? t.dh2[i] * s.keep2[c] : 0.f;
    t.dc2[(c * H2 + 2 * py + (d >> 1)) * H2 + 2 * px + (d & 1)] = g;
  }
  __syncthreads();

  // conv2: dW[co][ci][kh][kw] = sum_pos dc2 * h1, db = sum_pos dc2
  for (int e = tid; e < C2 * C1 * K5 * K5; e += NT) {
    const int co = e / (C1 * K5 * K5), ci = (e / (K5 * K5)) % C1, kh = (e / K5) % K5, kw = e % K5;
    const float* dc = t.dc2 + co * H2 * H2;
    const float* h = s.h1 + ci * P1 * P1 + kh * P1 + kw;
    float acc = 0.f;
#pragma unroll
    for (int oy = 0; oy < H2; ++oy)
#pragma unroll
      for (int ox = 0; ox < H2; ++ox) acc = fmaf(dc[oy * H2 + ox], h[oy * P1 + ox], acc);
    pr[O_W2 + e] += acc;
  }
  if (tid < C2) {
    float acc = 0.f;
    for (int q = 0; q < H2 * H2; ++q) acc += t.dc2[tid * H2 * H2 + q];
    pr[O_B2 + tid] += acc;
  }
  // conv2 data gradient (full correlation with the flipped kernel), then relu -> pool1
  for (int i = tid; i < C1 * P1 * P1; i += NT) {
    const int ci = i / (P1 * P1), y = (i / P1) % P1, x = i % P1;
    float acc = 0.f;
    for (int co = 0; co < C2; ++co) {
      const float* w = s.w2 + (co * C1 + ci) * K5 * K5;
      const float* dc = t.dc2 + co * H2 * H2;
#pragma unroll
      for (int kh = 0; kh < K5; ++kh) {
        const int oy = y - kh;
        if (oy < 0 || oy >= H2) continue;
#pragma unroll
        for (int kw = 0; kw < K5; ++kw) {
          const int ox = x - kw;
          if (ox >= 0 && ox < H2) acc = fmaf(w[kh * K5 + kw], dc[oy * H2 + ox], acc);
        }
      }
    }
    t.dh1[i] = acc;
    t.dp1[i] = s.h1[i] > 0.f ? acc : 0.f;  // relu(max_pool(.)) backward, still at the pooled cell
  }
  __syncthreads();

  // conv1: dW[c][kh][kw] = sum over pooled cells of dp1 * x at the window's argmax, db = sum dp1
  for (int e = tid; e < C1 * K5 * K5; e += NT) {
    const int c = e / (K5 * K5), kh = (e / K5) % K5, kw = e % K5;
    float acc = 0.f;
    for (int q = 0; q < P1 * P1; ++q) {
      const int i = c * P1 * P1 + q, d = s.a1[i];
      const int oy = 2 * (q / P1) + (d >> 1), ox = 2 * (q % P1) + (d & 1);
      acc = fmaf(t.dp1[i], s.x[(oy + kh) * IH + ox + kw], acc);
    }
    pr[O_W1 + e] += acc;
  }
  if (tid < C1) {
    float acc = 0.f;
    for (int q = 0; q < P1 * P1; ++q) acc += t.dp1[tid * P1 * P1 + q];
    pr[O_B1 + tid] += acc;
  }
  __syncthreads();  // the next image overwrites the forward / backward scratch
  }
  float* out = part + (size_t)blockIdx.x * row;
  for (int i = tid; i < row; i += NT) out[i] = pr[i];
}

// out[j] = sum_b part[b][j] (fixed order: deterministic)
__global__ void __launch_bounds__(NT) lenet_grad_reduce_kernel(const float* __restrict__ part, int B, int row,
                                                               float* __restrict__ out) {
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= row) return;
  float acc = 0.f;
  for (int b = 0; b < B; ++b) acc += part[(size_t)b * row + j];
  out[j] = acc;
}

// NLL loss (mean over targets != ignore_index) of log-probabilities [B][C].
// A target outside [0, C) that is not ignore_index is an error (torch raises): the
// kernel counts them into bad[0] (the host checks it lazily, without a sync in the
// step) and poisons the loss with a NaN so the error cannot train silently.
__global__ void __launch_bounds__(NT) nll_fwd_kernel(const float* __restrict__ logp, const int64_t* __restrict__ tgt,
                                                     int B, int C, int ignore, float* __restrict__ loss,
                                                     float* __restrict__ count, float* __restrict__ bad) {
  __shared__ float rs[NT / 64], rc[NT / 64], rb[NT / 64];
  float s = 0.f, n = 0.f, nb = 0.f;
  for (int i = threadIdx.x; i < B; i += NT) {
    const int64_t t = tgt[i];
    if (t == ignore) continue;
    if (t < 0 || t >= C) {
      nb += 1.f;
      continue;
    }
    s -= logp[(size_t)i * C + t];
    n += 1.f;
  }
  s = warp_sum(s);
  n = warp_sum(n);
  nb = warp_sum(nb);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { rs[wave] = s; rc[wave] = n; rb[wave] = nb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float S = 0.f, Nn = 0.f, Nb = 0.f;
    for (int w = 0; w < NT / 64; ++w) { S += rs[w]; Nn += rc[w]; Nb += rb[w]; }
    loss[0] = Nb > 0.f ? __builtin_nanf("") : S / Nn;  // NaN when every target is ignored, as torch
    count[0] = Nn;
    bad[0] = Nb;
  }
}

__global__ void __launch_bounds__(NT) nll_bwd_kernel(const int64_t* __restrict__ tgt, const float* __restrict__ g,
                                                     const float* __restrict__ count, int B, int C, int ignore,
                                                     float* __restrict__ dlogp) {
  const int e = blockIdx.x * NT + threadIdx.x;
  if (e >= B * C) return;
  const int i = e / C, c = e % C;
  const int64_t t = tgt[i];
  dlogp[e] = (t == c && t != ignore) ? -g[0] / count[0] : 0.f;  // (out-of-range t never equals c)
}

bool bad_args(const LeNetArgs& a) { return a.B <= 0 || a.NC <= 0 || a.NC > MAXNC; }

}  // namespace

PDT_API int pdt_lenet_grad_row(int nc) { return grad_row(nc); }

PDT_API int pdt_lenet_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                          const float* wf1, const float* bf1, const float* wf2, const float* bf2, int B, int NC,
                          int training, float p2, float p1, unsigned seed, float* logp, uint8_t* mask2,
                          uint8_t* mask1, hipStream_t st) {
  LeNetArgs a{x, w1, b1, w2, b2, wf1, bf1, wf2, bf2, B, NC, training, p2, p1, seed};
  if (bad_args(a)) return -1;
  hipLaunchKernelGGL(lenet_fwd_kernel, dim3(B), dim3(NT), 0, st, a, logp, mask2, mask1);
  PDT_RETURN_LAUNCH();
}

// part: [B][grad_row(NC)] scratch (the first ceil(B / ceil(B / 256)) rows are used); grads:
// [grad_row(NC)] flat output (see O_* layout)
PDT_API int pdt_lenet_bwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                          const float* wf1, const float* bf1, const float* wf2, const float* bf2, int B, int NC,
                          int training, float p2, float p1, unsigned seed, const float* dlogp, float* part,
                          float* grads, hipStream_t st) {
  LeNetArgs a{x, w1, b1, w2, b2, wf1, bf1, wf2, bf2, B, NC, training, p2, p1, seed};
  if (bad_args(a)) return -1;
  // one workgroup per CU at most (the LDS gradient row), each looping over `per` images
  const int per = (B + 255) / 256, nwg = (B + per - 1) / per;
  hipLaunchKernelGGL(lenet_bwd_kernel, dim3(nwg), dim3(NT), 0, st, a, dlogp, part, per);
  const int row = grad_row(NC);
  hipLaunchKernelGGL(lenet_grad_reduce_kernel, dim3((row + NT - 1) / NT), dim3(NT), 0, st, part, nwg, row, grads);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_nll_fwd(const float* logp, const int64_t* tgt, int B, int C, int ignore, float* loss, float* count,
                        float* bad, hipStream_t st) {
  if (B <= 0 || C <= 0) return -1;
  hipLaunchKernelGGL(nll_fwd_kernel, dim3(1), dim3(NT), 0, st, logp, tgt, B, C, ignore, loss, count, bad);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_nll_bwd(const int64_t* tgt, const float* g, const float* count, int B, int C, int ignore,
                        float* dlogp, hipStream_t st) {
  if (B <= 0 || C <= 0) return -1;
  hipLaunchKernelGGL(nll_bwd_kernel, dim3((B * C + NT - 1) / NT), dim3(NT), 0, st, tgt, g, count, B, C, ignore,
                     dlogp);
  PDT_RETURN_LAUNCH();
}
