// Multi-tensor fused optimizer steps (one launch for every parameter tensor).
// Reference: torch.optim.Adam(amsgrad) step (/root/reference/config/config.json:38-45,
// /root/reference/trainer/trainer.py:58); SGD-momentum is the ResNet recipe.
//
// Work list: the host builds, once per parameter set, a device table of
// chunks {tensor id, element offset, length}; each workgroup walks chunks with
// a grid-stride loop and reads the tensor's pointers from a pointer table.
// fp32 master params / grads / states; optionally a bf16 shadow copy of each
// param is written in the same pass (the copy the bf16 conv/GEMM kernels read),
// so no separate cast kernel runs per step.
#include "pdt_common.h"

namespace {

struct Chunk {
  int tensor;
  int pad;
  long offset;
  long len;
};

constexpr int NT = 256;

// SGD (torch semantics): g += wd*p; buf = mom*buf + (1-damp)*g (buf = g on
// first step); g = nesterov ? g + mom*buf : buf; p -= lr*g
__global__ void sgd_kernel(const Chunk* __restrict__ chunks, int nchunks, float* const* __restrict__ params,
                           const float* const* __restrict__ grads, float* const* __restrict__ bufs,
                           u16* const* __restrict__ shadows, float lr, float momentum, float dampening, float wd,
                           int nesterov, int first, float grad_scale, const float* __restrict__ dev) {
  if (dev != nullptr) lr = dev[0];  // capturable: the lr a replayed graph must not freeze
  // one element: returns the new parameter, updates the momentum buffer value in place
  auto upd = [&](float gi, float pi, float& bi, bool has_b) {
    gi *= grad_scale;
    if (wd != 0.f) gi += wd * pi;
    if (momentum != 0.f && has_b) {
      bi = first ? gi : momentum * bi + (1.f - dampening) * gi;
      gi = nesterov ? gi + momentum * bi : bi;
    }
    return pi - lr * gi;
  };
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const Chunk ch = chunks[c];
    float* p = params[ch.tensor] + ch.offset;
    const float* g = grads[ch.tensor] + ch.offset;
    float* b = bufs ? (bufs[ch.tensor] ? bufs[ch.tensor] + ch.offset : nullptr) : nullptr;
    u16* sh = shadows ? (shadows[ch.tensor] ? shadows[ch.tensor] + ch.offset : nullptr) : nullptr;
    const bool hb = b != nullptr;
    long i0 = 0;
    // 16-B vector path when every stream is aligned (gradients can be unaligned views
    // into DDP's buckets): 4 elements per lane, all loads issued before the math
    const uintptr_t al = (uintptr_t)p | (uintptr_t)g | (hb ? (uintptr_t)b : 0);
    if ((al & 15) == 0 && (!sh || ((uintptr_t)sh & 7) == 0)) {
      const long n4 = ch.len >> 2;
      for (long j = threadIdx.x; j < n4; j += NT) {
        const f32x4 gv = reinterpret_cast<const f32x4*>(g)[j];
        f32x4 pv = reinterpret_cast<const f32x4*>(p)[j];
        f32x4 bv = hb ? reinterpret_cast<const f32x4*>(b)[j] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float be = bv[e];
          pv[e] = upd(gv[e], pv[e], be, hb);
          bv[e] = be;
        }
        reinterpret_cast<f32x4*>(p)[j] = pv;
        if (hb && momentum != 0.f) reinterpret_cast<f32x4*>(b)[j] = bv;
        if (sh) {
          uint2 w;
          w.x = pack2bf(pv[0], pv[1]);
          w.y = pack2bf(pv[2], pv[3]);
          reinterpret_cast<uint2*>(sh)[j] = w;
        }
      }
      i0 = n4 << 2;
    }
    for (long i = i0 + threadIdx.x; i < ch.len; i += NT) {
      float bi = hb ? b[i] : 0.f;
      const float pi = upd(g[i], p[i], bi, hb);
      if (hb && momentum != 0.f) b[i] = bi;
      p[i] = pi;
      if (sh) sh[i] = f2bf(pi);
    }
  }
}

// Adam / AdamW (decoupled=1), optional AMSGrad. bc1 = 1-b1^t, bc2 = 1-b2^t.
__global__ void adam_kernel(const Chunk* __restrict__ chunks, int nchunks, float* const* __restrict__ params,
                            const float* const* __restrict__ grads, float* const* __restrict__ exp_avg,
                            float* const* __restrict__ exp_avg_sq, float* const* __restrict__ max_sq,
                            u16* const* __restrict__ shadows, float lr, float b1, float b2, float eps, float wd,
                            int decoupled, float bc1, float bc2, float grad_scale, const float* __restrict__ dev) {
  if (dev != nullptr) {  // capturable: lr and the step count t live in device memory
    lr = dev[0];
    bc1 = 1.f - powf(b1, dev[1]);
    bc2 = 1.f - powf(b2, dev[1]);
  }
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const Chunk ch = chunks[c];
    float* p = params[ch.tensor] + ch.offset;
    const float* g = grads[ch.tensor] + ch.offset;
    float* m = exp_avg[ch.tensor] + ch.offset;
    float* v = exp_avg_sq[ch.tensor] + ch.offset;
    float* vm = max_sq ? max_sq[ch.tensor] + ch.offset : nullptr;
    u16* sh = shadows ? (shadows[ch.tensor] ? shadows[ch.tensor] + ch.offset : nullptr) : nullptr;
    for (long i = threadIdx.x; i < ch.len; i += NT) {
      float gi = g[i] * grad_scale;
      float pi = p[i];
      if (wd != 0.f) {
        if (decoupled) pi *= (1.f - lr * wd);
        else gi += wd * pi;
      }
      float mi = b1 * m[i] + (1.f - b1) * gi;
      float vi = b2 * v[i] + (1.f - b2) * gi * gi;
      m[i] = mi;
      v[i] = vi;
      float vv = vi;
      if (vm) {
        vv = fmaxf(vm[i], vi);
        vm[i] = vv;
      }
      float denom = sqrtf(vv) * inv_sqrt_bc2 + eps;
      pi -= step_size * mi / denom;
      p[i] = pi;
      if (sh) sh[i] = f2bf(pi);
    }
  }
}

int grid_for(int n) { return n < 2048 ? (n < 1 ? 1 : n) : 2048; }

// capturable Adam: t += 1 on the device, ahead of the step kernel in the same stream
__global__ void opt_tick_kernel(float* dev) {
  if (threadIdx.x == 0) dev[1] += 1.f;
}

}  // namespace

PDT_API int pdt_chunk_struct_size() { return (int)sizeof(Chunk); }

// dev (optional, "capturable"): [lr] for SGD, [lr, t] for Adam in device memory, read by the
// kernels instead of the lr / bias-correction arguments, so a HIP graph that captured the step
// replays it with the current learning rate and step count (the host rewrites dev[0] when the
// lr changes; Adam's t is incremented on the device by opt_tick_kernel when tick != 0).
PDT_API int pdt_sgd_step2(const void* chunks, int nchunks, void* params, const void* grads, void* bufs, void* shadows,
                          float lr, float momentum, float dampening, float wd, int nesterov, int first,
                          float grad_scale, const float* dev, hipStream_t st) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(nchunks)), dim3(NT), 0, st, (const Chunk*)chunks, nchunks,
                     (float* const*)params, (const float* const*)grads, (float* const*)bufs,
                     (u16* const*)shadows, lr, momentum, dampening, wd, nesterov, first, grad_scale, dev);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_sgd_step(const void* chunks, int nchunks, void* params, const void* grads, void* bufs, void* shadows,
                         float lr, float momentum, float dampening, float wd, int nesterov, int first,
                         float grad_scale, hipStream_t st) {
  return pdt_sgd_step2(chunks, nchunks, params, grads, bufs, shadows, lr, momentum, dampening, wd, nesterov, first,
                       grad_scale, nullptr, st);
}

PDT_API int pdt_adam_step2(const void* chunks, int nchunks, void* params, const void* grads, void* exp_avg,
                           void* exp_avg_sq, void* max_sq, void* shadows, float lr, float b1, float b2, float eps,
                           float wd, int decoupled, float bc1, float bc2, float grad_scale, float* dev, int tick,
                           hipStream_t st) {
  if (tick && dev == nullptr) return -1;
  if (tick) {
    hipLaunchKernelGGL(opt_tick_kernel, dim3(1), dim3(64), 0, st, dev);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(nchunks)), dim3(NT), 0, st, (const Chunk*)chunks, nchunks,
                     (float* const*)params, (const float* const*)grads, (float* const*)exp_avg,
                     (float* const*)exp_avg_sq, (float* const*)max_sq, (u16* const*)shadows, lr, b1, b2, eps, wd,
                     decoupled, bc1, bc2, grad_scale, (const float*)dev);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_adam_step(const void* chunks, int nchunks, void* params, const void* grads, void* exp_avg,
                          void* exp_avg_sq, void* max_sq, void* shadows, float lr, float b1, float b2, float eps,
                          float wd, int decoupled, float bc1, float bc2, float grad_scale, hipStream_t st) {
  return pdt_adam_step2(chunks, nchunks, params, grads, exp_avg, exp_avg_sq, max_sq, shadows, lr, b1, b2, eps, wd,
                        decoupled, bc1, bc2, grad_scale, nullptr, 0, st);
}
