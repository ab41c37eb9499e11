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
                           int nesterov, int first, float grad_scale) {
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const Chunk ch = chunks[c];
    float* p = params[ch.tensor] + ch.offset;
    const float* g = grads[ch.tensor] + ch.offset;
    float* b = bufs ? (bufs[ch.tensor] ? bufs[ch.tensor] + ch.offset : nullptr) : nullptr;
    u16* sh = shadows ? (shadows[ch.tensor] ? shadows[ch.tensor] + ch.offset : nullptr) : nullptr;
    for (long i = threadIdx.x; i < ch.len; i += NT) {
      float gi = g[i] * grad_scale;
      float pi = p[i];
      if (wd != 0.f) gi += wd * pi;
      if (momentum != 0.f && b) {
        float bi = first ? gi : momentum * b[i] + (1.f - dampening) * gi;
        b[i] = bi;
        gi = nesterov ? gi + momentum * bi : bi;
      }
      pi -= lr * gi;
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
                            int decoupled, float bc1, float bc2, float grad_scale) {
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

}  // namespace

PDT_API int pdt_chunk_struct_size() { return (int)sizeof(Chunk); }

PDT_API int pdt_sgd_step(const void* chunks, int nchunks, void* params, const void* grads, void* bufs, void* shadows,
                         float lr, float momentum, float dampening, float wd, int nesterov, int first,
                         float grad_scale, hipStream_t st) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(nchunks)), dim3(NT), 0, st, (const Chunk*)chunks, nchunks,
                     (float* const*)params, (const float* const*)grads, (float* const*)bufs,
                     (u16* const*)shadows, lr, momentum, dampening, wd, nesterov, first, grad_scale);
  PDT_RETURN_LAUNCH();
}

PDT_API int pdt_adam_step(const void* chunks, int nchunks, void* params, const void* grads, void* exp_avg,
                          void* exp_avg_sq, void* max_sq, void* shadows, float lr, float b1, float b2, float eps,
                          float wd, int decoupled, float bc1, float bc2, float grad_scale, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(nchunks)), dim3(NT), 0, st, (const Chunk*)chunks, nchunks,
                     (float* const*)params, (const float* const*)grads, (float* const*)exp_avg,
                     (float* const*)exp_avg_sq, (float* const*)max_sq, (u16* const*)shadows, lr, b1, b2, eps, wd,
                     decoupled, bc1, bc2, grad_scale);
  PDT_RETURN_LAUNCH();
}
