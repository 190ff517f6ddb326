// Gradient clipping + Adam over a parameter list in two launches
// (reference: scripts/train.py:418-427 / :472-482 -- optional
// nn.utils.clip_grad_norm_ then optim.Adam.step, lr 1e-3 D / 1e-4 G).
//
// torch runs ~9 launches for clip_grad_norm_ (per-tensor norms, stack, norm,
// coefficient, clamp, scale) and 2 for a fused Adam (step increment + update).
// Here:
//   adam_prep_kernel    per-workgroup partial sums of squares of the
//                       concatenated gradients (clip only); block 0 increments
//                       every tensor's device step and forms its step scalars;
//   adam_update_kernel  every workgroup reduces the partials in the same fixed
//                       order (deterministic, identical in all workgroups),
//                       coef = min(max_norm / (||g|| + 1e-6), 1), writes the
//                       clipped gradient back (as clip_grad_norm_ does) and
//                       applies torch's Adam update:
//                         m = lerp(m, g, 1 - b1);  v = b2 v + (1 - b2) g^2
//                         p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// Every tensor keeps its own step counter (torch's per-parameter
// state['step'], float32 on the device as in capturable Adam), so the state
// stays interchangeable with torch.optim.Adam's.
// The tensor list travels by value in the kernel arguments (<= 48 tensors),
// so the launch is graph-capturable without a device pointer table.
#include "sgg_common.h"

namespace sgg {

constexpr int kAdamMaxTensors = 48;
constexpr int kAdamThreads = 256;
constexpr int kAdamChunk = 1024;   // elements per workgroup (4 per thread: ~50-75 workgroups for G / D)

struct AdamList {
  float* p[kAdamMaxTensors];
  float* g[kAdamMaxTensors];
  float* m[kAdamMaxTensors];
  float* v[kAdamMaxTensors];
  float* step[kAdamMaxTensors];         // per-tensor device step counters (torch's state['step'])
  long long off[kAdamMaxTensors + 1];   // prefix offsets of the concatenation
  int n;
};

__device__ __forceinline__ float block_sum(float x, float* red) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = x;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < kAdamThreads / 64; ++w) s += red[w];
  __syncthreads();
  return s;
}

// step scalars per tensor, as torch's Adam forms them (Python doubles, cast
// once to fp32): scal[2k] = lr / (1 - b1^t), scal[2k + 1] = sqrt(1 - b2^t)
__global__ void __launch_bounds__(kAdamThreads) adam_prep_kernel(AdamList L, int clip, float* __restrict__ partial,
                                                                 float* __restrict__ scal, double lr, double beta1,
                                                                 double beta2) {
  __shared__ float red[kAdamThreads / 64];
  if (blockIdx.x == 0 && (int)threadIdx.x < L.n) {
    const float t = L.step[threadIdx.x][0] + 1.f;
    L.step[threadIdx.x][0] = t;
    scal[2 * threadIdx.x] = (float)(lr / (1.0 - pow(beta1, (double)t)));
    scal[2 * threadIdx.x + 1] = (float)sqrt(1.0 - pow(beta2, (double)t));
  }
  if (!clip) return;
  const long long e0 = (long long)blockIdx.x * kAdamChunk, e1 = e0 + kAdamChunk;
  float acc = 0.f;
  for (int t = 0; t < L.n; ++t) {
    const long long lo = e0 > L.off[t] ? e0 : L.off[t];
    const long long hi = e1 < L.off[t + 1] ? e1 : L.off[t + 1];
    const float* g = L.g[t];
    for (long long e = lo + threadIdx.x; e < hi; e += kAdamThreads) {
      const float x = g[e - L.off[t]];
      acc = fmaf(x, x, acc);
    }
  }
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void __launch_bounds__(kAdamThreads) adam_update_kernel(AdamList L, int nparts, float max_norm,
                                                                   const float* __restrict__ partial,
                                                                   const float* __restrict__ scal, float beta2,
                                                                   float w1, float w2, float eps) {
  __shared__ float red[kAdamThreads / 64];
  float coef = 1.f;
  if (max_norm > 0.f) {
    float acc = 0.f;
    for (int q = threadIdx.x; q < nparts; q += kAdamThreads) acc += partial[q];
    const float norm = sqrtf(block_sum(acc, red));
    coef = fminf(max_norm / (norm + 1e-6f), 1.f);
  }
  const long long e0 = (long long)blockIdx.x * kAdamChunk, e1 = e0 + kAdamChunk;
  for (int k = 0; k < L.n; ++k) {
    const long long lo = e0 > L.off[k] ? e0 : L.off[k];
    const long long hi = e1 < L.off[k + 1] ? e1 : L.off[k + 1];
    if (lo >= hi) continue;
    float *p = L.p[k], *g = L.g[k], *m = L.m[k], *v = L.v[k];
    const float step_size = scal[2 * k], bc2s = scal[2 * k + 1];
    for (long long e = lo + threadIdx.x; e < hi; e += kAdamThreads) {
      const long long i = e - L.off[k];
      float gr = g[i];
      if (max_norm > 0.f) {
        gr *= coef;
        g[i] = gr;
      }
      const float mi = m[i] + w1 * (gr - m[i]);                 // exp_avg.lerp_(g, 1 - b1)
      const float vi = v[i] * beta2 + w2 * gr * gr;     // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
      m[i] = mi;
      v[i] = vi;
      p[i] += -step_size * (mi / (sqrtf(vi) / bc2s + eps));   // addcdiv_(m, denom, -step_size)
    }
  }
}

}  // namespace sgg

using namespace sgg;

// workspace floats: one partial per workgroup + 2 step scalars per tensor
extern "C" int sgg_adam_parts(long long total) {
  return (int)((total + kAdamChunk - 1) / kAdamChunk) + 2 * kAdamMaxTensors;
}

extern "C" int sgg_adam_step(float* const* params, float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, const long long* numel, int n, double lr, double beta1,
                             double beta2, float eps, float max_norm, float* const* step, float* ws,
                             size_t ws_bytes, void* stream) {
  SGG_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && numel && step, "sgg_adam_step: null pointer");
  SGG_CHECK_ARG(n >= 1 && n <= kAdamMaxTensors, "sgg_adam_step: %d tensors (1..%d)", n, kAdamMaxTensors);
  AdamList L;
  L.n = n;
  L.off[0] = 0;
  for (int i = 0; i < n; ++i) {
    SGG_CHECK_ARG(params[i] && grads[i] && exp_avg[i] && exp_avg_sq[i] && step[i] && numel[i] >= 0,
                  "sgg_adam_step: tensor %d", i);
    L.p[i] = params[i];
    L.g[i] = grads[i];
    L.m[i] = exp_avg[i];
    L.v[i] = exp_avg_sq[i];
    L.step[i] = step[i];
    L.off[i + 1] = L.off[i] + numel[i];
  }
  const int parts = sgg_adam_parts(L.off[n]) - 2 * kAdamMaxTensors;
  if (parts == 0) return 0;
  const int clip = max_norm > 0.f;
  SGG_CHECK_ARG(ws && ws_bytes >= sizeof(float) * ((size_t)parts + 2 * kAdamMaxTensors), "sgg_adam_step: workspace");
  hipStream_t st = (hipStream_t)stream;
  float* scal = ws + parts;
  hipLaunchKernelGGL(adam_prep_kernel, dim3(clip ? parts : 1), dim3(kAdamThreads), 0, st, L, clip, ws, scal, lr,
                     beta1, beta2);
  hipLaunchKernelGGL(adam_update_kernel, dim3(parts), dim3(kAdamThreads), 0, st, L, parts, clip ? max_norm : 0.f,
                     ws, scal, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), eps);
  SGG_RETURN_LAUNCH("sgg_adam_step");
}
