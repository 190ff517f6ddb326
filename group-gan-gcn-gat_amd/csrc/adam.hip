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

// A workgroup's chunk [e0, e0 + kAdamChunk) of the concatenation spans a few
// tensors; each thread takes kAdamPer elements (stride kAdamThreads).  The
// tensor table is read ONCE per wave, lane t holding tensor t's offsets and
// pointers (vector loads of the kernel arguments, all in flight together --
// a walk of scalar loads, one dependent load per tensor, was the cost of the
// previous form); an element finds its tensor among the chunk's few with
// s_readlane'd bounds and takes its pointers by a lane shuffle.  All loads of
// a thread's elements are then issued together: one memory latency per chunk.
constexpr int kAdamPer = kAdamChunk / kAdamThreads;

struct Tab {   // lane t: tensor t (t < n)
  long long lo, hi;
  unsigned long long p, g, m, v;
};

__device__ __forceinline__ Tab lane_tab(const AdamList& L) {
  const int t = threadIdx.x & 63;
  Tab r = {0, 0, 0, 0, 0, 0};
  if (t < L.n) {
    r.lo = L.off[t];
    r.hi = L.off[t + 1];
    r.p = reinterpret_cast<unsigned long long>(L.p[t]);
    r.g = reinterpret_cast<unsigned long long>(L.g[t]);
    r.m = reinterpret_cast<unsigned long long>(L.m[t]);
    r.v = reinterpret_cast<unsigned long long>(L.v[t]);
  }
  return r;
}

__device__ __forceinline__ long long rl64(long long x, int k) {
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)(unsigned long long)x, k);
  const int hi = __builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)x >> 32), k);
  return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ unsigned long long shfl64(unsigned long long x, int k) {
  const unsigned lo = (unsigned)__shfl((int)(unsigned)x, k), hi = (unsigned)__shfl((int)(unsigned)(x >> 32), k);
  return ((unsigned long long)hi << 32) | lo;
}

// tensor (-1 past the end) and in-tensor index of the thread's elements
__device__ __forceinline__ void chunk_elems(const AdamList& L, const Tab& T, long long e0, int (&ek)[kAdamPer],
                                            long long (&ei)[kAdamPer]) {
  const long long total = L.off[L.n];
  const long long e1 = (e0 + kAdamChunk < total ? e0 + kAdamChunk : total) - 1;   // last element
  const int t = threadIdx.x & 63;
  // the chunk's tensors k0 .. k1: the lanes holding e0 / e1
  const unsigned long long b0 = __ballot(t < L.n && T.lo <= e0 && e0 < T.hi);
  const unsigned long long b1 = __ballot(t < L.n && T.lo <= e1 && e1 < T.hi);
  const int k0 = b0 ? __ffsll((long long)b0) - 1 : 0, k1 = b1 ? __ffsll((long long)b1) - 1 : k0;
#pragma unroll
  for (int u = 0; u < kAdamPer; ++u) {
    ek[u] = -1;
    ei[u] = 0;
  }
  for (int k = k0; k <= k1; ++k) {   // (uniform; empty tensors have lo == hi)
    const long long lo = rl64(T.lo, k), hi = rl64(T.hi, k);
#pragma unroll
    for (int u = 0; u < kAdamPer; ++u) {
      const long long e = e0 + threadIdx.x + (long long)u * kAdamThreads;
      if (e >= lo && e < hi) {
        ek[u] = k;
        ei[u] = e - lo;
      }
    }
  }
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
  const long long e0 = (long long)blockIdx.x * kAdamChunk;
  const Tab T = lane_tab(L);
  int ek[kAdamPer];
  long long ei[kAdamPer];
  chunk_elems(L, T, e0, ek, ei);
  float x[kAdamPer];
#pragma unroll
  for (int u = 0; u < kAdamPer; ++u) {
    const float* g = reinterpret_cast<const float*>(shfl64(T.g, ek[u] < 0 ? 0 : ek[u]));
    x[u] = ek[u] >= 0 ? g[ei[u]] : 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < kAdamPer; ++u) acc = fmaf(x[u], x[u], acc);
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// fused (no clipping): the step scalars are formed here from step + 1 (lane t
// of every wave: tensor t, adam_prep's expressions), and the LAST workgroup to
// finish -- an atomic ticket in ws, left at 0 -- writes the incremented step
// counters: every workgroup has read them (and used the values) before
// taking its ticket, so none sees the new value.  One launch instead of two.
__global__ void __launch_bounds__(kAdamThreads) adam_update_kernel(AdamList L, int nparts, float max_norm,
                                                                   const float* __restrict__ partial,
                                                                   const float* __restrict__ scal, float beta2,
                                                                   float w1, float w2, float eps,
                                                                   unsigned* __restrict__ ticket, double lr,
                                                                   double beta1d, double beta2d) {
  __shared__ float red[kAdamThreads / 64];
  __shared__ int last;
  const long long e0 = (long long)blockIdx.x * kAdamChunk;
  const Tab T = lane_tab(L);
  float tstep = 0.f, lss = 0.f, lbc = 1.f;   // fused: lane t's step + 1 and step scalars
  if (ticket && (int)(threadIdx.x & 63) < L.n) {
    tstep = L.step[threadIdx.x & 63][0] + 1.f;
    lss = (float)(lr / (1.0 - pow(beta1d, (double)tstep)));
    lbc = (float)sqrt(1.0 - pow(beta2d, (double)tstep));
  }
  int ek[kAdamPer];
  long long ei[kAdamPer];
  chunk_elems(L, T, e0, ek, ei);
  float coef = 1.f;
  if (max_norm > 0.f) {
    float acc = 0.f;
    for (int q = threadIdx.x; q < nparts; q += kAdamThreads) acc += partial[q];
    const float norm = sqrtf(block_sum(acc, red));
    coef = fminf(max_norm / (norm + 1e-6f), 1.f);
  }
  float* pp[kAdamPer];
  float* gp[kAdamPer];
  float* mp[kAdamPer];
  float* vp[kAdamPer];
  float gr[kAdamPer], m0[kAdamPer], v0[kAdamPer], p0[kAdamPer], ss[kAdamPer], bc[kAdamPer];
#pragma unroll
  for (int u = 0; u < kAdamPer; ++u) {
    const int k = ek[u] >= 0 ? ek[u] : 0;
    const long long i = ek[u] >= 0 ? ei[u] : 0;
    pp[u] = reinterpret_cast<float*>(shfl64(T.p, k)) + i;
    gp[u] = reinterpret_cast<float*>(shfl64(T.g, k)) + i;
    mp[u] = reinterpret_cast<float*>(shfl64(T.m, k)) + i;
    vp[u] = reinterpret_cast<float*>(shfl64(T.v, k)) + i;
    if (ticket) {
      ss[u] = __shfl(lss, k);
      bc[u] = __shfl(lbc, k);
    } else {
      ss[u] = scal[2 * k];
      bc[u] = scal[2 * k + 1];
    }
  }
  // every load of the thread's elements first, then the updates
#pragma unroll
  for (int u = 0; u < kAdamPer; ++u) {
    gr[u] = *gp[u];
    m0[u] = *mp[u];
    v0[u] = *vp[u];
    p0[u] = *pp[u];
  }
#pragma unroll
  for (int u = 0; u < kAdamPer; ++u) {
    if (ek[u] < 0) continue;
    float g = gr[u];
    if (max_norm > 0.f) {
      g *= coef;
      *gp[u] = g;
    }
    const float mi = m0[u] + w1 * (g - m0[u]);        // exp_avg.lerp_(g, 1 - b1)
    const float vi = v0[u] * beta2 + w2 * g * g;      // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    *mp[u] = mi;
    *vp[u] = vi;
    *pp[u] = p0[u] + -ss[u] * (mi / (sqrtf(vi) / bc[u] + eps));   // addcdiv_(m, denom, -step_size)
  }
  if (ticket) {
    __syncthreads();   // (every lane's step read has been consumed above)
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last) {
      if ((int)threadIdx.x < L.n) L.step[threadIdx.x][0] = tstep;
      if (threadIdx.x == 0) *ticket = 0u;
    }
  }
}

}  // namespace sgg

using namespace sgg;

// workspace floats: the fused launch's ticket at the FIXED word ws[0] (zero
// when the workspace is first used, every call leaves it at zero, and nothing
// else ever writes it -- whatever the parameter count or clipping of the
// call), then one partial per workgroup, then 2 step scalars per tensor
extern "C" int sgg_adam_parts(long long total) {
  return (int)((total + kAdamChunk - 1) / kAdamChunk) + 2 * kAdamMaxTensors + 1;
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
  const int parts = sgg_adam_parts(L.off[n]) - 2 * kAdamMaxTensors - 1;
  if (parts == 0) return 0;
  const int clip = max_norm > 0.f;
  SGG_CHECK_ARG(ws && ws_bytes >= sizeof(float) * ((size_t)parts + 2 * kAdamMaxTensors + 1),
                "sgg_adam_step: workspace");
  hipStream_t st = (hipStream_t)stream;
  unsigned* ticket = reinterpret_cast<unsigned*>(ws);
  float* partial = ws + 1;
  float* scal = partial + parts;
  if (clip)   // the norm's partials need every workgroup: a launch of their own
    hipLaunchKernelGGL(adam_prep_kernel, dim3(parts), dim3(kAdamThreads), 0, st, L, clip, partial, scal, lr, beta1,
                       beta2);
  hipLaunchKernelGGL(adam_update_kernel, dim3(parts), dim3(kAdamThreads), 0, st, L, parts, clip ? max_norm : 0.f,
                     partial, scal, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), eps, clip ? nullptr : ticket,
                     lr, beta1, beta2);
  SGG_RETURN_LAUNCH("sgg_adam_step");
}
