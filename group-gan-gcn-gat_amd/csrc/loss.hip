// Adversarial loss of the training step (sgan/losses.py:5-21 bce_loss, as
// combined by gan_d_loss :36-49 / gan_g_loss :24-33 and weighted by the
// data-parallel shard fraction):
//   loss = w * ( mean_{i <  split} f(x_i, y_a) + mean_{i >= split} f(x_i, y_b) )
//   f(x, y) = max(x, 0) - x y + log(1 + exp(-|x|))
// The reference spends ~12 elementwise/reduction launches per bce_loss call
// plus their backward; here it is one launch forward and one backward.  The
// targets are device scalars so the step stays graph-capturable with fresh
// label-smoothing draws per replay.  nvalid (optional, device): only the
// first *nvalid scores of each half are real (a padded batch, PaddedScenes);
// the means run over those, the rest get a zero gradient.
#include "sgg_common.h"

namespace sgg {

__device__ __forceinline__ float bce_term(float x, float y) {
  return fmaxf(x, 0.f) - x * y + logf(1.f + expf(-fabsf(x)));
}

// d f / d x as torch's autograd forms it: clamp_min passes where x >= 0,
// abs' = sign(x) (0 at 0)
__device__ __forceinline__ float bce_grad(float x, float y) {
  const float e = expf(-fabsf(x));
  const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
  return (x >= 0.f ? 1.f : 0.f) - y - sg * (e / (1.f + e));
}

// the score i counts: inside its half's first nv scores
__device__ __forceinline__ bool bce_live(int i, int split, int nv) { return i < split ? i < nv : i - split < nv; }

__global__ void __launch_bounds__(256) bce_fwd_kernel(const float* __restrict__ x, int n, int split,
                                                      const float* __restrict__ ya, const float* __restrict__ yb,
                                                      float w, float* __restrict__ loss,
                                                      const float* __restrict__ addend, float* __restrict__ total,
                                                      const int32_t* __restrict__ nvalid) {
  __shared__ float red[2][4];
  const float a = *ya, b = *yb;
  const int nv = nvalid ? *nvalid : n;
  float s0 = 0.f, s1 = 0.f;
  constexpr int kPre = 16;   // up to 4,096 scores: every load in flight at once (one round trip)
  if (n <= kPre * 256) {
    float v[kPre];
#pragma unroll
    for (int m = 0; m < kPre; ++m) {
      const int i = threadIdx.x + 256 * m;
      v[m] = i < n ? x[i] : 0.f;
    }
#pragma unroll
    for (int m = 0; m < kPre; ++m) {   // the same per-thread order as the loop below
      const int i = threadIdx.x + 256 * m;
      if (i < n && bce_live(i, split, nv)) {
        if (i < split) s0 += bce_term(v[m], a);
        else s1 += bce_term(v[m], b);
      }
    }
  } else {
#pragma unroll 4
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      if (!bce_live(i, split, nv)) continue;
      if (i < split) s0 += bce_term(x[i], a);
      else s1 += bce_term(x[i], b);
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = s0;
    red[1][wave] = s1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t0 = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    const float t1 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    const int c0 = min(split, nv), c1 = min(n - split, nv);
    const float m0 = c0 > 0 ? t0 / (float)c0 : 0.f;
    const float m1 = c1 > 0 ? t1 / (float)c1 : 0.f;
    const float l = w * (m0 + m1);
    *loss = l;
    if (total) *total = l + *addend;
  }
}

__global__ void bce_bwd_kernel(const float* __restrict__ x, int n, int split, const float* __restrict__ ya,
                               const float* __restrict__ yb, float w, const float* __restrict__ gout,
                               float* __restrict__ dx, const int32_t* __restrict__ nvalid) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int nv = nvalid ? *nvalid : n;
  const bool first = i < split;
  const float cnt = first ? (float)min(split, nv) : (float)min(n - split, nv);
  dx[i] = bce_live(i, split, nv) ? (*gout * w / cnt) * bce_grad(x[i], first ? *ya : *yb) : 0.f;
}

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_bce_fwd(const float* x, int n, int split, const float* ya, const float* yb, float w, float* loss,
                           const float* addend, float* total, const int32_t* nvalid, void* stream) {
  SGG_CHECK_ARG(loss && ya && yb && (n == 0 || x), "sgg_bce_fwd: null pointer");
  SGG_CHECK_ARG(!total || addend, "sgg_bce_fwd: total needs the addend");
  SGG_CHECK_ARG(n >= 0 && split >= 0 && split <= n, "sgg_bce_fwd: bad sizes n=%d split=%d", n, split);
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, x, n, split, ya, yb, w, loss,
                     addend, total, nvalid);
  SGG_RETURN_LAUNCH("sgg_bce_fwd");
}

extern "C" int sgg_bce_bwd(const float* x, int n, int split, const float* ya, const float* yb, float w,
                           const float* gout, float* dx, const int32_t* nvalid, void* stream) {
  SGG_CHECK_ARG(ya && yb && gout && (n == 0 || (x && dx)), "sgg_bce_bwd: null pointer");
  SGG_CHECK_ARG(n >= 0 && split >= 0 && split <= n, "sgg_bce_bwd: bad sizes n=%d split=%d", n, split);
  if (n == 0) return 0;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, n, split, ya, yb,
                     w, gout, dx, nvalid);
  SGG_RETURN_LAUNCH("sgg_bce_bwd");
}
