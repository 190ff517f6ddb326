// Instance normalisation over the rows of each segment (the InstanceNorm1d,
// affine = False, in front of every layer of the sgangat batched GAT,
// sgan/GAT.py:71-74 and :80 of the commented text).  The reference runs it on
// a (1, F, N) view of one scene; here one workgroup owns one scene and lanes
// run along the features, so every row read is a coalesced F-float vector:
//   256 threads = 64 feature lanes x 4 row phases; each (phase, feature)
//   thread accumulates its rows, the 4 phases are combined in LDS.
// Two passes (mean, then centred sum of squares), biased variance; the
// per-feature sums are accumulated in fp64 (the backward's two means feed a
// gradient whose sum over the scene's rows cancels to ~0 -- the next
// layer's bias gradient -- so their rounding is what that sum sees).
#include "sgg_common.h"

namespace sgg {

constexpr int kNormThreads = 256;

__device__ __forceinline__ double phase_sum(double v, double (*red)[64], int ph, int fl) {
  red[ph][fl] = v;
  __syncthreads();
  const double s = (red[0][fl] + red[1][fl]) + (red[2][fl] + red[3][fl]);
  __syncthreads();
  return s;
}

__global__ void __launch_bounds__(kNormThreads) seg_norm_fwd_kernel(const float* __restrict__ x, int ldx, int F,
                                                                    const int32_t* __restrict__ seg_off, int nseg,
                                                                    float eps, float* __restrict__ y, int ldy,
                                                                    float* __restrict__ rstd_out) {
  __shared__ double red[4][64];
  const int fl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  for (int g = blockIdx.x; g < nseg; g += gridDim.x) {
    const int o = seg_off[g], n = seg_off[g + 1] - o;
    for (int f0 = 0; f0 < F; f0 += 64) {
      const int f = f0 + fl;
      const bool fok = f < F;
      double s = 0.0;
      if (fok)
        for (int r = ph; r < n; r += 4) s += (double)x[(size_t)(o + r) * ldx + f];
      const double meand = n > 0 ? phase_sum(s, red, ph, fl) / n : phase_sum(s, red, ph, fl);
      const float mean = (float)meand;
      double q = 0.0;
      if (fok)
        for (int r = ph; r < n; r += 4) {
          const double d = (double)x[(size_t)(o + r) * ldx + f] - meand;
          q = fma(d, d, q);
        }
      const double qs = phase_sum(q, red, ph, fl);
      const float var = n > 0 ? (float)(qs / n) : 0.f;
      const float rs = 1.f / sqrtf(var + eps);
      if (fok) {
        for (int r = ph; r < n; r += 4) y[(size_t)(o + r) * ldy + f] = (x[(size_t)(o + r) * ldx + f] - mean) * rs;
        if (ph == 0) rstd_out[(size_t)g * F + f] = rs;
      }
    }
  }
}

__global__ void __launch_bounds__(kNormThreads) seg_norm_bwd_kernel(const float* __restrict__ y, int ldy,
                                                                    const float* __restrict__ dy, int lddy, int F,
                                                                    const int32_t* __restrict__ seg_off, int nseg,
                                                                    const float* __restrict__ rstd,
                                                                    float* __restrict__ dx, int lddx) {
  __shared__ double red[4][64];
  const int fl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  for (int g = blockIdx.x; g < nseg; g += gridDim.x) {
    const int o = seg_off[g], n = seg_off[g + 1] - o;
    for (int f0 = 0; f0 < F; f0 += 64) {
      const int f = f0 + fl;
      const bool fok = f < F;
      double sd = 0.0, sdy = 0.0;
      if (fok)
        for (int r = ph; r < n; r += 4) {
          const double d = (double)dy[(size_t)(o + r) * lddy + f];
          sd += d;
          sdy = fma(d, (double)y[(size_t)(o + r) * ldy + f], sdy);
        }
      const double md = n > 0 ? phase_sum(sd, red, ph, fl) / n : phase_sum(sd, red, ph, fl);
      const double mdy = n > 0 ? phase_sum(sdy, red, ph, fl) / n : phase_sum(sdy, red, ph, fl);
      if (fok) {
        const double rs = (double)rstd[(size_t)g * F + f];
        for (int r = ph; r < n; r += 4) {
          const double d = (double)dy[(size_t)(o + r) * lddy + f];
          dx[(size_t)(o + r) * lddx + f] = (float)(rs * ((d - md) - (double)y[(size_t)(o + r) * ldy + f] * mdy));
        }
      }
    }
  }
}

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_seg_norm_fwd(const float* x, int ldx, int F, const int32_t* seg_off, int nseg, float eps,
                                float* y, int ldy, float* rstd, void* stream) {
  SGG_CHECK_ARG(x && seg_off && y && rstd, "sgg_seg_norm_fwd: null pointer");
  SGG_CHECK_ARG(F >= 1 && nseg >= 0 && ldx >= F && ldy >= F && eps > 0.f, "sgg_seg_norm_fwd: bad sizes");
  if (nseg == 0) return 0;
  const int grid = nseg < 16384 ? nseg : 16384;
  hipLaunchKernelGGL(seg_norm_fwd_kernel, dim3(grid), dim3(kNormThreads), 0, (hipStream_t)stream, x, ldx, F, seg_off,
                     nseg, eps, y, ldy, rstd);
  SGG_RETURN_LAUNCH("sgg_seg_norm_fwd");
}

extern "C" int sgg_seg_norm_bwd(const float* y, int ldy, const float* dy, int lddy, int F, const int32_t* seg_off,
                                int nseg, const float* rstd, float* dx, int lddx, void* stream) {
  SGG_CHECK_ARG(y && dy && seg_off && rstd && dx, "sgg_seg_norm_bwd: null pointer");
  SGG_CHECK_ARG(F >= 1 && nseg >= 0 && ldy >= F && lddy >= F && lddx >= F, "sgg_seg_norm_bwd: bad sizes");
  if (nseg == 0) return 0;
  const int grid = nseg < 16384 ? nseg : 16384;
  hipLaunchKernelGGL(seg_norm_bwd_kernel, dim3(grid), dim3(kNormThreads), 0, (hipStream_t)stream, y, ldy, dy, lddy,
                     F, seg_off, nseg, rstd, dx, lddx);
  SGG_RETURN_LAUNCH("sgg_seg_norm_bwd");
}
