// The split-K pass of C = X^T Y as a device body (xtw.hip's
// xtw_partial_kernel, and the pooling backward's two-product launch in
// xw.hip): one workgroup (256 threads) = one 64 x 64 output tile of one row
// split.  See xtw.hip for the scheme.
#pragma once
#include "sgg_common.h"

namespace sgg {

constexpr int kXtwRedFloats = 64 * 65 + 64;   // LDS of one workgroup

template <int MT>
__device__ __forceinline__ void xtw_partial_body(const float* __restrict__ X, int ldx, const float* __restrict__ Y,
                                                 int ldy, const float* __restrict__ Ym, int ldm, int R, int M, int N,
                                                 int rows_per_split, float* __restrict__ slab,
                                                 float* __restrict__ colslab, int bx, int by, int split,
                                                 float* red /* LDS, kXtwRedFloats */) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, kq = lane >> 4;
  const int m0 = bx * 64;
  const int n0 = by * 64;
  const int r0 = split * rows_per_split;
  const int r1 = min(R, r0 + rows_per_split);
  const bool do_col = colslab && bx == 0;
  // clamped columns: values of columns >= M / >= N are never stored; only rows
  // >= r1 must contribute zero (the last 16-row step of a wave alone)
  int mcl[MT], ncl[4];
#pragma unroll
  for (int u = 0; u < MT; ++u) mcl[u] = min(m0 + 16 * u + c16, M - 1);
#pragma unroll
  for (int t = 0; t < 4; ++t) ncl[t] = min(n0 + 16 * t + c16, N - 1);
  floatx4 acc[MT][4];
  float col[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < MT; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  float a[4][MT], b[4][4], an[4][MT], bnx[4][4];
  auto load16 = [&](int r, float (&aa)[4][MT], float (&bb)[4][4]) {
    if (r + 16 <= r1) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const size_t row = (size_t)(r + 4 * s + kq);
#pragma unroll
        for (int u = 0; u < MT; ++u) aa[s][u] = X[row * ldx + mcl[u]];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          bb[s][t] = Ym ? keep_if(Y[row * ldy + ncl[t]], Ym[row * ldm + ncl[t]] > 0.f) : Y[row * ldy + ncl[t]];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int row = r + 4 * s + kq;
        const size_t rc = (size_t)min(row, r1 - 1);
#pragma unroll
        for (int u = 0; u < MT; ++u) aa[s][u] = keep_if(X[rc * ldx + mcl[u]], row < r1);
#pragma unroll
        for (int t = 0; t < 4; ++t)
          bb[s][t] = keep_if(Y[rc * ldy + ncl[t]], row < r1 && (!Ym || Ym[rc * ldm + ncl[t]] > 0.f));
      }
    }
  };
  const int rw = r0 + 16 * wave;
  if (rw < r1) load16(rw, a, b);
  for (int r = rw; r < r1; r += 64) {
    const bool more = r + 64 < r1;
    if (more) load16(r + 64, an, bnx);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int u = 0; u < MT; ++u) acc[u][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][u], b[s][t], acc[u][t], 0, 0, 0);
        if (do_col) col[t] += b[s][t];
      }
    if (more) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int u = 0; u < MT; ++u) a[s][u] = an[s][u];
#pragma unroll
        for (int t = 0; t < 4; ++t) b[s][t] = bnx[s][t];
      }
    }
  }
  if (do_col) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {  // sum the 4 row phases (lanes c16, c16+16, +32, +48)
      col[t] += __shfl_xor(col[t], 16);
      col[t] += __shfl_xor(col[t], 32);
    }
  }
  // wave-ordered sum of the four partial tiles in LDS (row stride 65)
  float* cred = red + 64 * 65;
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int u = 0; u < MT; ++u)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            float* d = red + (16 * u + 4 * kq + rr) * 65 + 16 * t + c16;
            *d = w == 0 ? acc[u][t][rr] : *d + acc[u][t][rr];
          }
      if (do_col && kq == 0) {
#pragma unroll
        for (int t = 0; t < 4; ++t) cred[16 * t + c16] = w == 0 ? col[t] : cred[16 * t + c16] + col[t];
      }
    }
    __syncthreads();
  }
  float* out = slab + (size_t)split * M * N;
  for (int e = threadIdx.x; e < 16 * MT * 64; e += 256) {
    const int mm = e >> 6, nn = e & 63;
    if (m0 + mm < M && n0 + nn < N) out[(size_t)(m0 + mm) * N + n0 + nn] = red[mm * 65 + nn];
  }
  if (do_col && threadIdx.x < 64 && n0 + (int)threadIdx.x < N) colslab[(size_t)split * N + n0 + threadIdx.x] = cred[threadIdx.x];
}


}  // namespace sgg
