// Parameter-gradient reductions  C = X^T Y  (X: R x M, Y: R x N, R >> M, N),
// plus optional column sums of Y (bias gradients), on fp32 MFMA with split-K.
//
// Every weight gradient of the path is such a reduction over all nodes /
// (time, ped) pairs: dW = X^T dY of a node transform, dW_hh = dG^T h_{t-1}
// summed over T x B, dW1h = dU^T h of the pooling, da = Wh^T [ds dt] of the
// attention.  R is 10^3..10^5 and M, N <= 512: a library GEMM sees a skinny
// problem with a huge K and launches a handful of workgroups.  Here the rows
// are split over enough workgroups to fill the chip; each writes its partial
// 64 x 64 tile to a slab, and a second pass sums the slabs in split order
// (deterministic).  v_mfma_f32_16x16x4_f32: A[m][k] = X[r0 + k][m] (lanes run
// along m: coalesced), B[k][n] = Y[r0 + k][n].
#include "sgg_common.h"

namespace sgg {

__global__ void __launch_bounds__(256) xtw_partial_kernel(const float* __restrict__ X, int ldx,
                                                          const float* __restrict__ Y, int ldy,
                                                          const float* __restrict__ Ym, int ldm, int R, int M,
                                                          int N, int rows_per_split, float* __restrict__ slab,
                                                          float* __restrict__ colslab) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, kq = lane >> 4;
  const int m0 = blockIdx.x * 64 + wave * 16;
  const int n0 = blockIdx.y * 64;
  const int split = blockIdx.z;
  const int r0 = split * rows_per_split;
  const int r1 = min(R, r0 + rows_per_split);
  const int m = m0 + c16;
  const bool mok = m < M;
  bool nok[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) nok[t] = n0 + 16 * t + c16 < N;
  const bool do_col = colslab && blockIdx.x == 0 && wave == 0;
  floatx4 acc[4];
  float col[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  // software pipeline: the next 16 rows' loads are in flight while the current
  // 16 rows run through the MFMAs
  float a[4], b[4][4], an[4], bnx[4][4];
  // Loads come from clamped addresses: columns >= M / >= N produce values
  // that are never stored; only rows >= r1 must contribute zero, which
  // concerns the last 16-row step alone -- a wave-uniform branch.
  const int mcl = mok ? m : M - 1;
  int ncl[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) ncl[t] = nok[t] ? n0 + 16 * t + c16 : N - 1;
  auto load16 = [&](int r, float (&aa)[4], float (&bb)[4][4]) {
    if (r + 16 <= r1) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const size_t row = (size_t)(r + 4 * s + kq);
        aa[s] = X[row * ldx + mcl];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          bb[s][t] = Ym ? keep_if(Y[row * ldy + ncl[t]], Ym[row * ldm + ncl[t]] > 0.f) : Y[row * ldy + ncl[t]];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int row = r + 4 * s + kq;
        const size_t rc = (size_t)min(row, r1 - 1);
        aa[s] = keep_if(X[rc * ldx + mcl], row < r1);
#pragma unroll
        for (int t = 0; t < 4; ++t)
          bb[s][t] = keep_if(Y[rc * ldy + ncl[t]], row < r1 && (!Ym || Ym[rc * ldm + ncl[t]] > 0.f));
      }
    }
  };
  if (r0 < r1) load16(r0, a, b);
  for (int r = r0; r < r1; r += 16) {
    const bool more = r + 16 < r1;
    if (more) load16(r + 16, an, bnx);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s][t], acc[t], 0, 0, 0);
        if (do_col) col[t] += b[s][t];
      }
    if (more) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a[s] = an[s];
#pragma unroll
        for (int t = 0; t < 4; ++t) b[s][t] = bnx[s][t];
      }
    }
  }
  float* out = slab + (size_t)split * M * N;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = n0 + 16 * t + c16;
    if (n >= N) continue;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int mm = m0 + kq * 4 + rr;
      if (mm < M) out[(size_t)mm * N + n] = acc[t][rr];
    }
  }
  if (do_col) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {  // sum the 4 row phases (lanes c16, c16+16, +32, +48)
      float v = col[t];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int n = n0 + 16 * t + c16;
      if (kq == 0 && n < N) colslab[(size_t)split * N + n] = v;
    }
  }
}

// slab sums: block = 64 outputs x 16 split phases (1024 threads), fixed
// order -> deterministic; the blocks past the C outputs sum the column-sum
// slab, so C and the bias gradient take ONE launch.  Each phase walks
// <= splits / 16 partials with 4 loads in flight (the partial slabs were just
// written: L2 hits, latency- not bandwidth-bound).
__global__ void __launch_bounds__(1024) xtw_reduce_kernel(const float* __restrict__ slab, int splits, int MN,
                                                          float* __restrict__ C, int N, int ldc, int trans_c,
                                                          const float* __restrict__ colslab,
                                                          float* __restrict__ colsum) {
  __shared__ float part[16][64];
  const int el = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int nbm = (MN + 63) / 64;
  const bool col = (int)blockIdx.x >= nbm;
  const float* src = col ? colslab : slab;
  const int cnt = col ? N : MN;
  const int e = (col ? (int)blockIdx.x - nbm : (int)blockIdx.x) * 64 + el;
  float s = 0.f;
  if (e < cnt) {
    int k = ph;
    for (; k + 48 < splits; k += 64) {
      const float v0 = src[(size_t)k * cnt + e], v1 = src[(size_t)(k + 16) * cnt + e];
      const float v2 = src[(size_t)(k + 32) * cnt + e], v3 = src[(size_t)(k + 48) * cnt + e];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; k < splits; k += 16) s += src[(size_t)k * cnt + e];
  }
  part[ph][el] = s;
  __syncthreads();
  if (ph == 0 && e < cnt) {
    float v = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) v += part[p][el];
    if (col) {
      colsum[e] = v;
    } else {
      const int mm = e / N, n = e - mm * N;
      if (trans_c) C[(size_t)n * ldc + mm] = v;
      else C[(size_t)mm * ldc + n] = v;
    }
  }
}

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_xtw_splits(int R, int M, int N) {
  // >= ~32 rows per split (two 16-row MFMA steps), capped by the grid
  // (<= 1024 workgroups: thousands of one-step workgroups cost more in
  // dispatch than they compute), by the slab (<= 2^21 floats, so the reduce
  // stays an L2-resident pass) and at 256 partials per output (the reduce's
  // phases walk <= 16 each)
  const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
  const long long mn = (long long)M * N;
  long long splits = (R + 31) / 32;
  const long long by_grid = 1024 / tiles > 0 ? 1024 / tiles : 1;
  const long long by_slab = (1ll << 21) / mn > 0 ? (1ll << 21) / mn : 1;
  if (splits > by_grid) splits = by_grid;
  if (splits > by_slab) splits = by_slab;
  if (splits > 256) splits = 256;
  return splits < 1 ? 1 : (int)splits;
}

extern "C" int sgg_xtw(const float* X, int ldx, const float* Y, int ldy, const float* Ymask, int ldm, int R, int M,
                       int N, float* C, int ldc, int trans_c, float* colsum, float* ws, size_t ws_bytes,
                       void* stream) {
  SGG_CHECK_ARG((R == 0 || (X && Y)) && C && ws, "sgg_xtw: null pointer");
  SGG_CHECK_ARG(R >= 0 && M > 0 && N > 0 && ldx >= M && ldy >= N && ldc >= (trans_c ? M : N),
                "sgg_xtw: bad sizes");
  const int splits = sgg_xtw_splits(R, M, N);
  const size_t need = sizeof(float) * (size_t)splits * ((size_t)M * N + N);
  SGG_CHECK_ARG(ws_bytes >= need, "sgg_xtw: workspace %zu < %zu bytes", ws_bytes, need);
  SGG_CHECK_ARG(!Ymask || ldm >= N, "sgg_xtw: mask leading dim %d < N", ldm);
  hipStream_t st = (hipStream_t)stream;
  const int rps = ((R + splits - 1) / splits + 15) & ~15;
  float* colslab = ws + (size_t)splits * M * N;
  dim3 grid((M + 63) / 64, (N + 63) / 64, splits);
  hipLaunchKernelGGL(xtw_partial_kernel, grid, dim3(256), 0, st, X, ldx, Y, ldy, Ymask, ldm, R, M, N, rps, ws,
                     colsum ? colslab : nullptr);
  const int MN = M * N;
  const int nb = (MN + 63) / 64 + (colsum ? (N + 63) / 64 : 0);
  hipLaunchKernelGGL(xtw_reduce_kernel, dim3(nb), dim3(1024), 0, st, ws, splits, MN, C, N, ldc, trans_c,
                     colsum ? colslab : nullptr, colsum);
  SGG_RETURN_LAUNCH("sgg_xtw");
}
