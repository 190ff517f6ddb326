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
#include "xtw_body.h"

namespace sgg {

// One workgroup = one 64 x 64 output tile of one split.  The four waves split
// the ROWS (wave w takes rows r0 + 16 w + 64 i), each wave accumulating the
// whole tile: per 4-row step a lane loads MT A values (one per 16-wide m-tile)
// and 4 B values and issues MT x 4 MFMAs, so every loaded Y element feeds MT
// MFMAs (the column tiles of M no longer each re-load the Y rows).  MT =
// ceil(min(M, 64) / 16): a narrow X (M = 16 / 32 / 48) skips the m-tiles it
// does not have instead of running idle waves.  The four partial tiles are
// summed in LDS in wave order (deterministic) and stored coalesced.
template <int MT>
__global__ void __launch_bounds__(256) xtw_partial_kernel(const float* __restrict__ X, int ldx,
                                                          const float* __restrict__ Y, int ldy,
                                                          const float* __restrict__ Ym, int ldm, int R, int M,
                                                          int N, int rows_per_split, float* __restrict__ slab,
                                                          float* __restrict__ colslab) {
  __shared__ float red[kXtwRedFloats];
  xtw_partial_body<MT>(X, ldx, Y, ldy, Ym, ldm, R, M, N, rows_per_split, slab, colslab, blockIdx.x, blockIdx.y,
                       blockIdx.z, red);
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
  // >= 64 rows per split (one 16-row MFMA step per wave), capped by the grid
  // (<= 1024 workgroups: thousands of one-step workgroups cost more in
  // dispatch than they compute), by the slab (<= 2^21 floats, so the reduce
  // stays an L2-resident pass) and at 256 partials per output (the reduce's
  // phases walk <= 16 each)
  const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
  const long long mn = (long long)M * N;
  long long splits = (R + 63) / 64;
  const long long by_grid = 1024 / tiles > 0 ? 1024 / tiles : 1;
  const long long by_slab = (1ll << 21) / mn > 0 ? (1ll << 21) / mn : 1;
  if (splits > by_grid) splits = by_grid;
  if (splits > by_slab) splits = by_slab;
  if (splits > 256) splits = 256;
  return splits < 1 ? 1 : (int)splits;
}

static void launch_partial(const float* X, int ldx, const float* Y, int ldy, const float* Ymask, int ldm, int R,
                           int M, int N, int splits, float* ws, float* cs, hipStream_t st) {
  const int rps = ((R + splits - 1) / splits + 63) & ~63;   // whole 64-row steps (16 rows per wave)
  dim3 grid((M + 63) / 64, (N + 63) / 64, splits);
  switch (M >= 64 ? 4 : (M + 15) / 16) {   // 16-wide m-tiles of a 64-row output block
    case 1: hipLaunchKernelGGL(xtw_partial_kernel<1>, grid, dim3(256), 0, st, X, ldx, Y, ldy, Ymask, ldm, R, M, N, rps, ws, cs); break;
    case 2: hipLaunchKernelGGL(xtw_partial_kernel<2>, grid, dim3(256), 0, st, X, ldx, Y, ldy, Ymask, ldm, R, M, N, rps, ws, cs); break;
    case 3: hipLaunchKernelGGL(xtw_partial_kernel<3>, grid, dim3(256), 0, st, X, ldx, Y, ldy, Ymask, ldm, R, M, N, rps, ws, cs); break;
    default: hipLaunchKernelGGL(xtw_partial_kernel<4>, grid, dim3(256), 0, st, X, ldx, Y, ldy, Ymask, ldm, R, M, N, rps, ws, cs); break;
  }
}

extern "C" int sgg_xtw_partial(const float* X, int ldx, const float* Y, int ldy, const float* Ymask, int ldm, int R,
                               int M, int N, int colsum, float* ws, size_t ws_bytes, void* stream) {
  SGG_CHECK_ARG(X && Y && ws, "sgg_xtw_partial: null pointer");
  SGG_CHECK_ARG(R >= 1 && M > 0 && N > 0 && ldx >= M && ldy >= N, "sgg_xtw_partial: bad sizes");
  const int splits = sgg_xtw_splits(R, M, N);
  const size_t need = sizeof(float) * (size_t)splits * ((size_t)M * N + (colsum ? N : 0));
  SGG_CHECK_ARG(ws_bytes >= need, "sgg_xtw_partial: workspace %zu < %zu bytes", ws_bytes, need);
  SGG_CHECK_ARG(!Ymask || ldm >= N, "sgg_xtw_partial: mask leading dim %d < N", ldm);
  launch_partial(X, ldx, Y, ldy, Ymask, ldm, R, M, N, splits, ws, colsum ? ws + (size_t)splits * M * N : nullptr,
                 (hipStream_t)stream);
  SGG_RETURN_LAUNCH("sgg_xtw_partial");
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
  float* colslab = ws + (size_t)splits * M * N;
  launch_partial(X, ldx, Y, ldy, Ymask, ldm, R, M, N, splits, ws, colsum ? colslab : nullptr, st);
  const int MN = M * N;
  const int nb = (MN + 63) / 64 + (colsum ? (N + 63) / 64 : 0);
  hipLaunchKernelGGL(xtw_reduce_kernel, dim3(nb), dim3(1024), 0, st, ws, splits, MN, C, N, ldc, trans_c,
                     colsum ? colslab : nullptr, colsum);
  SGG_RETURN_LAUNCH("sgg_xtw");
}
