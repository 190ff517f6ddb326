// Dense node-feature transform Y = act(X @ W (+ bias)) on fp32 MFMA.
//
// v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain, no xf32):
//   A lane map: A[l & 15][l >> 4]    (16 rows x 4 k)
//   B lane map: B[l >> 4][l & 15]    (4 k x 16 cols)
//   C/D map   : row = (l >> 4) * 4 + r, col = l & 15   (r = 0..3)
// Workgroup = 4 waves = 64 rows x 64 cols of Y; each wave owns 16 rows x 64
// cols (4 accumulator tiles).  K is small on this path (2..144, 512 for the
// pooling backward), so operands are read straight from L1/L2: the X row
// fragment is reused across the 4 column tiles in registers, the W fragment
// is shared by the 4 waves through L1.  These launches are latency-bound
// (a few dozen workgroups), hence the deep register prefetch below.
#include "sgg_common.h"

namespace sgg {

template <bool TRANS_W>
__global__ void __launch_bounds__(256) xw_kernel(const float* __restrict__ X, int ldx,
                                                 const float* __restrict__ Xmask, int ldm,
                                                 const float* __restrict__ W, int ldw,
                                                 const float* __restrict__ bias, float* __restrict__ Y,
                                                 int ldy, int M, int K, int N, int act) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int row0 = blockIdx.x * 64 + wave * 16;
  const int col0 = blockIdx.y * 64;
  const int ar = lane & 15;   // A row / B col within the 16x16 tile
  const int kq = lane >> 4;   // k within the 4-deep step
  const int arow = row0 + ar;
  const bool arow_ok = arow < M;
  const float* xrow = X + (size_t)(arow_ok ? arow : 0) * ldx;
  // ReLU backward fused into the operand: X[m, k] counts where Xmask[m, k] > 0
  const float* mrow = Xmask ? Xmask + (size_t)(arow_ok ? arow : 0) * ldm : nullptr;

  floatx4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};

  // K is walked in 32-deep chunks (8 MFMA k-steps), double-buffered in
  // registers: the next chunk's loads are all in flight while the current
  // chunk computes, so a K <= 144 transform costs ~K/32 load latencies
  // instead of one per 4-deep step.  Out-of-range k / n read as 0 (adds 0).
  constexpr int KC = 32, S4 = KC / 4;
  // Loads come from clamped (in-bounds) addresses: rows >= M and columns
  // >= N compute values that the epilogue never stores, so they need no
  // mask; only k >= K must contribute zero, which concerns the last chunk
  // alone -- a wave-uniform branch.  (A per-load `cond ? v : 0` makes the
  // compiler sink each load into an exec-masked branch that waits for it.)
  int ncl[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) ncl[t] = min(col0 + 16 * t + ar, N - 1);
  auto load_chunk = [&](int kb, float (&aa)[S4], float (&bb)[S4][4]) {
    if (kb + KC <= K) {
#pragma unroll
      for (int s = 0; s < S4; ++s) {
        const int k = kb + 4 * s + kq;
        aa[s] = mrow ? keep_if(xrow[k], mrow[k] > 0.f) : xrow[k];
#pragma unroll
        for (int t = 0; t < 4; ++t) bb[s][t] = TRANS_W ? W[ncl[t] * ldw + k] : W[k * ldw + ncl[t]];
      }
    } else {
#pragma unroll
      for (int s = 0; s < S4; ++s) {
        const int k = kb + 4 * s + kq;
        const int kc = min(k, K - 1);
        aa[s] = keep_if(xrow[kc], k < K && (!mrow || mrow[kc] > 0.f));
#pragma unroll
        for (int t = 0; t < 4; ++t) bb[s][t] = TRANS_W ? W[ncl[t] * ldw + kc] : W[kc * ldw + ncl[t]];
      }
    }
  };
  float a0[S4], b0[S4][4], a1[S4], b1[S4][4];
  load_chunk(0, a0, b0);
  for (int k0 = 0; k0 < K; k0 += 2 * KC) {
    if (k0 + KC < K) load_chunk(k0 + KC, a1, b1);
#pragma unroll
    for (int s = 0; s < S4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b0[s][t], acc[t], 0, 0, 0);
    if (k0 + KC >= K) break;
    if (k0 + 2 * KC < K) load_chunk(k0 + 2 * KC, a0, b0);
#pragma unroll
    for (int s = 0; s < S4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], b1[s][t], acc[t], 0, 0, 0);
  }

  // epilogue (direct stores: an LDS-staged full-row variant measured slower,
  // 67 vs 42 us on the 25600 x 512 pooling U -- L2 merges the 64-B pieces)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = col0 + 16 * t + ar;
    if (n >= N) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = row0 + kq * 4 + r;
      if (m < M) {
        float v = acc[t][r] + bv;
        if (act == 1) v = v > 0.f ? v : 0.f;
        Y[(size_t)m * ldy + n] = v;
      }
    }
  }
}

}  // namespace sgg

extern "C" int sgg_xw(const float* X, int ldx, const float* Xmask, int ldm, const float* W, int ldw, int trans_w,
                      const float* bias, float* Y, int ldy, int M, int K, int N, int act, void* stream) {
  SGG_CHECK_ARG(X && W && Y, "sgg_xw: null pointer");
  SGG_CHECK_ARG(M >= 0 && K > 0 && N > 0, "sgg_xw: bad sizes M=%d K=%d N=%d", M, K, N);
  SGG_CHECK_ARG(ldx >= K && ldy >= N && ldw >= (trans_w ? K : N), "sgg_xw: bad leading dims ldx=%d ldw=%d ldy=%d",
                ldx, ldw, ldy);
  SGG_CHECK_ARG(act == 0 || act == 1, "sgg_xw: act must be 0 or 1");
  SGG_CHECK_ARG(!Xmask || ldm >= K, "sgg_xw: mask leading dim %d < K", ldm);
  if (M == 0) return 0;
  dim3 grid((M + 63) / 64, (N + 63) / 64);
  hipStream_t s = (hipStream_t)stream;
  if (trans_w)
    hipLaunchKernelGGL(sgg::xw_kernel<true>, grid, dim3(256), 0, s, X, ldx, Xmask, ldm, W, ldw, bias, Y, ldy, M, K, N, act);
  else
    hipLaunchKernelGGL(sgg::xw_kernel<false>, grid, dim3(256), 0, s, X, ldx, Xmask, ldm, W, ldw, bias, Y, ldy, M, K, N, act);
  SGG_RETURN_LAUNCH("sgg_xw");
}
