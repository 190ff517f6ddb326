// Dense node-feature transform Y = act(X @ W (+ bias)) on fp32 MFMA.
//
// v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain, no xf32):
//   A lane map: A[l & 15][l >> 4]    (16 rows x 4 k)
//   B lane map: B[l >> 4][l & 15]    (4 k x 16 cols)
//   C/D map   : row = (l >> 4) * 4 + r, col = l & 15   (r = 0..3)
// Workgroup = 4 waves = 64 rows x 64 cols of Y; each wave owns 16 rows x 64
// cols (4 accumulator tiles).  K is small on most of this path (2..144), so
// the X fragments are read straight from L1/L2 with a deep register prefetch
// (these launches are latency-bound: a few dozen workgroups).  A weight in the
// nn.Linear layout (N x K, TRANS_W) with K <= 256 is staged once per
// workgroup in LDS -- its 64 rows read along k, coalesced -- instead of a
// lane-per-column fragment read that touches one cache line per lane.
// Large K (>= 256: the pooling backward dh = dU W1h, K = 512) takes the
// split-K form: a workgroup = 16 rows x 64 cols whose 4 waves each walk a
// quarter of K, the partial tiles summed through LDS in wave order.
#include <stdlib.h>

#include "sgg_common.h"
#include "xtw_body.h"

namespace sgg {

constexpr int kXwKC = 16;            // K chunk: 4 MFMA k-steps, double-buffered in registers
constexpr int kXwS4 = kXwKC / 4;
constexpr int kXwStageMaxK = 256;    // TRANS_W weights staged in LDS up to this K

// Operand fetch of one 16-row x 64-col wave tile over k in [kb, kend):
// X rows from global, W from global (row-major K x N, or N x K if TRANS_W)
// or from the LDS image `ws` (64 rows x K at pitch K + 1, TRANS_W staged).
// Loads use clamped (in-bounds) addresses; only k >= kend must contribute
// zero, which concerns the last chunk alone -- a wave-uniform branch (a
// per-load `cond ? v : 0` makes the compiler sink each load into an
// exec-masked branch that waits for it).
template <bool TRANS_W, bool STAGED>
struct XwFrag {
  const float* xrow;
  const float* mrow;
  const float* W;
  const float* ws;
  int ldw, kp, kend;
  int ncl[4];   // clamped global output columns (unstaged) / local rows of ws (staged)
  int kq;

  __device__ __forceinline__ float wval(int t, int k) const {
    if (STAGED) return ws[ncl[t] * kp + k];
    return TRANS_W ? W[(size_t)ncl[t] * ldw + k] : W[(size_t)k * ldw + ncl[t]];
  }
  // k order within a 16-deep chunk is permuted: k-step s of lane quarter kq
  // takes k = kb + 4 kq + s (the same for both operands), so a lane's four
  // A values of a chunk are one 16-byte load (full 64-byte lines per wave
  // instruction instead of 16-byte pieces of 16 lines)
  bool vec;   // X (and the mask) rows 16-byte aligned
  __device__ __forceinline__ void load_a(int kb, float (&aa)[kXwS4]) const {
    if (kb + kXwKC <= kend) {
      if (vec) {
        const float4 v = *reinterpret_cast<const float4*>(xrow + kb + 4 * kq);
        aa[0] = v.x;
        aa[1] = v.y;
        aa[2] = v.z;
        aa[3] = v.w;
        if (mrow) {
          const float4 mv = *reinterpret_cast<const float4*>(mrow + kb + 4 * kq);
          aa[0] = keep_if(aa[0], mv.x > 0.f);
          aa[1] = keep_if(aa[1], mv.y > 0.f);
          aa[2] = keep_if(aa[2], mv.z > 0.f);
          aa[3] = keep_if(aa[3], mv.w > 0.f);
        }
        return;
      }
#pragma unroll
      for (int s = 0; s < kXwS4; ++s) {
        const int k = kb + 4 * kq + s;
        aa[s] = mrow ? keep_if(xrow[k], mrow[k] > 0.f) : xrow[k];
      }
    } else {
#pragma unroll
      for (int s = 0; s < kXwS4; ++s) {
        const int k = kb + 4 * kq + s;
        const int kc = min(k, kend - 1);
        aa[s] = keep_if(xrow[kc], k < kend && (!mrow || mrow[kc] > 0.f));
      }
    }
  }
  __device__ __forceinline__ void load_b(int kb, float (&bb)[kXwS4][4]) const {
#pragma unroll
    for (int s = 0; s < kXwS4; ++s) {
      const int kc = min(kb + 4 * kq + s, kend - 1);   // past kend the A operand is zero
#pragma unroll
      for (int t = 0; t < 4; ++t) bb[s][t] = wval(t, kc);
    }
  }
  __device__ __forceinline__ void load(int kb, float (&aa)[kXwS4], float (&bb)[kXwS4][4]) const {
    load_a(kb, aa);
    load_b(kb, bb);
  }
};

// acc[t] += X[rows, kb0..kend) W[kb0..kend), cols]: the next chunk's loads are
// in flight while the current chunk runs through the MFMAs
// apre: the first chunk's A fragments, already loaded by the caller (issued
// before the weight staging, so the two memory latencies overlap)
template <bool TRANS_W, bool STAGED>
__device__ __forceinline__ void xw_walk(const XwFrag<TRANS_W, STAGED>& f, int kb0, floatx4 (&acc)[4],
                                        const float (*apre)[kXwS4] = nullptr) {
  if (kb0 >= f.kend) return;
  float a0[kXwS4], b0[kXwS4][4], a1[kXwS4], b1[kXwS4][4];
  if (apre) {
#pragma unroll
    for (int s = 0; s < kXwS4; ++s) a0[s] = (*apre)[s];
    f.load_b(kb0, b0);
  } else {
    f.load(kb0, a0, b0);
  }
  for (int k0 = kb0; k0 < f.kend; k0 += 2 * kXwKC) {
    if (k0 + kXwKC < f.kend) f.load(k0 + kXwKC, a1, b1);
#pragma unroll
    for (int s = 0; s < kXwS4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b0[s][t], acc[t], 0, 0, 0);
    if (k0 + kXwKC >= f.kend) break;
    if (k0 + 2 * kXwKC < f.kend) f.load(k0 + 2 * kXwKC, a0, b0);
#pragma unroll
    for (int s = 0; s < kXwS4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], b1[s][t], acc[t], 0, 0, 0);
  }
}

__device__ __forceinline__ float xw_epi(float v, const float* bias, int n, int act) {
  if (bias) v += bias[n];
  if (act & 1) v = v > 0.f ? v : 0.f;
  return v;
}

template <bool TRANS_W, bool STAGED>
__global__ void __launch_bounds__(256) xw_kernel(const float* __restrict__ X, int ldx,
                                                 const float* __restrict__ Xmask, int ldm,
                                                 const float* __restrict__ W, int ldw,
                                                 const float* __restrict__ bias, float* __restrict__ Y,
                                                 int ldy, int M, int K, int N, int act) {
  extern __shared__ float wsm[];   // STAGED: this workgroup's 64 W rows x K at pitch K + 1
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int row0 = blockIdx.x * 64 + wave * 16;
  const int col0 = blockIdx.y * 64;
  const int ar = lane & 15;   // A row / B col within the 16x16 tile
  const int kq = lane >> 4;   // k within the 4-deep step
  const int arow = row0 + ar;
  const bool arow_ok = arow < M;
  XwFrag<TRANS_W, STAGED> f;
  f.xrow = X + (size_t)(arow_ok ? arow : 0) * ldx;
  // ReLU backward fused into the operand: X[m, k] counts where Xmask[m, k] > 0
  f.mrow = Xmask ? Xmask + (size_t)(arow_ok ? arow : 0) * ldm : nullptr;
  f.W = W;
  f.ws = wsm;
  f.ldw = ldw;
  f.kp = K + 1;
  f.kend = K;
  f.kq = kq;
  f.vec = ((reinterpret_cast<uintptr_t>(X) | (uintptr_t)ldx * 4 |
            (Xmask ? (reinterpret_cast<uintptr_t>(Xmask) | (uintptr_t)ldm * 4) : 0)) & 15) == 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) f.ncl[t] = STAGED ? min(16 * t + ar, N - 1 - col0) : min(col0 + 16 * t + ar, N - 1);
  // the lane's four bias values, fetched up front (not a memory round trip in the epilogue)
  float bcol[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) bcol[t] = bias ? bias[min(col0 + 16 * t + ar, N - 1)] : 0.f;
  float apre[kXwS4];
  if (STAGED) {
    f.load_a(0, apre);   // the first X chunk in flight across the weight staging
    // the 64 rows of the N x K weight this workgroup needs: four threads per
    // row, thread k0 takes k = k0, k0 + 4, ... (no index division), 16 loads
    // in flight before the LDS stores (one round trip for K <= 64)
    const int kp = K + 1;
    const int nl = threadIdx.x >> 2, k0 = threadIdx.x & 3;
    const float* wrow = W + (size_t)min(col0 + nl, N - 1) * ldw;
    float* srow = wsm + nl * kp;
    for (int j0 = 0; j0 < K; j0 += 64) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = wrow[min(j0 + k0 + 4 * u, K - 1)];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = j0 + k0 + 4 * u;
        if (k < K) srow[k] = v[u];
      }
    }
    __syncthreads();
  }
  floatx4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  xw_walk(f, 0, acc, STAGED ? &apre : nullptr);

  // epilogue (direct stores: an LDS-staged full-row variant measured slower,
  // 67 vs 42 us on the 25600 x 512 pooling U -- L2 merges the 64-B pieces)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = col0 + 16 * t + ar;
    if (n >= N) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = row0 + kq * 4 + r;
      if (m < M) {
        float* py = Y + (size_t)m * ldy + n;
        float v = acc[t][r] + bcol[t];
        if (act & 1) v = v > 0.f ? v : 0.f;
        *py = v + ((act & 2) ? *py : 0.f);
      }
    }
  }
}

constexpr int kXwSplitLds = 4 * 16 * 65;   // LDS floats of one split-K workgroup

template <bool TRANS_W>
__device__ __forceinline__ void xw_splitk_body(const float* __restrict__ X, int ldx, const float* __restrict__ Xmask,
                                               int ldm, const float* __restrict__ W, int ldw,
                                               const float* __restrict__ bias, float* __restrict__ Y, int ldy, int M,
                                               int K, int N, int act, int bx, int by, float* smem) {
  float (*part)[16][65] = reinterpret_cast<float (*)[16][65]>(smem);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int row0 = bx * 16;
  const int col0 = by * 64;
  const int ar = lane & 15, kq = lane >> 4;
  const int arow = row0 + ar;
  const bool arow_ok = arow < M;
  const int span = (((K + 3) / 4) + kXwKC - 1) / kXwKC * kXwKC;   // this wave's K range
  XwFrag<TRANS_W, false> f;
  f.xrow = X + (size_t)(arow_ok ? arow : 0) * ldx;
  f.mrow = Xmask ? Xmask + (size_t)(arow_ok ? arow : 0) * ldm : nullptr;
  f.W = W;
  f.ws = nullptr;
  f.ldw = ldw;
  f.kp = 0;
  f.kend = min(K, (wave + 1) * span);
  f.kq = kq;
  f.vec = ((reinterpret_cast<uintptr_t>(X) | (uintptr_t)ldx * 4 |
            (Xmask ? (reinterpret_cast<uintptr_t>(Xmask) | (uintptr_t)ldm * 4) : 0)) & 15) == 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) f.ncl[t] = min(col0 + 16 * t + ar, N - 1);
  floatx4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  xw_walk(f, wave * span, acc);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wave][kq * 4 + r][16 * t + ar] = acc[t][r];
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * 64; e += 256) {
    const int rr = e >> 6, cc = e & 63;
    const int m = row0 + rr, n = col0 + cc;
    if (m < M && n < N) {
      float* py = Y + (size_t)m * ldy + n;
      *py = xw_epi(((part[0][rr][cc] + part[1][rr][cc]) + part[2][rr][cc]) + part[3][rr][cc], bias, n, act) +
            ((act & 2) ? *py : 0.f);
    }
  }
}

template <bool TRANS_W>
__global__ void __launch_bounds__(256) xw_splitk_kernel(const float* __restrict__ X, int ldx,
                                                        const float* __restrict__ Xmask, int ldm,
                                                        const float* __restrict__ W, int ldw,
                                                        const float* __restrict__ bias, float* __restrict__ Y,
                                                        int ldy, int M, int K, int N, int act) {
  __shared__ float part[kXwSplitLds];
  xw_splitk_body<TRANS_W>(X, ldx, Xmask, ldm, W, ldw, bias, Y, ldy, M, K, N, act, blockIdx.x, blockIdx.y, part);
}

// The pooling backward's two independent products of dU (B x 512) in ONE
// launch: dh (+)= dU W1h (split-K, as sgg_xw with K >= 256) and the split-K
// partials of dW1h^T = h^T dU with the column sums of dU (as
// sgg_xtw_partial); the first nxw workgroups take the former, the rest the
// latter.  (Two launches of ~7-8 us each before.)
template <int MT>
__global__ void __launch_bounds__(256) xw_xtw_kernel(const float* __restrict__ dU, int ldu, const float* __restrict__ W,
                                                     int ldw, float* __restrict__ dh, int ldh, int act, int B, int K,
                                                     int H, int nxw_x, int nxw, const float* __restrict__ X, int ldx,
                                                     int rows_per_split, int gx, int gy, float* __restrict__ slab,
                                                     float* __restrict__ colslab) {
  __shared__ float smem[kXwSplitLds > kXtwRedFloats ? kXwSplitLds : kXtwRedFloats];
  const int b = blockIdx.x;
  if (b < nxw) {
    xw_splitk_body<false>(dU, ldu, nullptr, 0, W, ldw, nullptr, dh, ldh, B, K, H, act, b % nxw_x, b / nxw_x, smem);
  } else {
    const int q = b - nxw;
    xtw_partial_body<MT>(X, ldx, dU, ldu, nullptr, 0, B, H, K, rows_per_split, slab, colslab, q % gx, (q / gx) % gy,
                         q / (gx * gy), smem);
  }
}

// ---------------------------------------------------------------------------
// bf16 variant (opt-in, BASELINE configs 3 and 5: "bf16 + MFMA XW"): X and W
// rounded to bf16 (round-to-nearest-even), v_mfma_f32_16x16x32_bf16, fp32
// accumulate, fp32 epilogue / output.  Same tiling as xw_kernel (4 waves x
// 16 rows x 64 cols); lane l holds A[row l & 15][k = 8 (l >> 4) + j] and
// B[k = 8 (l >> 4) + j][col l & 15], j = 0..7, so one k-step covers 32 k.
// Operands are read straight from global (L2-resident: K <= 512 here).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <bool TRANS_W>
__global__ void __launch_bounds__(256) xw_bf16_kernel(const float* __restrict__ X, int ldx,
                                                      const float* __restrict__ Xmask, int ldm,
                                                      const float* __restrict__ W, int ldw,
                                                      const float* __restrict__ bias, float* __restrict__ Y,
                                                      int ldy, int M, int K, int N, int act) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int row0 = blockIdx.x * 64 + wave * 16;
  const int col0 = blockIdx.y * 64;
  const int ar = lane & 15, kg = lane >> 4;
  const int arow = min(row0 + ar, M - 1);
  const float* xrow = X + (size_t)arow * ldx;
  const float* mrow = Xmask ? Xmask + (size_t)arow * ldm : nullptr;
  int ncl[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) ncl[t] = min(col0 + 16 * t + ar, N - 1);
  floatx4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 32) {
    const int kb = k0 + 8 * kg;
    bf16x8 a;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kb + j, kc = min(k, K - 1);
      const bool keep = k < K && (!mrow || mrow[kc] > 0.f);
      a[j] = (__bf16)keep_if(xrow[kc], keep);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bf16x8 b;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kc = min(kb + j, K - 1);   // k >= K meets a zero A element
        b[j] = (__bf16)(TRANS_W ? W[(size_t)ncl[t] * ldw + kc] : W[(size_t)kc * ldw + ncl[t]]);
      }
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = col0 + 16 * t + ar;
    if (n >= N) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = row0 + kg * 4 + r;
      if (m < M) {
        float* py = Y + (size_t)m * ldy + n;
        *py = xw_epi(acc[t][r], bias, n, act) + ((act & 2) ? *py : 0.f);
      }
    }
  }
}

}  // namespace sgg

extern "C" int sgg_xw_bf16(const float* X, int ldx, const float* Xmask, int ldm, const float* W, int ldw, int trans_w,
                           const float* bias, float* Y, int ldy, int M, int K, int N, int act, void* stream) {
  SGG_CHECK_ARG(X && W && Y, "sgg_xw_bf16: null pointer");
  SGG_CHECK_ARG(M >= 0 && K > 0 && N > 0, "sgg_xw_bf16: bad sizes M=%d K=%d N=%d", M, K, N);
  // (the row stride of a one-row weight is never used: torch reports any value for it)
  SGG_CHECK_ARG(ldx >= K && ldy >= N && (trans_w ? (N == 1 || ldw >= K) : (K == 1 || ldw >= N)),
                "sgg_xw_bf16: bad leading dims ldx=%d ldw=%d ldy=%d (M=%d K=%d N=%d trans=%d)", ldx, ldw, ldy, M, K, N,
                trans_w);
  SGG_CHECK_ARG(act >= 0 && act <= 3, "sgg_xw_bf16: act must be 0..3 (bit 0 ReLU, bit 1 accumulate)");
  SGG_CHECK_ARG(!Xmask || ldm >= K, "sgg_xw_bf16: mask leading dim %d < K", ldm);
  if (M == 0) return 0;
  dim3 grid((M + 63) / 64, (N + 63) / 64);
  hipStream_t s = (hipStream_t)stream;
  if (trans_w)
    hipLaunchKernelGGL(sgg::xw_bf16_kernel<true>, grid, dim3(256), 0, s, X, ldx, Xmask, ldm, W, ldw, bias, Y, ldy, M, K,
                       N, act);
  else
    hipLaunchKernelGGL(sgg::xw_bf16_kernel<false>, grid, dim3(256), 0, s, X, ldx, Xmask, ldm, W, ldw, bias, Y, ldy, M,
                       K, N, act);
  SGG_RETURN_LAUNCH("sgg_xw_bf16");
}

extern "C" int sgg_xw(const float* X, int ldx, const float* Xmask, int ldm, const float* W, int ldw, int trans_w,
                      const float* bias, float* Y, int ldy, int M, int K, int N, int act, void* stream) {
  SGG_CHECK_ARG(X && W && Y, "sgg_xw: null pointer");
  SGG_CHECK_ARG(M >= 0 && K > 0 && N > 0, "sgg_xw: bad sizes M=%d K=%d N=%d", M, K, N);
  SGG_CHECK_ARG(ldx >= K && ldy >= N && (trans_w ? (N == 1 || ldw >= K) : (K == 1 || ldw >= N)),
                "sgg_xw: bad leading dims ldx=%d ldw=%d ldy=%d", ldx, ldw, ldy);
  SGG_CHECK_ARG(act >= 0 && act <= 3, "sgg_xw: act must be 0..3 (bit 0 ReLU, bit 1 accumulate)");
  SGG_CHECK_ARG(!Xmask || ldm >= K, "sgg_xw: mask leading dim %d < K", ldm);
  if (M == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (K >= 256) {
    dim3 grid((M + 15) / 16, (N + 63) / 64);
    if (trans_w)
      hipLaunchKernelGGL(sgg::xw_splitk_kernel<true>, grid, dim3(256), 0, s, X, ldx, Xmask, ldm, W, ldw, bias, Y, ldy,
                         M, K, N, act);
    else
      hipLaunchKernelGGL(sgg::xw_splitk_kernel<false>, grid, dim3(256), 0, s, X, ldx, Xmask, ldm, W, ldw, bias, Y, ldy,
                         M, K, N, act);
    SGG_RETURN_LAUNCH("sgg_xw");
  }
  dim3 grid((M + 63) / 64, (N + 63) / 64);
  if (trans_w && K <= sgg::kXwStageMaxK)
    hipLaunchKernelGGL((sgg::xw_kernel<true, true>), grid, dim3(256), sizeof(float) * 64 * (K + 1), s, X, ldx, Xmask,
                       ldm, W, ldw, bias, Y, ldy, M, K, N, act);
  else if (trans_w)
    hipLaunchKernelGGL((sgg::xw_kernel<true, false>), grid, dim3(256), 0, s, X, ldx, Xmask, ldm, W, ldw, bias, Y, ldy,
                       M, K, N, act);
  else
    hipLaunchKernelGGL((sgg::xw_kernel<false, false>), grid, dim3(256), 0, s, X, ldx, Xmask, ldm, W, ldw, bias, Y,
                       ldy, M, K, N, act);
  SGG_RETURN_LAUNCH("sgg_xw");
}

extern "C" int sgg_xtw_splits(int R, int M, int N);
using sgg::kHidden;

extern "C" int sgg_pool_dh_dw(const float* dU, int ldu, const float* W, int ldw, float* dh, int ldh, int accumulate,
                              const float* h, int ldx, int B, int H, float* ws, size_t ws_bytes, void* stream) {
  SGG_CHECK_ARG(dU && W && dh && h && ws, "sgg_pool_dh_dw: null pointer");
  SGG_CHECK_ARG(B >= 1 && H >= 1 && H <= 64 && ldu >= kHidden && ldw >= H && ldh >= H && ldx >= H,
                "sgg_pool_dh_dw: bad sizes B=%d H=%d", B, H);
  const int splits = sgg_xtw_splits(B, H, kHidden);
  const size_t need = sizeof(float) * (size_t)splits * ((size_t)H * kHidden + kHidden);
  SGG_CHECK_ARG(ws_bytes >= need, "sgg_pool_dh_dw: workspace %zu < %zu bytes", ws_bytes, need);
  const int nxw_x = (B + 15) / 16, nxw = nxw_x * ((H + 63) / 64);
  const int gx = (H + 63) / 64, gy = kHidden / 64;
  const int rps = ((B + splits - 1) / splits + 63) & ~63;   // (xtw.hip launch_partial)
  const dim3 grid(nxw + gx * gy * splits);
  float* colslab = ws + (size_t)splits * H * kHidden;
  hipStream_t st = (hipStream_t)stream;
  const int act = accumulate ? 2 : 0;
#define SGG_XWXTW(MT)                                                                                               \
  hipLaunchKernelGGL(sgg::xw_xtw_kernel<MT>, grid, dim3(256), 0, st, dU, ldu, W, ldw, dh, ldh, act, B, kHidden, H, \
                     nxw_x, nxw, h, ldx, rps, gx, gy, ws, colslab)
  switch (H >= 64 ? 4 : (H + 15) / 16) {
    case 1: SGG_XWXTW(1); break;
    case 2: SGG_XWXTW(2); break;
    case 3: SGG_XWXTW(3); break;
    default: SGG_XWXTW(4); break;
  }
#undef SGG_XWXTW
  SGG_RETURN_LAUNCH("sgg_pool_dh_dw");
}
