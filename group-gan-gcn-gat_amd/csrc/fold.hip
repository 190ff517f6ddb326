// Input-embedding fold of the path's first layers (one launch each way).
//
// Every Linear(2, E) embedding of a displacement feeds a linear layer
// straight away: the LSTM input weights of Encoder/Decoder (reference
// sgan/models.py:52-59, 121-125; W_ih (4H x E), biases b_ih + b_hh) and the
// first pooling layer (models.py:477-481, 530-538: W1[:, :E], b1).  Folding
//   W (We r + be) + b1 (+ b2)  =  A r + bias,   A = W We (R x 2),
//                                              bias = W be + b1 (+ b2)
// turns the per-(ped, step) / per-pair embedding into two FMAs.  The fold
// runs once per forward; its backward maps (dA, dbias) back to
//   dW = dA We^T + dbias be^T,  dWe = W^T dA,  dbe = W^T dbias,
//   db1 = db2 = dbias (left to the caller: no copy needed).
// R <= 512, E <= 128: one workgroup, latency-bound -- the point is one
// launch instead of the ~3 forward / ~5 backward BLAS + elementwise launches
// autograd would issue for the same algebra.
#include "sgg_common.h"

namespace sgg {

__global__ void __launch_bounds__(512) fold_fwd_kernel(const float* __restrict__ W, int ldw, int R, int E,
                                                       const float* __restrict__ We, const float* __restrict__ be,
                                                       const float* __restrict__ b1, const float* __restrict__ b2,
                                                       float* __restrict__ A, float* __restrict__ bias) {
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    float a0 = 0.f, a1 = 0.f, bb = 0.f;
    const float* w = W + (size_t)r * ldw;
#pragma unroll 8
    for (int e = 0; e < E; ++e) {
      const float we = w[e];
      a0 = fmaf(we, We[2 * e], a0);
      a1 = fmaf(we, We[2 * e + 1], a1);
      bb = fmaf(we, be[e], bb);
    }
    A[2 * r] = a0;
    A[2 * r + 1] = a1;
    bias[r] = bb + b1[r] + (b2 ? b2[r] : 0.f);
  }
}

// every fold of a module set in one launch: workgroup k computes fold k
struct FoldList {
  SggFold f[SGG_FOLD_MAX];
};

__global__ void __launch_bounds__(512) fold_fwd_multi_kernel(FoldList L) {
  const SggFold& d = L.f[blockIdx.x];
  for (int r = threadIdx.x; r < d.R; r += blockDim.x) {
    float a0 = 0.f, a1 = 0.f, bb = 0.f;
    const float* w = d.W + (size_t)r * d.ldw;
#pragma unroll 8
    for (int e = 0; e < d.E; ++e) {
      const float we = w[e];
      a0 = fmaf(we, d.We[2 * e], a0);
      a1 = fmaf(we, d.We[2 * e + 1], a1);
      bb = fmaf(we, d.be[e], bb);
    }
    d.A[2 * r] = a0;
    d.A[2 * r + 1] = a1;
    d.bias[r] = bb + d.b1[r] + (d.b2 ? d.b2[r] : 0.f);
  }
}

// (dA, dbias) staged in LDS once; thread t owns column e = t % E of row group
// g = t / E (ng = 512 / E groups): its dW entries need no global load (We, be
// of its column in registers), and its three column sums walk the group's
// rows with the W loads all independent (many in flight); the groups are
// summed in LDS in a fixed order.
__device__ __forceinline__ void fold_bwd_body(const float* __restrict__ W, int ldw, int R, int E,
                                              const float* __restrict__ We, const float* __restrict__ be,
                                              const float* __restrict__ dA, const float* __restrict__ dbias,
                                              float* __restrict__ dW, int lddw, float* __restrict__ dWe,
                                              float* __restrict__ dbe, float* __restrict__ dbias_copy) {
  __shared__ float g3[3 * 512];        // (dA_x, dA_y, dbias) per row, R <= 512
  __shared__ float part[3 * 512];      // per (group, column) sums
  for (int r = threadIdx.x; r < R; r += blockDim.x) {
    const float2 a = reinterpret_cast<const float2*>(dA)[r];
    const float b = dbias[r];
    g3[3 * r] = a.x;
    g3[3 * r + 1] = a.y;
    g3[3 * r + 2] = b;
    // the second bias leaf (b_hh next to b_ih) gets its own copy of dbias
    if (dbias_copy) dbias_copy[r] = b;
  }
  __syncthreads();
  const int ng = blockDim.x / E;
  const int t = threadIdx.x;
  if (t < ng * E) {
    const int e = t % E, g = t / E;
    const float we0 = We[2 * e], we1 = We[2 * e + 1], bee = be[e];
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll 8
    for (int r = g; r < R; r += ng) {
      const float a0 = g3[3 * r], a1 = g3[3 * r + 1], b = g3[3 * r + 2];
      dW[(size_t)r * lddw + e] = fmaf(a0, we0, fmaf(a1, we1, b * bee));
      const float w = W[(size_t)r * ldw + e];
      s0 = fmaf(w, a0, s0);
      s1 = fmaf(w, a1, s1);
      s2 = fmaf(w, b, s2);
    }
    part[3 * t] = s0;
    part[3 * t + 1] = s1;
    part[3 * t + 2] = s2;
  }
  __syncthreads();
  if (t < 3 * E) {   // output (e, j): dWe[e][j] (j < 2) or dbe[e] (j = 2)
    const int e = t / 3, j = t - 3 * e;
    float s = 0.f;
    for (int g = 0; g < ng; ++g) s += part[3 * (g * E + e) + j];
    if (j < 2) dWe[2 * e + j] = s;
    else dbe[e] = s;
  }
}

__global__ void __launch_bounds__(512) fold_bwd_kernel(const float* __restrict__ W, int ldw, int R, int E,
                                                       const float* __restrict__ We, const float* __restrict__ be,
                                                       const float* __restrict__ dA, const float* __restrict__ dbias,
                                                       float* __restrict__ dW, int lddw, float* __restrict__ dWe,
                                                       float* __restrict__ dbe, float* __restrict__ dbias_copy) {
  fold_bwd_body(W, ldw, R, E, We, be, dA, dbias, dW, lddw, dWe, dbe, dbias_copy);
}

// every fold backward of a grad finish in one launch: workgroup k runs fold k
// on its summed (dA, dbias) (dA_src / db_src point at the sums)
struct FoldBwdList {
  SggFoldBwd f[SGG_FOLDB_MAX];
};

__global__ void __launch_bounds__(512) fold_bwd_multi_kernel(FoldBwdList L) {
  const SggFoldBwd& d = L.f[blockIdx.x];
  fold_bwd_body(d.W, d.ldw, d.R, d.E, d.We, d.be, d.dA_src, d.db_src, d.dW, d.lddw, d.dWe, d.dbe, d.dbias_copy);
}

void fold_bwd_multi(const SggFoldBwd* folds, int n, hipStream_t st) {
  FoldBwdList L;
  for (int k = 0; k < n; ++k) L.f[k] = folds[k];
  hipLaunchKernelGGL(fold_bwd_multi_kernel, dim3(n), dim3(512), 0, st, L);
}

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_fold_fwd(const float* W, int ldw, int R, int E, const float* We, const float* be, const float* b1,
                            const float* b2, float* A, float* bias, void* stream) {
  SGG_CHECK_ARG(W && We && be && b1 && A && bias, "sgg_fold_fwd: null pointer");
  SGG_CHECK_ARG(R >= 1 && E >= 1 && ldw >= E, "sgg_fold_fwd: bad sizes R=%d E=%d ldw=%d", R, E, ldw);
  hipLaunchKernelGGL(fold_fwd_kernel, dim3(1), dim3(512), 0, (hipStream_t)stream, W, ldw, R, E, We, be, b1, b2, A,
                     bias);
  SGG_RETURN_LAUNCH("sgg_fold_fwd");
}

extern "C" int sgg_fold_fwd_multi(const SggFold* folds, int n, void* stream) {
  SGG_CHECK_ARG(folds && n >= 1 && n <= SGG_FOLD_MAX, "sgg_fold_fwd_multi: 1 <= n <= %d folds (got %d)", SGG_FOLD_MAX, n);
  FoldList L;
  for (int k = 0; k < n; ++k) {
    const SggFold& d = folds[k];
    SGG_CHECK_ARG(d.W && d.We && d.be && d.b1 && d.A && d.bias, "sgg_fold_fwd_multi: null pointer in fold %d", k);
    SGG_CHECK_ARG(d.R >= 1 && d.E >= 1 && d.ldw >= d.E, "sgg_fold_fwd_multi: bad sizes in fold %d", k);
    L.f[k] = d;
  }
  hipLaunchKernelGGL(fold_fwd_multi_kernel, dim3(n), dim3(512), 0, (hipStream_t)stream, L);
  SGG_RETURN_LAUNCH("sgg_fold_fwd_multi");
}

extern "C" int sgg_fold_bwd(const float* W, int ldw, int R, int E, const float* We, const float* be, const float* dA,
                            const float* dbias, float* dW, int lddw, float* dWe, float* dbe, float* dbias_copy,
                            void* stream) {
  SGG_CHECK_ARG(W && We && be && dA && dbias && dW && dWe && dbe, "sgg_fold_bwd: null pointer");
  SGG_CHECK_ARG(R >= 1 && R <= 512 && E >= 1 && E <= 128 && ldw >= E && lddw >= E, "sgg_fold_bwd: bad sizes");
  hipLaunchKernelGGL(fold_bwd_kernel, dim3(1), dim3(512), 0, (hipStream_t)stream, W, ldw, R, E, We, be, dA, dbias,
                     dW, lddw, dWe, dbe, dbias_copy);
  SGG_RETURN_LAUNCH("sgg_fold_bwd");
}
