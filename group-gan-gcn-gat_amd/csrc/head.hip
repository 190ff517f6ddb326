// The discriminator's scoring head in one launch per direction:
//   real_classifier = make_mlp([h_dim, mlp_dim, 1]) (reference sgan/models.py:
//   958-965, make_mlp :7-20, called at :991): Linear(K, N1) -> ReLU ->
//   Linear(N1, 1) -> ReLU.
// Forward (sgg_head_fwd): hid = act1(X W1^T + b1) on v_mfma_f32_16x16x4_f32
// (exact fp32), then y = act2(hid . w2 + b2) from the accumulator tiles
// (per-lane partial over the column tiles, then a 16-lane xor tree) -- the
// hidden layer never makes a second pass through memory; hid is stored for
// the backward's ReLU mask.
// Backward (sgg_head_bwd): g2 = dY (Y > 0), dhid = g2 w2 (hid > 0) staged in
// LDS, dX = dhid W1 on the MFMA, and (wslab != NULL) one slab row per
// workgroup [dW1 (N1 x K) | db1 (N1) | dW2 (N1) | db2] over its 64 rows:
// dW1 = dhid^T X on the MFMA (each wave a quarter of the output tiles over all
// 64 rows: no cross-wave sum), the vector sums in row order.  sgg_grad_finish
// sums the rows.  Replaces 2 forward and up to 6 backward launches (two node
// transforms, two input-gradient transforms, two split-K reductions).
#include "sgg_common.h"

namespace sgg {

namespace {

constexpr int kHeadRows = 64;   // rows per workgroup (4 waves x 16)

// d bce / d x, the expression of loss.hip's bce_grad (torch autograd's form)
__device__ __forceinline__ float bce_grad(float x, float y) {
  const float e = expf(-fabsf(x));
  const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
  return (x >= 0.f ? 1.f : 0.f) - y - sg * (e / (1.f + e));
}

template <int NT, int KT>   // NT = N1 / 16 hidden column tiles, K = 16 KT inputs
__global__ void __launch_bounds__(256) head_fwd_kernel(const float* __restrict__ X, int ldx, int M,
                                                       const float* __restrict__ W1, const float* __restrict__ b1,
                                                       const float* __restrict__ w2, const float* __restrict__ b2,
                                                       int act, float* __restrict__ hid, float* __restrict__ Y) {
  constexpr int K = 16 * KT, KS = 4 * KT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * kHeadRows + wave * 16;
  const float* xr = X + (size_t)min(row0 + c16, M - 1) * ldx;
  // every operand of the lane issued up front: one memory round trip.  The k
  // order is permuted (k-step 4 m + i, lane quarter q <-> k = 16 m + 4 q + i),
  // the same for both operands, so a lane's four k values of block m are one
  // 16-byte load of X and of each W1 row (full 64-byte lines per instruction)
  float a[KS], b[KS][NT], bc[NT], wc[NT];
#pragma unroll
  for (int m = 0; m < KT; ++m) {
    const float4 xv = *reinterpret_cast<const float4*>(xr + 16 * m + 4 * q);
    a[4 * m] = xv.x;
    a[4 * m + 1] = xv.y;
    a[4 * m + 2] = xv.z;
    a[4 * m + 3] = xv.w;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float4 wv = *reinterpret_cast<const float4*>(W1 + (size_t)(16 * t + c16) * K + 16 * m + 4 * q);
      b[4 * m][t] = wv.x;
      b[4 * m + 1][t] = wv.y;
      b[4 * m + 2][t] = wv.z;
      b[4 * m + 3][t] = wv.w;
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bc[t] = b1[16 * t + c16];
    wc[t] = w2[16 * t + c16];
  }
  const float bb2 = b2[0];
  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s][t], acc[t], 0, 0, 0);
  // epilogue: lane holds rows 4 q + r, columns 16 t + c16
  const int N1 = 16 * NT;
  float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float h = acc[t][r] + bc[t];
      if (act & 1) h = h > 0.f ? h : 0.f;
      const int m = row0 + 4 * q + r;
      if (m < M) hid[(size_t)m * N1 + 16 * t + c16] = h;
      p[r] = fmaf(h, wc[t], p[r]);
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) p[r] += __shfl_xor(p[r], o);
    float y = p[r] + bb2;
    if (act & 2) y = y > 0.f ? y : 0.f;
    const int m = row0 + 4 * q + r;
    if (c16 == 0 && m < M) Y[m] = y;
  }
}

// the backward after dhid is staged: dX = dhid W1 (the W1 fragments wb were
// loaded before the staging barrier) and, with wslab, the workgroup's slab row
template <int NT, int KT, int DP>
__device__ __forceinline__ void head_bwd_tail(const float* __restrict__ X, int ldx, int M, int rb,
                                              const float (&dh)[kHeadRows][DP], const float (&hg)[kHeadRows][DP],
                                              const float (&g2s)[kHeadRows], const float (&wb)[4 * NT][KT],
                                              float* __restrict__ dX, int lddx, float* __restrict__ wslab) {
  constexpr int N1 = 16 * NT, K = 16 * KT;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  // dX (this wave's 16 rows) = dhid W1: A[row][k = n] from LDS, B[n][col] = W1[n][col]
  {
    floatx4 acc[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < N1 / 4; ++s) {
      const float a = dh[16 * wave + c16][4 * s + q];
#pragma unroll
      for (int t = 0; t < KT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, wb[s][t], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = rb + 16 * wave + 4 * q + r;
        if (m < M) dX[(size_t)m * lddx + 16 * t + c16] = acc[t][r];
      }
  }
  if (!wslab) return;
  float* row = wslab + (size_t)blockIdx.x * (N1 * K + 2 * N1 + 1);
  // dW1 = dhid^T X over the 64 rows: output tiles (mt, nt) dealt to the waves
  for (int tile = wave; tile < NT * KT; tile += 4) {
    const int mt = tile / KT, nt = tile - mt * KT;
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
    float xb[kHeadRows / 4];
#pragma unroll
    for (int s = 0; s < kHeadRows / 4; ++s)   // row r >= M: dh is zero
      xb[s] = X[(size_t)min(rb + 4 * s + q, M - 1) * ldx + 16 * nt + c16];
#pragma unroll
    for (int s = 0; s < kHeadRows / 4; ++s) {
      const float a = dh[4 * s + q][16 * mt + c16];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, xb[s], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) row[(size_t)(16 * mt + 4 * q + r) * K + 16 * nt + c16] = acc[r];
  }
  // db1, dW2 (column sums in row order), db2
  for (int n = tid; n < N1; n += 256) {
    float s1 = 0.f, s2 = 0.f;
    for (int r = 0; r < kHeadRows; ++r) {
      s1 += dh[r][n];
      s2 += hg[r][n];
    }
    row[N1 * K + n] = s1;
    row[N1 * K + N1 + n] = s2;
  }
  if (tid == 0) {
    float s = 0.f;
    for (int r = 0; r < kHeadRows; ++r) s += g2s[r];
    row[N1 * K + 2 * N1] = s;
  }
}

// dY of the BCE loss on score y of row m (bce_bwd_kernel's expression, loss.hip)
__device__ __forceinline__ float bce_dy(float y, int m, int M, float gw, float ya, float yb, int split, int nv) {
  const bool first = m < split;
  const float cnt = first ? (float)min(split, nv) : (float)min(M - split, nv);
  const bool live = first ? m < nv : m - split < nv;
  return live ? (gw / cnt) * bce_grad(y, first ? ya : yb) : 0.f;
}

template <int NT, int KT>   // N1 = 16 NT hidden units, K = 16 KT inputs
__global__ void __launch_bounds__(256) head_bwd_kernel(const float* __restrict__ X, int ldx, int M,
                                                       const float* __restrict__ W1, const float* __restrict__ w2,
                                                       const float* __restrict__ hid, const float* __restrict__ Y,
                                                       const float* __restrict__ dY, int act,
                                                       float* __restrict__ dX, int lddx, float* __restrict__ wslab,
                                                       const float* __restrict__ bce_g, const float* __restrict__ bce_ya,
                                                       const float* __restrict__ bce_yb, int bce_split, float bce_w,
                                                       const int32_t* __restrict__ bce_nvalid) {
  constexpr int N1 = 16 * NT, K = 16 * KT;
  constexpr int DP = N1 + 4;   // dhid row pitch
  __shared__ float dh[kHeadRows][DP];
  __shared__ float hg[kHeadRows][DP];   // g2 * hid (the dW2 terms)
  __shared__ float g2s[kHeadRows];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int c16 = lane & 15, q = lane >> 4;
  const int rb = blockIdx.x * kHeadRows;
  // the dX product's W1 fragments, in flight across the staging
  float wb[N1 / 4][KT];
#pragma unroll
  for (int s = 0; s < N1 / 4; ++s)
#pragma unroll
    for (int t = 0; t < KT; ++t) wb[s][t] = W1[(size_t)(4 * s + q) * K + 16 * t + c16];
  // stage dhid (rows past M are zero: they add nothing to the weight sums):
  // thread = (column n, row phase), every global load of the thread issued
  // before any is used (one memory round trip)
  {
    constexpr int RPT = kHeadRows * N1 / 256;   // rows per thread
    constexpr int RS = 256 / N1;                // row stride
    const int n = tid % N1, r0 = tid / N1;
    const float wn = w2[n];
    float hv[RPT], yv[RPT], dyv[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int mc = min(rb + r0 + RS * i, M - 1);
      hv[i] = hid[(size_t)mc * N1 + n];
      yv[i] = Y[mc];
      dyv[i] = bce_g ? 0.f : dY[mc];
    }
    if (bce_g) {   // dY of the BCE loss on Y
      const float gw = *bce_g * bce_w, ya = *bce_ya, yb = *bce_yb;
      const int nv = bce_nvalid ? *bce_nvalid : M;   // a padded batch: the real rows of each range
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int mc = min(rb + r0 + RS * i, M - 1);
        dyv[i] = bce_dy(yv[i], mc, M, gw, ya, yb, bce_split, nv);
      }
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = r0 + RS * i, m = rb + r;
      const float g = (m < M && (!(act & 2) || yv[i] > 0.f)) ? dyv[i] : 0.f;
      dh[r][n] = (!(act & 1) || hv[i] > 0.f) ? g * wn : 0.f;
      hg[r][n] = g * hv[i];
      if (n == 0) g2s[r] = g;
    }
  }
  __syncthreads();
  head_bwd_tail<NT, KT, DP>(X, ldx, M, rb, dh, hg, g2s, wb, dX, lddx, wslab);
}

// Forward and the BCE backward in ONE launch (sgg_head_fwdbwd): the
// workgroup's 64 rows go forward as in head_fwd_kernel (Y written for the
// loss value; hid stays in registers), each lane forms dY of its rows from
// its Y and the BCE targets, and stages dhid / g2 hid / g2 from its own
// accumulators -- the values head_bwd_kernel would re-read from hid and Y --
// then the backward tail runs as in head_bwd_kernel.  Bitwise the results of
// the two launches with the same upstream gradient *bce_g.
template <int NT, int KT>
__global__ void __launch_bounds__(256) head_fwdbwd_kernel(
    const float* __restrict__ X, int ldx, int M, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, int act, float* __restrict__ Y,
    float* __restrict__ dX, int lddx, float* __restrict__ wslab, const float* __restrict__ bce_g,
    const float* __restrict__ bce_ya, const float* __restrict__ bce_yb, int bce_split, float bce_w,
    const int32_t* __restrict__ bce_nvalid) {
  constexpr int N1 = 16 * NT, K = 16 * KT, KS = 4 * KT;
  constexpr int DP = N1 + 4;
  __shared__ float dh[kHeadRows][DP];
  __shared__ float hg[kHeadRows][DP];
  __shared__ float g2s[kHeadRows];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int rb = blockIdx.x * kHeadRows;
  const int row0 = rb + wave * 16;
  const float* xr = X + (size_t)min(row0 + c16, M - 1) * ldx;
  float a[KS], b[KS][NT], bc[NT], wc[NT];
#pragma unroll
  for (int m = 0; m < KT; ++m) {
    const float4 xv = *reinterpret_cast<const float4*>(xr + 16 * m + 4 * q);
    a[4 * m] = xv.x;
    a[4 * m + 1] = xv.y;
    a[4 * m + 2] = xv.z;
    a[4 * m + 3] = xv.w;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float4 wv = *reinterpret_cast<const float4*>(W1 + (size_t)(16 * t + c16) * K + 16 * m + 4 * q);
      b[4 * m][t] = wv.x;
      b[4 * m + 1][t] = wv.y;
      b[4 * m + 2][t] = wv.z;
      b[4 * m + 3][t] = wv.w;
    }
  }
  float wb[N1 / 4][KT];   // the backward's W1 fragments, in flight with the forward's operands
#pragma unroll
  for (int s = 0; s < N1 / 4; ++s)
#pragma unroll
    for (int t = 0; t < KT; ++t) wb[s][t] = W1[(size_t)(4 * s + q) * K + 16 * t + c16];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bc[t] = b1[16 * t + c16];
    wc[t] = w2[16 * t + c16];
  }
  const float bb2 = b2[0];
  const float gw = *bce_g * bce_w, ya = *bce_ya, yb = *bce_yb;
  const int nv = bce_nvalid ? *bce_nvalid : M;
  floatx4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s][t], acc[t], 0, 0, 0);
  // forward epilogue (head_fwd_kernel's): lane holds rows 4 q + r, columns 16 t + c16
  float h[NT][4];
  float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = acc[t][r] + bc[t];
      if (act & 1) v = v > 0.f ? v : 0.f;
      h[t][r] = v;
      p[r] = fmaf(v, wc[t], p[r]);
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) p[r] += __shfl_xor(p[r], o);
    float y = p[r] + bb2;
    if (act & 2) y = y > 0.f ? y : 0.f;
    const int lr = wave * 16 + 4 * q + r, m = rb + lr;
    if (c16 == 0 && m < M) Y[m] = y;
    // the backward's staging of row m (head_bwd_kernel's expressions on the same values)
    const float dy = bce_dy(y, min(m, M - 1), M, gw, ya, yb, bce_split, nv);
    const float g = (m < M && (!(act & 2) || y > 0.f)) ? dy : 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = 16 * t + c16;
      dh[lr][n] = (!(act & 1) || h[t][r] > 0.f) ? g * wc[t] : 0.f;
      hg[lr][n] = g * h[t][r];
    }
    if (c16 == 0) g2s[lr] = g;
  }
  __syncthreads();
  head_bwd_tail<NT, KT, DP>(X, ldx, M, rb, dh, hg, g2s, wb, dX, lddx, wslab);
}

template <int NT>
int launch_fwd_nt(const float* X, int ldx, int M, int K, const float* W1, const float* b1, const float* w2,
                  const float* b2, int act, float* hid, float* Y, hipStream_t st) {
  const dim3 grid((M + kHeadRows - 1) / kHeadRows);
  switch (K) {
    case 16: hipLaunchKernelGGL((head_fwd_kernel<NT, 1>), grid, dim3(256), 0, st, X, ldx, M, W1, b1, w2, b2, act, hid, Y); break;
    case 32: hipLaunchKernelGGL((head_fwd_kernel<NT, 2>), grid, dim3(256), 0, st, X, ldx, M, W1, b1, w2, b2, act, hid, Y); break;
    case 48: hipLaunchKernelGGL((head_fwd_kernel<NT, 3>), grid, dim3(256), 0, st, X, ldx, M, W1, b1, w2, b2, act, hid, Y); break;
    default: hipLaunchKernelGGL((head_fwd_kernel<NT, 4>), grid, dim3(256), 0, st, X, ldx, M, W1, b1, w2, b2, act, hid, Y); break;
  }
  SGG_RETURN_LAUNCH("sgg_head_fwd");
}

struct BceArgs {
  const float *g, *ya, *yb;
  int split;
  float w;
  const int32_t* nvalid;
};

template <int NT, int KT>
int launch_bwd_nt(const float* X, int ldx, int M, const float* W1, const float* w2, const float* hid, const float* Y,
                  const float* dY, int act, float* dX, int lddx, float* wslab, const BceArgs& bc, hipStream_t st) {
  hipLaunchKernelGGL((head_bwd_kernel<NT, KT>), dim3((M + kHeadRows - 1) / kHeadRows), dim3(256), 0, st, X, ldx, M,
                     W1, w2, hid, Y, dY, act, dX, lddx, wslab, bc.g, bc.ya, bc.yb, bc.split, bc.w,
                     bc.nvalid);
  SGG_RETURN_LAUNCH("sgg_head_bwd");
}

template <int NT>
int launch_bwd_k(const float* X, int ldx, int M, int K, const float* W1, const float* w2, const float* hid,
                 const float* Y, const float* dY, int act, float* dX, int lddx, float* wslab, const BceArgs& bc,
                 hipStream_t st) {
  switch (K) {
    case 16: return launch_bwd_nt<NT, 1>(X, ldx, M, W1, w2, hid, Y, dY, act, dX, lddx, wslab, bc, st);
    case 32: return launch_bwd_nt<NT, 2>(X, ldx, M, W1, w2, hid, Y, dY, act, dX, lddx, wslab, bc, st);
    case 48: return launch_bwd_nt<NT, 3>(X, ldx, M, W1, w2, hid, Y, dY, act, dX, lddx, wslab, bc, st);
    default: return launch_bwd_nt<NT, 4>(X, ldx, M, W1, w2, hid, Y, dY, act, dX, lddx, wslab, bc, st);
  }
}

template <int NT, int KT>
int launch_fwdbwd_nt(const float* X, int ldx, int M, const float* W1, const float* b1, const float* w2, const float* b2,
                     int act, float* Y, float* dX, int lddx, float* wslab, const BceArgs& bc, hipStream_t st) {
  hipLaunchKernelGGL((head_fwdbwd_kernel<NT, KT>), dim3((M + kHeadRows - 1) / kHeadRows), dim3(256), 0, st, X, ldx, M,
                     W1, b1, w2, b2, act, Y, dX, lddx, wslab, bc.g, bc.ya, bc.yb, bc.split, bc.w, bc.nvalid);
  SGG_RETURN_LAUNCH("sgg_head_fwdbwd");
}

template <int NT>
int launch_fwdbwd_k(const float* X, int ldx, int M, int K, const float* W1, const float* b1, const float* w2,
                    const float* b2, int act, float* Y, float* dX, int lddx, float* wslab, const BceArgs& bc,
                    hipStream_t st) {
  switch (K) {
    case 16: return launch_fwdbwd_nt<NT, 1>(X, ldx, M, W1, b1, w2, b2, act, Y, dX, lddx, wslab, bc, st);
    case 32: return launch_fwdbwd_nt<NT, 2>(X, ldx, M, W1, b1, w2, b2, act, Y, dX, lddx, wslab, bc, st);
    case 48: return launch_fwdbwd_nt<NT, 3>(X, ldx, M, W1, b1, w2, b2, act, Y, dX, lddx, wslab, bc, st);
    default: return launch_fwdbwd_nt<NT, 4>(X, ldx, M, W1, b1, w2, b2, act, Y, dX, lddx, wslab, bc, st);
  }
}

}  // namespace

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_head_ok(int K, int N1) {
  return (K == 16 || K == 32 || K == 48 || K == 64) && (N1 == 16 || N1 == 32 || N1 == 64);
}

extern "C" int sgg_head_slab_cols(int K, int N1) { return N1 * K + 2 * N1 + 1; }

extern "C" int sgg_head_fwd(const float* X, int ldx, int M, int K, int N1, const float* W1, const float* b1,
                            const float* w2, const float* b2, int act, float* hid, float* Y, void* stream) {
  SGG_CHECK_ARG(X && W1 && b1 && w2 && b2 && hid && Y, "sgg_head_fwd: null pointer");
  SGG_CHECK_ARG(M >= 0 && sgg_head_ok(K, N1) && ldx >= K && act >= 0 && act <= 3,
                "sgg_head_fwd: unsupported shape M=%d K=%d N1=%d ldx=%d act=%d", M, K, N1, ldx, act);
  SGG_CHECK_ARG(((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W1)) & 15) == 0 && ldx % 4 == 0,
                "sgg_head_fwd: X and W1 must be 16-byte aligned with ldx %% 4 == 0 (ldx=%d)", ldx);
  if (M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (N1) {
    case 16: return launch_fwd_nt<1>(X, ldx, M, K, W1, b1, w2, b2, act, hid, Y, st);
    case 32: return launch_fwd_nt<2>(X, ldx, M, K, W1, b1, w2, b2, act, hid, Y, st);
    default: return launch_fwd_nt<4>(X, ldx, M, K, W1, b1, w2, b2, act, hid, Y, st);
  }
}

extern "C" int sgg_head_bwd(const float* X, int ldx, int M, int K, int N1, const float* W1, const float* w2,
                            const float* hid, const float* Y, const float* dY, int act, float* dX, int lddx,
                            float* wslab, const float* bce_g, const float* bce_ya, const float* bce_yb,
                            int bce_split, float bce_w, const int32_t* bce_nvalid, void* stream) {
  SGG_CHECK_ARG(X && W1 && w2 && hid && Y && (dY || bce_g) && dX, "sgg_head_bwd: null pointer");
  SGG_CHECK_ARG(!bce_g || (bce_ya && bce_yb && bce_split >= 0 && bce_split <= M),
                "sgg_head_bwd: BCE targets / split (split=%d, M=%d)", bce_split, M);
  const BceArgs bc{bce_g, bce_ya, bce_yb, bce_split, bce_w, bce_nvalid};
  SGG_CHECK_ARG(M >= 0 && sgg_head_ok(K, N1) && ldx >= K && lddx >= K && act >= 0 && act <= 3,
                "sgg_head_bwd: unsupported shape M=%d K=%d N1=%d", M, K, N1);
  if (M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (N1) {
    case 16: return launch_bwd_k<1>(X, ldx, M, K, W1, w2, hid, Y, dY, act, dX, lddx, wslab, bc, st);
    case 32: return launch_bwd_k<2>(X, ldx, M, K, W1, w2, hid, Y, dY, act, dX, lddx, wslab, bc, st);
    default: return launch_bwd_k<4>(X, ldx, M, K, W1, w2, hid, Y, dY, act, dX, lddx, wslab, bc, st);
  }
}

extern "C" int sgg_head_fwdbwd(const float* X, int ldx, int M, int K, int N1, const float* W1, const float* b1,
                               const float* w2, const float* b2, int act, float* Y, float* dX, int lddx,
                               float* wslab, const float* bce_g, const float* bce_ya, const float* bce_yb,
                               int bce_split, float bce_w, const int32_t* bce_nvalid, void* stream) {
  SGG_CHECK_ARG(X && W1 && b1 && w2 && b2 && Y && dX && bce_g && bce_ya && bce_yb, "sgg_head_fwdbwd: null pointer");
  SGG_CHECK_ARG(M >= 0 && sgg_head_ok(K, N1) && ldx >= K && lddx >= K && act >= 0 && act <= 3,
                "sgg_head_fwdbwd: unsupported shape M=%d K=%d N1=%d ldx=%d act=%d", M, K, N1, ldx, act);
  SGG_CHECK_ARG(((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W1)) & 15) == 0 && ldx % 4 == 0,
                "sgg_head_fwdbwd: X and W1 must be 16-byte aligned with ldx %% 4 == 0 (ldx=%d)", ldx);
  SGG_CHECK_ARG(bce_split >= 0 && bce_split <= M, "sgg_head_fwdbwd: BCE split %d outside [0, %d]", bce_split, M);
  if (M == 0) return 0;
  const BceArgs bc{bce_g, bce_ya, bce_yb, bce_split, bce_w, bce_nvalid};
  hipStream_t st = (hipStream_t)stream;
  switch (N1) {
    case 16: return launch_fwdbwd_k<1>(X, ldx, M, K, W1, b1, w2, b2, act, Y, dX, lddx, wslab, bc, st);
    case 32: return launch_fwdbwd_k<2>(X, ldx, M, K, W1, b1, w2, b2, act, Y, dX, lddx, wslab, bc, st);
    default: return launch_fwdbwd_k<4>(X, ldx, M, K, W1, b1, w2, b2, act, Y, dX, lddx, wslab, bc, st);
  }
}
