// Social pooling (PoolHiddenNet, reference sgan/models.py:458-549) on gfx950.
//
// The reference materialises, per scene, the (N^2 x (E+H)) pair matrix
// [Linear(2,E)(p_j - p_i) ; h_j], runs Linear(E+H, 512) -> ReLU ->
// Linear(512, bn) -> ReLU on it and takes max over j.  We fold the
// embedding into the first layer (A = W1e We, U = h W1h^T + W1e be + b1, the
// latter one MFMA node transform, see sgg_xw) so a pair only needs
//   hidden_k = ReLU(U[j,k] + A[k,0] r_x + A[k,1] r_y)      (2 FMA + max)
//   z_c      = ReLU(sum_k W2[c,k] hidden_k + b2[c])         (bn FMA per k)
// and never leaves registers.
//
// Forward: one workgroup per scene (grid-stride), the scene's U rows
// LDS-resident (row stride 516 floats: 16-B aligned, +4 banks per row so the
// few distinct rows a wave touches never share a bank slot), one pair per
// thread with i fastest (a wave reads <= 4 distinct U rows -> near-broadcast
// LDS reads; A and W2 are wave-uniform -> scalar loads).  The max over j is a
// 64-bit LDS atomic max on (float bits << 32 | ~j): post-ReLU values are >= 0
// so their bit patterns order like the floats, and ties resolve to the
// smallest j.  The winning j is kept for the backward.
//
// Backward: only (i, argmax[i,c]) carries gradient.  One workgroup of 512
// threads, thread k = hidden unit k, walks the scene's selected pairs grouped
// by j (lists built with a wave ballot, deterministic order): U[j,k] is read
// once per j (coalesced), dU[j,k] is produced in a register and stored once,
// dW2[:,k] lives in LDS (thread-owned column: no atomics), dA in registers.
#include "sgg_common.h"

namespace sgg {

constexpr int kURow = kHidden + 4;  // padded LDS row (floats)

template <int BN>
__global__ void __launch_bounds__(256) pool_fwd_kernel(
    const float* __restrict__ U, const float* __restrict__ pos, const float* __restrict__ A,
    const float* __restrict__ W2T /* 512 x BN */, const float* __restrict__ b2,
    const int32_t* __restrict__ scene_off, int S, float* __restrict__ out, int32_t* __restrict__ argmax) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int max_n = SGG_POOL_MAX_PEDS;
  (void)max_n;
  for (int s = blockIdx.x; s < S; s += gridDim.x) {
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    float* Us = reinterpret_cast<float*>(smem);
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(Us + (size_t)n * kURow);
    float2* ps = reinterpret_cast<float2*>(keys + (size_t)n * BN);

    // stage U rows (float4 granules) and positions
    const float4* Ug = reinterpret_cast<const float4*>(U + (size_t)o * kHidden);
    for (int q = threadIdx.x; q < n * (kHidden / 4); q += blockDim.x) {
      const int r = q / (kHidden / 4), c4 = q - r * (kHidden / 4);
      *reinterpret_cast<float4*>(Us + (size_t)r * kURow + 4 * c4) = Ug[q];
    }
    for (int q = threadIdx.x; q < n; q += blockDim.x) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
    for (int q = threadIdx.x; q < n * BN; q += blockDim.x) keys[q] = 0ull;
    __syncthreads();

    const int npairs = n * n;
    for (int p = threadIdx.x; p < npairs; p += blockDim.x) {
      const int j = p / n;
      const int i = p - j * n;
      const float rx = ps[j].x - ps[i].x;
      const float ry = ps[j].y - ps[i].y;
      const float* ur = Us + (size_t)j * kURow;
      float acc[BN];
#pragma unroll
      for (int c = 0; c < BN; ++c) acc[c] = 0.f;
      for (int k4 = 0; k4 < kHidden; k4 += 4) {
        const float4 u = *reinterpret_cast<const float4*>(ur + k4);
        const float uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = k4 + q;
          float h = fmaf(A[2 * k + 1], ry, fmaf(A[2 * k], rx, uu[q]));
          h = h > 0.f ? h : 0.f;
#pragma unroll
          for (int c = 0; c < BN; ++c) acc[c] = fmaf(W2T[k * BN + c], h, acc[c]);
        }
      }
      const unsigned long long jkey = 0xFFFFFFFFull - (unsigned long long)j;
#pragma unroll
      for (int c = 0; c < BN; ++c) {
        float v = acc[c] + b2[c];
        v = v > 0.f ? v : 0.f;
        const unsigned long long key = ((unsigned long long)__float_as_uint(v) << 32) | jkey;
        atomicMax(&keys[i * BN + c], key);
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < n * BN; q += blockDim.x) {
      const unsigned long long key = keys[q];
      out[(size_t)o * BN + q] = __uint_as_float((unsigned)(key >> 32));
      argmax[(size_t)o * BN + q] = o + (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
    }
    __syncthreads();  // LDS reused by the next scene
  }
}

template <int BN>
__global__ void __launch_bounds__(512) pool_bwd_kernel(
    const float* __restrict__ U, const float* __restrict__ pos, const float* __restrict__ A,
    const float* __restrict__ W2 /* BN x 512 */, const float* __restrict__ out,
    const int32_t* __restrict__ argmax, const float* __restrict__ dout, const int32_t* __restrict__ scene_off,
    int S, int max_n, float* __restrict__ dU, float* __restrict__ dW2_part, float* __restrict__ dA_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int k = threadIdx.x;  // hidden unit, blockDim.x == 512
  const int lane = k & 63;
  const int wave = k >> 6;
  float* dW2s = reinterpret_cast<float*>(smem);                 // BN x 512
  float* gs = dW2s + BN * kHidden;                               // max_n*BN
  int* js = reinterpret_cast<int*>(gs + max_n * BN);             // max_n*BN (local j)
  int* lst = js + max_n * BN;                                    // max_n*BN entries
  int* loff = lst + max_n * BN;                                  // max_n + 1
  float2* ps = reinterpret_cast<float2*>(loff + ((max_n + 2) & ~1));

#pragma unroll
  for (int c = 0; c < BN; ++c) dW2s[c * kHidden + k] = 0.f;
  const float a0 = A[2 * k], a1 = A[2 * k + 1];
  float dA0 = 0.f, dA1 = 0.f;

  for (int s = blockIdx.x; s < S; s += gridDim.x) {
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    const int ne = n * BN;
    for (int e = k; e < ne; e += blockDim.x) {
      const size_t ge = (size_t)o * BN + e;
      gs[e] = out[ge] > 0.f ? dout[ge] : 0.f;
      js[e] = argmax[ge] - o;
    }
    for (int q = k; q < n; q += blockDim.x) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
    __syncthreads();
    if (wave == 0) {  // stable bucket of the selected (i, c) entries by j
      int cnt = 0;
      for (int j = 0; j < n; ++j) {
        if (lane == 0) loff[j] = cnt;
        for (int b = 0; b < ne; b += 64) {
          const int e = b + lane;
          const bool pred = e < ne && js[e] == j && gs[e] != 0.f;
          const unsigned long long m = __ballot(pred);
          if (pred) lst[cnt + __popcll(m & ((1ull << lane) - 1ull))] = e;
          cnt += __popcll(m);
        }
      }
      if (lane == 0) loff[n] = cnt;
    }
    __syncthreads();
    const float* Us = U + (size_t)o * kHidden + k;
    float u_next = n > 0 ? Us[0] : 0.f;
    for (int j = 0; j < n; ++j) {
      const float u = u_next;
      if (j + 1 < n) u_next = Us[(size_t)(j + 1) * kHidden];
      const float2 pj = ps[j];
      float du = 0.f;
      const int e1 = loff[j + 1];
      for (int q = loff[j]; q < e1; ++q) {
        const int e = lst[q];
        const int i = e / BN;
        const int c = e - i * BN;
        const float g = gs[e];
        const float rx = pj.x - ps[i].x;
        const float ry = pj.y - ps[i].y;
        const float pre = fmaf(a1, ry, fmaf(a0, rx, u));
        if (pre > 0.f) {
          dW2s[c * kHidden + k] += g * pre;
          const float d = g * W2[c * kHidden + k];
          du += d;
          dA0 = fmaf(d, rx, dA0);
          dA1 = fmaf(d, ry, dA1);
        }
      }
      dU[(size_t)(o + j) * kHidden + k] = du;
    }
    __syncthreads();  // lists / gs reused by the next scene
  }
#pragma unroll
  for (int c = 0; c < BN; ++c) dW2_part[((size_t)blockIdx.x * BN + c) * kHidden + k] = dW2s[c * kHidden + k];
  dA_part[((size_t)blockIdx.x * kHidden + k) * 2 + 0] = dA0;
  dA_part[((size_t)blockIdx.x * kHidden + k) * 2 + 1] = dA1;
}

static size_t pool_fwd_lds(int bn, int max_n) {
  return (size_t)max_n * kURow * 4 + (size_t)max_n * bn * 8 + (size_t)max_n * 8 + 16;
}
static size_t pool_bwd_lds(int bn, int max_n) {
  return (size_t)bn * kHidden * 4 + (size_t)max_n * bn * 12 + (size_t)(((max_n + 2) & ~1) * 4) +
         (size_t)max_n * 8 + 16;
}

template <int BN>
static int launch_fwd(const float* U, const float* pos, const float* A, const float* W2T, const float* b2,
                      const int32_t* off, int S, int max_n, float* out, int32_t* am, hipStream_t st) {
  const size_t lds = pool_fwd_lds(BN, max_n);
  const int grid = S < 8192 ? S : 8192;
  hipLaunchKernelGGL(pool_fwd_kernel<BN>, dim3(grid), dim3(256), lds, st, U, pos, A, W2T, b2, off, S, out, am);
  SGG_RETURN_LAUNCH("sgg_pool_fwd");
}

template <int BN>
static int launch_bwd(const float* U, const float* pos, const float* A, const float* W2, const float* out,
                      const int32_t* am, const float* dout, const int32_t* off, int S, int max_n, float* dU,
                      float* dW2p, float* dAp, hipStream_t st) {
  const size_t lds = pool_bwd_lds(BN, max_n);
  hipLaunchKernelGGL(pool_bwd_kernel<BN>, dim3(sgg_pool_bwd_grid(S)), dim3(512), lds, st, U, pos, A, W2, out,
                     am, dout, off, S, max_n, dU, dW2p, dAp);
  SGG_RETURN_LAUNCH("sgg_pool_bwd");
}

}  // namespace sgg

using namespace sgg;

static bool pool_bn_ok(int bn) { return bn == 8 || bn == 16 || bn == 32 || bn == 48 || bn == 64; }

extern "C" int sgg_pool_fwd(const float* U, const float* pos, const float* A, const float* W2T, const float* b2,
                            const int32_t* scene_off, int S, int B, int bn, int max_n, float* out,
                            int32_t* argmax, void* stream) {
  SGG_CHECK_ARG(U && pos && A && W2T && b2 && scene_off && out && argmax, "sgg_pool_fwd: null pointer");
  SGG_CHECK_ARG(pool_bn_ok(bn), "sgg_pool_fwd: bottleneck %d not built (8/16/32/48/64)", bn);
  SGG_CHECK_ARG(S >= 0 && B >= 0, "sgg_pool_fwd: bad sizes");
  SGG_CHECK_ARG(max_n >= 1 && max_n <= SGG_POOL_MAX_PEDS, "sgg_pool_fwd: max scene size %d outside [1, %d]",
                max_n, SGG_POOL_MAX_PEDS);
  if (S == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (bn) {
    case 8: return launch_fwd<8>(U, pos, A, W2T, b2, scene_off, S, max_n, out, argmax, st);
    case 16: return launch_fwd<16>(U, pos, A, W2T, b2, scene_off, S, max_n, out, argmax, st);
    case 32: return launch_fwd<32>(U, pos, A, W2T, b2, scene_off, S, max_n, out, argmax, st);
    case 48: return launch_fwd<48>(U, pos, A, W2T, b2, scene_off, S, max_n, out, argmax, st);
    default: return launch_fwd<64>(U, pos, A, W2T, b2, scene_off, S, max_n, out, argmax, st);
  }
}

extern "C" int sgg_pool_bwd_grid(int S) { return S < 1 ? 1 : (S < 256 ? S : 256); }

extern "C" int sgg_pool_bwd(const float* U, const float* pos, const float* A, const float* W2, const float* out,
                            const int32_t* argmax, const float* dout, const int32_t* scene_off, int S, int B,
                            int bn, int max_n, float* dU, float* dW2_part, float* dA_part, void* stream) {
  SGG_CHECK_ARG(U && pos && A && W2 && out && argmax && dout && scene_off && dU && dW2_part && dA_part,
                "sgg_pool_bwd: null pointer");
  SGG_CHECK_ARG(pool_bn_ok(bn), "sgg_pool_bwd: bottleneck %d not built", bn);
  SGG_CHECK_ARG(max_n >= 1 && max_n <= SGG_POOL_MAX_PEDS, "sgg_pool_bwd: max scene size %d outside [1, %d]",
                max_n, SGG_POOL_MAX_PEDS);
  SGG_CHECK_ARG(S >= 0 && B >= 0, "sgg_pool_bwd: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (S == 0) return 0;
  switch (bn) {
    case 8: return launch_bwd<8>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, dW2_part, dA_part, st);
    case 16: return launch_bwd<16>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, dW2_part, dA_part, st);
    case 32: return launch_bwd<32>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, dW2_part, dA_part, st);
    case 48: return launch_bwd<48>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, dW2_part, dA_part, st);
    default: return launch_bwd<64>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, dW2_part, dA_part, st);
  }
}
