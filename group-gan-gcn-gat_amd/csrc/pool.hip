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
// Backward: only (i, argmax[i,c]) carries gradient; selected entries indexed
// by (j, c) bitmasks, thread = hidden unit, W2 column and dW2 partial in
// registers (see pool_bwd_kernel).
#include <stdlib.h>
#include <string.h>

#include "sgg_common.h"

namespace sgg {


// ---- forward: MFMA layer 2 ---------------------------------------------------
// Work unit = a chunk of whole i-rows [i0, i1) of one scene (host plan,
// sgg_pool_plan): every pair (i, j) of those rows, j fastest, cut into 16-pair
// MFMA groups, GPW groups per wave (the tail groups of a chunk are padding).
// Keeping whole i-rows in one workgroup makes max_j complete there (LDS
// atomics only).  The 512 hidden units are walked in k-tiles of 64 staged in
// LDS (U rows of the scene, W2^T tile, A tile); per 4-deep k-step a lane builds
// ONE hidden value per group (pair l&15, unit l>>4: 2 FMA + max) -- the A
// operand of v_mfma_f32_16x16x4_f32 against the W2^T fragment, NT = bn/16
// column tiles.  fp32 in, fp32 accumulate (exact fmaf chains).  The next
// k-step's LDS operands are loaded before the current step's MFMAs.
constexpr int kKT = 64;          // hidden units per LDS k-tile
constexpr int kKTP = kKT + 2;    // U tile row stride: (2j + k) mod 32 -> conflict-free b32 reads
constexpr int kPoolWaves = 4;

// One batch of a forward launch.  A launch serves one batch, or two of the
// same pooling net (sgg_pool_fwd2, weights shared): workgroups [0, g1) walk
// s1's chunks and [g1, grid) s2's (g1 a multiple of 8, so each range keeps
// the XCD-aware chunk order); the set is picked once per workgroup.
struct PoolSet {
  const float* U;
  const float* pos;
  const int32_t* scene_off;
  const int4* chunks;
  int nchunks;
  const int32_t* nchunks_dev;   // a fixed-capacity plan: the count is device data
  float* out;
  int32_t* argmax;
};

// this workgroup's batch: its pointers, chunk count, first chunk and stride
#define SGG_POOL_PICK(s1, s2, g1)                                                       \
  const bool two_ = (int)blockIdx.x >= (g1);                                            \
  const float* __restrict__ U = two_ ? s2.U : s1.U;                                     \
  const float* __restrict__ pos = two_ ? s2.pos : s1.pos;                               \
  const int32_t* __restrict__ scene_off = two_ ? s2.scene_off : s1.scene_off;           \
  const int4* __restrict__ chunks = two_ ? s2.chunks : s1.chunks;                       \
  float* __restrict__ out = two_ ? s2.out : s1.out;                                     \
  int32_t* __restrict__ argmax = two_ ? s2.argmax : s1.argmax;                          \
  const int32_t* ncd_ = two_ ? s2.nchunks_dev : s1.nchunks_dev;                         \
  const int nch = ncd_ ? *ncd_ : (two_ ? s2.nchunks : s1.nchunks);                      \
  const int gb_ = (int)blockIdx.x - (two_ ? (g1) : 0);                                  \
  const int gstride = two_ ? (int)gridDim.x - (g1) : (g1);                              \
  const int xb = (gb_ & 7) * (gstride >> 3) + (gb_ >> 3)   /* XCD-aware (pool_fwd_kernel) */

template <int BN>
struct PoolCfg {
  static constexpr int NT = (BN + 15) / 16;                      // 16-wide column tiles
  static constexpr int BNP = NT * 16 + ((NT % 2 == 0) ? 16 : 0); // odd multiple of 16: conflict-free B reads
};

// UNR: k-steps unrolled per k-tile.  Fully unrolled (16) the LDS operand
// prefetch is plain register renaming -- no in-step wait for the reads --
// but the wave holds ~40 % more VGPRs; that pays only while the grid is at
// most a couple of workgroups per CU (occupancy does not matter then): the
// host picks it for small grids (launch_fwd).
// (occupancy hint: <8, 1> keeps 5 waves per SIMD without spilling)
template <int BN, int GPW, int UNR>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(BN == 8 && GPW == 1 ? 5 : 1))) pool_fwd_kernel(
    const PoolSet s1, const PoolSet s2, int g1, const float* __restrict__ A,
    const float* __restrict__ W2 /* BN x 512 */, const float* __restrict__ b2) {
  using C = PoolCfg<BN>;
  constexpr int NT = C::NT, BNP = C::BNP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Us = reinterpret_cast<float*>(smem);                              // 64 x kKTP
  float* W2s = Us + SGG_POOL_MAX_PEDS * kKTP;                              // kKT x BNP
  float* As = W2s + kKT * BNP;                                             // kKT x 2
  float2* ps = reinterpret_cast<float2*>(As + 2 * kKT);                    // scene positions (<= 64)
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(ps + SGG_POOL_MAX_PEDS);  // 64 x BN
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kq = lane >> 4;
  // b2 of the lane's columns, loaded once: read in the epilogue's guarded
  // branches each load was a memory round trip of its own (NT x 4 x GPW per chunk)
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bv[t] = b2[min(16 * t + c16, BN - 1)];

  // XCD-aware chunk order: the grid is a multiple of 8 and blocks b, b + 8,
  // b + 16, ... share an XCD (round-robin dispatch; speed only, never
  // correctness), so they take CONSECUTIVE chunks -- the chunks of one scene,
  // which all stage the same U rows, then hit one XCD's L2 instead of
  // fetching those rows once per XCD.
  SGG_POOL_PICK(s1, s2, g1);
  for (int ch = xb; ch < nch; ch += gstride) {
    const int4 cd = chunks[ch];
    const int s = cd.x, i0 = cd.y, i1 = cd.z;
    if (i1 <= i0) continue;   // an empty padding chunk (fixed-capacity plan), uniform over the workgroup
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    const int rows = i1 - i0;
    const int npairs = rows * n;

    for (int q = threadIdx.x; q < n; q += blockDim.x) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
    for (int q = threadIdx.x; q < rows * BN; q += blockDim.x) keys[q] = 0ull;
    __syncthreads();  // ps visible for the per-lane pair set-up below

    // per-lane A-row pair of each group (padding pairs -> j = 0, r = 0)
    int uoff[GPW];
    float rx[GPW], ry[GPW];
    floatx4 acc[GPW][NT];
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int p = (wave * GPW + g) * 16 + c16;
      int il = 0, j = 0;
      if (p < npairs) { il = p / n; j = p - il * n; }
      uoff[g] = j * kKTP + kq;
      const float2 pj = ps[j], pi = ps[i0 + il];
      rx[g] = p < npairs ? pj.x - pi.x : 0.f;
      ry[g] = p < npairs ? pj.y - pi.y : 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }

    // k-tiles of 64 hidden units, register-staged one tile ahead (the next
    // tile's global loads are in flight while the current tile computes)
    constexpr int kUQ = (SGG_POOL_MAX_PEDS * (kKT / 4) + 255) / 256;   // float4 of U per thread
    constexpr int kWQ = (kKT * BNP + 255) / 256;                       // W2^T floats per thread
    float4 ureg[kUQ];
    float wreg[kWQ];
    float areg = 0.f;
    auto load_tile = [&](int k0) {
#pragma unroll
      for (int e = 0; e < kUQ; ++e) {
        const int q = threadIdx.x + 256 * e;
        const int r = q / (kKT / 4), c4 = q - r * (kKT / 4);
        if (r < n) ureg[e] = *reinterpret_cast<const float4*>(U + (size_t)(o + r) * kHidden + k0 + 4 * c4);
      }
#pragma unroll
      for (int e = 0; e < kWQ; ++e) {   // W2 (BN x 512, nn.Linear layout), read transposed:
        const int q = threadIdx.x + 256 * e;   // c fastest, so the LDS stores below are conflict-free
        const int kk = q / BNP, cc = q - kk * BNP;
        wreg[e] = (kk < kKT && cc < BN) ? W2[(size_t)cc * kHidden + k0 + kk] : 0.f;
      }
      if (threadIdx.x < 2 * kKT) areg = A[2 * k0 + threadIdx.x];
    };
    auto store_tile = [&]() {
#pragma unroll
      for (int e = 0; e < kUQ; ++e) {
        const int q = threadIdx.x + 256 * e;
        const int r = q / (kKT / 4), c4 = q - r * (kKT / 4);
        if (r < n) {
          float* d = Us + r * kKTP + 4 * c4;
          d[0] = ureg[e].x; d[1] = ureg[e].y; d[2] = ureg[e].z; d[3] = ureg[e].w;
        }
      }
#pragma unroll
      for (int e = 0; e < kWQ; ++e) {   // the W2^T tile
        const int q = threadIdx.x + 256 * e;
        if (q < kKT * BNP) W2s[q] = wreg[e];
      }
      if (threadIdx.x < 2 * kKT) As[threadIdx.x] = areg;
    };
    load_tile(0);
    __syncthreads();  // (ps / keys init visible; previous chunk's readers done)
    store_tile();
    __syncthreads();
    for (int k0 = 0; k0 < kHidden; k0 += kKT) {
      if (k0 + kKT < kHidden) load_tile(k0 + kKT);
      float b[NT], u[GPW];
      float2 a;
#pragma unroll
      for (int t = 0; t < NT; ++t) b[t] = W2s[kq * BNP + 16 * t + c16];
      a = *reinterpret_cast<const float2*>(As + 2 * kq);
#pragma unroll
      for (int g = 0; g < GPW; ++g) u[g] = Us[uoff[g]];
#pragma unroll UNR
      for (int s4 = 0; s4 < kKT / 4; ++s4) {
        float h[GPW], bc[NT];
#pragma unroll
        for (int g = 0; g < GPW; ++g) h[g] = fmaxf(fmaf(a.y, ry[g], fmaf(a.x, rx[g], u[g])), 0.f);
#pragma unroll
        for (int t = 0; t < NT; ++t) bc[t] = b[t];
        if (s4 + 1 < kKT / 4) {  // prefetch the next k-step's operands
          const int kn = 4 * (s4 + 1);
#pragma unroll
          for (int t = 0; t < NT; ++t) b[t] = W2s[(kn + kq) * BNP + 16 * t + c16];
          a = *reinterpret_cast<const float2*>(As + 2 * (kn + kq));
#pragma unroll
          for (int g = 0; g < GPW; ++g) u[g] = Us[uoff[g] + kn];
        }
#pragma unroll
        for (int g = 0; g < GPW; ++g)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(h[g], bc[t], acc[g][t], 0, 0, 0);
      }
      __syncthreads();  // tile consumed
      if (k0 + kKT < kHidden) {
        store_tile();
        __syncthreads();
      }
    }

    // epilogue: bias, ReLU, max over j (LDS atomic max on (bits << 32 | ~j))
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int grp = wave * GPW + g;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = grp * 16 + kq * 4 + r;
        if (p < npairs) {
          const int il = p / n, j = p - il * n;
          const unsigned long long jkey = 0xFFFFFFFFull - (unsigned long long)j;
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int cc = 16 * t + c16;
            if (cc < BN) {
              float v = acc[g][t][r] + bv[t];
              v = v > 0.f ? v : 0.f;
              atomicMax(&keys[il * BN + cc], ((unsigned long long)__float_as_uint(v) << 32) | jkey);
            }
          }
        }
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < rows * BN; q += blockDim.x) {
      const unsigned long long key = keys[q];
      const size_t oi = (size_t)(o + i0) * BN + q;
      out[oi] = __uint_as_float((unsigned)(key >> 32));
      argmax[oi] = o + (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
    }
    __syncthreads();
  }
}

// ---- forward, fragment-native tiles ------------------------------------------
// Same work units, chunk order, arithmetic and epilogue as pool_fwd_kernel, but
// each 64-unit k-tile is stored in LDS in the order the MFMA lanes consume it:
// unit k = 4 s + kq of the tile (k-step s, lane quarter kq) sits at column
// 16 kq + s, so a lane's 16 k-steps of U[j, .], W2[c, .] and (A_x, A_y) are
// contiguous and come in with a few ds_read_b128 issued together at the top of
// the tile -- one LDS latency per 16 k-steps instead of one per k-step -- and
// the next tile's global loads are in flight meanwhile (register-staged).
constexpr int kVP = kKT + 4;     // row pitch (16-B aligned rows; 4 j mod 64 -> b128 reads spread over the banks)

__device__ __forceinline__ int perm16(int k) { return (k & 3) * 16 + (k >> 2); }

template <int BN, int GPW>
__global__ void __launch_bounds__(256) pool_fwd_v_kernel(
    const PoolSet s1, const PoolSet s2, int g1, const float* __restrict__ A,
    const float* __restrict__ W2 /* BN x 512 */, const float* __restrict__ b2) {
  constexpr int NT = PoolCfg<BN>::NT;
  constexpr int TB = (SGG_POOL_MAX_PEDS + 16 * NT) * kVP + 2 * kKT;   // one tile buffer: U | W2 | A
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* const tb0 = reinterpret_cast<float*>(smem);
  float* const tb1 = tb0 + TB;
  float2* ps = reinterpret_cast<float2*>(tb0 + 2 * TB);                                      // scene positions
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(ps + SGG_POOL_MAX_PEDS);  // 64 x BN
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kq = lane >> 4;
  // b2 of the lane's columns, loaded once: read in the epilogue's guarded
  // branches each load was a memory round trip of its own (NT x 4 x GPW per chunk)
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bv[t] = b2[min(16 * t + c16, BN - 1)];

  SGG_POOL_PICK(s1, s2, g1);
  for (int ch = xb; ch < nch; ch += gstride) {
    const int4 cd = chunks[ch];
    const int s = cd.x, i0 = cd.y, i1 = cd.z;
    if (i1 <= i0) continue;   // an empty padding chunk (fixed-capacity plan), uniform over the workgroup
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    const int rows = i1 - i0;
    const int npairs = rows * n;

    for (int q = threadIdx.x; q < n; q += blockDim.x) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
    for (int q = threadIdx.x; q < rows * BN; q += blockDim.x) keys[q] = 0ull;
    __syncthreads();

    int uoff[GPW];
    float rx[GPW], ry[GPW];
    floatx4 acc[GPW][NT];
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int p = (wave * GPW + g) * 16 + c16;
      int il = 0, j = 0;
      if (p < npairs) { il = p / n; j = p - il * n; }
      uoff[g] = j * kVP + 16 * kq;
      const float2 pj = ps[j], pi = ps[i0 + il];
      rx[g] = p < npairs ? pj.x - pi.x : 0.f;
      ry[g] = p < npairs ? pj.y - pi.y : 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }

    constexpr int kUQ = (SGG_POOL_MAX_PEDS * (kKT / 4) + 255) / 256;   // float4 of U per thread
    constexpr int kWQ = (16 * NT * (kKT / 4) + 255) / 256;            // float4 of W2 per thread
    // a register set of one staged tile (U rows, W2 rows, A)
    struct Stage {
      float4 u[kUQ], w[kWQ];
      float a;
    };
    Stage sx;
    auto load_tile = [&](Stage& st, int k0) {
      float4 (&ureg)[kUQ] = st.u;
      float4 (&wreg)[kWQ] = st.w;
      float& areg = st.a;
#pragma unroll
      for (int e = 0; e < kUQ; ++e) {
        const int q = threadIdx.x + 256 * e;
        const int r = q / (kKT / 4), c4 = q - r * (kKT / 4);
        if (r < n) ureg[e] = *reinterpret_cast<const float4*>(U + (size_t)(o + r) * kHidden + k0 + 4 * c4);
      }
#pragma unroll
      for (int e = 0; e < kWQ; ++e) {   // W2 rows (nn.Linear layout), rows >= BN are zero
        const int q = threadIdx.x + 256 * e;
        const int c = q / (kKT / 4), c4 = q - c * (kKT / 4);
        wreg[e] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c < BN) wreg[e] = *reinterpret_cast<const float4*>(W2 + (size_t)c * kHidden + k0 + 4 * c4);
      }
      if (threadIdx.x < 2 * kKT) areg = A[2 * k0 + threadIdx.x];
    };
    // float4 c4 of a row holds units 4 c4 .. 4 c4 + 3 = k-step c4 of lane quarters 0..3
    auto store_tile = [&](const Stage& st, float* tb) {
      const float4 (&ureg)[kUQ] = st.u;
      const float4 (&wreg)[kWQ] = st.w;
      const float areg = st.a;
      float* Us = tb;
      float* W2s = tb + SGG_POOL_MAX_PEDS * kVP;
      float* As = W2s + 16 * NT * kVP;
#pragma unroll
      for (int e = 0; e < kUQ; ++e) {
        const int q = threadIdx.x + 256 * e;
        const int r = q / (kKT / 4), c4 = q - r * (kKT / 4);
        if (r < n) {
          float* d = Us + r * kVP + c4;
          d[0] = ureg[e].x; d[16] = ureg[e].y; d[32] = ureg[e].z; d[48] = ureg[e].w;
        }
      }
#pragma unroll
      for (int e = 0; e < kWQ; ++e) {
        const int q = threadIdx.x + 256 * e;
        const int c = q / (kKT / 4), c4 = q - c * (kKT / 4);
        if (c < 16 * NT) {
          float* d = W2s + c * kVP + c4;
          d[0] = wreg[e].x; d[16] = wreg[e].y; d[32] = wreg[e].z; d[48] = wreg[e].w;
        }
      }
      if (threadIdx.x < 2 * kKT) {   // (A_x, A_y) of unit k at [kq][s]
        const int k = threadIdx.x >> 1;
        As[2 * perm16(k) + (threadIdx.x & 1)] = areg;
      }
    };
    // the lane's 16 k-steps of operands of one tile, in the order they are consumed
    struct Frag {
      float uu[GPW][16], aa[32], bb[NT][16];
    };
    auto read_frag = [&](const float* tb, Frag& F) {
      const float* Us = tb;
      const float* W2s = tb + SGG_POOL_MAX_PEDS * kVP;
      const float* As = W2s + 16 * NT * kVP;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int g = 0; g < GPW; ++g)
          *reinterpret_cast<float4*>(&F.uu[g][4 * v]) = *reinterpret_cast<const float4*>(Us + uoff[g] + 4 * v);
        *reinterpret_cast<float4*>(&F.aa[8 * v]) = *reinterpret_cast<const float4*>(As + 32 * kq + 8 * v);
        *reinterpret_cast<float4*>(&F.aa[8 * v + 4]) = *reinterpret_cast<const float4*>(As + 32 * kq + 8 * v + 4);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          *reinterpret_cast<float4*>(&F.bb[t][4 * v]) =
              *reinterpret_cast<const float4*>(W2s + (16 * t + c16) * kVP + 16 * kq + 4 * v);
      }
    };
    auto compute = [&](const Frag& F) {
#pragma unroll
      for (int s4 = 0; s4 < kKT / 4; ++s4) {
#pragma unroll
        for (int g = 0; g < GPW; ++g) {
          const float h = fmaxf(fmaf(F.aa[2 * s4 + 1], ry[g], fmaf(F.aa[2 * s4], rx[g], F.uu[g][s4])), 0.f);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(h, F.bb[t][s4], acc[g][t], 0, 0, 0);
        }
      }
    };
    // two LDS tile buffers, one barrier per tile: while tile k computes (its
    // fragments in registers), tile k + 1's fragments come in from the other
    // buffer and tile k + 2's global loads are in flight; tile k + 2 is then
    // stored over tile k (whose fragments every wave read before the last
    // barrier).  (Two register sets -- loads two tiles ahead -- measured no
    // faster for the small G tiles: 21.4 vs 21.3 us.)
    constexpr int NKT = kHidden / kKT;   // 8 (even)
    Frag F0, F1;
    load_tile(sx, 0);
    __syncthreads();  // (ps / keys init visible; previous chunk's readers done)
    store_tile(sx, tb0);
    load_tile(sx, kKT);
    __syncthreads();
    read_frag(tb0, F0);
    store_tile(sx, tb1);
    __syncthreads();
#pragma unroll
    for (int kt = 0; kt < NKT; kt += 2) {
      if (kt + 2 < NKT) load_tile(sx, (kt + 2) * kKT);
      read_frag(tb1, F1);
      compute(F0);
      if (kt + 2 < NKT) store_tile(sx, tb0);
      __syncthreads();
      if (kt + 3 < NKT) load_tile(sx, (kt + 3) * kKT);
      if (kt + 2 < NKT) read_frag(tb0, F0);
      compute(F1);
      if (kt + 3 < NKT) store_tile(sx, tb1);
      __syncthreads();
    }

    // epilogue: bias, ReLU, max over j (as pool_fwd_kernel)
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int grp = wave * GPW + g;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = grp * 16 + kq * 4 + r;
        if (p < npairs) {
          const int il = p / n, j = p - il * n;
          const unsigned long long jkey = 0xFFFFFFFFull - (unsigned long long)j;
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int cc = 16 * t + c16;
            if (cc < BN) {
              float v = acc[g][t][r] + bv[t];
              v = v > 0.f ? v : 0.f;
              atomicMax(&keys[il * BN + cc], ((unsigned long long)__float_as_uint(v) << 32) | jkey);
            }
          }
        }
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < rows * BN; q += blockDim.x) {
      const unsigned long long key = keys[q];
      const size_t oi = (size_t)(o + i0) * BN + q;
      out[oi] = __uint_as_float((unsigned)(key >> 32));
      argmax[oi] = o + (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
    }
    __syncthreads();
  }
}

// ---- forward, split-bf16 layer 2 (fp32 results) -----------------------------
// pool_fwd_v_kernel's work units, tiles, chunk order and epilogue, with the
// 512 -> bn contraction on v_mfma_f32_16x16x32_bf16 in the split form of
// sgg_common.h (mfma_x3: fp32 operands as exact sums of three bf16 pieces,
// six products per K = 32 chunk; within a few fp32 roundings of the fp32
// MFMA sum, not bitwise).  Per 64-unit tile a lane consumes two K = 32 chunks:
// unit 32 c + 8 q + j of the tile is k-element j of lane quarter q in chunk c,
// stored at column 16 q + 8 c + j, so the lane's 16 units of U and (A_x, A_y)
// are contiguous as in the v kernel.  Per chunk a lane forms its 8 hidden
// values per group (2 FMA + max each, fp32), splits them (the A operand) and
// runs NT x 6 MFMAs against the W2^T pieces, which store_tile splits once
// into LDS (bf16, 144-byte rows: conflict-free 16-byte reads).  Per chunk
// and group: 8 x 16 + NT x 96 cycles of the matrix pipe here against
// 8 NT x 32 for the fp32 16x16x4 form, half of each MFMA's cycles free for
// the VALU.  The U tile holds the batch's largest scene (umax rows).
constexpr int kWXP = kKT + 8;    // W2 piece row pitch in bf16 (144 B)

__device__ __forceinline__ int permx(int k) { return ((k >> 3) & 3) * 16 + (k >> 5) * 8 + (k & 7); }

template <int BN>
__host__ __device__ constexpr int pool_x3_tb_fixed() {   // W2 pieces + A of one tile buffer, in floats
  return (3 * 16 * PoolCfg<BN>::NT * kWXP) / 2 + 2 * kKT;
}

template <int BN, int GPW>
__global__ void __launch_bounds__(256, 2) pool_fwd_x3_kernel(
    const PoolSet s1, const PoolSet s2, int g1, const float* __restrict__ A,
    const float* __restrict__ W2 /* BN x 512 */, const float* __restrict__ b2, int umax) {
  constexpr int NT = PoolCfg<BN>::NT;
  const int TB = umax * kVP + pool_x3_tb_fixed<BN>();   // one tile buffer: U | W2 pieces | A
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* const tb0 = reinterpret_cast<float*>(smem);
  float* const tb1 = tb0 + TB;
  float2* ps = reinterpret_cast<float2*>(tb0 + 2 * TB);                                      // scene positions
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(ps + SGG_POOL_MAX_PEDS);  // rows x BN
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kq = lane >> 4;
  // b2 of the lane's columns, loaded once: read in the epilogue's guarded
  // branches each load was a memory round trip of its own (NT x 4 x GPW per chunk)
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bv[t] = b2[min(16 * t + c16, BN - 1)];

  SGG_POOL_PICK(s1, s2, g1);
  for (int ch = xb; ch < nch; ch += gstride) {
    const int4 cd = chunks[ch];
    const int s = cd.x, i0 = cd.y, i1 = cd.z;
    if (i1 <= i0) continue;   // an empty padding chunk (fixed-capacity plan), uniform over the workgroup
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    const int rows = i1 - i0;
    const int npairs = rows * n;

    for (int q = threadIdx.x; q < n; q += blockDim.x) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
    for (int q = threadIdx.x; q < rows * BN; q += blockDim.x) keys[q] = 0ull;
    __syncthreads();

    int uoff[GPW];
    float rx[GPW], ry[GPW];
    floatx4 acc[GPW][NT];
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int p = (wave * GPW + g) * 16 + c16;
      int il = 0, j = 0;
      if (p < npairs) { il = p / n; j = p - il * n; }
      uoff[g] = j * kVP + 16 * kq;
      const float2 pj = ps[j], pi = ps[i0 + il];
      rx[g] = p < npairs ? pj.x - pi.x : 0.f;
      ry[g] = p < npairs ? pj.y - pi.y : 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }

    constexpr int kUQ = (SGG_POOL_MAX_PEDS * (kKT / 4) + 255) / 256;   // float4 of U per thread
    constexpr int kWQ = (16 * NT * (kKT / 4) + 255) / 256;            // float4 of W2 per thread
    struct Stage {   // (native vector registers: a HIP float4 struct copied under a guard goes to scratch)
      floatx4 u[kUQ], w[kWQ];
      float a;
    };
    Stage sx;
    auto load_tile = [&](Stage& st, int k0) {
#pragma unroll
      for (int e = 0; e < kUQ; ++e) {
        const int q = threadIdx.x + 256 * e;
        const int r = q / (kKT / 4), c4 = q - r * (kKT / 4);
        if (r < n) st.u[e] = *reinterpret_cast<const floatx4*>(U + (size_t)(o + r) * kHidden + k0 + 4 * c4);
      }
#pragma unroll
      for (int e = 0; e < kWQ; ++e) {   // W2 rows (nn.Linear layout), rows >= BN are zero
        const int q = threadIdx.x + 256 * e;
        const int c = q / (kKT / 4), c4 = q - c * (kKT / 4);
        st.w[e] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (c < BN) st.w[e] = *reinterpret_cast<const floatx4*>(W2 + (size_t)c * kHidden + k0 + 4 * c4);
      }
      if (threadIdx.x < 2 * kKT) st.a = A[2 * k0 + threadIdx.x];
    };
    // float4 c4 of a row holds units 4 c4 .. 4 c4 + 3: columns permx(4 c4) .. + 3
    auto store_tile = [&](const Stage& st, float* tb) {
      float* Us = tb;
      unsigned* Wp = reinterpret_cast<unsigned*>(tb + umax * kVP);   // 3 pieces x 16 NT rows x kWXP bf16
      float* As = tb + umax * kVP + (3 * 16 * NT * kWXP) / 2;
#pragma unroll
      for (int e = 0; e < kUQ; ++e) {
        const int q = threadIdx.x + 256 * e;
        const int r = q / (kKT / 4), c4 = q - r * (kKT / 4);
        if (r < n && r < umax) *reinterpret_cast<floatx4*>(Us + r * kVP + permx(4 * c4)) = st.u[e];
      }
#pragma unroll
      for (int e = 0; e < kWQ; ++e) {
        const int q = threadIdx.x + 256 * e;
        const int c = q / (kKT / 4), c4 = q - c * (kKT / 4);
        if (c < 16 * NT) {
          float h[4], m[4], l[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) split3(st.w[e][x], h[x], m[x], l[x]);
          const int wo = (c * kWXP + permx(4 * c4)) >> 1;   // in dwords
          *reinterpret_cast<uint2*>(Wp + wo) = make_uint2(bf16_pack_top(h[0], h[1]), bf16_pack_top(h[2], h[3]));
          *reinterpret_cast<uint2*>(Wp + (16 * NT * kWXP) / 2 + wo) =
              make_uint2(bf16_pack_top(m[0], m[1]), bf16_pack_top(m[2], m[3]));
          *reinterpret_cast<uint2*>(Wp + 16 * NT * kWXP + wo) =
              make_uint2(bf16_pack_top(l[0], l[1]), bf16_pack_top(l[2], l[3]));
        }
      }
      if (threadIdx.x < 2 * kKT) {   // (A_x, A_y) of unit k at column permx(k)
        const int k = threadIdx.x >> 1;
        As[2 * permx(k) + (threadIdx.x & 1)] = st.a;
      }
    };
    // the lane's U and (A_x, A_y) of a tile; the W2 pieces are read per chunk
    // (compute), which keeps the wave within two per SIMD
    struct Frag {
      float uu[GPW][16], aa[32];
    };
    auto read_frag = [&](const float* tb, Frag& F) {
      const float* Us = tb;
      const float* As = tb + umax * kVP + (3 * 16 * NT * kWXP) / 2;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int g = 0; g < GPW; ++g)
          *reinterpret_cast<float4*>(&F.uu[g][4 * v]) = *reinterpret_cast<const float4*>(Us + uoff[g] + 4 * v);
        *reinterpret_cast<float4*>(&F.aa[8 * v]) = *reinterpret_cast<const float4*>(As + 32 * kq + 8 * v);
        *reinterpret_cast<float4*>(&F.aa[8 * v + 4]) = *reinterpret_cast<const float4*>(As + 32 * kq + 8 * v + 4);
      }
    };
    auto compute = [&](const float* tb, const Frag& F) {
      const bf16x8* Wp = reinterpret_cast<const bf16x8*>(tb + umax * kVP);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        bf16x8 wp[NT][3];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int pc = 0; pc < 3; ++pc)
            wp[t][pc] = Wp[(pc * 16 * NT * kWXP + (16 * t + c16) * kWXP + 16 * kq + 8 * c) >> 3];
#pragma unroll
        for (int g = 0; g < GPW; ++g) {
          float hv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int k = 8 * c + j;
            hv[j] = fmaxf(fmaf(F.aa[2 * k + 1], ry[g], fmaf(F.aa[2 * k], rx[g], F.uu[g][k])), 0.f);
          }
          bf16x8 hp[3];
          split8(hv, hp);
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = mfma_x3(hp, wp[t], acc[g][t]);
        }
      }
    };
    // two LDS tile buffers, one barrier per tile: tile kt's fragments are read
    // into registers, tile kt + 1 is stored into the other buffer (whose tile
    // kt - 1 every wave read before the last barrier), tile kt + 2's global
    // loads go out, then tile kt computes
    constexpr int NKT = kHidden / kKT;
    Frag F;
    load_tile(sx, 0);
    __syncthreads();  // (ps / keys init visible; previous chunk's readers done)
    store_tile(sx, tb0);
    load_tile(sx, kKT);
    __syncthreads();
#pragma unroll 1
    for (int kt = 0; kt < NKT; ++kt) {
      const float* tb = (kt & 1) ? tb1 : tb0;
      read_frag(tb, F);
      if (kt + 1 < NKT) store_tile(sx, (kt & 1) ? tb0 : tb1);
      if (kt + 2 < NKT) load_tile(sx, (kt + 2) * kKT);
      compute(tb, F);
      __syncthreads();
    }

    // epilogue: bias, ReLU, max over j (as pool_fwd_kernel)
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int grp = wave * GPW + g;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = grp * 16 + kq * 4 + r;
        if (p < npairs) {
          const int il = p / n, j = p - il * n;
          const unsigned long long jkey = 0xFFFFFFFFull - (unsigned long long)j;
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int cc = 16 * t + c16;
            if (cc < BN) {
              float v = acc[g][t][r] + bv[t];
              v = v > 0.f ? v : 0.f;
              atomicMax(&keys[il * BN + cc], ((unsigned long long)__float_as_uint(v) << 32) | jkey);
            }
          }
        }
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < rows * BN; q += blockDim.x) {
      const unsigned long long key = keys[q];
      const size_t oi = (size_t)(o + i0) * BN + q;
      out[oi] = __uint_as_float((unsigned)(key >> 32));
      argmax[oi] = o + (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
    }
    __syncthreads();
  }
}

// ---- forward, bf16 layer 2 ----------------------------------------------------
// The opt-in bf16 precision (sgg_pool_fwd_bf16; BASELINE configs 3 and 5): the
// 512 -> bn contraction on v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
// The hidden unit is formed exactly as in the fp32 kernels (2 FMA + max in
// fp32) and only then rounded to bf16 (round-to-nearest-even) as the A
// operand; W2 is rounded when it is staged.  A 32-deep k-step gives a lane 8
// consecutive units 8 kq .. 8 kq + 7 of its pair (A[row = pair][k]) and of
// its column (B[k][col] = W2[col][k]): the U row, (A_x, A_y) and W2 reads
// are 16-byte LDS reads, and one bf16 MFMA does the work of eight f32 ones.
//
// With the matrix cores 16x faster, what the fp32 kernels hide behind the
// MFMA -- staging the scene's U rows and W2 once per few hundred pairs --
// would dominate, so the form differs: 512-thread persistent workgroups stage
// W2 (bf16) and A ONCE for their lifetime; a chunk of whole i-rows of one
// scene (sgg_pool_plan_bf16: up to 1024 pairs) runs in passes of up to
// 8 waves x GPW 16-pair groups, its U rows streamed through two LDS k-tile
// buffers (one barrier per 64-unit tile; the next-but-one tile's global loads
// in flight in registers).  Any chunk table works (a chunk larger than a pass
// takes several); the chunk order, epilogue and argmax contract (max over j,
// smallest j on ties) are the fp32 kernels'.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef short short2v __attribute__((ext_vector_type(2)));
typedef short short4v __attribute__((ext_vector_type(4)));
constexpr int kBfWaves = 8;
constexpr int kBfThreads = 64 * kBfWaves;
constexpr int kBfUP = kKT + 4;         // U tile row pitch (floats; 16-B rows)
constexpr int kBfWP = kHidden + 8;     // W2 row pitch (bf16; 16-B rows, +4 banks per row)
constexpr int kBfMaxRows = 64;         // i-rows of one pass (keys)

template <int BN>
__host__ __device__ constexpr size_t pool_bf16_lds_bytes() {
  return sizeof(__bf16) * (size_t)16 * PoolCfg<BN>::NT * kBfWP + sizeof(float) * 2 * kHidden +
         sizeof(float) * 2 * (size_t)SGG_POOL_MAX_PEDS * kBfUP + sizeof(float2) * SGG_POOL_MAX_PEDS +
         sizeof(unsigned long long) * (size_t)kBfMaxRows * BN;
}

template <int BN, int GPW>
__global__ void __launch_bounds__(kBfThreads) pool_fwd_bf16_kernel(
    const PoolSet s1, const PoolSet s2, int g1, const float* __restrict__ A,
    const float* __restrict__ W2 /* BN x 512 */, const float* __restrict__ b2) {
  constexpr int NT = PoolCfg<BN>::NT;
  constexpr int CAP = kBfWaves * GPW * 16;   // pairs per pass
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* W2s = reinterpret_cast<__bf16*>(smem);                                // 16 NT rows x kBfWP
  float* As = reinterpret_cast<float*>(W2s + 16 * NT * kBfWP);                  // 512 units x (A_x, A_y)
  float* Ut = As + 2 * kHidden;                                                 // 2 x 64 rows x kBfUP
  float2* ps = reinterpret_cast<float2*>(Ut + 2 * SGG_POOL_MAX_PEDS * kBfUP);   // scene positions
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(ps + SGG_POOL_MAX_PEDS);  // rows x BN
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, kq = lane >> 4;
  // b2 of the lane's columns, loaded once: read in the epilogue's guarded
  // branches each load was a memory round trip of its own (NT x 4 x GPW per chunk)
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bv[t] = b2[min(16 * t + c16, BN - 1)];

  // W2 (rounded to bf16; rows >= BN zero) and A, once per workgroup
  for (int q = tid; q < 16 * NT * (kHidden / 4); q += kBfThreads) {
    const int c = q / (kHidden / 4), c4 = q - c * (kHidden / 4);
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < BN) w = *reinterpret_cast<const float4*>(W2 + (size_t)c * kHidden + 4 * c4);
    __bf16* d = W2s + c * kBfWP + 4 * c4;
    d[0] = (__bf16)w.x;
    d[1] = (__bf16)w.y;
    d[2] = (__bf16)w.z;
    d[3] = (__bf16)w.w;
  }
  // A planar (A_x of the 512 units, then A_y): a lane's consecutive units are
  // adjacent registers, the operand pairs of v_pk_fma_f32
  for (int q = tid; q < kHidden; q += kBfThreads) {
    const float2 a = reinterpret_cast<const float2*>(A)[q];
    As[q] = a.x;
    As[kHidden + q] = a.y;
  }

  SGG_POOL_PICK(s1, s2, g1);
  for (int ch = xb; ch < nch; ch += gstride) {
    const int4 cd = chunks[ch];
    const int s = cd.x;
    if (cd.z <= cd.y) continue;   // an empty padding chunk (fixed-capacity plan), uniform
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    int rpp = CAP / n;
    rpp = rpp < 1 ? 1 : (rpp > kBfMaxRows ? kBfMaxRows : rpp);
    for (int i0 = cd.y; i0 < cd.z; i0 += rpp) {
      const int rows = min(rpp, cd.z - i0);
      const int npairs = rows * n;
      __syncthreads();   // (W2s / As staged; the previous pass's readers of Ut, ps, keys done)
      for (int q = tid; q < n; q += kBfThreads) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
      for (int q = tid; q < rows * BN; q += kBfThreads) keys[q] = 0ull;

      // U tiles of 64 units: n rows x 16 float4, two per thread (n <= 64)
      constexpr int kUQ = (SGG_POOL_MAX_PEDS * (kKT / 4) + kBfThreads - 1) / kBfThreads;
      // (native vector registers: HIP's float4 struct, copied under the row
      // guard, was kept in scratch memory)
      floatx4 ra[kUQ], rb[kUQ];
      auto load_tile = [&](floatx4 (&r)[kUQ], int k0) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < kUQ; ++e) {
          const int q = tid + kBfThreads * e;
          const int row = q / (kKT / 4), c4 = q - row * (kKT / 4);
          if (row < n) r[e] = *reinterpret_cast<const floatx4*>(U + (size_t)(o + row) * kHidden + k0 + 4 * c4);
        }
      };
      auto store_tile = [&](const floatx4 (&r)[kUQ], int buf) __attribute__((always_inline)) {
        float* d = Ut + buf * SGG_POOL_MAX_PEDS * kBfUP;
#pragma unroll
        for (int e = 0; e < kUQ; ++e) {
          const int q = tid + kBfThreads * e;
          const int row = q / (kKT / 4), c4 = q - row * (kKT / 4);
          if (row < n) *reinterpret_cast<floatx4*>(d + row * kBfUP + 4 * c4) = r[e];
        }
      };
      load_tile(ra, 0);
      load_tile(rb, kKT);
      __syncthreads();   // ps / keys visible
      store_tile(ra, 0);

      // the lane's pair of each group (padding pairs: j = 0, r = 0)
      int uoff[GPW];
      float2v rxy[GPW];
      floatx4 acc[GPW][NT];
#pragma unroll
      for (int g = 0; g < GPW; ++g) {
        const int p = (wave * GPW + g) * 16 + c16;
        int il = 0, j = 0;
        if (p < npairs) { il = p / n; j = p - il * n; }
        uoff[g] = j * kBfUP + 8 * kq;
        const float2 pj = ps[j], pi = ps[i0 + il];
        rxy[g] = p < npairs ? float2v{pj.x - pi.x, pj.y - pi.y} : float2v{0.f, 0.f};
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      const int ngr = (npairs + 15) >> 4;   // groups with pairs (wave-uniform tests below)
      __syncthreads();   // tile 0 staged

      constexpr int NKT = kHidden / kKT;   // (even)
      // the k-steps of tile kt from LDS buffer kt & 1
      auto compute = [&](int kt) __attribute__((always_inline)) {
        const float* ut = Ut + (kt & 1) * SGG_POOL_MAX_PEDS * kBfUP;
#pragma unroll 1
        for (int sk = 0; sk < kKT / 32; ++sk) {
          const int ku = kt * kKT + 32 * sk + 8 * kq;   // the lane's 8 units of this k-step
          float2v ax[4], ay[4];
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const float4 x = *reinterpret_cast<const float4*>(As + ku + 4 * v);
            const float4 y = *reinterpret_cast<const float4*>(As + kHidden + ku + 4 * v);
            ax[2 * v] = float2v{x.x, x.y};
            ax[2 * v + 1] = float2v{x.z, x.w};
            ay[2 * v] = float2v{y.x, y.y};
            ay[2 * v + 1] = float2v{y.z, y.w};
          }
          bf16x8_t bfr[NT];
#pragma unroll
          for (int t = 0; t < NT; ++t)
            bfr[t] = *reinterpret_cast<const bf16x8_t*>(W2s + (16 * t + c16) * kBfWP + ku);
#pragma unroll
          for (int g = 0; g < GPW; ++g) {
            if (wave * GPW + g < ngr) {   // (wave-uniform)
              const float4 u0 = *reinterpret_cast<const float4*>(ut + uoff[g] + 32 * sk);
              const float4 u1 = *reinterpret_cast<const float4*>(ut + uoff[g] + 32 * sk + 4);
              const float2v uv[4] = {{u0.x, u0.y}, {u0.z, u0.w}, {u1.x, u1.y}, {u1.z, u1.w}};
              const float2v rx2 = rxy[g].xx, ry2 = rxy[g].yy;   // (op_sel broadcasts of one register pair)
              // two units per instruction: fma(A_y, r_y, fma(A_x, r_x, U)) in fp32
              // (v_pk_fma_f32), rounded to bf16 (v_cvt_pk_bf16_f32), then the
              // ReLU on the bf16 bits as signed 16-bit max with 0
              // (v_pk_max_i16: a negative value's sign bit makes it < 0) --
              // the same bits as rounding max(x, 0), in 16 instead of 28
              // vector instructions per 8 units
              // (register values combined by shuffles and bit casts: a union
              // or an indexed array here lived in scratch memory)
              short2v hi[4];
#pragma unroll
              for (int m = 0; m < 4; ++m) {
                const float2v pre = __builtin_elementwise_fma(ay[m], ry2, __builtin_elementwise_fma(ax[m], rx2, uv[m]));
                const short2v b = __builtin_bit_cast(short2v, __builtin_convertvector(pre, bf16x2v));
                hi[m] = __builtin_elementwise_max(b, short2v{0, 0});
              }
              const short4v h01 = __builtin_shufflevector(hi[0], hi[1], 0, 1, 2, 3);
              const short4v h23 = __builtin_shufflevector(hi[2], hi[3], 0, 1, 2, 3);
              const bf16x8_t hv = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(h01, h23, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
              for (int t = 0; t < NT; ++t)
                acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hv, bfr[t], acc[g][t], 0, 0, 0);
            }
          }
        }
      };
      // two register sets in turn (no copy between them): the loads of tile
      // kt + 2, issued before tile kt's k-steps, are stored to LDS only after
      // tile kt + 1's -- a whole tile of MFMAs in flight over their latency
      // (a copy ra -> rb at the end of each tile waited for the loads just issued)
#pragma unroll 1
      for (int kt = 0; kt < NKT; kt += 2) {
        // rb holds tile kt + 1 (loaded a tile ago); ra takes tile kt + 2
        if (kt + 2 < NKT) load_tile(ra, (kt + 2) * kKT);
        compute(kt);
        store_tile(rb, (kt + 1) & 1);   // (buffer (kt + 1) & 1 was last read in tile kt - 1)
        __syncthreads();
        // ra holds tile kt + 2; rb takes tile kt + 3
        if (kt + 3 < NKT) load_tile(rb, (kt + 3) * kKT);
        compute(kt + 1);
        if (kt + 2 < NKT) store_tile(ra, kt & 1);
        __syncthreads();
      }

      // epilogue: bias, ReLU, max over j (LDS atomic max on (bits << 32 | ~j)).
      // (ne: n through an empty asm, so the pairs' (il, j) are formed here and
      // not hoisted ahead of the k-loop, where 16 x GPW of them sat in registers
      // through it and pushed GPW 4 into scratch)
      int ne = n;
      asm volatile("" : "+s"(ne));
      const int npe = rows * ne;
#pragma unroll
      for (int g = 0; g < GPW; ++g) {
        const int grp = wave * GPW + g;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = grp * 16 + kq * 4 + r;
          if (p < npe) {
            const int il = p / ne, j = p - il * ne;
            const unsigned long long jkey = 0xFFFFFFFFull - (unsigned long long)j;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const int cc = 16 * t + c16;
              if (cc < BN) {
                float v = acc[g][t][r] + bv[t];
                v = v > 0.f ? v : 0.f;
                atomicMax(&keys[il * BN + cc], ((unsigned long long)__float_as_uint(v) << 32) | jkey);
              }
            }
          }
        }
      }
      __syncthreads();
      for (int q = tid; q < rows * BN; q += kBfThreads) {
        const unsigned long long key = keys[q];
        const size_t oi = (size_t)(o + i0) * BN + q;
        out[oi] = __uint_as_float((unsigned)(key >> 32));
        argmax[oi] = o + (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
      }
    }
  }
}


// ---- bf16 forward, j-block form (scenes of >= 32 peds) ----------------------
// The pairs of a chunk (i-rows [i0, i1) of one scene, R <= 64 rows) in
// j-blocks of 16: a 16-pair MFMA group is ONE i-row against 16 consecutive j,
// so
//   * a j-block's 16 U rows (16 x 512 fp32, 32 KiB) are staged in LDS ONCE for
//     all the chunk's rows and all 512 hidden units -- the next block's rows
//     loaded into registers while this one computes, double-buffered: two
//     barriers per j-block instead of one per 64-unit k-tile, and a scene's U
//     crosses L2 -> LDS n / R times per row instead of once per pass of 512
//     pairs;
//   * the max over the group's 16 j of each output column is formed in
//     registers (the D fragment's 4 rows in-lane, then two lane-swap steps over
//     the four lane quarters on the 64-bit (bits << 32 | ~j) key), so one LDS
//     atomic max per (row, column) and j-block instead of one per pair;
//   * rows of a round: 8 waves x GPW groups (rounds for more rows).
// Hidden units, rounding and ReLU exactly as pool_fwd_bf16_kernel (fp32
// pre-activation U + A_x r_x + A_y r_y, rounded to bf16 once, ReLU on the
// bits); the same argmax contract (max over j, smallest j on ties).
constexpr int kJbRows = 16;             // j per block (the MFMA's 16 pair rows)
constexpr int kJbUP = kHidden + 4;      // U row pitch (floats; 16-B rows)
constexpr int kJbUQ = kJbRows * (kHidden / 4) / kBfThreads;   // U float4 per thread per block (4)

template <int BN>
__host__ __device__ constexpr size_t pool_jb_lds_bytes() {
  return sizeof(__bf16) * (size_t)16 * PoolCfg<BN>::NT * kBfWP + sizeof(float) * 2 * kHidden +
         sizeof(float) * 2 * (size_t)kJbRows * kJbUP + sizeof(float2) * SGG_POOL_MAX_PEDS +
         sizeof(unsigned long long) * (size_t)kBfMaxRows * BN;
}

__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
// max of a 64-bit key over the four 16-lane rows of the wave (every lane gets it)
__device__ __forceinline__ unsigned long long rows_max64(unsigned long long v) {
  unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
  const auto l1 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h1 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  v = umax64(((unsigned long long)h1[0] << 32) | l1[0], ((unsigned long long)h1[1] << 32) | l1[1]);
  lo = (unsigned)v;
  hi = (unsigned)(v >> 32);
  const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return umax64(((unsigned long long)h2[0] << 32) | l2[0], ((unsigned long long)h2[1] << 32) | l2[1]);
}

template <int BN, int GPW>
__global__ void __launch_bounds__(kBfThreads) pool_fwd_bf16_jb_kernel(
    const PoolSet s1, const PoolSet s2, int g1, const float* __restrict__ A,
    const float* __restrict__ W2 /* BN x 512 */, const float* __restrict__ b2) {
  constexpr int NT = PoolCfg<BN>::NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* W2s = reinterpret_cast<__bf16*>(smem);                                // 16 NT rows x kBfWP
  float* As = reinterpret_cast<float*>(W2s + 16 * NT * kBfWP);                  // 512 units x (A_x, A_y)
  float* Uj = As + 2 * kHidden;                                                 // 2 x 16 rows x kJbUP
  float2* ps = reinterpret_cast<float2*>(Uj + 2 * kJbRows * kJbUP);             // scene positions
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(ps + SGG_POOL_MAX_PEDS);  // rows x BN
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15, kq = lane >> 4;
  // b2 of the lane's columns, loaded once: read in the epilogue's guarded
  // branches each load was a memory round trip of its own (NT x 4 x GPW per chunk)
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bv[t] = b2[min(16 * t + c16, BN - 1)];

  // W2 (rounded to bf16; rows >= BN zero) and A, once per workgroup
  for (int q = tid; q < 16 * NT * (kHidden / 4); q += kBfThreads) {
    const int c = q / (kHidden / 4), c4 = q - c * (kHidden / 4);
    float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < BN) w = *reinterpret_cast<const float4*>(W2 + (size_t)c * kHidden + 4 * c4);
    __bf16* d = W2s + c * kBfWP + 4 * c4;
    d[0] = (__bf16)w.x;
    d[1] = (__bf16)w.y;
    d[2] = (__bf16)w.z;
    d[3] = (__bf16)w.w;
  }
  for (int q = tid; q < kHidden; q += kBfThreads) {
    const float2 a = reinterpret_cast<const float2*>(A)[q];
    As[q] = a.x;
    As[kHidden + q] = a.y;
  }

  SGG_POOL_PICK(s1, s2, g1);
  for (int ch = xb; ch < nch; ch += gstride) {
    const int4 cd = chunks[ch];
    const int s = cd.x;
    if (cd.z <= cd.y) continue;   // an empty padding chunk (fixed-capacity plan), uniform
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    const int i0 = cd.y, R = min(cd.z - cd.y, kBfMaxRows);
    const int nj = (n + kJbRows - 1) / kJbRows;
    __syncthreads();   // (W2s / As staged; the previous chunk's readers of Uj, ps, keys done)
    for (int q = tid; q < n; q += kBfThreads) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
    for (int q = tid; q < R * BN; q += kBfThreads) keys[q] = 0ull;

    // U rows of j-block jb: 16 rows x 128 float4, four per thread (rows >= n: zeros)
    floatx4 ur[kJbUQ];
    auto load_block = [&](int jb) __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < kJbUQ; ++e) {
        const int q = tid + kBfThreads * e;
        const int row = q / (kHidden / 4), c4 = q - row * (kHidden / 4);
        const int j = jb * kJbRows + row;
        ur[e] = j < n ? *reinterpret_cast<const floatx4*>(U + (size_t)(o + j) * kHidden + 4 * c4)
                      : floatx4{0.f, 0.f, 0.f, 0.f};
      }
    };
    auto store_block = [&](int buf) __attribute__((always_inline)) {
      float* d = Uj + buf * kJbRows * kJbUP;
#pragma unroll
      for (int e = 0; e < kJbUQ; ++e) {
        const int q = tid + kBfThreads * e;
        const int row = q / (kHidden / 4), c4 = q - row * (kHidden / 4);
        *reinterpret_cast<floatx4*>(d + row * kJbUP + 4 * c4) = ur[e];
      }
    };
    load_block(0);
    store_block(0);
    if (nj > 1) load_block(1);
    __syncthreads();   // ps, keys, block 0 staged

    for (int jb = 0; jb < nj; ++jb) {
      const float* ut = Uj + (jb & 1) * kJbRows * kJbUP;
      const int j = jb * kJbRows + c16;                 // this lane's j (pair row c16 of every group)
      const bool jok = j < n;
      const float2 pj = ps[jok ? j : 0];
      for (int r0 = 0; r0 < R; r0 += kBfWaves * GPW) {   // rounds of 8 waves x GPW rows
        float2v rxy[GPW];
        floatx4 acc[GPW][NT];
#pragma unroll
        for (int g = 0; g < GPW; ++g) {
          const int il = r0 + wave * GPW + g;
          const float2 pi = ps[i0 + min(il, R - 1)];
          rxy[g] = jok ? float2v{pj.x - pi.x, pj.y - pi.y} : float2v{0.f, 0.f};
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        const int ngr = min(GPW, max(0, R - r0 - wave * GPW));   // this wave's rows this round (uniform)
        const float* urow = ut + c16 * kJbUP + 8 * kq;
#pragma unroll 2
        for (int ks = 0; ks < kHidden / 32; ++ks) {
          const int ku = 32 * ks + 8 * kq;   // the lane's 8 units of this k-step
          float2v ax[4], ay[4];
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const float4 x = *reinterpret_cast<const float4*>(As + ku + 4 * v);
            const float4 y = *reinterpret_cast<const float4*>(As + kHidden + ku + 4 * v);
            ax[2 * v] = float2v{x.x, x.y};
            ax[2 * v + 1] = float2v{x.z, x.w};
            ay[2 * v] = float2v{y.x, y.y};
            ay[2 * v + 1] = float2v{y.z, y.w};
          }
          bf16x8_t bfr[NT];
#pragma unroll
          for (int t = 0; t < NT; ++t)
            bfr[t] = *reinterpret_cast<const bf16x8_t*>(W2s + (16 * t + c16) * kBfWP + ku);
          const float4 u0 = *reinterpret_cast<const float4*>(urow + 32 * ks);
          const float4 u1 = *reinterpret_cast<const float4*>(urow + 32 * ks + 4);
          const float2v uv[4] = {{u0.x, u0.y}, {u0.z, u0.w}, {u1.x, u1.y}, {u1.z, u1.w}};
#pragma unroll
          for (int g = 0; g < GPW; ++g) {
            if (g < ngr) {   // (wave-uniform)
              const float2v rx2 = rxy[g].xx, ry2 = rxy[g].yy;
              short2v hi[4];
#pragma unroll
              for (int m = 0; m < 4; ++m) {
                const float2v pre = __builtin_elementwise_fma(ay[m], ry2, __builtin_elementwise_fma(ax[m], rx2, uv[m]));
                const short2v b = __builtin_bit_cast(short2v, __builtin_convertvector(pre, bf16x2v));
                hi[m] = __builtin_elementwise_max(b, short2v{0, 0});
              }
              const short4v h01 = __builtin_shufflevector(hi[0], hi[1], 0, 1, 2, 3);
              const short4v h23 = __builtin_shufflevector(hi[2], hi[3], 0, 1, 2, 3);
              const bf16x8_t hv =
                  __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(h01, h23, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
              for (int t = 0; t < NT; ++t)
                acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hv, bfr[t], acc[g][t], 0, 0, 0);
            }
          }
        }
        // epilogue: bias, ReLU, key (bits << 32 | ~j) per D element (rows 4 kq + r
        // = j0 + 4 kq + r, column 16 t + c16), max over the group's 16 j, one
        // LDS atomic per (row, column)
#pragma unroll
        for (int g = 0; g < GPW; ++g) {
          if (g < ngr) {
            const int il = r0 + wave * GPW + g;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const int cc = 16 * t + c16;
              const float bb = cc < BN ? bv[t] : 0.f;
              unsigned long long best = 0ull;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int jj = jb * kJbRows + 4 * kq + r;
                float v = acc[g][t][r] + bb;
                v = v > 0.f ? v : 0.f;
                const unsigned long long key =
                    jj < n ? (((unsigned long long)__float_as_uint(v) << 32) | (0xFFFFFFFFull - (unsigned)jj)) : 0ull;
                best = umax64(best, key);
              }
              best = rows_max64(best);
              if (kq == 0 && cc < BN) atomicMax(&keys[il * BN + cc], best);
            }
          }
        }
      }
      // next block: its registers to the other buffer (its last readers were
      // block jb - 1's, all past the barrier below of that block), then the
      // block after it into registers
      if (jb + 1 < nj) {
        store_block((jb + 1) & 1);
        if (jb + 2 < nj) load_block(jb + 2);
      }
      __syncthreads();
    }
    for (int q = tid; q < R * BN; q += kBfThreads) {
      const unsigned long long key = keys[q];
      const size_t oi = (size_t)(o + i0) * BN + q;
      out[oi] = __uint_as_float((unsigned)(key >> 32));
      argmax[oi] = o + (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
    }
  }
}


// ---- forward, resident form -------------------------------------------------// ---- forward, resident form -------------------------------------------------
// When the whole W2^T (bn rows x 512, rows padded to 16 NT with zeros) and a
// scene's U rows fit in LDS beside each other: the workgroup stages W2 and A
// once for its lifetime (persistent grid over the chunk table) and the U rows
// of a chunk's scene when the scene changes, then runs all 128 k-steps with
// no barrier.  Same chunk table, pair set-up, MFMA step and epilogue as the
// tiled kernel above (bitwise the same results).
constexpr int kUP = kHidden + 2;   // resident row pitch (U rows, W2 rows): 2 mod 32 -> conflict-free b32 reads

// rows x 512 row-major block -> LDS at pitch kUP (rows >= zrow read as 0,
// zrow >= 1): float4 loads, 8 per thread in flight before the stores
__device__ inline void stage_rows512(float* dst, const float* __restrict__ src, int rows, int zrow) {
  const int tot = rows * (kHidden / 4);
  for (int e0 = threadIdx.x; e0 < tot; e0 += 8 * (int)blockDim.x) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = min(e0 + u * (int)blockDim.x, tot - 1);
      const int r = e / (kHidden / 4), c4 = e - r * (kHidden / 4);
      const float4 x = *reinterpret_cast<const float4*>(src + (size_t)min(r, zrow - 1) * kHidden + 4 * c4);
      const bool ok = r < zrow;
      v[u] = make_float4(keep_if(x.x, ok), keep_if(x.y, ok), keep_if(x.z, ok), keep_if(x.w, ok));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * (int)blockDim.x;
      if (e < tot) {
        const int r = e / (kHidden / 4), c4 = e - r * (kHidden / 4);
        float2* d = reinterpret_cast<float2*>(dst + r * kUP + 4 * c4);
        d[0] = make_float2(v[u].x, v[u].y);
        d[1] = make_float2(v[u].z, v[u].w);
      }
    }
  }
}

template <int BN, int GPW>
__global__ void __launch_bounds__(256) pool_fwd_res_kernel(
    const float* __restrict__ U, const float* __restrict__ pos, const float* __restrict__ A,
    const float* __restrict__ W2 /* BN x 512 */, const float* __restrict__ b2,
    const int32_t* __restrict__ scene_off, const int4* __restrict__ chunks, int nchunks, const int32_t* __restrict__ nchunks_dev, int max_n,
    float* __restrict__ out, int32_t* __restrict__ argmax) {
  constexpr int NT = PoolCfg<BN>::NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* W2s = reinterpret_cast<float*>(smem);                                    // 16 NT rows x kUP
  float* As = W2s + 16 * NT * kUP;                                                // 512 x 2
  float* Us = As + 2 * kHidden;                                                   // max_n rows x kUP
  float2* ps = reinterpret_cast<float2*>(Us + (size_t)max_n * kUP);               // max_n
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(ps + max_n);   // rows x BN
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, kq = lane >> 4;
  // b2 of the lane's columns, loaded once: read in the epilogue's guarded
  // branches each load was a memory round trip of its own (NT x 4 x GPW per chunk)
  float bv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bv[t] = b2[min(16 * t + c16, BN - 1)];

  stage_rows512(W2s, W2, 16 * NT, BN);
  for (int e = threadIdx.x; e < 2 * kHidden; e += 256) As[e] = A[e];
  int cur = -1;
  const int nch = nchunks_dev ? *nchunks_dev : nchunks;   // a fixed-capacity plan: the count is device data
  for (int ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const int4 cd = chunks[ch];
    const int s = cd.x, i0 = cd.y, i1 = cd.z;
    if (i1 <= i0) continue;   // an empty padding chunk (fixed-capacity plan), uniform over the workgroup
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    const int rows = i1 - i0;
    const int npairs = rows * n;
    __syncthreads();   // W2s / As staged (first chunk); the previous chunk's readers of Us, ps, keys done
    if (s != cur) {
      stage_rows512(Us, U + (size_t)o * kHidden, n, n);
      for (int q = threadIdx.x; q < n; q += 256) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
      cur = s;
    }
    for (int q = threadIdx.x; q < rows * BN; q += 256) keys[q] = 0ull;
    __syncthreads();

    int uoff[GPW];
    float rx[GPW], ry[GPW];
    bool gv[GPW];
    floatx4 acc[GPW][NT];
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int p = (wave * GPW + g) * 16 + c16;
      gv[g] = (wave * GPW + g) * 16 < npairs;   // wave-uniform: a group with pairs
      int il = 0, j = 0;
      if (p < npairs) { il = p / n; j = p - il * n; }
      uoff[g] = j * kUP + kq;
      const float2 pj = ps[j], pi = ps[i0 + il];
      rx[g] = p < npairs ? pj.x - pi.x : 0.f;
      ry[g] = p < npairs ? pj.y - pi.y : 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[g][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    float b[NT], u[GPW];
    float2 a;
#pragma unroll
    for (int t = 0; t < NT; ++t) b[t] = W2s[(16 * t + c16) * kUP + kq];
    a = *reinterpret_cast<const float2*>(As + 2 * kq);
#pragma unroll
    for (int g = 0; g < GPW; ++g) u[g] = Us[uoff[g]];
#pragma unroll 2
    for (int s4 = 0; s4 < kHidden / 4; ++s4) {
      float h[GPW], bc[NT];
#pragma unroll
      for (int g = 0; g < GPW; ++g) h[g] = fmaxf(fmaf(a.y, ry[g], fmaf(a.x, rx[g], u[g])), 0.f);
#pragma unroll
      for (int t = 0; t < NT; ++t) bc[t] = b[t];
      if (s4 + 1 < kHidden / 4) {  // prefetch the next k-step's operands
        const int kn = 4 * (s4 + 1);
#pragma unroll
        for (int t = 0; t < NT; ++t) b[t] = W2s[(16 * t + c16) * kUP + kn + kq];
        a = *reinterpret_cast<const float2*>(As + 2 * (kn + kq));
#pragma unroll
        for (int g = 0; g < GPW; ++g) u[g] = Us[uoff[g] + kn];
      }
#pragma unroll
      for (int g = 0; g < GPW; ++g)
        if (gv[g])
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(h[g], bc[t], acc[g][t], 0, 0, 0);
    }

    // epilogue: bias, ReLU, max over j (LDS atomic max on (bits << 32 | ~j))
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const int grp = wave * GPW + g;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = grp * 16 + kq * 4 + r;
        if (p < npairs) {
          const int il = p / n, j = p - il * n;
          const unsigned long long jkey = 0xFFFFFFFFull - (unsigned long long)j;
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int cc = 16 * t + c16;
            if (cc < BN) {
              float v = acc[g][t][r] + bv[t];
              v = v > 0.f ? v : 0.f;
              atomicMax(&keys[il * BN + cc], ((unsigned long long)__float_as_uint(v) << 32) | jkey);
            }
          }
        }
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < rows * BN; q += 256) {
      const unsigned long long key = keys[q];
      const size_t oi = (size_t)(o + i0) * BN + q;
      out[oi] = __uint_as_float((unsigned)(key >> 32));
      argmax[oi] = o + (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
    }
  }
}

// ---- backward ---------------------------------------------------------------
// Only (i, argmax[i, c]) carries gradient.  Work unit = (scene, j range): the
// scene's pooled-from peds j are cut into jq ranges so that S x jq units fill
// the chip (sgg_pool_bwd_grid).  The selected entries of the scene are indexed
// by (j, c) as 64-bit masks over i, built with LDS atomic OR (order-free, so
// deterministic).  Thread k = hidden unit k walks its unit's j range and, per
// j, the statically unrolled c loop over the set bits i of mask (j, c): W2[c][k]
// and the dW2[c][k] partial stay in registers (no memory access on the
// per-entry chain), U[j, k] is read once (coalesced) and dU[j, k] stored
// once; the per-entry operands (g, p_i) are wave-uniform LDS broadcasts and
// the bit walk is scalar.  Each workgroup writes its [dW2 | dA | db2] partial
// to its own slab row; WGRAD = false (frozen weights) computes dU only.
// STAGE: the unit's U rows (<= kBwdStageRows) are copied to LDS in the
// prologue, issued together with the out / dout / argmax / position loads (one
// memory round trip before the walk instead of three)
constexpr int kBwdStageRows = 16;

template <int BN, bool WGRAD, bool STAGE>
__global__ void __launch_bounds__(512) pool_bwd_kernel(
    const float* __restrict__ U, const float* __restrict__ pos, const float* __restrict__ A,
    const float* __restrict__ W2 /* BN x 512 */, const float* __restrict__ out,
    const int32_t* __restrict__ argmax, const float* __restrict__ dout, const int32_t* __restrict__ scene_off,
    int S, int jq, float* __restrict__ dU, float* __restrict__ part) {
  __shared__ unsigned long long msk[SGG_POOL_MAX_PEDS * BN];   // (j, c) -> set of i
  __shared__ float gs[SGG_POOL_MAX_PEDS * BN];                 // masked dout (i, c)
  __shared__ int jsel[SGG_POOL_MAX_PEDS * BN];                 // argmax j of (i, c) (scene-local)
  __shared__ float2 ps[SGG_POOL_MAX_PEDS];
  extern __shared__ float Us[];                                // STAGE: rows j0 .. j1 of U
  const int k = threadIdx.x;   // hidden unit, blockDim.x == 512
  float w2[BN], dw2[BN];
#pragma unroll
  for (int c = 0; c < BN; ++c) {
    w2[c] = W2[c * kHidden + k];
    dw2[c] = 0.f;
  }
  const float a0 = A[2 * k], a1 = A[2 * k + 1];
  float dA0 = 0.f, dA1 = 0.f, db2 = 0.f;
  for (int un = blockIdx.x; un < S * jq; un += gridDim.x) {
    const int s = un / jq, jp = un - s * jq;
    const int o = scene_off[s];
    const int n = scene_off[s + 1] - o;
    const int ne = n * BN;
    const int j0 = (n * jp) / jq, j1 = (n * (jp + 1)) / jq;
    if (STAGE) {   // this thread's column of the unit's U rows (coalesced rows)
      const float* Ur = U + (size_t)(o + j0) * kHidden + k;
#pragma unroll 4
      for (int r = 0; r < j1 - j0; ++r) Us[r * kHidden + k] = Ur[(size_t)r * kHidden];
    }
#pragma unroll 2
    for (int e = k; e < ne; e += kHidden) {
      const size_t ge = (size_t)o * BN + e;
      const float ov = out[ge], dv = dout[ge];
      const int av = argmax[ge];
      gs[e] = ov > 0.f ? dv : 0.f;
      jsel[e] = av - o;
      msk[e] = 0ull;
    }
    for (int q = k; q < n; q += kHidden) ps[q] = make_float2(pos[2 * (o + q)], pos[2 * (o + q) + 1]);
    __syncthreads();
    for (int e = k; e < ne; e += kHidden) {
      if (gs[e] != 0.f) {
        const int i = e / BN, c = e - i * BN;
        atomicOr(&msk[jsel[e] * BN + c], 1ull << i);
      }
    }
    if (WGRAD && jp == 0 && k < BN)
      for (int i = 0; i < n; ++i) db2 += gs[i * BN + k];
    __syncthreads();
    const float* Uc = U + (size_t)o * kHidden + k;
    float u_next = STAGE ? 0.f : (j0 < j1 ? Uc[(size_t)j0 * kHidden] : 0.f);
    for (int j = j0; j < j1; ++j) {
      float u;
      if (STAGE) {
        u = Us[(j - j0) * kHidden + k];
      } else {
        u = u_next;
        if (j + 1 < j1) u_next = Uc[(size_t)(j + 1) * kHidden];
      }
      const float2 pj = ps[j];
      float du = 0.f;
      // the row's masks in blocks of 16 up front: one LDS latency per block,
      // not per (j, c) (blocks bound the registers at bn 64)
      constexpr int CB = BN < 16 ? BN : 16;
      unsigned long long mrow[CB];
#pragma unroll
      for (int c = 0; c < BN; ++c) {
        if (c % CB == 0) {
#pragma unroll
          for (int cc = 0; cc < CB; ++cc) mrow[cc] = msk[j * BN + c + cc];
        }
        const unsigned long long mv = mrow[c % CB];
        // (readfirstlane returns int: go through unsigned, no sign extension)
        const unsigned mhi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(mv >> 32));
        const unsigned mlo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)mv);
        unsigned long long m = ((unsigned long long)mhi << 32) | (unsigned long long)mlo;
        // two set bits per trip: both entries' LDS operands are in flight
        // together (the walk is scalar and the reads are broadcasts, so the
        // per-entry cost is their latency); entries are still taken in
        // ascending i, one at a time, so every sum keeps its order
        auto entry = [&](float g, float2 pi) {
          const float rx = pj.x - pi.x, ry = pj.y - pi.y;
          const float pre = fmaf(a1, ry, fmaf(a0, rx, u));
          const float gm = pre > 0.f ? g : 0.f;
          const float d = gm * w2[c];
          du += d;
          if (WGRAD) {
            dw2[c] = fmaf(gm, pre, dw2[c]);
            dA0 = fmaf(d, rx, dA0);
            dA1 = fmaf(d, ry, dA1);
          }
        };
        while (m) {
          const int i = __builtin_ctzll(m);
          m &= m - 1;
          const bool two = m != 0;   // uniform
          const int i2 = two ? __builtin_ctzll(m) : i;
          if (two) m &= m - 1;
          const float g = gs[i * BN + c], g2 = gs[i2 * BN + c];
          const float2 pi = ps[i], pi2 = ps[i2];
          entry(g, pi);
          if (two) entry(g2, pi2);
        }
      }
      dU[(size_t)(o + j) * kHidden + k] = du;
    }
    __syncthreads();   // msk / gs / ps reused by the next unit
  }
  if (WGRAD) {   // this workgroup's row of the parameter-gradient slab: [dW2 (BN x 512) | dA (512 x 2) | db2 (BN)]
    float* row = part + (size_t)blockIdx.x * (BN * kHidden + 2 * kHidden + BN);
#pragma unroll
    for (int c = 0; c < BN; ++c) row[c * kHidden + k] = dw2[c];
    row[BN * kHidden + 2 * k] = dA0;
    row[BN * kHidden + 2 * k + 1] = dA1;
    if (k < BN) row[BN * kHidden + 2 * kHidden + k] = db2;
  }
}

template <int BN>
static size_t pool_fwd_lds(int max_rows) {
  using C = PoolCfg<BN>;
  return sizeof(float) * ((size_t)SGG_POOL_MAX_PEDS * kKTP + (size_t)kKT * C::BNP + 2 * kKT) +
         sizeof(float2) * SGG_POOL_MAX_PEDS + sizeof(unsigned long long) * (size_t)max_rows * BN;
}

static int device_cus();

// workgroups of one batch's range: a multiple of 8 (XCD-aware order), <= 32768
static int pool_range(int nchunks) { return nchunks < 32768 ? (nchunks + 7) & ~7 : 32768; }

template <int BN, int GPW>
static void launch_fwd_g(const PoolSet& s1, const PoolSet& s2, const float* A, const float* W2, const float* b2,
                         int max_rows, int max_n, hipStream_t st) {
  // one workgroup per chunk (host counts) in each batch's range
  const int g1 = pool_range(s1.nchunks), grid = g1 + (s2.chunks ? pool_range(s2.nchunks) : 0);
  const int nchunks = s1.nchunks + (s2.chunks ? s2.nchunks : 0);
  const size_t lds = pool_fwd_lds<BN>(max_rows);
  // bn 32 / 48 (the discriminator's pooling): the split-bf16 contraction
  // (SGG_POOL_X3=0: the fp32 MFMA forms below)
  if constexpr (GPW <= 2 && BN >= 32 && BN <= 48) {
    const char* xe = getenv("SGG_POOL_X3");
    if (!(xe && xe[0] == '0') && max_n >= 1 && max_n <= SGG_POOL_MAX_PEDS) {
      const int umax = (max_n + 3) & ~3;
      const size_t lx = sizeof(float) * 2 * ((size_t)umax * kVP + pool_x3_tb_fixed<BN>()) +
                        sizeof(float2) * SGG_POOL_MAX_PEDS + sizeof(unsigned long long) * (size_t)max_rows * BN;
      hipLaunchKernelGGL((pool_fwd_x3_kernel<BN, GPW>), dim3(grid), dim3(256), lx, st, s1, s2, g1, A, W2, b2, umax);
      return;
    }
  }
  // small grids (<= 4 chunks per CU, <= 2 pair groups per wave): the
  // fragment-native tiles (measured 1.25-1.45x faster at 64-128 scenes;
  // slower at gpw 4 / >= 1024 scenes, where occupancy hides the LDS latency)
  if constexpr (GPW <= 2) {
    const char* vv = getenv("SGG_POOL_V");
    if (nchunks <= 4 * device_cus() && !(vv && vv[0] == '0')) {
      const size_t lv = sizeof(float) * 2 * ((size_t)(SGG_POOL_MAX_PEDS + 16 * PoolCfg<BN>::NT) * kVP + 2 * kKT) +
                        sizeof(float2) * SGG_POOL_MAX_PEDS + sizeof(unsigned long long) * (size_t)max_rows * BN;
      hipLaunchKernelGGL((pool_fwd_v_kernel<BN, GPW>), dim3(grid), dim3(256), lv, st, s1, s2, g1, A, W2, b2);
      return;
    }
  }
  hipLaunchKernelGGL((pool_fwd_kernel<BN, GPW, 2>), dim3(grid), dim3(256), lds, st, s1, s2, g1, A, W2, b2);
}
// j ranges per scene of the backward: S x jq units ~ one round of the chip
static int pool_bwd_jq(int S) {
  if (S < 1) return 1;
  const int jq = 256 / S;
  return jq < 1 ? 1 : (jq > 8 ? 8 : jq);
}

template <int BN>
static size_t pool_res_lds(int max_n, int max_rows) {
  return sizeof(float) * ((size_t)16 * PoolCfg<BN>::NT * kUP + 2 * kHidden + (size_t)max_n * kUP) +
         sizeof(float2) * (size_t)max_n + sizeof(unsigned long long) * (size_t)max_rows * BN;
}

static int device_cus() {
  static int ncu = 0;
  if (ncu == 0) {
    int d = 0, v = 0;
    if (hipGetDevice(&d) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess)
      ncu = v > 0 ? v : 256;
    else
      ncu = 256;
  }
  return ncu;
}

template <int BN, int GPW>
static void launch_fwd_res(const float* U, const float* pos, const float* A, const float* W2, const float* b2,
                           const int32_t* off, const int32_t* chunks, int nchunks, const int32_t* ncd, int max_n,
                           size_t lds, float* out,
                           int32_t* am, hipStream_t st) {
  const int per_cu = (int)((160u * 1024u) / lds);
  long long grid = (long long)device_cus() * (per_cu < 1 ? 1 : per_cu);
  if (grid > nchunks) grid = nchunks;
  hipLaunchKernelGGL((pool_fwd_res_kernel<BN, GPW>), dim3((unsigned)grid), dim3(256), lds, st, U, pos, A,
                     W2, b2, off, reinterpret_cast<const int4*>(chunks), nchunks, ncd, max_n, out, am);
}

template <int BN>
static int launch_fwd(const PoolSet& s1, const PoolSet& s2, const float* A, const float* W2, const float* b2,
                      int max_rows, int max_n, int gpw, hipStream_t st) {
  const size_t res = pool_res_lds<BN>(max_n, max_rows);
  // measured (tools/bench_kernels.py, round 1): the resident form is slower
  // than the tiled one at the training shapes (one workgroup of four waves
  // per CU cannot hide its LDS latency; the tiled form runs two per CU), so
  // it is opt-in (SGG_POOL_RESIDENT=1; single-batch launches)
  const char* rs = getenv("SGG_POOL_RESIDENT");
  if (res <= 160u * 1024u && rs && rs[0] == '1' && !s2.chunks) {
    const int32_t* ck = reinterpret_cast<const int32_t*>(s1.chunks);
#define SGG_POOL_RES(G) launch_fwd_res<BN, G>(s1.U, s1.pos, A, W2, b2, s1.scene_off, ck, s1.nchunks, s1.nchunks_dev, \
                                              max_n, res, s1.out, s1.argmax, st)
    switch (gpw) {
      case 1: SGG_POOL_RES(1); break;
      case 2: SGG_POOL_RES(2); break;
      case 4: SGG_POOL_RES(4); break;
      default: SGG_POOL_RES(8); break;
    }
#undef SGG_POOL_RES
    SGG_RETURN_LAUNCH("sgg_pool_fwd");
  }
  switch (gpw) {
    case 1: launch_fwd_g<BN, 1>(s1, s2, A, W2, b2, max_rows, max_n, st); break;
    case 2: launch_fwd_g<BN, 2>(s1, s2, A, W2, b2, max_rows, max_n, st); break;
    case 4: launch_fwd_g<BN, 4>(s1, s2, A, W2, b2, max_rows, max_n, st); break;
    default: launch_fwd_g<BN, 8>(s1, s2, A, W2, b2, max_rows, max_n, st); break;
  }
  SGG_RETURN_LAUNCH("sgg_pool_fwd");
}

template <int BN>
static int launch_fwd_bf16(const PoolSet& s1, const PoolSet& s2, const float* A, const float* W2, const float* b2,
                           int gpw, int max_rows, int max_n, hipStream_t st) {
  // persistent: one 512-thread workgroup per CU (its LDS plan), each batch's
  // range a multiple of 8 (XCD-aware order) sized by its share of the chunks
  const int n1 = s1.nchunks, n2 = s2.chunks ? s2.nchunks : 0;
  int grid = device_cus();
  if (grid > n1 + n2) grid = n1 + n2;
  grid = (grid + 7) & ~7;
  int g1 = grid;
  if (n2 > 0) {
    if (n1 == 0) {
      g1 = 0;
    } else {
      if (grid < 16) grid = 16;
      g1 = (int)(((long long)grid * n1 / (n1 + n2) + 4) & ~7LL);
      g1 = g1 < 8 ? 8 : (g1 > grid - 8 ? grid - 8 : g1);
    }
  }
  // scenes of >= 32 peds: the j-block form (SGG_POOL_JB=0: the pass form)
  const char* jbe = getenv("SGG_POOL_JB");
  const bool jb_off = jbe && strcmp(jbe, "0") == 0;
  if (max_n >= 32 && !jb_off && pool_jb_lds_bytes<BN>() <= 160 * 1024) {
    const size_t ljb = pool_jb_lds_bytes<BN>();
#define SGG_POOL_JB(G) \
  hipLaunchKernelGGL((pool_fwd_bf16_jb_kernel<BN, G>), dim3(grid), dim3(kBfThreads), ljb, st, s1, s2, g1, A, W2, b2)
    if (max_rows > 16)
      SGG_POOL_JB(4);
    else if (max_rows > 8)
      SGG_POOL_JB(2);
    else
      SGG_POOL_JB(1);
#undef SGG_POOL_JB
    SGG_RETURN_LAUNCH("sgg_pool_fwd_bf16");
  }
  const size_t lds = pool_bf16_lds_bytes<BN>();
#define SGG_POOL_BF(G) \
  hipLaunchKernelGGL((pool_fwd_bf16_kernel<BN, G>), dim3(grid), dim3(kBfThreads), lds, st, s1, s2, g1, A, W2, b2)
  if (gpw >= 4 && BN <= 48)
    SGG_POOL_BF(4);
  else if (gpw >= 2)
    SGG_POOL_BF(2);
  else
    SGG_POOL_BF(1);
#undef SGG_POOL_BF
  SGG_RETURN_LAUNCH("sgg_pool_fwd_bf16");
}

template <int BN>
static int launch_bwd(const float* U, const float* pos, const float* A, const float* W2, const float* out,
                      const int32_t* am, const float* dout, const int32_t* off, int S, int max_n, float* dU,
                      float* part, hipStream_t st) {
  const int grid = sgg_pool_bwd_grid(S), jq = pool_bwd_jq(S);
  const int rows = (max_n + jq - 1) / jq + 1;   // a unit's j range (floor boundaries: <= ceil + 1)
  const bool stage = rows <= kBwdStageRows;
  const size_t lds = stage ? sizeof(float) * (size_t)rows * kHidden : 0;
#define SGG_POOL_BWD(W, SG)                                                                                          \
  hipLaunchKernelGGL((pool_bwd_kernel<BN, W, SG>), dim3(grid), dim3(512), lds, st, U, pos, A, W2, out, am, dout, off, \
                     S, jq, dU, part)
  if (part) {
    if (stage) SGG_POOL_BWD(true, true); else SGG_POOL_BWD(true, false);
  } else {
    if (stage) SGG_POOL_BWD(false, true); else SGG_POOL_BWD(false, false);
  }
#undef SGG_POOL_BWD
  SGG_RETURN_LAUNCH("sgg_pool_bwd");
}

}  // namespace sgg

using namespace sgg;

static bool pool_bn_ok(int bn) { return bn == 8 || bn == 16 || bn == 32 || bn == 48 || bn == 64; }

static int plan_rows(int n, int gpw) {
  int rows = (16 * kPoolWaves * gpw) / n;
  if (rows > 64) rows = 64;
  return rows < 1 ? 1 : rows;
}

extern "C" int sgg_pool_plan(const int32_t* host_scene_off, int S, int bn, int target_chunks, int max_gpw,
                             int32_t* chunks, int cap, int* max_rows, int* gpw_out) {
  // host helper: pick the widest per-wave group count whose chunking still
  // yields >= target_chunks workgroups, then split every scene into chunks
  // of whole i-rows (see pool_fwd_kernel).
  if (!host_scene_off || !chunks || !max_rows || !gpw_out || S < 0 || cap < 0) {
    sgg::set_error("sgg_pool_plan: bad argument");
    return SGG_E_ARG;
  }
  int gpw = bn > 16 ? 4 : 2;  // measured best caps (register budget vs LDS re-staging)
  if (max_gpw > 0) {
    while (gpw > max_gpw && gpw > 1) gpw >>= 1;
  }
  for (; gpw > 1; gpw >>= 1) {
    long nc = 0;
    for (int s = 0; s < S; ++s) {
      const int n = host_scene_off[s + 1] - host_scene_off[s];
      if (n > 0) nc += (n + plan_rows(n, gpw) - 1) / plan_rows(n, gpw);
    }
    if (nc >= target_chunks) break;
  }
  int nc = 0, mr = 1;
  for (int s = 0; s < S; ++s) {
    const int n = host_scene_off[s + 1] - host_scene_off[s];
    if (n <= 0) continue;
    // the fewest chunks of <= plan_rows rows each, rows spread evenly over them
    const int rmax = plan_rows(n, gpw), nck = (n + rmax - 1) / rmax, rows = (n + nck - 1) / nck;
    for (int i0 = 0; i0 < n; i0 += rows) {
      const int i1 = i0 + rows < n ? i0 + rows : n;
      if (nc >= cap) {
        sgg::set_error("sgg_pool_plan: chunk table capacity %d exceeded", cap);
        return SGG_E_ARG;
      }
      chunks[4 * nc + 0] = s;
      chunks[4 * nc + 1] = i0;
      chunks[4 * nc + 2] = i1;
      chunks[4 * nc + 3] = gpw;
      if (i1 - i0 > mr) mr = i1 - i0;
      ++nc;
    }
  }
  *max_rows = mr;
  *gpw_out = gpw;
  return nc;
}

extern "C" int sgg_pool_plan_bf16(const int32_t* host_scene_off, int S, int bn, int target_chunks, int32_t* chunks,
                                  int cap, int* max_rows, int* gpw_out) {
  // host helper for pool_fwd_bf16_kernel: chunks of whole i-rows of up to a
  // pair budget Pb (the largest of 2048 .. 128 that still gives >= target_chunks
  // chunks: the j-block form stages a scene's U once per chunk, so the fewer,
  // larger chunks the better while every CU has one), rows spread evenly over
  // a scene's chunks; gpw = the 16-pair groups per wave that one pass of the
  // widest chunk needs (8 waves per workgroup)
  if (!host_scene_off || !chunks || !max_rows || !gpw_out || S < 0 || cap < 0 || !pool_bn_ok(bn)) {
    sgg::set_error("sgg_pool_plan_bf16: bad argument");
    return SGG_E_ARG;
  }
  auto rows_of = [&](int n, int pb) { const int r = pb / n; return r < 1 ? 1 : (r > n ? n : r); };
  int pb = 2048;
  for (; pb > 128; pb >>= 1) {
    long nc = 0;
    for (int s = 0; s < S; ++s) {
      const int n = host_scene_off[s + 1] - host_scene_off[s];
      if (n > 0) nc += (n + rows_of(n, pb) - 1) / rows_of(n, pb);
    }
    if (nc >= target_chunks) break;
  }
  int nc = 0, mr = 1, mp = 1;
  for (int s = 0; s < S; ++s) {
    const int n = host_scene_off[s + 1] - host_scene_off[s];
    if (n <= 0) continue;
    const int rmax = rows_of(n, pb), nck = (n + rmax - 1) / rmax, rows = (n + nck - 1) / nck;
    for (int i0 = 0; i0 < n; i0 += rows) {
      const int i1 = i0 + rows < n ? i0 + rows : n;
      if (nc >= cap) {
        sgg::set_error("sgg_pool_plan_bf16: chunk table capacity %d exceeded", cap);
        return SGG_E_ARG;
      }
      chunks[4 * nc + 0] = s;
      chunks[4 * nc + 1] = i0;
      chunks[4 * nc + 2] = i1;
      chunks[4 * nc + 3] = 0;
      if (i1 - i0 > mr) mr = i1 - i0;
      if ((i1 - i0) * n > mp) mp = (i1 - i0) * n;
      ++nc;
    }
  }
  // (register budget at two waves per SIMD: gpw <= 4, and <= 2 at bn 64 --
  // a chunk wider than one pass runs in several)
  const int gmax = bn > 48 ? 2 : 4;
  int gpw = 1;
  while (gpw < gmax && 16 * kBfWaves * gpw < mp) gpw <<= 1;
  for (int c = 0; c < nc; ++c) chunks[4 * c + 3] = gpw;
  *max_rows = mr;
  *gpw_out = gpw;
  return nc;
}

// the checks every forward entry makes on one batch
static int pool_batch_check(const char* fn, const float* U, const float* pos, const int32_t* scene_off,
                            const int32_t* chunks, int nchunks, int max_rows, int gpw, int B, int max_n,
                            const float* out, const int32_t* argmax) {
  SGG_CHECK_ARG(U && pos && scene_off && chunks && out && argmax, "%s: null pointer", fn);
  SGG_CHECK_ARG(nchunks >= 0 && B >= 0, "%s: bad sizes", fn);
  SGG_CHECK_ARG(max_n >= 1 && max_n <= SGG_POOL_MAX_PEDS, "%s: max scene size %d outside [1, %d]", fn, max_n,
                SGG_POOL_MAX_PEDS);
  SGG_CHECK_ARG(max_rows >= 1 && max_rows <= 64, "%s: chunk rows %d outside [1, 64]", fn, max_rows);
  SGG_CHECK_ARG(gpw == 1 || gpw == 2 || gpw == 4 || gpw == 8, "%s: gpw %d not in {1,2,4,8}", fn, gpw);
  return 0;
}

// one forward launch over one or two batches (nchunks: their total)
static int pool_fwd_sets(const PoolSet& s1, const PoolSet& s2, const float* A, const float* W2, const float* b2,
                         int max_rows, int max_n, int gpw, int bn, bool bf16, hipStream_t st) {
  if (s1.nchunks + (s2.chunks ? s2.nchunks : 0) == 0) return 0;
  if (bf16) {
    switch (bn) {
      case 8: return launch_fwd_bf16<8>(s1, s2, A, W2, b2, gpw, max_rows, max_n, st);
      case 16: return launch_fwd_bf16<16>(s1, s2, A, W2, b2, gpw, max_rows, max_n, st);
      case 32: return launch_fwd_bf16<32>(s1, s2, A, W2, b2, gpw, max_rows, max_n, st);
      case 48: return launch_fwd_bf16<48>(s1, s2, A, W2, b2, gpw, max_rows, max_n, st);
      default: return launch_fwd_bf16<64>(s1, s2, A, W2, b2, gpw, max_rows, max_n, st);
    }
  }
  switch (bn) {
    case 8: return launch_fwd<8>(s1, s2, A, W2, b2, max_rows, max_n, gpw, st);
    case 16: return launch_fwd<16>(s1, s2, A, W2, b2, max_rows, max_n, gpw, st);
    case 32: return launch_fwd<32>(s1, s2, A, W2, b2, max_rows, max_n, gpw, st);
    case 48: return launch_fwd<48>(s1, s2, A, W2, b2, max_rows, max_n, gpw, st);
    default: return launch_fwd<64>(s1, s2, A, W2, b2, max_rows, max_n, gpw, st);
  }
}

static int pool_fwd_one(const char* fn, bool bf16, const float* U, const float* pos, const float* A, const float* W2,
                        const float* b2, const int32_t* scene_off, const int32_t* chunks, int nchunks, int max_rows,
                        int gpw, int B, int bn, int max_n, float* out, int32_t* argmax, const int32_t* nchunks_dev,
                        void* stream) {
  SGG_CHECK_ARG(A && W2 && b2, "%s: null pointer", fn);
  SGG_CHECK_ARG(pool_bn_ok(bn), "%s: bottleneck %d not built (8/16/32/48/64)", fn, bn);
  const int rc = pool_batch_check(fn, U, pos, scene_off, chunks, nchunks, max_rows, gpw, B, max_n, out, argmax);
  if (rc != 0) return rc;
  const PoolSet s1 = {U, pos, scene_off, reinterpret_cast<const int4*>(chunks), nchunks, nchunks_dev, out, argmax};
  const PoolSet none = {};
  return pool_fwd_sets(s1, none, A, W2, b2, max_rows, max_n, gpw, bn, bf16, (hipStream_t)stream);
}

extern "C" int sgg_pool_fwd(const float* U, const float* pos, const float* A, const float* W2, const float* b2,
                            const int32_t* scene_off, const int32_t* chunks, int nchunks, int max_rows, int gpw,
                            int B, int bn, int max_n, float* out, int32_t* argmax, const int32_t* nchunks_dev,
                            void* stream) {
  return pool_fwd_one("sgg_pool_fwd", false, U, pos, A, W2, b2, scene_off, chunks, nchunks, max_rows, gpw, B, bn,
                      max_n, out, argmax, nchunks_dev, stream);
}

extern "C" int sgg_pool_fwd_bf16(const float* U, const float* pos, const float* A, const float* W2, const float* b2,
                                 const int32_t* scene_off, const int32_t* chunks, int nchunks, int max_rows, int gpw,
                                 int B, int bn, int max_n, float* out, int32_t* argmax, const int32_t* nchunks_dev,
                                 void* stream) {
  return pool_fwd_one("sgg_pool_fwd_bf16", true, U, pos, A, W2, b2, scene_off, chunks, nchunks, max_rows, gpw, B,
                      bn, max_n, out, argmax, nchunks_dev, stream);
}

extern "C" int sgg_pool_fwd2(const SggPoolBatch* a, const SggPoolBatch* b, const float* A, const float* W2,
                             const float* b2, int bn, int bf16, void* stream) {
  SGG_CHECK_ARG(a && b && A && W2 && b2, "sgg_pool_fwd2: null pointer");
  SGG_CHECK_ARG(pool_bn_ok(bn), "sgg_pool_fwd2: bottleneck %d not built (8/16/32/48/64)", bn);
  for (const SggPoolBatch* p : {a, b}) {
    const int rc = pool_batch_check("sgg_pool_fwd2", p->U, p->pos, p->scene_off, p->chunks, p->nchunks, p->max_rows,
                                    p->gpw, p->B, p->max_n, p->out, p->argmax);
    if (rc != 0) return rc;
  }
  // one kernel instance (its pair groups per wave) serves both batches
  SGG_CHECK_ARG(a->gpw == b->gpw, "sgg_pool_fwd2: the batches' plans differ in gpw (%d, %d)", a->gpw, b->gpw);
  const PoolSet s1 = {a->U, a->pos, a->scene_off, reinterpret_cast<const int4*>(a->chunks), a->nchunks,
                      a->nchunks_dev, a->out, a->argmax};
  const PoolSet s2 = {b->U, b->pos, b->scene_off, reinterpret_cast<const int4*>(b->chunks), b->nchunks,
                      b->nchunks_dev, b->out, b->argmax};
  const int mr = a->max_rows > b->max_rows ? a->max_rows : b->max_rows;
  const int mn = a->max_n > b->max_n ? a->max_n : b->max_n;
  return pool_fwd_sets(s1, s2, A, W2, b2, mr, mn, a->gpw, bn, bf16 != 0, (hipStream_t)stream);
}

extern "C" int sgg_pool_bwd_grid(int S) {
  if (S < 1) return 1;
  const long long u = (long long)S * pool_bwd_jq(S);
  return (int)(u < 256 ? u : 256);
}

extern "C" int sgg_pool_bwd(const float* U, const float* pos, const float* A, const float* W2, const float* out,
                            const int32_t* argmax, const float* dout, const int32_t* scene_off, int S, int B,
                            int bn, int max_n, float* dU, float* part, void* stream) {
  SGG_CHECK_ARG(U && pos && A && W2 && out && argmax && dout && scene_off && dU, "sgg_pool_bwd: null pointer");
  SGG_CHECK_ARG(pool_bn_ok(bn), "sgg_pool_bwd: bottleneck %d not built", bn);
  SGG_CHECK_ARG(max_n >= 1 && max_n <= SGG_POOL_MAX_PEDS, "sgg_pool_bwd: max scene size %d outside [1, %d]",
                max_n, SGG_POOL_MAX_PEDS);
  SGG_CHECK_ARG(S >= 0 && B >= 0, "sgg_pool_bwd: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (S == 0) return 0;
  switch (bn) {
    case 8: return launch_bwd<8>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, part, st);
    case 16: return launch_bwd<16>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, part, st);
    case 32: return launch_bwd<32>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, part, st);
    case 48: return launch_bwd<48>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, part, st);
    default: return launch_bwd<64>(U, pos, A, W2, out, argmax, dout, scene_off, S, max_n, dU, part, st);
  }
}
