// The whole GCNModule of a scene in one workgroup (reference
// sgan/models.py:628-712 with GCN.forward :573-580 and normalize :607-613),
// forward and backward.
//
// Per scene (n <= 64 peds):
//   groups     M_ij = (i == j) | (lab_i == lab_j != 0) on the last-observed
//              labels (:651-657); group g(i) = i's first member
//   gcn_intra  H <- ReLU((A H) W_l), l = 0, 1 with A = D^-1 M (:661-665).
//              A averages a row's group, so after the first aggregation the
//              rows of a group are equal: the two layers run on the G group
//              rows only -- Xb = group mean of X, H1 = ReLU(Xb W0) (fin -> 72),
//              H2 = ReLU(H1 W1) (72 -> 16); ped i's intra row is H2[g(i)]
//   pool       gin = R intra, R the row-normalised distinct rows of M
//              (:667-686): gin_g = H2[g]
//   gcn_inter  the same GCN (16 -> 72 -> 16) with A = 1/G on the complete
//              group graph (:688-694): every group row is m = mean_g gin_g
//              after the first aggregation, so G1 = ReLU(m W0'), G2 = ReLU(G1 W1')
//   un-pool    inter_i = G2 / |g(i)|  (R^T with R normalised, :700)
//   out        out_embedding([intra_i, inter_i])                (:703-708)
//
// The node transforms run on the MFMA (v_mfma_f32_16x16x4f32; with bf16 set,
// bf16 operands on v_mfma_f32_16x16x32_bf16 with fp32 accumulation -- the
// "bf16 + MFMA XW" of BASELINE configs 3 / 5), group structure by one wave
// (ballot / shuffles), everything else in LDS.  The backward recomputes the
// forward (a few hundred kFLOP per scene) and back-propagates in the same
// workgroup; the parameter gradients of the workgroup's scenes accumulate in
// its own row of a slab (fixed tile -> lane ownership: deterministic) that
// sgg_slab_reduce sums in row order.
#include "sgg_common.h"

// phase timestamps of workgroup 0's first scene (tools/gcnmod_probe.hip)
#ifdef SGG_GCN_PROF
__device__ long long g_gcn_prof[64];
#define CPMARK(i) \
  if (threadIdx.x == 0 && blockIdx.x == 0 && first) g_gcn_prof[i] = wall_clock64();
#else
#define CPMARK(i)
#endif

namespace sgg {

namespace {

constexpr int kThreads = 256, kWaves = kThreads / kWave;
constexpr int FH = 72, FO = 16, FC = 2 * FO;   // GCN hidden / out width (GCNModule(hidden 72, out 16)), [intra | inter]
constexpr int PH = FH + 1, PO = FO + 1, PC = FC + 1;
constexpr int kMaxPeds = 64;                   // one wavefront holds a scene's group structure
constexpr int kMaxIn = 64, kMaxOut = 64;
constexpr int kFwdGridCap = 65536, kBwdGridCap = 512;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__host__ __device__ inline int odd(int n) { return n | 1; }

// LDS plan (float offsets) for scenes of at most np peds
struct Geo {
  int PX, PE;                                   // pitches of the fin- / fe-wide rows
  int grp, gl, goff, gcnt, mem, Mv;             // int arrays (np each), M
  int inv;                                      // 1 / |g| per group
  int Xb, H1, H2;                               // group rows
  int vm, vG1, vG2, vT, vD2, vE1, vdg;          // per-scene vectors (16 / 72)
  int W0i, W1i, W0g, W1g, Woe, boe;             // weights, staged once per workgroup
  int dY, dcat, Sg, Eg;                         // backward
  int total;
};

__host__ __device__ inline Geo make_geo(int np, int fin, int fe, bool bwd) {
  Geo L;
  L.PX = odd(fin);
  L.PE = odd(fe);
  int o = 0;
  auto take = [&](int n) { const int r = o; o += (n + 3) & ~3; return r; };
  L.grp = take(np); L.gl = take(np); L.goff = take(np); L.gcnt = take(np); L.mem = take(np); L.Mv = take(1);
  L.inv = take(np);
  L.Xb = take(np * L.PX);
  L.H1 = take(np * PH);
  L.H2 = take(np * PO);
  L.vm = take(FO); L.vG1 = take(FH); L.vG2 = take(FO); L.vT = take(FO); L.vD2 = take(FO); L.vE1 = take(FH);
  L.vdg = take(FO);
  L.W0i = take(fin * PH);
  L.W1i = take(FH * PO);
  L.W0g = take(FO * PH);
  L.W1g = take(FH * PO);
  L.Woe = take(fe * PC);
  L.boe = take(fe);
  if (bwd) {
    L.dY = take(np * L.PE);
    L.dcat = take(np * PC);
    L.Sg = take(np * PO);
    L.Eg = take(np * PH);
  } else {
    L.dY = L.dcat = L.Sg = L.Eg = 0;
  }
  L.total = o;
  return L;
}

// parameter-gradient slab row: the module's parameters in registration order
// (gcn_intra.W.0, gcn_intra.W.1, gcn_inter.W.0, gcn_inter.W.1,
// out_embedding.weight, out_embedding.bias)
struct PLay {
  int W0i, W1i, W0g, W1g, Woe, boe, total;
};
__host__ __device__ inline PLay make_play(int fin, int fe) {
  PLay P;
  int o = 0;
  P.W0i = o; o += fin * FH;
  P.W1i = o; o += FH * FO;
  P.W0g = o; o += FO * FH;
  P.W1g = o; o += FH * FO;
  P.Woe = o; o += fe * FC;
  P.boe = o; o += fe;
  P.total = o;
  return P;
}

__device__ __forceinline__ float bf16r(float x) { return (float)(__bf16)x; }   // round to nearest even
__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// LDS exchange inside one wavefront (release / acquire at wavefront scope)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One 16 x 16 tile of C = A B: A(r, k) for rows r0 + (lane & 15), B(k, c) for
// columns c0 + (lane & 15), reduction over k < K (the accessors clamp rows /
// columns past the edge; k >= K meets a zero A element).  fp32:
// v_mfma_f32_16x16x4f32, lane holds A[i][k0 + lane >> 4]; BF: bf16 operands,
// v_mfma_f32_16x16x32_bf16, lane holds A[i][k0 + 8 (lane >> 4) + j], j < 8.
// D lane: rows r0 + 4 (lane >> 4) + r, column c0 + (lane & 15).
template <bool BF, class FA, class FB>
__device__ __forceinline__ floatx4 tile(int r0, int c0, int K, FA fa, FB fb) {
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if constexpr (BF) {
    for (int k0 = 0; k0 < K; k0 += 32) {
      bf16x8 a, b;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = k0 + 8 * kq + j;
        const bool ok = k < K;
        const int kc = ok ? k : K - 1;
        a[j] = (__bf16)keep_if(fa(r0 + i, kc), ok);
        b[j] = (__bf16)fb(kc, c0 + i);
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
  } else {
    for (int k0 = 0; k0 < K; k0 += 4) {
      const int k = k0 + kq;
      const bool ok = k < K;
      const int kc = ok ? k : K - 1;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(keep_if(fa(r0 + i, kc), ok), fb(kc, c0 + i), acc, 0, 0, 0);
    }
  }
  return acc;
}

// C (rows x N) = A B over K on waves [w0, w0 + nw) of the workgroup, tiles
// dealt round-robin; epi(row, col, value) stores each element
template <bool BF, class FA, class FB, class FE>
__device__ __forceinline__ void mm(int rows, int N, int K, int w0, int nw, FA fa, FB fb, FE epi) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
  if (wave < w0 || wave >= w0 + nw) return;
  const int ct = (N + 15) >> 4, nt = ((rows + 15) >> 4) * ct;
  for (int t = wave - w0; t < nt; t += nw) {
    const int r0 = (t / ct) << 4, c0 = (t % ct) << 4;
    const floatx4 acc = tile<BF>(r0, c0, K, fa, fb);
    const int c = c0 + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + 4 * kq + r;
      if (row < rows && c < N) epi(row, c, acc[r]);
    }
  }
}

struct Scene {
  int p0, n, M;
};

// Group structure of the scene by wavefront 0 (lane = ped, n <= 64): leader
// (first member), group rank = rank of the leader, member count, the member
// CSR in group order; writes grp / gl / goff / gcnt / mem / inv / M.
__device__ void groups(const float* __restrict__ labels, int p0, int n, float* lds, const Geo& L) {
  int* grp = (int*)(lds + L.grp);
  int* gl = (int*)(lds + L.gl);
  int* goff = (int*)(lds + L.goff);
  int* gcnt = (int*)(lds + L.gcnt);
  int* mem = (int*)(lds + L.mem);
  float* inv = lds + L.inv;
  const int lane = threadIdx.x & 63;
  const bool act = lane < n;
  const float li = act ? labels[p0 + lane] : 0.f;
  int l = lane;
  // (j is uniform: readlane, a VALU read, instead of a shuffle's LDS round trip)
  for (int j = 0; j < n; ++j) {   // the first member with the same nonzero label (:651-657)
    const float lj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(li), j));
    if (j < lane && l == lane && li != 0.f && lj == li) l = j;
  }
  const bool lead = act && l == lane;
  const unsigned long long lm = __ballot(lead);
  const int rank = __popcll(lm & ((1ull << lane) - 1ull));
  int cnt = 0, before = 0;
  for (int j = 0; j < n; ++j) {
    const int lj = __builtin_amdgcn_readlane(l, j);
    cnt += lj == lane;
    before += (j < lane) & (lj == l);
  }
  int v = lead ? cnt : 0;   // inclusive scan of the leaders' counts (leader order == rank order)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  const int excl = v - (lead ? cnt : 0);
  const int g = __shfl(rank, l), off = __shfl(excl, l);
  if (act) {
    grp[lane] = g;
    mem[off + before] = lane;
    if (lead) {
      gl[rank] = lane;
      goff[rank] = excl;
      gcnt[rank] = cnt;
      inv[rank] = 1.f / (float)cnt;   // normalize(): row sum ^ -1 (:607-613)
    }
  }
  if (lane == 0) ((int*)(lds + L.Mv))[0] = __popcll(lm);
}

// Xb[g][c] = (sum over g's members of X[p][c]) / |g|   (A X on the group rows).
// The scene's X rows are first staged in the H1 region (free until
// intra_fwd_h1) with 16 loads in flight per thread -- a member walk over
// global rows waits a memory latency per load -- then summed from LDS.
__device__ void group_mean_x(const SggGcnModArgs& a, int p0, int n, int M, float* lds, const Geo& L) {
  const int* goff = (const int*)(lds + L.goff);
  const int* gcnt = (const int*)(lds + L.gcnt);
  const int* mem = (const int*)(lds + L.mem);
  const float* inv = lds + L.inv;
  float* Xb = lds + L.Xb;
  const int fin = a.fin;
  if (L.PX <= PH) {
    float* Xs = lds + L.H1;   // n x fin at pitch PX (n PX <= np PH)
    constexpr int kU = 16;
    const int tot = n * fin;
    for (int base = 0; base < tot; base += kU * kThreads) {
      float v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = min(base + u * kThreads + (int)threadIdx.x, tot - 1);
        const int r = e / fin, c = e - r * fin;
        const bool second = a.X2 && c >= a.kx1;
        v[u] = second ? a.X2[(size_t)(p0 + r) * a.ldx2 + (c - a.kx1)] : a.X[(size_t)(p0 + r) * a.ldx + c];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = base + u * kThreads + (int)threadIdx.x;
        if (e < tot) {
          const int r = e / fin, c = e - r * fin;
          Xs[r * L.PX + c] = v[u];
        }
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < M * fin; e += blockDim.x) {
      const int g = e / fin, c = e - g * fin;
      float s = 0.f;
      for (int q = goff[g], qe = q + gcnt[g]; q < qe; ++q) s += Xs[mem[q] * L.PX + c];
      Xb[g * L.PX + c] = s * inv[g];
    }
    return;
  }
  for (int e = threadIdx.x; e < M * fin; e += blockDim.x) {
    const int g = e / fin, c = e - g * fin;
    const bool second = a.X2 && c >= a.kx1;
    const float* src = second ? a.X2 + (c - a.kx1) : a.X + c;
    const int ld = second ? a.ldx2 : a.ldx;
    float s = 0.f;
    for (int q = goff[g], qe = q + gcnt[g]; q < qe; ++q) s += src[(size_t)(p0 + mem[q]) * ld];
    Xb[g * L.PX + c] = s * inv[g];
  }
}

// Forward of the intra GCN on the group rows: H1 = ReLU(Xb W0), then H2 = ReLU(H1 W1)
template <bool BF>
__device__ void intra_fwd_h1(int M, int fin, float* lds, const Geo& L) {
  const float* Xb = lds + L.Xb;
  const float* W = lds + L.W0i;
  float* H1 = lds + L.H1;
  mm<BF>(M, FH, fin, 0, kWaves, [&](int r, int k) { return Xb[min(r, M - 1) * L.PX + k]; },
         [&](int k, int c) { return W[k * PH + min(c, FH - 1)]; },
         [&](int r, int c, float v) { H1[r * PH + c] = relu(v); });
}
template <bool BF>
__device__ void intra_fwd_h2(int M, float* lds, const Geo& L) {
  const float* H1 = lds + L.H1;
  const float* W = lds + L.W1i;
  float* H2 = lds + L.H2;
  mm<BF>(M, FO, FH, 0, kWaves, [&](int r, int k) { return H1[min(r, M - 1) * PH + k]; },
         [&](int k, int c) { return W[k * PO + c]; }, [&](int r, int c, float v) { H2[r * PO + c] = relu(v); });
}

// The inter GCN (wavefront 0): m = mean over groups of gin (= H2), G1 =
// ReLU(m W0'), G2 = ReLU(G1 W1')
template <bool BF>
__device__ void inter_fwd(int M, float* lds, const Geo& L) {
  const int lane = threadIdx.x & 63;
  const float* H2 = lds + L.H2;
  const float* W0g = lds + L.W0g;
  const float* W1g = lds + L.W1g;
  float* m = lds + L.vm;
  float* G1 = lds + L.vG1;
  float* G2 = lds + L.vG2;
  const float iM = 1.f / (float)M;
  auto q = [](float x) { return BF ? bf16r(x) : x; };
  if (lane < FO) {
    float s = 0.f;
    for (int g = 0; g < M; ++g) s += H2[g * PO + lane];
    m[lane] = s * iM;
  }
  wave_sync();
  for (int k = lane; k < FH; k += 64) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < FO; ++c) s += q(m[c]) * q(W0g[c * PH + k]);
    G1[k] = relu(s);
  }
  wave_sync();
  if (lane < FO) {
    float s = 0.f;
    for (int k = 0; k < FH; ++k) s += q(G1[k]) * q(W1g[k * PO + lane]);
    G2[lane] = relu(s);
  }
}

// [intra_i | inter_i] = [H2[g(i)] | G2 / |g(i)|]
__device__ __forceinline__ float cat_at(const float* lds, const Geo& L, int i, int c) {
  const int g = ((const int*)(lds + L.grp))[i];
  return c < FO ? lds[L.H2 + g * PO + c] : lds[L.vG2 + c - FO] * lds[L.inv + g];
}

// the module's six weight arrays into LDS as one virtual concatenation, 16
// loads in flight per thread (one load + one store per trip would wait a
// memory latency per element)
template <bool BF>
__device__ void stage_weights(const SggGcnModArgs& a, float* lds, const Geo& L) {
  const int n0 = a.fin * FH, n1 = n0 + FH * FO, n2 = n1 + FO * FH, n3 = n2 + FH * FO, n4 = n3 + a.fe * FC,
            tot = n4 + a.fe;
  auto where = [&](int e, const float*& src, int& le, int& cols, int& dst, int& pitch) {
    if (e < n0) { src = a.W0i; le = e; cols = FH; dst = L.W0i; pitch = PH; }
    else if (e < n1) { src = a.W1i; le = e - n0; cols = FO; dst = L.W1i; pitch = PO; }
    else if (e < n2) { src = a.W0g; le = e - n1; cols = FH; dst = L.W0g; pitch = PH; }
    else if (e < n3) { src = a.W1g; le = e - n2; cols = FO; dst = L.W1g; pitch = PO; }
    else if (e < n4) { src = a.Woe; le = e - n3; cols = FC; dst = L.Woe; pitch = PC; }
    else { src = a.boe; le = e - n4; cols = a.fe; dst = L.boe; pitch = 0; }
  };
  constexpr int kU = 16;
  for (int base = 0; base < tot; base += kU * kThreads) {
    float v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int e = min(base + u * kThreads + (int)threadIdx.x, tot - 1);
      const float* src;
      int le, cols, dst, pitch;
      where(e, src, le, cols, dst, pitch);
      v[u] = src[le];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int e = base + u * kThreads + (int)threadIdx.x;
      if (e < tot) {
        const float* src;
        int le, cols, dst, pitch;
        where(e, src, le, cols, dst, pitch);
        const int r = le / cols, c = le - r * cols;
        lds[dst + r * pitch + c] = v[u];
      }
    }
  }
}

// the per-batch fields of a forward: batch a's, or (two) the second batch's
// of sgg_gcnmod_fwd2 -- per-field uniform selects (weights, np, fin, fe, bf16
// are shared)
__device__ __forceinline__ SggGcnModArgs pick_batch(const SggGcnModArgs& a, const SggGcnModArgs& b, bool two) {
  SggGcnModArgs q = a;
  q.X = two ? b.X : a.X;
  q.ldx = two ? b.ldx : a.ldx;
  q.X2 = two ? b.X2 : a.X2;
  q.ldx2 = two ? b.ldx2 : a.ldx2;
  q.kx1 = two ? b.kx1 : a.kx1;
  q.labels = two ? b.labels : a.labels;
  q.scene_off = two ? b.scene_off : a.scene_off;
  q.S = two ? b.S : a.S;
  q.y = two ? b.y : a.y;
  q.ldy = two ? b.ldy : a.ldy;
  return q;
}

template <bool BF>
__global__ void __launch_bounds__(kThreads) gcnmod_fwd_kernel(const SggGcnModArgs a1, const SggGcnModArgs a2,
                                                              int S2) {
  extern __shared__ float lds[];
  const Geo L = make_geo(a1.np, a1.fin, a1.fe, false);
  stage_weights<BF>(a1, lds, L);
  for (int vs = blockIdx.x; vs < a1.S + S2; vs += gridDim.x) {
    const bool two = vs >= a1.S;   // uniform
    const SggGcnModArgs a = pick_batch(a1, a2, two);
    const int s = two ? vs - a1.S : vs;
    const int p0 = a.scene_off[s], n = a.scene_off[s + 1] - p0;
    if (n <= 0) continue;
    if (threadIdx.x < 64) groups(a.labels, p0, n, lds, L);
    __syncthreads();
    const int M = ((const int*)(lds + L.Mv))[0];
    group_mean_x(a, p0, n, M, lds, L);
    __syncthreads();
    intra_fwd_h1<BF>(M, a.fin, lds, L);
    __syncthreads();
    intra_fwd_h2<BF>(M, lds, L);
    __syncthreads();
    if (threadIdx.x < 64) inter_fwd<BF>(M, lds, L);
    __syncthreads();
    // y = [intra | inter] Woe^T + b
    const float* Woe = lds + L.Woe;
    const float* boe = lds + L.boe;
    mm<BF>(n, a.fe, FC, 0, kWaves, [&](int r, int k) { return cat_at(lds, L, min(r, n - 1), k); },
           [&](int k, int c) { return Woe[min(c, a.fe - 1) * PC + k]; },
           [&](int r, int c, float v) { a.y[(size_t)(p0 + r) * a.ldy + c] = v + boe[c]; });
    __syncthreads();
  }
}

template <bool BF>
__global__ void __launch_bounds__(kThreads) gcnmod_bwd_kernel(const SggGcnModArgs a) {
  extern __shared__ float lds[];
  const Geo L = make_geo(a.np, a.fin, a.fe, true);
  const PLay P = make_play(a.fin, a.fe);
  float* slab = a.slab + (size_t)blockIdx.x * P.total;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fin = a.fin, fe = a.fe;
#ifdef SGG_GCN_PROF
  if (threadIdx.x == 0 && blockIdx.x == 0) g_gcn_prof[0] = wall_clock64();
#endif
  stage_weights<BF>(a, lds, L);
  bool first = true;   // the workgroup's first scene writes its slab row, later ones add
  auto acc = [&](int off, float v) { float* p = slab + off; *p = first ? v : *p + v; };
  const int copies = a.dy_copies > 1 ? a.dy_copies : 1;
  CPMARK(1);
  for (int s = blockIdx.x; s < a.S; s += gridDim.x) {
    const int p0 = a.scene_off[s], n = a.scene_off[s + 1] - p0;
    if (n <= 0) continue;
    const int* grp = (const int*)(lds + L.grp);
    const int* goff = (const int*)(lds + L.goff);
    const int* gcnt = (const int*)(lds + L.gcnt);
    const int* mem = (const int*)(lds + L.mem);
    const float* inv = lds + L.inv;
    float* dY = lds + L.dY;
    float* dcat = lds + L.dcat;
    // -- recompute the forward; dY (the copies summed) to LDS
    if (wave == 0) {
      groups(a.labels, p0, n, lds, L);
    } else {
      // 8 elements per thread in flight, one copy at a time (the copies
      // summed in order, as one element at a time did)
      constexpr int kU = 8;
      const int tot = n * fe, nt = kThreads - 64, t = threadIdx.x - 64;
      for (int base = 0; base < tot; base += kU * nt) {
        const float* src[kU];
        float v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int e = min(base + u * nt + t, tot - 1);
          const int r = e / fe, c = e - r * fe;
          src[u] = a.dy + (size_t)(p0 + r) * a.lddy + c;
          v[u] = src[u][0];
        }
        for (int k = 1; k < copies; ++k) {
#pragma unroll
          for (int u = 0; u < kU; ++u) v[u] += src[u][(size_t)k * a.dy_cstride];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int e = base + u * nt + t;
          if (e < tot) {
            const int r = e / fe, c = e - r * fe;
            dY[r * L.PE + c] = v[u];
          }
        }
      }
    }
    __syncthreads();
    CPMARK(2);
    const int M = ((const int*)(lds + L.Mv))[0];
    group_mean_x(a, p0, n, M, lds, L);
    __syncthreads();
    CPMARK(3);
    intra_fwd_h1<BF>(M, fin, lds, L);
    __syncthreads();
    intra_fwd_h2<BF>(M, lds, L);
    __syncthreads();
    CPMARK(4);
    // wave 0: the inter GCN; waves 1..3: dcat = dY Woe
    const float* Woe = lds + L.Woe;
    if (wave == 0) inter_fwd<BF>(M, lds, L);
    mm<false>(n, FC, fe, 1, kWaves - 1, [&](int r, int k) { return dY[min(r, n - 1) * L.PE + k]; },
              [&](int k, int c) { return Woe[k * PC + c]; }, [&](int r, int c, float v) { dcat[r * PC + c] = v; });
    __syncthreads();
    CPMARK(5);
    const float* H1 = lds + L.H1;
    const float* H2 = lds + L.H2;
    const float* Xb = lds + L.Xb;
    const float* G1 = lds + L.vG1;
    const float* G2 = lds + L.vG2;
    const float* m = lds + L.vm;
    float* T = lds + L.vT;
    float* D2 = lds + L.vD2;
    float* E1 = lds + L.vE1;
    float* dgin = lds + L.vdg;
    float* Sg = lds + L.Sg;
    if (wave == 0) {
      // inter GCN backward on the scene vector: T = sum_i dinter_i / |g(i)|
      // (R^T), D2 = T [G2 > 0], E1 = (D2 W1'^T) [G1 > 0], dgin = E1 W0'^T / G
      if (lane < FO) {
        float t = 0.f;
        for (int i = 0; i < n; ++i) t += dcat[i * PC + FO + lane] * inv[grp[i]];
        T[lane] = t;
        D2[lane] = G2[lane] > 0.f ? t : 0.f;
      }
      wave_sync();
      const float* W1g = lds + L.W1g;
      for (int k = lane; k < FH; k += 64) {
        float e = 0.f;
#pragma unroll
        for (int c = 0; c < FO; ++c) e += D2[c] * W1g[k * PO + c];
        E1[k] = G1[k] > 0.f ? e : 0.f;
      }
      wave_sync();
      const float* W0g = lds + L.W0g;
      if (lane < FO) {
        float d = 0.f;
        for (int k = 0; k < FH; ++k) d += E1[k] * W0g[lane * PH + k];
        dgin[lane] = d * (1.f / (float)M);
      }
    } else {
      // out_embedding: dWoe += dY^T [intra | inter], dboe += column sums of dY
      mm<false>(fe, FC, n, 1, kWaves - 1, [&](int o, int r) { return dY[r * L.PE + min(o, fe - 1)]; },
                [&](int r, int c) { return cat_at(lds, L, r, min(c, FC - 1)); },
                [&](int o, int c, float v) { acc(P.Woe + o * FC + c, v); });
      for (int e = threadIdx.x - 64; e < fe + M * FO; e += blockDim.x - 64) {
        if (e < fe) {
          float b = 0.f;
          for (int i = 0; i < n; ++i) b += dY[i * L.PE + e];
          acc(P.boe + e, b);
        } else {   // Sg[g] = sum over g's members of dintra
          const int g = (e - fe) / FO, c = (e - fe) - g * FO;
          float v = 0.f;
          for (int q = goff[g], qe = q + gcnt[g]; q < qe; ++q) v += dcat[mem[q] * PC + c];
          Sg[g * PO + c] = v;
        }
      }
    }
    __syncthreads();
    CPMARK(6);
    // Dg = (Sg + dgin) [H2 > 0] (each member's dintra plus its share of
    // dgin, summed over the group); dW1' += G1 (x) D2; dW0' += m (x) E1
    for (int e = threadIdx.x; e < M * FO + 2 * FH * FO; e += blockDim.x) {
      if (e < M * FO) {
        const int g = e / FO, c = e - g * FO;
        Sg[g * PO + c] = H2[g * PO + c] > 0.f ? Sg[g * PO + c] + dgin[c] : 0.f;
      } else if (e < M * FO + FH * FO) {
        const int q = e - M * FO, k = q / FO, c = q - k * FO;
        acc(P.W1g + q, G1[k] * D2[c]);
      } else {
        const int q = e - M * FO - FH * FO, c = q / FH, k = q - c * FH;
        acc(P.W0g + q, m[c] * E1[k]);
      }
    }
    __syncthreads();
    CPMARK(7);
    // intra layer 2: dW1 += H1^T Dg; Eg = (Dg W1^T) [H1 > 0]
    float* Eg = lds + L.Eg;
    const float* W1i = lds + L.W1i;
    mm<false>(FH, FO, M, 0, 2, [&](int k, int g) { return H1[g * PH + min(k, FH - 1)]; },
              [&](int g, int c) { return Sg[g * PO + c]; }, [&](int k, int c, float v) { acc(P.W1i + k * FO + c, v); });
    mm<false>(M, FH, FO, 2, 2, [&](int g, int c) { return Sg[min(g, M - 1) * PO + c]; },
              [&](int c, int k) { return W1i[min(k, FH - 1) * PO + c]; },
              [&](int g, int k, float v) { Eg[g * PH + k] = H1[g * PH + k] > 0.f ? v : 0.f; });
    __syncthreads();
    CPMARK(8);
    // intra layer 1: dW0 += Xb^T Eg; dX_p = (Eg W0^T)[g(p)] / |g(p)| for every member p
    const float* W0i = lds + L.W0i;
    mm<false>(fin, FH, M, 0, 2, [&](int k, int g) { return Xb[g * L.PX + min(k, fin - 1)]; },
              [&](int g, int c) { return Eg[g * PH + min(c, FH - 1)]; },
              [&](int k, int c, float v) { acc(P.W0i + k * FH + c, v); });
    mm<false>(M, fin, FH, 2, 2, [&](int g, int k) { return Eg[min(g, M - 1) * PH + k]; },
              [&](int k, int c) { return W0i[min(c, fin - 1) * PH + k]; },
              [&](int g, int c, float v) {
                const float d = v * inv[g];
                const bool second = a.dX2 && c >= a.kx1;
                float* dst = second ? a.dX2 + (c - a.kx1) : a.dX + c;
                const int ld = second ? a.lddx2 : a.lddx;
                for (int q = goff[g], qe = q + gcnt[g]; q < qe; ++q) dst[(size_t)(p0 + mem[q]) * ld] = d;
              });
    __syncthreads();
    CPMARK(9);
    first = false;
  }
  if (first) {   // no non-empty scene: the row still enters the sum
    for (int e = threadIdx.x; e < P.total; e += blockDim.x) slab[e] = 0.f;
  }
}

int gcnmod_check(const char* who, const SggGcnModArgs* a, int bwd) {
  SGG_CHECK_ARG(a, "%s: null args", who);
  SGG_CHECK_ARG(a->S >= 0 && a->scene_off && a->labels && a->X, "%s: null input", who);
  SGG_CHECK_ARG(a->np >= 1 && a->np <= kMaxPeds, "%s: np = %d (1 .. %d peds per scene)", who, a->np, kMaxPeds);
  SGG_CHECK_ARG(a->fin >= 1 && a->fin <= kMaxIn && a->fe >= 1 && a->fe <= kMaxOut, "%s: fin = %d, fe = %d", who,
                a->fin, a->fe);
  SGG_CHECK_ARG(a->W0i && a->W1i && a->W0g && a->W1g && a->Woe && a->boe, "%s: null weight", who);
  SGG_CHECK_ARG(!a->X2 || (a->kx1 >= 1 && a->kx1 < a->fin), "%s: kx1 = %d", who, a->kx1);
  SGG_CHECK_ARG(a->ldx >= (a->X2 ? a->kx1 : a->fin), "%s: ldx = %d", who, a->ldx);
  if (!bwd) {
    SGG_CHECK_ARG(a->y && a->ldy >= a->fe, "%s: y / ldy", who);
  } else {
    SGG_CHECK_ARG(a->dy && a->lddy >= a->fe && a->dX && a->slab, "%s: dy / dX / slab", who);
    SGG_CHECK_ARG(a->lddx >= (a->X2 ? a->kx1 : a->fin), "%s: lddx = %d", who, a->lddx);
    SGG_CHECK_ARG(!a->X2 || (a->dX2 && a->lddx2 >= a->fin - a->kx1), "%s: dX2 / lddx2", who);
  }
  return 0;
}

}  // namespace

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_gcnmod_param_size(int fin, int fe) {
  if (fin < 1 || fin > kMaxIn || fe < 1 || fe > kMaxOut) return -1;
  return make_play(fin, fe).total;
}

extern "C" int sgg_gcnmod_slab_rows(int S) { return S < 1 ? 1 : (S < kBwdGridCap ? S : kBwdGridCap); }

extern "C" long long sgg_gcnmod_lds_bytes(int max_n, int fin, int fe, int bwd) {
  if (max_n < 1 || max_n > kMaxPeds || fin < 1 || fin > kMaxIn || fe < 1 || fe > kMaxOut) return -1;
  return 4ll * make_geo(max_n, fin, fe, bwd != 0).total;
}

extern "C" int sgg_gcnmod_fwd(const SggGcnModArgs* a, void* stream) {
  const int rc = gcnmod_check("sgg_gcnmod_fwd", a, 0);
  if (rc) return rc;
  if (a->S == 0) return 0;
  const size_t lds = 4 * (size_t)make_geo(a->np, a->fin, a->fe, false).total;
  const dim3 grid(a->S < kFwdGridCap ? a->S : kFwdGridCap);
  if (a->bf16)
    hipLaunchKernelGGL(gcnmod_fwd_kernel<true>, grid, dim3(kThreads), lds, (hipStream_t)stream, *a, *a, 0);
  else
    hipLaunchKernelGGL(gcnmod_fwd_kernel<false>, grid, dim3(kThreads), lds, (hipStream_t)stream, *a, *a, 0);
  SGG_RETURN_LAUNCH("sgg_gcnmod_fwd");
}

extern "C" int sgg_gcnmod_fwd2(const SggGcnModArgs* a, const SggGcnModArgs* b, void* stream) {
  if (int rc = gcnmod_check("sgg_gcnmod_fwd2 (a)", a, 0)) return rc;
  if (int rc = gcnmod_check("sgg_gcnmod_fwd2 (b)", b, 0)) return rc;
  SGG_CHECK_ARG(a->np == b->np && a->fin == b->fin && a->fe == b->fe && a->bf16 == b->bf16 && a->W0i == b->W0i &&
                    a->W1i == b->W1i && a->W0g == b->W0g && a->W1g == b->W1g && a->Woe == b->Woe && a->boe == b->boe,
                "sgg_gcnmod_fwd2: the two batches must share the weights, np, fin, fe and precision");
  const int S = a->S + b->S;
  if (S == 0) return 0;
  const size_t lds = 4 * (size_t)make_geo(a->np, a->fin, a->fe, false).total;
  const dim3 grid(S < kFwdGridCap ? S : kFwdGridCap);
  if (a->bf16)
    hipLaunchKernelGGL(gcnmod_fwd_kernel<true>, grid, dim3(kThreads), lds, (hipStream_t)stream, *a, *b, b->S);
  else
    hipLaunchKernelGGL(gcnmod_fwd_kernel<false>, grid, dim3(kThreads), lds, (hipStream_t)stream, *a, *b, b->S);
  SGG_RETURN_LAUNCH("sgg_gcnmod_fwd2");
}

extern "C" int sgg_gcnmod_bwd(const SggGcnModArgs* a, void* stream) {
  const int rc = gcnmod_check("sgg_gcnmod_bwd", a, 1);
  if (rc) return rc;
  if (a->S == 0) return 0;
  const size_t lds = 4 * (size_t)make_geo(a->np, a->fin, a->fe, true).total;
  const dim3 grid(sgg_gcnmod_slab_rows(a->S));
  if (a->bf16)
    hipLaunchKernelGGL(gcnmod_bwd_kernel<true>, grid, dim3(kThreads), lds, (hipStream_t)stream, *a);
  else
    hipLaunchKernelGGL(gcnmod_bwd_kernel<false>, grid, dim3(kThreads), lds, (hipStream_t)stream, *a);
  SGG_RETURN_LAUNCH("sgg_gcnmod_bwd");
}
