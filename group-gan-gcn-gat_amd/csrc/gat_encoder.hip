// The whole group GAT encoder of a scene in one workgroup (GATEncoder,
// reference sgan/models.py:254-294, with GAT :222-237 and
// GraphAttentionLayer :184-220), forward and backward.
//
// Per scene (n <= 64 peds, the workgroup's LDS holds everything):
//   groups      M_ij = (i == j) | (lab_i == lab_j != 0) on the last-observed
//               labels (:263-266); group g(i) = index of i's first member
//   intra GAT   per head h: Wh = X W_h (40 -> 72), masked softmax attention,
//               ELU; heads concatenated; out layer (72 nh -> 16) + ELU +
//               log_softmax over features                      (:269, :231-237)
//   group mean  gin = R intra, R the row-normalised distinct rows of M
//                                                               (:271-280)
//   inter GAT   the same GAT (16 -> 72 -> 16) on the complete graph of the
//               scene's groups                                  (:282-285)
//   un-pool     inter_i = gout[g(i)] / |g(i)|  (R^T with R normalised, :286)
//   out         Linear(32, 24)([intra, inter])                   (:288-289)
//
// One launch replaces the ~14 launches of the per-op path (sgg_xw +
// sgg_gat_fwd per layer, group pooling kernels, concat, Linear).  The
// backward recomputes the forward in LDS (it is ~0.3 MFLOP per 20-ped scene)
// and back-propagates through every layer in the same workgroup; each
// scene's parameter gradients go to its own row of a slab (no atomics) that
// sgg_slab_reduce sums in scene order (deterministic).
//
// Attention: e_ij = LeakyReLU(a[:F].Wh_i + a[F:].Wh_j) (the s_i + t_j
// decomposition of the reference's (N, N, 2F) concatenation), masked to
// -inf outside the graph, softmax over j; one wavefront per attention row
// with lane j (n <= 64), row max / sum by wave shuffles.
#include "sgg_common.h"

namespace sgg {

namespace {

// forward 1024 threads (16 waves: attention rows and output elements of a
// 20-ped scene are ~1 per wave / thread, so the dependent chains overlap);
// the same for the backward
constexpr int kFwdThreads = 1024, kBwdThreads = 1024;
constexpr int kMaxWaves = kFwdThreads / 64;
constexpr int FI = 40, FH = 72, FO = 16, FE = 24;   // GATEncoder dims (models.py:242-244)
constexpr int P40 = FI + 1, P72 = FH + 1, P16 = FO + 1;

// LDS image of the weights: W (K x N) rows at pitch N + 1 (odd: a column walk
// across rows, lane = row, is bank-conflict free; a row walk is contiguous)
constexpr int PW72 = FH + 1, PW16 = FO + 1, PWE = 2 * FO + 1;
__host__ __device__ inline int weights_floats(int nh) {
  return nh * (FI * PW72 + 2 * FH) + (FH * nh * PW16 + 2 * FO) + nh * (FO * PW72 + 2 * FH) + (FH * nh * PW16 + 2 * FO) +
         FE * PWE + FE;
}

struct LW {
  const float* Wi[kGatEncMaxHeads];
  const float* ai[kGatEncMaxHeads];
  const float* Wio;
  const float* aio;
  const float* Wg[kGatEncMaxHeads];
  const float* ag[kGatEncMaxHeads];
  const float* Wgo;
  const float* ago;
  const float* Woe;
  const float* boe;
};

// copy a K x N row-major global matrix to LDS at pitch N + 1; each thread
// issues its (up to 4 per round) loads before any store, so a matrix costs
// one memory latency per 4 trips instead of one per trip
__device__ inline float* stage_mat(float* dst, const float* __restrict__ src, int K, int N, int nthreads) {
  const int tot = K * N;
  for (int e0 = threadIdx.x; e0 < tot; e0 += 4 * nthreads) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = src[min(e0 + u * nthreads, tot - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * nthreads;
      if (e < tot) {
        const int k = e / N, c = e - k * N;
        dst[k * (N + 1) + c] = v[u];
      }
    }
  }
  return dst + K * (N + 1);
}
__device__ inline float* stage_vec(float* dst, const float* __restrict__ src, int n, int nthreads) {
  for (int e = threadIdx.x; e < n; e += nthreads) dst[e] = src[e];
  return dst + n;
}

struct Layout {
  // float offsets into the workgroup's LDS
  int X, H1, yI, preI, gin, G1, preG, gout, Wh, s, t, ds, dt, att;   // forward
  int dWh, dH, dI, dG, dpre, attm;                                    // backward
  int ints;       // int region: lab (float), gidl, grank, cnt, M
  int wts;        // the module's weights, staged once per workgroup (odd row pitches)
  int total;      // floats
  int PH, NP, NPP;
};

__host__ __device__ inline Layout make_layout(int np, int nh, bool bwd) {
  Layout L;
  L.NP = np;
  L.PH = FH * nh + 1;
  L.NPP = np | 1;
  int o = 0;
  auto take = [&](int n) { const int r = o; o += (n + 3) & ~3; return r; };
  L.X = take(np * P40);
  L.H1 = take(np * L.PH);
  L.yI = take(np * P16);
  L.preI = take(np * P16);
  L.gin = take(np * P16);
  L.G1 = take(np * L.PH);
  L.preG = take(np * P16);
  L.gout = take(np * P16);
  L.Wh = take(np * P72);
  L.s = take(np);
  L.t = take(np);
  L.ds = take(np);
  L.dt = take(np);
  L.att = take(kMaxWaves * 64);
  if (bwd) {
    L.dWh = take(np * P72);
    L.dH = take(np * L.PH);
    L.dI = take(np * P16);
    L.dG = take(np * P16);
    L.dpre = take(np * P16);
    L.attm = take(np * L.NPP);
  } else {
    L.dWh = L.dH = L.dI = L.dG = L.dpre = L.attm = 0;
  }
  L.ints = take(5 * np + 4);
  L.wts = take(weights_floats(nh));
  L.total = o;
  return L;
}

// parameter-gradient slab layout (floats per scene)
struct PLayout {
  int Wi[kGatEncMaxHeads], ai[kGatEncMaxHeads], Wio, aio, Wg[kGatEncMaxHeads], ag[kGatEncMaxHeads], Wgo, ago, Woe,
      boe, total;
};

__host__ __device__ inline PLayout make_playout(int nh) {
  PLayout P;
  int o = 0;
#pragma unroll
  for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
      if (h >= nh) break;
    P.Wi[h] = o; o += FI * FH;
    P.ai[h] = o; o += 2 * FH;
  }
  P.Wio = o; o += FH * nh * FO;
  P.aio = o; o += 2 * FO;
#pragma unroll
  for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
      if (h >= nh) break;
    P.Wg[h] = o; o += FO * FH;
    P.ag[h] = o; o += 2 * FH;
  }
  P.Wgo = o; o += FH * nh * FO;
  P.ago = o; o += 2 * FO;
  P.Woe = o; o += FE * 2 * FO;
  P.boe = o; o += FE;
  P.total = o;
  return P;
}

// forward state of one scene kept for the backward (floats; written by the
// forward when args.saved != NULL, read back by the backward instead of
// recomputing the four attention layers): every layer's Wh, the head / out
// activations, the group structure
struct SLayout {
  int Whi[kGatEncMaxHeads], Whio, Whg[kGatEncMaxHeads], Whgo, H1, yI, preI, gin, G1, preG, gout, ints, total;
};

__host__ __device__ inline SLayout make_slayout(int np, int nh) {
  SLayout S;
  int o = 0;
  for (int h = 0; h < kGatEncMaxHeads; ++h) {
    S.Whi[h] = o;
    if (h < nh) o += np * FH;
  }
  S.Whio = o; o += np * FO;
  for (int h = 0; h < kGatEncMaxHeads; ++h) {
    S.Whg[h] = o;
    if (h < nh) o += np * FH;
  }
  S.Whgo = o; o += np * FO;
  S.H1 = o; o += np * FH * nh;
  S.yI = o; o += np * FO;
  S.preI = o; o += np * FO;
  S.gin = o; o += np * FO;
  S.G1 = o; o += np * FH * nh;
  S.preG = o; o += np * FO;
  S.gout = o; o += np * FO;
  S.ints = o; o += 5 * np + 4;
  S.total = (o + 3) & ~3;
  return S;
}

// rows x cols between an LDS image at pitch ld and a dense global block
__device__ inline void rows_to_global(float* __restrict__ dst, const float* src, int ld, int rows, int cols) {
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
    const int r = e / cols, c = e - r * cols;
    dst[e] = src[r * ld + c];
  }
}
__device__ inline void rows_from_global(float* dst, int ld, const float* __restrict__ src, int rows, int cols) {
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
    const int r = e / cols, c = e - r * cols;
    dst[r * ld + c] = src[e];
  }
}

__device__ __forceinline__ float lrelu(float x, float a) { return x > 0.f ? x : a * x; }

// out[r][c] = sum_k in[r][k] W[k][c]   (W: K x N in LDS at pitch ldw, K % 4 == 0)
__device__ void lin(const float* in, int ldi, int rows, int K, const float* W, int ldw, int N, float* out, int ldo) {
  for (int e = threadIdx.x; e < rows * N; e += blockDim.x) {
    const int r = e / N, c = e - r * N;
    const float* x = in + r * ldi;
    const float* w = W + c;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int k = 0; k < K; k += 4) {
      a0 = fmaf(x[k], w[k * ldw], a0);
      a1 = fmaf(x[k + 1], w[(k + 1) * ldw], a1);
      a2 = fmaf(x[k + 2], w[(k + 2) * ldw], a2);
      a3 = fmaf(x[k + 3], w[(k + 3) * ldw], a3);
    }
    out[r * ldo + c] = (a0 + a1) + (a2 + a3);
  }
}

// out[r][k] (+)= sum_c d[r][c] W[k][c]   (input gradient of lin; N % 4 == 0)
__device__ void lin_t(const float* d, int ldd, int rows, int N, const float* W, int ldw, int K, float* out, int ldo,
                      bool acc) {
  for (int e = threadIdx.x; e < rows * K; e += blockDim.x) {
    const int r = e / K, k = e - r * K;
    const float* dr = d + r * ldd;
    const float* wr = W + k * ldw;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int c = 0; c < N; c += 4) {
      a0 = fmaf(dr[c], wr[c], a0);
      a1 = fmaf(dr[c + 1], wr[c + 1], a1);
      a2 = fmaf(dr[c + 2], wr[c + 2], a2);
      a3 = fmaf(dr[c + 3], wr[c + 3], a3);
    }
    const float v = (a0 + a1) + (a2 + a3);
    out[r * ldo + k] = acc ? out[r * ldo + k] + v : v;
  }
}

// dst[k][c] = sum_r x[r][k] d[r][c]   (weight gradient of lin, to the slab)
__device__ void wgrad(const float* x, int ldx, int rows, int K, const float* d, int ldd, int N, float* dst) {
  for (int e = threadIdx.x; e < K * N; e += blockDim.x) {
    const int k = e / N, c = e - k * N;
    float a0 = 0.f, a1 = 0.f;
    int r = 0;
    for (; r + 1 < rows; r += 2) {
      a0 = fmaf(x[r * ldx + k], d[r * ldd + c], a0);
      a1 = fmaf(x[(r + 1) * ldx + k], d[(r + 1) * ldd + c], a1);
    }
    if (r < rows) a0 = fmaf(x[r * ldx + k], d[r * ldd + c], a0);
    dst[e] = a0 + a1;
  }
}

// s_i = a[:F].Wh_i, t_i = a[F:].Wh_i: one wavefront per dot product (lanes
// over the F <= 128 features, a wave-shuffle sum) instead of an F-long
// serial chain of LDS reads per thread
__device__ void scores(const float* Wh, int ldw, int rows, int F, const float* a, float* s, float* t) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int e = wave; e < 2 * rows; e += nw) {
    const int r = e >> 1, w = e & 1;
    const float* av = a + w * F;
    const float* x = Wh + r * ldw;
    float v = lane < F ? x[lane] * av[lane] : 0.f;
    if (lane + 64 < F) v = fmaf(x[lane + 64], av[lane + 64], v);
    v = wave_sum(v);
    if (lane == 0) (w ? t : s)[r] = v;
  }
}

__device__ __forceinline__ bool edge(const int* gidl, int i, int j) { return gidl == nullptr || gidl[i] == gidl[j]; }

// softmax row i of the attention, lane j (n <= 64)
__device__ __forceinline__ float att_row(int i, int rows, const int* gidl, const float* s, const float* t, float alpha,
                                         int lane) {
  const bool ok = lane < rows && edge(gidl, i, lane);
  const float e = ok ? lrelu(s[i] + t[lane], alpha) : -INFINITY;
  const float m = wave_max(e);
  const float p = ok ? __expf(e - m) : 0.f;
  const float sum = wave_sum(p);
  return p / sum;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// attention layer forward: out = epi(att . Wh); pre (optional) = att . Wh
// epi: 1 ELU, 2 ELU + log_softmax over the F features
__device__ void att_fwd(const float* Wh, int ldw, int rows, int F, const int* gidl, const float* s, const float* t,
                        float alpha, int epi, float* out, int ldo, float* pre, int ldp, float* attw) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* aw = attw + wave * 64;
  for (int i = wave; i < rows; i += (int)(blockDim.x >> 6)) {
    aw[lane] = att_row(i, rows, gidl, s, t, alpha, lane);
    wave_lds_sync();
    float hv[2], zv[2], zmax = -INFINITY;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = lane + 64 * c;
      float acc = 0.f, acc2 = 0.f;
      if (f < F) {
        int j = 0;
        for (; j + 1 < rows; j += 2) {
          acc = fmaf(aw[j], Wh[j * ldw + f], acc);
          acc2 = fmaf(aw[j + 1], Wh[(j + 1) * ldw + f], acc2);
        }
        if (j < rows) acc = fmaf(aw[j], Wh[j * ldw + f], acc);
        acc += acc2;
      }
      hv[c] = acc;
      zv[c] = elu(acc);
      if (f < F) zmax = fmaxf(zmax, zv[c]);
    }
    float lse = 0.f;
    if (epi == 2) {
      zmax = wave_max(zmax);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (lane + 64 * c < F) se += __expf(zv[c] - zmax);
      lse = zmax + __logf(wave_sum(se));
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = lane + 64 * c;
      if (f < F) {
        if (pre) pre[i * ldp + f] = hv[c];
        out[i * ldo + f] = epi == 2 ? zv[c] - lse : zv[c];
      }
    }
    wave_lds_sync();   // aw is rewritten by the wave's next row
  }
}

// gradient through the epilogue: d (in: d out, out: d pre), one wave per row
__device__ void epi_bwd(float* d, int ldd, const float* pre, int ldp, int rows, int F, int epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = wave; i < rows; i += (int)(blockDim.x >> 6)) {
    float dv[2], hv[2], zv[2];
    float zmax = -INFINITY, sdy = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = lane + 64 * c;
      dv[c] = f < F ? d[i * ldd + f] : 0.f;
      hv[c] = f < F ? pre[i * ldp + f] : 0.f;
      zv[c] = elu(hv[c]);
      if (f < F) {
        zmax = fmaxf(zmax, zv[c]);
        sdy += dv[c];
      }
    }
    float lse = 0.f;
    if (epi == 2) {
      zmax = wave_max(zmax);
      sdy = wave_sum(sdy);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (lane + 64 * c < F) se += __expf(zv[c] - zmax);
      lse = zmax + __logf(wave_sum(se));
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = lane + 64 * c;
      if (f < F) {
        float v = dv[c];
        if (epi == 2) v -= __expf(zv[c] - lse) * sdy;
        d[i * ldd + f] = v * elu_grad(hv[c]);
      }
    }
  }
}

// attention layer backward.  dpre: gradient of the aggregate (rows x F);
// writes dWh (rows x F) and the a-gradient (2F) to da; attm scratch rows x npp
__device__ void att_bwd(const float* Wh, int ldw, int rows, int F, const int* gidl, float* s, float* t, float alpha,
                        const float* a, const float* dpre, int ldd, float* dWh, int lddw, float* ds,
                        float* dt, float* attm, int npp, float* da) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  scores(Wh, ldw, rows, F, a, s, t);
  __syncthreads();
  for (int i = wave; i < rows; i += (int)(blockDim.x >> 6)) {
    const float v = att_row(i, rows, gidl, s, t, alpha, lane);
    if (lane < rows) attm[i * npp + lane] = v;
  }
  __syncthreads();
  // attention-weighted part: dWh_j = sum_i att_ij dpre_i
  for (int e = threadIdx.x; e < rows * F; e += blockDim.x) {
    const int j = e / F, f = e - j * F;
    float acc = 0.f;
    for (int i = 0; i < rows; ++i) acc = fmaf(attm[i * npp + j], dpre[i * ldd + f], acc);
    dWh[j * lddw + f] = acc;
  }
  __syncthreads();   // attm is overwritten with dz below
  for (int i = wave; i < rows; i += (int)(blockDim.x >> 6)) {
    const int j = lane;
    float datt = 0.f, at = 0.f;
    if (j < rows) {
      at = attm[i * npp + j];
      for (int f = 0; f < F; ++f) datt = fmaf(dpre[i * ldd + f], Wh[j * ldw + f], datt);
    }
    const float dot = wave_sum(at * datt);
    float dz = 0.f;
    if (j < rows) {
      const float de = at * (datt - dot);
      dz = (s[i] + t[j]) > 0.f ? de : alpha * de;
      attm[i * npp + j] = dz;
    }
    const float dsum = wave_sum(dz);
    if (lane == 0) ds[i] = dsum;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < rows; j += blockDim.x) {
    float acc = 0.f;
    for (int i = 0; i < rows; ++i) acc += attm[i * npp + j];
    dt[j] = acc;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < rows * F; e += blockDim.x) {
    const int j = e / F, f = e - j * F;
    dWh[j * lddw + f] += ds[j] * a[f] + dt[j] * a[F + f];
  }
  // da[f] = sum_i ds_i Wh_i[f], da[F + f] = sum_j dt_j Wh_j[f]
  for (int e = threadIdx.x; e < 2 * F; e += blockDim.x) {
    const int w = e / F, f = e - w * F;
    const float* g = w ? dt : ds;
    float acc = 0.f;
    for (int r = 0; r < rows; ++r) acc = fmaf(g[r], Wh[r * ldw + f], acc);
    da[e] = acc;
  }
  __syncthreads();
}

template <bool BWD>
__global__ void __launch_bounds__(BWD ? kBwdThreads : kFwdThreads) gatenc_kernel(GatEncArgs p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const Layout L = make_layout(p.np, p.nh, BWD);
  const PLayout PL = make_playout(p.nh);
  const SLayout SL = make_slayout(p.np, p.nh);
  const int nh = p.nh, PH = L.PH;
  float* X = sm + L.X;
  float* H1 = sm + L.H1;
  float* yI = sm + L.yI;
  float* preI = sm + L.preI;
  float* gin = sm + L.gin;
  float* G1 = sm + L.G1;
  float* preG = sm + L.preG;
  float* gout = sm + L.gout;
  float* Wh = sm + L.Wh;
  float* s = sm + L.s;
  float* t = sm + L.t;
  float* ds = sm + L.ds;
  float* dt = sm + L.dt;
  float* attw = sm + L.att;
  float* lab = sm + L.ints;
  int* gidl = reinterpret_cast<int*>(lab + L.NP);
  int* grank = gidl + L.NP;
  int* cnt = grank + L.NP;
  float* ginv = reinterpret_cast<float*>(cnt + L.NP);
  int* Mp = reinterpret_cast<int*>(ginv + L.NP);
  const int tid = threadIdx.x;
  LW lw;
  {
    float* q = sm + L.wts;
#pragma unroll
    for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
      if (h >= nh) break;
      lw.Wi[h] = q; q = stage_mat(q, p.w.Wi[h], FI, FH, blockDim.x);
      lw.ai[h] = q; q = stage_vec(q, p.w.ai[h], 2 * FH, blockDim.x);
    }
    lw.Wio = q; q = stage_mat(q, p.w.Wio, FH * nh, FO, blockDim.x);
    lw.aio = q; q = stage_vec(q, p.w.aio, 2 * FO, blockDim.x);
#pragma unroll
    for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
      if (h >= nh) break;
      lw.Wg[h] = q; q = stage_mat(q, p.w.Wg[h], FO, FH, blockDim.x);
      lw.ag[h] = q; q = stage_vec(q, p.w.ag[h], 2 * FH, blockDim.x);
    }
    lw.Wgo = q; q = stage_mat(q, p.w.Wgo, FH * nh, FO, blockDim.x);
    lw.ago = q; q = stage_vec(q, p.w.ago, 2 * FO, blockDim.x);
    lw.Woe = q; q = stage_mat(q, p.w.Woe, FE, 2 * FO, blockDim.x);
    lw.boe = q; q = stage_vec(q, p.w.boe, FE, blockDim.x);
  }
  // (the first scene's input loads are followed by a barrier before any use)

  for (int sc = blockIdx.x; sc < p.S; sc += gridDim.x) {
    const int o = p.scene_off[sc];
    const int n = p.scene_off[sc + 1] - o;
    if (n <= 0) continue;   // uniform over the workgroup
    float* saved = p.saved ? p.saved + (size_t)sc * SL.total : nullptr;
    // ---- inputs and group structure ------------------------------------
    for (int e = tid; e < n * FI; e += blockDim.x) {
      const int r = e / FI, k = e - r * FI;
      X[r * P40 + k] = p.X[(size_t)(o + r) * p.ldx + k];
    }
    for (int i = tid; i < n; i += blockDim.x) lab[i] = p.labels[o + i];
    __syncthreads();
    if (!BWD || !p.saved) {
      // group structure (models.py:263-278) in ONE wave, lane = ped (n <= 64):
      // g(i) = first ped with i's non-zero label (or i), groups ranked by
      // their first member, sizes by a lane sweep -- no workgroup barrier
      if (tid < 64) {
        const int i = tid;
        const float li = i < n ? lab[i] : 0.f;
        int g = i;
        for (int j = 0; j < n; ++j) {
          const float lj = __shfl(li, j);
          if (li != 0.f && lj == li && j < g) g = j;
        }
        const bool lead = i < n && g == i;
        const unsigned long long leaders = __ballot(lead);
        int c = 0;
        for (int j = 0; j < n; ++j) c += __shfl(g, j) == g;
        const int r = __popcll(leaders & ((1ull << g) - 1ull));
        if (i < n) {
          gidl[i] = g;
          grank[i] = r;
          ginv[i] = 1.f / (float)c;
          if (lead) cnt[r] = c;
        }
        if (i == 0) *Mp = __popcll(leaders);
      }
      __syncthreads();
    } else {
      rows_from_global(lab, 5 * L.NP + 4, saved + SL.ints, 1, 5 * L.NP + 4);
      __syncthreads();
    }
    const int M = *Mp;

    if (!BWD || !saved) {
    // ---- intra GAT: heads (40 -> 72, ELU), out (72 nh -> 16, ELU, log_softmax)
#pragma unroll
    for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
      if (h >= nh) break;
      lin(X, P40, n, FI, lw.Wi[h], PW72, FH, Wh, P72);
      __syncthreads();
      if (saved) rows_to_global(saved + SL.Whi[h], Wh, P72, n, FH);
      scores(Wh, P72, n, FH, lw.ai[h], s, t);
      __syncthreads();
      att_fwd(Wh, P72, n, FH, gidl, s, t, p.alpha, 1, H1 + h * FH, PH, nullptr, 0, attw);
      __syncthreads();
    }
    lin(H1, PH, n, FH * nh, lw.Wio, PW16, FO, Wh, P72);
    __syncthreads();
    if (saved) rows_to_global(saved + SL.Whio, Wh, P72, n, FO);
    scores(Wh, P72, n, FO, lw.aio, s, t);
    __syncthreads();
    att_fwd(Wh, P72, n, FO, gidl, s, t, p.alpha, 2, yI, P16, preI, P16, attw);
    __syncthreads();
    // ---- group mean (R intra) ------------------------------------------
    for (int e = tid; e < M * FO; e += blockDim.x) {
      const int g = e / FO, f = e - g * FO;
      float acc = 0.f;
      for (int i = 0; i < n; ++i)
        if (grank[i] == g) acc = fmaf(ginv[i], yI[i * P16 + f], acc);
      gin[g * P16 + f] = acc;
    }
    __syncthreads();
    // ---- inter GAT on the complete graph of the M groups ----------------
#pragma unroll
    for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
      if (h >= nh) break;
      lin(gin, P16, M, FO, lw.Wg[h], PW72, FH, Wh, P72);
      __syncthreads();
      if (saved) rows_to_global(saved + SL.Whg[h], Wh, P72, M, FH);
      scores(Wh, P72, M, FH, lw.ag[h], s, t);
      __syncthreads();
      att_fwd(Wh, P72, M, FH, nullptr, s, t, p.alpha, 1, G1 + h * FH, PH, nullptr, 0, attw);
      __syncthreads();
    }
    lin(G1, PH, M, FH * nh, lw.Wgo, PW16, FO, Wh, P72);
    __syncthreads();
    if (saved) rows_to_global(saved + SL.Whgo, Wh, P72, M, FO);
    scores(Wh, P72, M, FO, lw.ago, s, t);
    __syncthreads();
    att_fwd(Wh, P72, M, FO, nullptr, s, t, p.alpha, 2, gout, P16, preG, P16, attw);
    __syncthreads();
    if (saved) {   // the activations and the group structure for the backward
      rows_to_global(saved + SL.H1, H1, PH, n, FH * nh);
      rows_to_global(saved + SL.yI, yI, P16, n, FO);
      rows_to_global(saved + SL.preI, preI, P16, n, FO);
      rows_to_global(saved + SL.gin, gin, P16, M, FO);
      rows_to_global(saved + SL.G1, G1, PH, M, FH * nh);
      rows_to_global(saved + SL.preG, preG, P16, M, FO);
      rows_to_global(saved + SL.gout, gout, P16, M, FO);
      rows_to_global(saved + SL.ints, lab, 5 * L.NP + 4, 1, 5 * L.NP + 4);
    }
    } else {
      // backward with the forward's saved state: no recompute
      rows_from_global(H1, PH, saved + SL.H1, n, FH * nh);
      rows_from_global(yI, P16, saved + SL.yI, n, FO);
      rows_from_global(preI, P16, saved + SL.preI, n, FO);
      rows_from_global(gin, P16, saved + SL.gin, M, FO);
      rows_from_global(G1, PH, saved + SL.G1, M, FH * nh);
      rows_from_global(preG, P16, saved + SL.preG, M, FO);
      rows_from_global(gout, P16, saved + SL.gout, M, FO);
      __syncthreads();
    }

    if (!BWD) {
      // ---- out = Woe [intra, gout[g(i)] / |g(i)|] + boe ------------------
      for (int e = tid; e < n * FE; e += blockDim.x) {
        const int i = e / FE, c = e - i * FE;
        const float* wr = lw.Woe + c * PWE;
        const float* gi = gout + grank[i] * P16;
        const float sc_i = ginv[i];
        float a0 = lw.boe[c], a1 = 0.f;
        for (int f = 0; f < FO; ++f) {
          a0 = fmaf(wr[f], yI[i * P16 + f], a0);
          a1 = fmaf(wr[FO + f], gi[f] * sc_i, a1);
        }
        p.y[(size_t)(o + i) * p.ldy + c] = a0 + a1;
      }
      __syncthreads();
      continue;
    }

    // ================= backward ===========================================
    float* dWh = sm + L.dWh;
    float* dH = sm + L.dH;
    float* dI = sm + L.dI;
    float* dG = sm + L.dG;
    float* dpre = sm + L.dpre;
    float* attm = sm + L.attm;
    float* slab = p.slab + (size_t)sc * PL.total;
    // the scene's dy rows to LDS first (the Wh scratch, pitch FE + 1): the
    // loops below walk them n-deep, one memory latency per step from global
    constexpr int PDY = FE + 1;
    float* dy = Wh;
    {
      const float* dyg = p.dy + (size_t)o * p.lddy;
      const int tot = n * FE;
      for (int e0 = tid; e0 < tot; e0 += 4 * blockDim.x) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = min(e0 + u * (int)blockDim.x, tot - 1);
          const int i = e / FE, k = e - i * FE;
          v[u] = dyg[(size_t)i * p.lddy + k];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = e0 + u * (int)blockDim.x;
          if (e < tot) {
            const int i = e / FE, k = e - i * FE;
            dy[i * PDY + k] = v[u];
          }
        }
      }
    }
    __syncthreads();
    // out embedding: d[intra | inter] = dy Woe; dWoe = dy^T [intra | inter]; dboe = sum dy
    for (int e = tid; e < n * 2 * FO; e += blockDim.x) {
      const int i = e / (2 * FO), c = e - i * 2 * FO;
      float acc = 0.f;
      for (int k = 0; k < FE; ++k) acc = fmaf(dy[i * PDY + k], lw.Woe[k * PWE + c], acc);
      if (c < FO) dI[i * P16 + c] = acc;
      else dpre[i * P16 + c - FO] = acc;   // d inter (scratch)
    }
    for (int e = tid; e < FE * 2 * FO; e += blockDim.x) {
      const int k = e / (2 * FO), c = e - k * 2 * FO;
      float acc = 0.f;
      for (int i = 0; i < n; ++i) {
        const float v = c < FO ? yI[i * P16 + c] : gout[grank[i] * P16 + c - FO] * ginv[i];
        acc = fmaf(dy[i * PDY + k], v, acc);
      }
      slab[PL.Woe + e] = acc;
    }
    for (int k = tid; k < FE; k += blockDim.x) {
      float acc = 0.f;
      for (int i = 0; i < n; ++i) acc += dy[i * PDY + k];
      slab[PL.boe + k] = acc;
    }
    __syncthreads();
    // un-pool backward: d gout[g] = sum_{i in g} d inter_i / |g|
    for (int e = tid; e < M * FO; e += blockDim.x) {
      const int g = e / FO, f = e - g * FO;
      float acc = 0.f;
      for (int i = 0; i < n; ++i)
        if (grank[i] == g) acc = fmaf(ginv[i], dpre[i * P16 + f], acc);
      dG[g * P16 + f] = acc;
    }
    __syncthreads();
    // ---- inter out layer ----
    epi_bwd(dG, P16, preG, P16, M, FO, 2);
    if (saved) rows_from_global(Wh, P72, saved + SL.Whgo, M, FO);
    else lin(G1, PH, M, FH * nh, lw.Wgo, PW16, FO, Wh, P72);
    __syncthreads();
    att_bwd(Wh, P72, M, FO, nullptr, s, t, p.alpha, lw.ago, dG, P16, dWh, P72, ds, dt, attm, L.NPP, slab + PL.ago);
    wgrad(G1, PH, M, FH * nh, dWh, P72, FO, slab + PL.Wgo);
    lin_t(dWh, P72, M, FO, lw.Wgo, PW16, FH * nh, dH, PH, false);
    __syncthreads();
    // ---- inter heads ----
    for (int e = tid; e < M * FO; e += blockDim.x) dG[(e / FO) * P16 + e % FO] = 0.f;   // becomes d gin
#pragma unroll
    for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
      if (h >= nh) break;
      // ELU backward from the stored output: elu'(x) = 1 (y > 0) | y + 1
      for (int e = tid; e < M * FH; e += blockDim.x) {
        const int r = e / FH, f = e - r * FH;
        const float yv = G1[r * PH + h * FH + f];
        dH[r * PH + h * FH + f] *= yv > 0.f ? 1.f : yv + 1.f;
      }
      if (saved) rows_from_global(Wh, P72, saved + SL.Whg[h], M, FH);
      else lin(gin, P16, M, FO, lw.Wg[h], PW72, FH, Wh, P72);
      __syncthreads();
      att_bwd(Wh, P72, M, FH, nullptr, s, t, p.alpha, lw.ag[h], dH + h * FH, PH, dWh, P72, ds, dt, attm, L.NPP,
              slab + PL.ag[h]);
      wgrad(gin, P16, M, FO, dWh, P72, FH, slab + PL.Wg[h]);
      lin_t(dWh, P72, M, FH, lw.Wg[h], PW72, FO, dG, P16, true);
      __syncthreads();
    }
    // group-mean backward: d intra_i += d gin[g(i)] / |g(i)|
    for (int e = tid; e < n * FO; e += blockDim.x) {
      const int i = e / FO, f = e - i * FO;
      dI[i * P16 + f] = fmaf(ginv[i], dG[grank[i] * P16 + f], dI[i * P16 + f]);
    }
    __syncthreads();
    // ---- intra out layer ----
    epi_bwd(dI, P16, preI, P16, n, FO, 2);
    if (saved) rows_from_global(Wh, P72, saved + SL.Whio, n, FO);
    else lin(H1, PH, n, FH * nh, lw.Wio, PW16, FO, Wh, P72);
    __syncthreads();
    att_bwd(Wh, P72, n, FO, gidl, s, t, p.alpha, lw.aio, dI, P16, dWh, P72, ds, dt, attm, L.NPP, slab + PL.aio);
    wgrad(H1, PH, n, FH * nh, dWh, P72, FO, slab + PL.Wio);
    lin_t(dWh, P72, n, FO, lw.Wio, PW16, FH * nh, dH, PH, false);
    __syncthreads();
    // ---- intra heads ----
    float* dXo = p.dX + (size_t)o * p.lddx;
#pragma unroll
    for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
      if (h >= nh) break;
      for (int e = tid; e < n * FH; e += blockDim.x) {
        const int r = e / FH, f = e - r * FH;
        const float yv = H1[r * PH + h * FH + f];
        dH[r * PH + h * FH + f] *= yv > 0.f ? 1.f : yv + 1.f;
      }
      if (saved) rows_from_global(Wh, P72, saved + SL.Whi[h], n, FH);
      else lin(X, P40, n, FI, lw.Wi[h], PW72, FH, Wh, P72);
      __syncthreads();
      att_bwd(Wh, P72, n, FH, gidl, s, t, p.alpha, lw.ai[h], dH + h * FH, PH, dWh, P72, ds, dt, attm, L.NPP,
              slab + PL.ai[h]);
      wgrad(X, P40, n, FI, dWh, P72, FH, slab + PL.Wi[h]);
      // dX (global) accumulates over heads in a fixed order
      for (int e = tid; e < n * FI; e += blockDim.x) {
        const int r = e / FI, k = e - r * FI;
        const float* dr = dWh + r * P72;
        const float* wr = lw.Wi[h] + k * PW72;
        float a0 = 0.f, a1 = 0.f;
        for (int c = 0; c < FH; c += 2) {
          a0 = fmaf(dr[c], wr[c], a0);
          a1 = fmaf(dr[c + 1], wr[c + 1], a1);
        }
        float* dst = dXo + (size_t)r * p.lddx + k;
        *dst = h ? *dst + (a0 + a1) : a0 + a1;
      }
      __syncthreads();
    }
  }
}

// out[c] = sum_s slab[s][c] in a fixed order (deterministic): block = 64
// columns x 16 row phases, phase p sums rows p, p + 16, ... with 4 loads in
// flight, then the 16 phase sums in order
__global__ void __launch_bounds__(1024) slab_reduce_kernel(const float* __restrict__ slab, int rows, int cols,
                                                          float* __restrict__ out) {
  __shared__ float part[16][64];
  const int el = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + el;
  float s = 0.f;
  if (c < cols) {
    int r = ph;
    for (; r + 48 < rows; r += 64) {
      const float v0 = slab[(size_t)r * cols + c], v1 = slab[(size_t)(r + 16) * cols + c];
      const float v2 = slab[(size_t)(r + 32) * cols + c], v3 = slab[(size_t)(r + 48) * cols + c];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; r < rows; r += 16) s += slab[(size_t)r * cols + c];
  }
  part[ph][el] = s;
  __syncthreads();
  if (ph == 0 && c < cols) {
    float v = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) v += part[p][el];
    out[c] = v;
  }
}

}  // namespace

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_gatenc_param_size(int nh) {
  if (nh < 1 || nh > kGatEncMaxHeads) return -1;
  return make_playout(nh).total;
}

extern "C" long long sgg_gatenc_saved_floats(int S, int max_n, int nh) {
  if (S < 0 || max_n < 1 || nh < 1 || nh > kGatEncMaxHeads) return -1;
  return (long long)S * make_slayout(max_n, nh).total;
}

extern "C" long long sgg_gatenc_lds_bytes(int max_n, int nh, int bwd) {
  if (max_n < 1 || nh < 1 || nh > kGatEncMaxHeads) return -1;
  return 4ll * make_layout(max_n, nh, bwd != 0).total;
}

static int gatenc_check(const char* who, const GatEncArgs* a, int bwd) {
  SGG_CHECK_ARG(a, "%s: null args", who);
  SGG_CHECK_ARG(a->X && a->labels && a->scene_off, "%s: null input", who);
  SGG_CHECK_ARG(a->nh >= 1 && a->nh <= kGatEncMaxHeads, "%s: heads %d outside [1, %d]", who, a->nh, kGatEncMaxHeads);
  SGG_CHECK_ARG(a->np >= 1 && a->np <= 64, "%s: max scene size %d outside [1, 64]", who, a->np);
  SGG_CHECK_ARG(a->S >= 0 && a->ldx >= FI, "%s: bad sizes", who);
  for (int h = 0; h < a->nh; ++h)
    SGG_CHECK_ARG(a->w.Wi[h] && a->w.ai[h] && a->w.Wg[h] && a->w.ag[h], "%s: null head weight %d", who, h);
  SGG_CHECK_ARG(a->w.Wio && a->w.aio && a->w.Wgo && a->w.ago && a->w.Woe && a->w.boe, "%s: null weight", who);
  if (bwd) {
    SGG_CHECK_ARG(a->dy && a->dX && a->slab && a->lddy >= FE && a->lddx >= FI, "%s: null / bad gradient buffer", who);
  } else {
    SGG_CHECK_ARG(a->y && a->ldy >= FE, "%s: null / bad output", who);
  }
  const long long lds = sgg_gatenc_lds_bytes(a->np, a->nh, bwd);
  SGG_CHECK_ARG(lds <= 160 * 1024, "%s: %d peds x %d heads need %lld B of LDS (> 160 KiB)", who, a->np, a->nh, lds);
  return 0;
}

extern "C" int sgg_gatenc_fwd(const GatEncArgs* args, void* stream) {
  const int rc = gatenc_check("sgg_gatenc_fwd", args, 0);
  if (rc) return rc;
  if (args->S == 0) return 0;
  const size_t lds = (size_t)sgg_gatenc_lds_bytes(args->np, args->nh, 0);
  hipLaunchKernelGGL(gatenc_kernel<false>, dim3(args->S < 65536 ? args->S : 65536), dim3(kFwdThreads), lds,
                     (hipStream_t)stream, *args);
  SGG_RETURN_LAUNCH("sgg_gatenc_fwd");
}

extern "C" int sgg_gatenc_bwd(const GatEncArgs* args, void* stream) {
  const int rc = gatenc_check("sgg_gatenc_bwd", args, 1);
  if (rc) return rc;
  if (args->S == 0) return 0;
  const size_t lds = (size_t)sgg_gatenc_lds_bytes(args->np, args->nh, 1);
  hipLaunchKernelGGL(gatenc_kernel<true>, dim3(args->S < 65536 ? args->S : 65536), dim3(kBwdThreads), lds,
                     (hipStream_t)stream, *args);
  SGG_RETURN_LAUNCH("sgg_gatenc_bwd");
}

extern "C" int sgg_slab_reduce(const float* slab, int rows, int cols, float* out, void* stream) {
  SGG_CHECK_ARG(slab && out, "sgg_slab_reduce: null pointer");
  SGG_CHECK_ARG(rows >= 0 && cols >= 0, "sgg_slab_reduce: bad sizes");
  if (cols == 0) return 0;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((cols + 63) / 64), dim3(1024), 0, (hipStream_t)stream, slab, rows, cols,
                     out);
  SGG_RETURN_LAUNCH("sgg_slab_reduce");
}
