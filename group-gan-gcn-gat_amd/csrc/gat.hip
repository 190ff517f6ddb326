// Graph attention over the nodes of each segment (GraphAttentionLayer,
// reference sgan/models.py:184-220; ELU / log_softmax of GAT.forward :236-237).
//
// The reference builds the (N, N, 2F) concatenation [Wh_i || Wh_j] and
// multiplies it by `a` (models.py:212-220): e_ij = a1.Wh_i + a2.Wh_j.  We use
// that decomposition directly (s_i + t_j, 2NF MACs instead of 2N^2F), which
// is exact up to fp32 reassociation.  One workgroup (4 waves) per segment
// (scene for the intra-group graph, the scene's groups for the inter-group
// graph); Wh is LDS-resident (odd row stride), the attention of a 16-row
// block lives in registers and both products (att @ Wh, and the backward's
// dhp @ Wh^T / att^T @ dhp) run on fp32 MFMA tiles (below).
//
// Multi-head (the batched GAT of the sgangat family, sgan/GAT.py:6-55 text):
// Wh holds all heads side by side (n x heads*F, the output of one X @ [w_0 |
// .. | w_{H-1}] transform), `a` is heads x [a_src | a_dst], and the workgroup
// grid runs over (segment, head) pairs; head h writes columns [hF, hF + F) of
// y, so the concatenation of heads (GAT.py:86) is free.  `bias` (F, shared by
// the heads, GAT.py:41) is added to the aggregate before the epilogue.
#include "sgg_common.h"

namespace sgg {

// phase timestamps of workgroup 0's first (segment, head) (tools/gat_layer_probe.hip)
#ifdef SGG_GAT_PROF
__device__ long long g_gat_prof[64];
#define GPMARK(i) \
  if (threadIdx.x == 0 && blockIdx.x == 0) g_gat_prof[i] = wall_clock64();
#else
#define GPMARK(i)
#endif

constexpr int kGatThreads = 256;
constexpr int kGatWaves = kGatThreads / 64;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float lrelu(float x, float alpha) { return x > 0.f ? x : alpha * x; }

// LDS row stride of a staged node tile: F rounded up to the 4-feature MFMA
// k-step (the pad columns hold zeros), odd
__host__ __device__ __forceinline__ int gat_fs(int F) { return ((F + 3) & ~3) | 1; }
__host__ __device__ __forceinline__ int gat_r16(int n) { return (n + 15) & ~15; }

// A rows x cols block into LDS with 16 loads in flight per thread (a loop
// of one load and one store per element waits a memory latency per
// element): ld(r, c) is called with indices clamped into [0, nv) x [0, cv)
// and its value masked to zero outside; st(r, c, v) stores it
template <typename Ld, typename St>
__device__ __forceinline__ void stage_block(int rows, int cols, int nv, int cv, Ld ld, St st) {
  constexpr int kU = 16;
  const int total = rows * cols;
  const int dq = kGatThreads / cols, dr = kGatThreads - dq * cols;   // one step of kGatThreads elements
  for (int base = 0; base < total; base += kU * kGatThreads) {
    const int e0 = base + (int)threadIdx.x;
    const int r0 = e0 / cols, c0 = e0 - r0 * cols;
    float v[kU];
    int r = r0, c = c0;
#pragma unroll
    for (int u = 0; u < kU; ++u) {   // (slots past the block load a clamped element: no branch)
      v[u] = keep_if(ld(min(r, nv - 1), min(c, cv - 1)), r < nv && c < cv);
      r += dq;
      c += dr;
      if (c >= cols) {
        c -= cols;
        ++r;
      }
    }
    r = r0;
    c = c0;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (e0 + u * kGatThreads < total) st(r, c, v[u]);
      r += dq;
      c += dr;
      if (c >= cols) {
        c -= cols;
        ++r;
      }
    }
  }
}

// Both kernels work on 16 x 16 x 4 fp32 MFMA tiles (exact fp32 products;
// v_mfma_f32_16x16x4_f32: A[i = lane & 15][k = lane >> 4], B[k = lane >> 4][c
// = lane & 15], C rows 4 (lane >> 4) + v, column lane & 15).  One workgroup
// per (segment, head); wave w takes the 16-node row blocks w, w + 4, ...
//
// Forward: the attention rows of a row block are built directly in the A
// operand layout (lane = row i, k-step m = nodes 4m + (lane >> 4)), so the
// softmax needs two cross-lane steps per reduction and the aggregation
// att @ Wh reads only Wh (LDS) -- no attention matrix is stored.

// s_i = Wh_i . a_src, t_i = Wh_i . a_dst (a_s / a_d: LDS copies) and the
// labels of rows [0, nr) (Ws rows >= n are zero): each row's dot products
// split over 256 / nr lanes (a shuffle tree joins them); the caller barriers
__device__ __forceinline__ void gat_scores(const float* Ws, int Fs, const float* a_s, const float* a_d, int F,
                                           const float* labels, int mode, int o, int n, int nr, float* ss, float* ts,
                                           float* lab, const float* Ds = nullptr, float* rsum = nullptr) {
  int sp = 1;   // lanes per row: a power of 2 (groups of aligned lanes)
  while (sp < 16 && 2 * sp * nr <= kGatThreads) sp *= 2;
  const int part = threadIdx.x & (sp - 1);
  for (int r = threadIdx.x / sp; r < nr; r += kGatThreads / sp) {
    // (fp64: the products of two floats are exact, so the scores are the
    // rounded exact dot products whatever the lane split)
    double s = 0.0, t = 0.0;
    float sd = 0.f;
    for (int f = part; f < F; f += sp) {
      const double w = Ws[r * Fs + f];
      s = fma(w, (double)a_s[f], s);
      t = fma(w, (double)a_d[f], t);
      if (Ds) sd += Ds[r * Fs + f];
    }
    for (int o2 = 1; o2 < sp; o2 <<= 1) {
      s += __shfl_xor(s, o2);
      t += __shfl_xor(t, o2);
      sd += __shfl_xor(sd, o2);
    }
    if (part == 0) {
      ss[r] = (float)s;
      ts[r] = (float)t;
      if (rsum) rsum[r] = sd;
      lab[r] = (mode == 0 && r < n) ? labels[o + r] : 0.f;
    }
  }
}

// softmax attention + aggregation + bias + epilogue of one (segment, head)
// from the LDS tile Ws (nr x Fs, zero rows past n) and its scores
template <int NM>
__device__ __forceinline__ void gat_attend(const float* Ws, int Fs, const float* ss, const float* ts,
                                           const float* lab, int o, int n, int nr, int F, int HF, int c0, float alpha,
                                           int mode, int epi, const float* __restrict__ bias, float* __restrict__ hp,
                                           float* __restrict__ y, int ldy) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int nct = (F + 15) >> 4;
  const int nm = nr >> 2;
  for (int rb = wave; 16 * rb < n; rb += kGatWaves) {
    const int i = 16 * rb + r16;
    const bool iv = i < n;
    const float si = ss[i], li = lab[i];
    float p[NM];
    float mx = -INFINITY;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      p[m] = -INFINITY;
      if (m < nm) {
        const int j = 4 * m + q;
        const bool edge = iv && j < n && (mode == 1 || i == j || (li != 0.f && li == lab[j]));
        if (edge) {
          p[m] = lrelu(si + ts[j], alpha);
          mx = fmaxf(mx, p[m]);
        }
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float sum = 0.f;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const float e = p[m] == -INFINITY ? 0.f : expf(p[m] - mx);
      p[m] = e;
      sum += e;
    }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float inv = iv ? 1.f / sum : 0.f;
#pragma unroll
    for (int m = 0; m < NM; ++m) p[m] *= inv;
    // out = att @ Wh (+ bias), 16-feature column tiles
    floatx4 hv[8];
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) {
      hv[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (ct < nct) {
        const int fb = min(16 * ct + r16, F - 1);
#pragma unroll
        for (int m = 0; m < NM; ++m)
          if (m < nm) hv[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(p[m], Ws[(4 * m + q) * Fs + fb], hv[ct], 0, 0, 0);
        const float bv = (bias && 16 * ct + r16 < F) ? bias[16 * ct + r16] : 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) hv[ct][v] += bv;
      }
    }
    // epilogue per output row 16 rb + 4 q + v, feature 16 ct + r16
    float lse[4] = {0.f, 0.f, 0.f, 0.f};
    if (epi == 2) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float zm = -INFINITY;
#pragma unroll
        for (int ct = 0; ct < 8; ++ct)
          if (ct < nct && 16 * ct + r16 < F) zm = fmaxf(zm, elu(hv[ct][v]));
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) zm = fmaxf(zm, __shfl_xor(zm, o2));
        float se = 0.f;
#pragma unroll
        for (int ct = 0; ct < 8; ++ct)
          if (ct < nct && 16 * ct + r16 < F) se += expf(elu(hv[ct][v]) - zm);
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) se += __shfl_xor(se, o2);
        lse[v] = zm + logf(se);
      }
    }
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) {
      const int f = 16 * ct + r16;
      if (ct < nct && f < F) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int io = 16 * rb + 4 * q + v;
          if (io < n) {
            const float h = hv[ct][v];
            const float z = epi ? elu(h) : h;
            if (epi) hp[(size_t)(o + io) * HF + c0 + f] = h;
            y[(size_t)(o + io) * ldy + c0 + f] = epi == 2 ? z - lse[v] : z;
          }
        }
      }
    }
  }
}

// rows past the last segment (zero-padded group buffers): zero outputs
// (blk / nblk: this workgroup's index among the nblk serving the rows)
__device__ __forceinline__ void gat_zero_pad_rows(int tot, int nrows, int HF, float* y, int ldy, float* hp,
                                                  int blk = -1, int nblk = 0) {
  if (blk < 0) {
    blk = blockIdx.x;
    nblk = gridDim.x;
  }
  for (size_t e = (size_t)tot * HF + (size_t)blk * kGatThreads + threadIdx.x; e < (size_t)nrows * HF;
       e += (size_t)nblk * kGatThreads) {
    const size_t r = e / HF, c = e - r * HF;
    y[r * ldy + c] = 0.f;
    if (hp) hp[e] = 0.f;
  }
}

template <int NM>   // 4-node k-steps held per lane: segments of <= 4 NM nodes
__global__ void __launch_bounds__(kGatThreads) gat_fwd_kernel(
    const float* __restrict__ Wh, int heads, const float* __restrict__ a_src, const float* __restrict__ a_dst, int lda,
    const float* __restrict__ bias, const float* __restrict__ labels, const int32_t* __restrict__ seg_off, int nseg,
    int nrows, int F, float alpha, int mode, int epi, int max_seg, float* __restrict__ hp, float* __restrict__ y,
    int ldy) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Fs = gat_fs(F), F4 = (F + 3) & ~3;
  const int nmax = gat_r16(max_seg);
  const int HF = heads * F;
  gat_zero_pad_rows(seg_off[nseg], nrows, HF, y, ldy, epi ? hp : nullptr);
  float* Ws = reinterpret_cast<float*>(smem);   // nmax x Fs
  float* ss = Ws + nmax * Fs;                   // nmax
  float* ts = ss + nmax;                        // nmax
  float* lab = ts + nmax;                       // nmax
  float* al = lab + nmax;                       // 2F: the head's a_src | a_dst
  for (int gh = blockIdx.x; gh < nseg * heads; gh += gridDim.x) {
    const int g = gh / heads, hd = gh - g * heads;
    const int o = seg_off[g];
    // (a segment larger than the caller's max_seg would overrun the LDS plan:
    // clamped, memory-safe; the host builds max_seg from the same offsets)
    const int n = min(seg_off[g + 1] - o, nmax);
    if (n <= 0) continue;
    const int c0 = hd * F;
    const int nr = gat_r16(n);
    stage_block(nr, F4, n, F, [&](int r, int f) { return Wh[(size_t)(o + r) * HF + c0 + f]; },
                [&](int r, int f, float v) { Ws[r * Fs + f] = v; });
    for (int f = threadIdx.x; f < 2 * F; f += kGatThreads)
      al[f] = f < F ? a_src[(size_t)lda * hd + f] : a_dst[(size_t)lda * hd + f - F];
    __syncthreads();
    gat_scores(Ws, Fs, al, al + F, F, labels, mode, o, n, nr, ss, ts, lab);
    __syncthreads();
    gat_attend<NM>(Ws, Fs, ss, ts, lab, o, n, nr, F, HF, c0, alpha, mode, epi, bias, hp, y, ldy);
    __syncthreads();  // LDS reused by the next segment
  }
}

// One batched-GAT layer of the sgangat family in one launch (GAT.py:71-86
// text: InstanceNorm1d over the scene's nodes, then the multi-head attention
// layer): per (segment, head) the segment's input rows (one or two column
// blocks: [h | pool_h] without a concatenation) are staged in LDS, normalised
// per feature (the two-pass fp64 statistics of seg_norm_fwd_kernel, norm.hip,
// same row phases and combine order), transformed by the head's W (K x F, the
// module's (heads, K, F) layout: no permuted copy) on the MFMA -- fp32 16x16x4,
// or bf16 16x16x32 with xw_bf16_kernel's rounding and k order -- and attended.
// When saving (training), head 0 writes the normalised rows and 1 / std and
// every head its Wh block: the backward's operands.
struct GatLayerArgs {
  const float *x1, *x2;
  int ld1, K1, ld2, K2;
  const float *w, *a_src, *a_dst, *bias;
  const int32_t* seg_off;
  int nseg, nrows, heads, F, epi, max_seg;
  float alpha, eps;
  float *xn, *rstd, *wh, *hp, *y;
  int ldy;
};

__host__ __device__ __forceinline__ int gat_layer_kp(int K) { return (K + 31) & ~31; }

// the layer over one set: workgroups blk = 0 .. nblk - 1 of those serving it
template <int NM, bool BF16>
__device__ __forceinline__ void gat_layer_fwd_body(const GatLayerArgs& p, int blk, int nblk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int F = p.F, K = p.K1 + p.K2, HF = p.heads * F;
  const int Fs = gat_fs(F);
  const int Kp = gat_layer_kp(K), Ks = Kp + 1;
  const int F16 = (F + 15) & ~15, Wp = F16 + 1;
  const int nmax = gat_r16(p.max_seg);
  GPMARK(0);
  // the first work item's offsets with the total (independent loads)
  const int gfirst = min(blk / p.heads, p.nseg);
  const int tot = p.seg_off[p.nseg], ofirst = p.seg_off[gfirst], efirst = p.seg_off[min(gfirst + 1, p.nseg)];
  gat_zero_pad_rows(tot, p.nrows, HF, p.y, p.ldy, p.epi ? p.hp : nullptr, blk, nblk);
  if (p.wh) {   // the saved operands too (the backward's products run over all rows)
    gat_zero_pad_rows(tot, p.nrows, HF, p.wh, HF, nullptr, blk, nblk);
    gat_zero_pad_rows(tot, p.nrows, K, p.xn, K, nullptr, blk, nblk);
  }
  double(*red)[64] = reinterpret_cast<double(*)[64]>(smem);   // 8 x 64
  float* Xs = reinterpret_cast<float*>(smem + 8 * 64 * sizeof(double));   // nmax x Ks
  float* Wl = Xs + nmax * Ks;                   // Kp x Wp
  float* Ws = Wl + Kp * Wp;                     // nmax x Fs
  float* ss = Ws + nmax * Fs;
  float* ts = ss + nmax;
  float* lab = ts + nmax;
  float* al = lab + nmax;                       // 3F: the head's a_src | a_dst, the bias
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int fl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  for (int gh = blk; gh < p.nseg * p.heads; gh += nblk) {
    const int g = gh / p.heads, hd = gh - g * p.heads;
    const int o = gh == blk ? ofirst : p.seg_off[g];
    const int n = min((gh == blk ? efirst : p.seg_off[g + 1]) - o, nmax);   // (LDS plan bound)
    if (n <= 0) continue;
    const int c0 = hd * F;
    const int nr = gat_r16(n);
    const bool save = p.wh != nullptr;
    GPMARK(1);
    const float* wg = p.w + (size_t)hd * K * F;
    float av = 0.f;   // thread t < 3F: a_src | a_dst | bias entry t (issued with the tiles' loads)
    {
      const int t = threadIdx.x;
      if (t < F) av = p.a_src[(size_t)F * hd + t];
      else if (t < 2 * F) av = p.a_dst[(size_t)F * hd + t - F];
      else if (t < 3 * F && p.bias) av = p.bias[t - 2 * F];
    }
    stage_block(
        nr, Kp, n, K,
        [&](int r, int k) {
          return k < p.K1 ? p.x1[(size_t)(o + r) * p.ld1 + k] : p.x2[(size_t)(o + r) * p.ld2 + (k - p.K1)];
        },
        [&](int r, int k, float v) { Xs[r * Ks + k] = v; });
    stage_block(Kp, F16, K, F, [&](int k, int f) { return wg[(size_t)k * F + f]; },
                [&](int k, int f, float v) { Wl[k * Wp + f] = v; });
    if ((int)threadIdx.x < 3 * F) al[threadIdx.x] = av;
    for (int t = threadIdx.x + kGatThreads; t < 3 * F; t += kGatThreads)   // (F > 85)
      al[t] = t < F ? p.a_src[(size_t)F * hd + t] : t < 2 * F ? p.a_dst[(size_t)F * hd + t - F]
                                                             : (p.bias ? p.bias[t - 2 * F] : 0.f);
    __syncthreads();
    GPMARK(2);
    // instance norm per feature over the segment's rows (in place)
    // (one pass: fp64 sum and sum of squares -- exact enough for fp32 data
    // that var = E[x^2] - mean^2 loses nothing at fp32 -- two chains each)
    for (int f0 = 0; f0 < K; f0 += 64) {
      const int f = f0 + fl;
      const bool fok = f < K;
      double s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
      if (fok) {
        int r = ph;
        for (; r + 4 < n; r += 8) {
          const double x0 = Xs[r * Ks + f], x1 = Xs[(r + 4) * Ks + f];
          s0 += x0;
          s1 += x1;
          q0 = fma(x0, x0, q0);
          q1 = fma(x1, x1, q1);
        }
        if (r < n) {
          const double x0 = Xs[r * Ks + f];
          s0 += x0;
          q0 = fma(x0, x0, q0);
        }
      }
      red[ph][fl] = s0 + s1;
      red[4 + ph][fl] = q0 + q1;
      __syncthreads();
      const double meand = ((red[0][fl] + red[1][fl]) + (red[2][fl] + red[3][fl])) / n;
      const double sq = ((red[4][fl] + red[5][fl]) + (red[6][fl] + red[7][fl])) / n;
      __syncthreads();
      const float mean = (float)meand;
      const double vard = sq - meand * meand;
      const float rs = 1.f / sqrtf((float)(vard > 0.0 ? vard : 0.0) + p.eps);
      if (fok) {
        for (int r = ph; r < n; r += 4) {
          const float v = (Xs[r * Ks + f] - mean) * rs;
          Xs[r * Ks + f] = v;
          if (save && hd == 0) p.xn[(size_t)(o + r) * K + f] = v;
        }
        if (save && hd == 0 && ph == 0) p.rstd[(size_t)g * K + f] = rs;
      }
    }
    __syncthreads();
    GPMARK(3);
    // Wh = Xn W_h: (row block, column tile) MFMA tiles over the waves
    const int nrb = nr >> 4, nct = F16 >> 4;
    for (int tile = wave; tile < nrb * nct; tile += kGatWaves) {
      const int rb = tile / nct, ct = tile - rb * nct;
      floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
      const float* xr = Xs + (16 * rb + r16) * Ks;
      if constexpr (BF16) {
        for (int k0 = 0; k0 < Kp; k0 += 32) {
          const int kb = k0 + 8 * q;
          bf16x8 a, b;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            a[j] = (__bf16)xr[kb + j];
            b[j] = (__bf16)Wl[(kb + j) * Wp + 16 * ct + r16];
          }
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
        }
      } else {
        for (int k0 = 0; k0 < K; k0 += 4)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[k0 + q], Wl[(k0 + q) * Wp + 16 * ct + r16], acc, 0, 0, 0);
      }
      const int f = 16 * ct + r16;
      if (f < F) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int r = 16 * rb + 4 * q + v;
          Ws[r * Fs + f] = acc[v];
          if (save && r < n) p.wh[(size_t)(o + r) * HF + c0 + f] = acc[v];
        }
      }
    }
    __syncthreads();
    GPMARK(4);
    gat_scores(Ws, Fs, al, al + F, F, nullptr, 1, o, n, nr, ss, ts, lab);
    __syncthreads();
    GPMARK(5);
    gat_attend<NM>(Ws, Fs, ss, ts, lab, o, n, nr, F, HF, c0, p.alpha, 1, p.epi, p.bias ? al + 2 * F : nullptr, p.hp,
                   p.y, p.ldy);
    GPMARK(6);
    __syncthreads();  // LDS reused by the next segment
    GPMARK(7);
  }
}

template <int NM, bool BF16>
__global__ void __launch_bounds__(kGatThreads) gat_layer_fwd_kernel(const GatLayerArgs p) {
  gat_layer_fwd_body<NM, BF16>(p, blockIdx.x, gridDim.x);
}

// two sets (batches) through the same layer weights in one launch
// (sgg_gat_layer_fwd2): workgroups [0, g1) serve set a, [g1, grid) set b
template <int NM, bool BF16>
__global__ void __launch_bounds__(kGatThreads) gat_layer_fwd2_kernel(const GatLayerArgs a, const GatLayerArgs b, int g1) {
  if ((int)blockIdx.x < g1)
    gat_layer_fwd_body<NM, BF16>(a, blockIdx.x, g1);
  else
    gat_layer_fwd_body<NM, BF16>(b, blockIdx.x - g1, gridDim.x - g1);
}

static size_t gat_layer_lds(int K, int F, int max_seg) {
  const size_t nm = gat_r16(max_seg), Kp = gat_layer_kp(K);
  return 8 * 64 * sizeof(double) +
         sizeof(float) * (nm * (Kp + 1) + Kp * (((F + 15) & ~15) + 1) + nm * gat_fs(F) + 3 * nm + 3 * F) + 16;
}

// Backward.  Per row block (in the C layout: lane = column j, rows 4 (lane >>
// 4) + v): the attention recomputed, datt = dhp @ Wh^T on MFMA, the softmax
// and LeakyReLU backward to dz, its row sums (ds) and per-block column sums
// (dt, summed over the blocks in order afterwards); the attention goes to LDS
// for dWh = att^T @ dhp (MFMA over the rows) + ds a_src + dt a_dst.
// With the slabs (sgg_gat_bwd_ex) each (segment, head) also writes its
// partials of the parameter gradients: da_src = Wh^T ds, da_dst = Wh^T dt
// (pda, 2F floats) and the bias gradient's column sums of dhp (pdb, F doubles:
// a near-cancelling sum, the next layer's instance norm removes each
// feature's scene mean); gat_param_reduce_kernel sums them in a fixed order.
template <int NJT>  // 16-node column tiles: segments of <= 16 NJT nodes
__global__ void __launch_bounds__(kGatThreads) gat_bwd_kernel(
    const float* __restrict__ Wh, int heads, const float* __restrict__ a_src, const float* __restrict__ a_dst, int lda,
    const float* __restrict__ labels, const int32_t* __restrict__ seg_off, int nseg, int nrows, int F, float alpha,
    int mode, int epi, int max_seg, const float* __restrict__ hp, const float* __restrict__ y,
    const float* __restrict__ dy, int lddy, float* __restrict__ dWh, float* __restrict__ ds_out,
    float* __restrict__ dt_out, float* __restrict__ pda, double* __restrict__ pdb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int gfirst = min((int)blockIdx.x / heads, nseg);
  const int tot = seg_off[nseg], ofirst = seg_off[gfirst], efirst = seg_off[min(gfirst + 1, nseg)];
  {  // rows past the last segment: zero gradients
    const size_t r0 = tot, w = (size_t)heads * (F + 2);
    for (size_t e = r0 * w + blockIdx.x * kGatThreads + threadIdx.x; e < (size_t)nrows * w;
         e += (size_t)gridDim.x * kGatThreads) {
      const size_t r = e / w, c = e - r * w;
      if (c < (size_t)heads * F) dWh[r * heads * F + c] = 0.f;
      else if (!ds_out) continue;
      else if (c < (size_t)heads * (F + 1)) ds_out[r * heads + c - (size_t)heads * F] = 0.f;
      else dt_out[r * heads + c - (size_t)heads * (F + 1)] = 0.f;
    }
  }
  const int Fs = gat_fs(F), F4 = (F + 3) & ~3;
  const int nmax = gat_r16(max_seg), Na = nmax + 4;
  float* Ws = reinterpret_cast<float*>(smem);  // nmax x Fs
  float* Ds = Ws + nmax * Fs;                  // nmax x Fs  (d hp)
  float* At = Ds + nmax * Fs;                  // nmax x Na  (att)
  float* ss = At + nmax * Na;
  float* ts = ss + nmax;
  float* lab = ts + nmax;
  float* dss = lab + nmax;
  float* dts = dss + nmax;
  float* rsum = dts + nmax;                    // epilogue 2: row sums of dy
  float* dtp = rsum + nmax;                    // (nmax / 16) x nmax column partials of dz
  float* al = dtp + (nmax / 16) * nmax;        // 2F: the head's a_src | a_dst
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int HF = heads * F;
  const int nct = (F + 15) >> 4;
  for (int gh = blockIdx.x; gh < nseg * heads; gh += gridDim.x) {
    const int g = gh / heads, hd = gh - g * heads;
    const int o = gh == (int)blockIdx.x ? ofirst : seg_off[g];
    const int n = min((gh == (int)blockIdx.x ? efirst : seg_off[g + 1]) - o, nmax);   // (LDS plan bound)
    if (n <= 0) {
      for (int c = threadIdx.x; c < 3 * F; c += kGatThreads) {
        if (c < 2 * F) {
          if (pda) pda[(size_t)gh * 2 * F + c] = 0.f;
        } else if (pdb) {
          pdb[(size_t)gh * F + c - 2 * F] = 0.0;
        }
      }
      continue;
    }
    const float* as = al;
    const float* ad = al + F;
    const int c0 = hd * F;
    const int nr = gat_r16(n), nrb = nr >> 4;
    for (int f = threadIdx.x; f < 2 * F; f += kGatThreads)
      al[f] = f < F ? a_src[(size_t)lda * hd + f] : a_dst[(size_t)lda * hd + f - F];
    stage_block(nr, F4, n, F, [&](int r, int f) { return Wh[(size_t)(o + r) * HF + c0 + f]; },
                [&](int r, int f, float v) { Ws[r * Fs + f] = v; });
    stage_block(
        nr, F4, n, F,
        [&](int r, int f) {
          const size_t row = (size_t)(o + r);
          const float d = dy[row * lddy + c0 + f];
          return epi == 1 ? d * elu_grad(hp[row * HF + c0 + f]) : d;
        },
        [&](int r, int f, float v) { Ds[r * Fs + f] = v; });
    __syncthreads();
    gat_scores(Ws, Fs, as, ad, F, labels, mode, o, n, nr, ss, ts, lab, Ds, rsum);
    __syncthreads();
    if (epi == 2) {   // d hp = (dy - softmax(y) sum(dy)) * ELU'(hp)
      stage_block(
          n, F, n, F,
          [&](int r, int f) {
            const size_t row = (size_t)(o + r);
            return (Ds[r * Fs + f] - expf(y[row * F + f]) * rsum[r]) * elu_grad(hp[row * HF + c0 + f]);
          },
          [&](int r, int f, float v) { Ds[r * Fs + f] = v; });
      __syncthreads();
    }
    for (int rb = wave; rb < nrb; rb += kGatWaves) {
      float sv[4], lv[4];
      bool iv[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int i = 16 * rb + 4 * q + v;
        iv[v] = i < n;
        sv[v] = ss[i];
        lv[v] = lab[i];
      }
      float tj[NJT], att[NJT][4];
      float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const int j = 16 * jt + r16;
        const bool jv = jt < nrb && j < n;
        tj[jt] = jt < nrb ? ts[j] : 0.f;
        const float lj = jt < nrb ? lab[j] : 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int i = 16 * rb + 4 * q + v;
          const bool edge = jv && iv[v] && (mode == 1 || i == j || (lv[v] != 0.f && lv[v] == lj));
          att[jt][v] = edge ? lrelu(sv[v] + tj[jt], alpha) : -INFINITY;
          mx[v] = fmaxf(mx[v], att[jt][v]);
        }
      }
      float inv[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) mx[v] = fmaxf(mx[v], __shfl_xor(mx[v], o2));
        float sum = 0.f;
#pragma unroll
        for (int jt = 0; jt < NJT; ++jt) {
          const float e = att[jt][v] == -INFINITY ? 0.f : expf(att[jt][v] - mx[v]);
          att[jt][v] = e;
          sum += e;
        }
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) sum += __shfl_xor(sum, o2);
        inv[v] = iv[v] ? 1.f / sum : 0.f;
      }
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt)
#pragma unroll
        for (int v = 0; v < 4; ++v) att[jt][v] *= inv[v];
      // datt_ij = dhp_i . Wh_j
      floatx4 da[NJT];
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) da[jt] = floatx4{0.f, 0.f, 0.f, 0.f};
      const float* Dr = Ds + (16 * rb + r16) * Fs + q;
      for (int k = 0; k < F4; k += 4) {
        const float av = Dr[k];
#pragma unroll
        for (int jt = 0; jt < NJT; ++jt)
          if (jt < nrb) da[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, Ws[(16 * jt + r16) * Fs + k + q], da[jt], 0, 0, 0);
      }
      float dot[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt)
#pragma unroll
        for (int v = 0; v < 4; ++v) dot[v] = fmaf(att[jt][v], da[jt][v], dot[v]);
      float dsr[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) dot[v] += __shfl_xor(dot[v], o2);
        dsr[v] = 0.f;
      }
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        if (jt < nrb) {
          float cp = 0.f;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const float de = att[jt][v] * (da[jt][v] - dot[v]);
            const float dz = (sv[v] + tj[jt]) > 0.f ? de : alpha * de;
            dsr[v] += dz;
            cp += dz;
            At[(16 * rb + 4 * q + v) * Na + 16 * jt + r16] = att[jt][v];
          }
          cp += __shfl_xor(cp, 16);
          cp += __shfl_xor(cp, 32);
          if (q == 0) dtp[rb * nmax + 16 * jt + r16] = cp;
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
#pragma unroll
        for (int o2 = 1; o2 < 16; o2 <<= 1) dsr[v] += __shfl_xor(dsr[v], o2);
        if (r16 == 0) dss[16 * rb + 4 * q + v] = dsr[v];
      }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < nr; j += kGatThreads) {
      float acc = 0.f;
      for (int rb = 0; rb < nrb; ++rb) acc += dtp[rb * nmax + j];
      dts[j] = acc;
      if (j < n && ds_out) {
        ds_out[(size_t)(o + j) * heads + hd] = dss[j];
        dt_out[(size_t)(o + j) * heads + hd] = acc;
      }
    }
    __syncthreads();
    // parameter-gradient partials of this (segment, head): LDS reads only
    for (int c = threadIdx.x; c < 3 * F; c += kGatThreads) {
      if (c < 2 * F) {
        if (pda) {
          const int f = c < F ? c : c - F;
          const float* wv = c < F ? dss : dts;
          float acc = 0.f;
          for (int i = 0; i < n; ++i) acc = fmaf(Ws[i * Fs + f], wv[i], acc);
          pda[(size_t)gh * 2 * F + c] = acc;
        }
      } else if (pdb) {
        const int f = c - 2 * F;
        double acc = 0.0;
        for (int i = 0; i < n; ++i) acc += (double)Ds[i * Fs + f];
        pdb[(size_t)gh * F + f] = acc;
      }
    }
    // dWh_j = sum_i att_ij dhp_i + ds_j a_src + dt_j a_dst
    for (int jb = wave; jb < nrb; jb += kGatWaves) {
      for (int ct = 0; ct < nct; ++ct) {
        const int fb = min(16 * ct + r16, F - 1);
        floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int m = 0; m < nr; m += 4)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(At[(m + q) * Na + 16 * jb + r16], Ds[(m + q) * Fs + fb], acc, 0,
                                                     0, 0);
        const int f = 16 * ct + r16;
        if (f < F) {
          const float sf = as[f], df = ad[f];
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int j = 16 * jb + 4 * q + v;
            if (j < n) dWh[(size_t)(o + j) * HF + c0 + f] = acc[v] + (dss[j] * sf + dts[j] * df);
          }
        }
      }
    }
    __syncthreads();  // LDS reused by the next segment
  }
}

// da_src / da_dst (heads x F each) and dbias (F, summed over the heads) from
// the (segment, head) partials of gat_bwd_kernel: one workgroup per output,
// a fixed-order fp64 tree over the segments
__global__ void __launch_bounds__(256) gat_param_reduce_kernel(const float* __restrict__ pda,
                                                               const double* __restrict__ pdb, int nseg, int heads,
                                                               int F, float* __restrict__ da_src,
                                                               float* __restrict__ da_dst, float* __restrict__ dbias) {
  __shared__ double red[256];
  const int e = blockIdx.x, na = heads * 2 * F;
  const int t = threadIdx.x;
  double acc = 0.0;
  if (e < na) {
    const int h = e / (2 * F), c = e - h * 2 * F;
    for (int g = t; g < nseg; g += 256) acc += (double)pda[((size_t)g * heads + h) * 2 * F + c];
  } else {
    const int f = e - na;
    for (int gh = t; gh < nseg * heads; gh += 256) acc += pdb[(size_t)gh * F + f];
  }
  red[t] = acc;
  __syncthreads();
  for (int s2 = 128; s2 > 0; s2 >>= 1) {
    if (t < s2) red[t] += red[t + s2];
    __syncthreads();
  }
  if (t == 0) {
    if (e < na) {
      const int h = e / (2 * F), c = e - h * 2 * F;
      if (c < F) da_src[h * F + c] = (float)red[0];
      else da_dst[h * F + c - F] = (float)red[0];
    } else {
      dbias[e - na] = (float)red[0];
    }
  }
}

static size_t gat_fwd_lds(int F, int max_seg) {
  const size_t nm = gat_r16(max_seg);
  return sizeof(float) * (nm * gat_fs(F) + 3 * nm + 2 * F) + 16;
}
static size_t gat_bwd_lds(int F, int max_seg) {
  const size_t nm = gat_r16(max_seg);
  return sizeof(float) * (2 * nm * gat_fs(F) + nm * (nm + 4) + 6 * nm + (nm / 16) * nm + 2 * F) + 16;
}

}  // namespace sgg

using namespace sgg;

static int gat_args_ok(const char* who, const float* Wh, int heads, const float* a, const float* labels,
                       const int32_t* off, int nseg, int n, int F, int mode, int epi, int max_seg) {
  SGG_CHECK_ARG(Wh && a && off, "%s: null pointer", who);
  SGG_CHECK_ARG(mode == 1 || labels, "%s: mask_mode 0 needs labels", who);
  SGG_CHECK_ARG(nseg >= 0 && n >= 0, "%s: bad sizes", who);
  SGG_CHECK_ARG(F >= 1 && F <= 128, "%s: F=%d outside [1, 128]", who, F);
  SGG_CHECK_ARG(heads >= 1 && heads <= 64, "%s: heads=%d outside [1, 64]", who, heads);
  SGG_CHECK_ARG(mode == 0 || mode == 1, "%s: bad mask_mode", who);
  SGG_CHECK_ARG(epi >= 0 && epi <= 2, "%s: bad epilogue", who);
  SGG_CHECK_ARG(epi != 2 || heads == 1, "%s: the log_softmax epilogue is single-head", who);
  SGG_CHECK_ARG(max_seg >= 1 && max_seg <= SGG_GAT_MAX_NODES, "%s: max segment %d outside [1, %d]", who, max_seg,
                SGG_GAT_MAX_NODES);
  return 0;
}

static int gat_grid(int nseg, int heads) {
  const long long w = (long long)nseg * heads;
  return w < 1 ? 1 : w < 16384 ? (int)w : 16384;
}

static int gat_fwd_launch(const char* who, const float* Wh, int heads, const float* as, const float* ad, int lda,
                          const float* bias, const float* labels, const int32_t* seg_off, int nseg, int n, int F,
                          float alpha, int mask_mode, int epilogue, int max_seg, float* hp, float* y, int ldy,
                          void* stream) {
  int rc = gat_args_ok(who, Wh, heads, as, labels, seg_off, nseg, n, F, mask_mode, epilogue, max_seg);
  if (rc) return rc;
  SGG_CHECK_ARG(ad, "%s: null a_dst", who);
  SGG_CHECK_ARG(y && (epilogue == 0 || hp), "%s: null output", who);
  SGG_CHECK_ARG(ldy >= heads * F, "%s: ldy < heads * F", who);
  SGG_CHECK_ARG(epilogue != 2 || ldy == F, "%s: log_softmax epilogue needs a dense y (ldy == F)", who);
  if (nseg == 0 && n == 0) return 0;   // (rows but no segments: the kernel zeroes the rows)
  auto k = max_seg <= 32 ? gat_fwd_kernel<8> : max_seg <= 64 ? gat_fwd_kernel<16> : gat_fwd_kernel<32>;
  hipLaunchKernelGGL(k, dim3(gat_grid(nseg, heads)), dim3(kGatThreads), gat_fwd_lds(F, max_seg), (hipStream_t)stream,
                     Wh, heads, as, ad, lda, bias, labels, seg_off, nseg, n, F, alpha, mask_mode, epilogue, max_seg,
                     hp, y, ldy);
  SGG_RETURN_LAUNCH(who);
}

static int gat_bwd_launch(const char* who, const float* Wh, int heads, const float* as, const float* ad, int lda,
                          const float* labels, const int32_t* seg_off, int nseg, int n, int F, float alpha,
                          int mask_mode, int epilogue, int max_seg, const float* hp, const float* y, const float* dy,
                          int lddy, float* dWh, float* ds, float* dt, float* pda, double* pdb, void* stream) {
  int rc = gat_args_ok(who, Wh, heads, as, labels, seg_off, nseg, n, F, mask_mode, epilogue, max_seg);
  if (rc) return rc;
  SGG_CHECK_ARG(ad && dy && dWh, "%s: null pointer", who);
  SGG_CHECK_ARG(epilogue == 0 || hp, "%s: epilogue needs hp", who);
  SGG_CHECK_ARG(epilogue != 2 || y, "%s: log_softmax epilogue needs y", who);
  SGG_CHECK_ARG(lddy >= heads * F, "%s: lddy < heads * F", who);
  if (nseg == 0 && n == 0) return 0;
  const size_t lds = gat_bwd_lds(F, max_seg);
  SGG_CHECK_ARG(lds <= 160 * 1024, "%s: segment %d x F %d needs %zu B of LDS", who, max_seg, F, lds);
  auto k = max_seg <= 32 ? gat_bwd_kernel<2> : max_seg <= 64 ? gat_bwd_kernel<4> : gat_bwd_kernel<8>;
  hipLaunchKernelGGL(k, dim3(gat_grid(nseg, heads)), dim3(kGatThreads), lds, (hipStream_t)stream, Wh, heads, as, ad,
                     lda, labels, seg_off, nseg, n, F, alpha, mask_mode, epilogue, max_seg, hp, y, dy, lddy, dWh, ds,
                     dt, pda, pdb);
  SGG_RETURN_LAUNCH(who);
}

extern "C" int sgg_gat_fwd(const float* Wh, int heads, const float* a, const float* bias, const float* labels,
                           const int32_t* seg_off, int nseg, int n, int F, float alpha, int mask_mode, int epilogue,
                           int max_seg, float* hp, float* y, int ldy, void* stream) {
  return gat_fwd_launch("sgg_gat_fwd", Wh, heads, a, a ? a + F : nullptr, 2 * F, bias, labels, seg_off, nseg, n, F,
                        alpha, mask_mode, epilogue, max_seg, hp, y, ldy, stream);
}

extern "C" int sgg_gat_bwd(const float* Wh, int heads, const float* a, const float* labels, const int32_t* seg_off,
                           int nseg, int n, int F, float alpha, int mask_mode, int epilogue, int max_seg,
                           const float* hp, const float* y, const float* dy, int lddy, float* dWh, float* ds,
                           float* dt, void* stream) {
  SGG_CHECK_ARG(ds && dt, "sgg_gat_bwd: null pointer");
  return gat_bwd_launch("sgg_gat_bwd", Wh, heads, a, a ? a + F : nullptr, 2 * F, labels, seg_off, nseg, n, F, alpha,
                        mask_mode, epilogue, max_seg, hp, y, dy, lddy, dWh, ds, dt, nullptr, nullptr, stream);
}

static size_t gat_pda_bytes(int nseg, int heads, int F) {
  return ((size_t)nseg * heads * 2 * F * sizeof(float) + 15) & ~(size_t)15;
}

extern "C" size_t sgg_gat_bwd_ex_work_bytes(int nseg, int heads, int F) {
  if (nseg < 0 || heads < 1 || F < 1) return 0;
  return gat_pda_bytes(nseg, heads, F) + (size_t)nseg * heads * F * sizeof(double);
}

extern "C" int sgg_gat_fwd_ex(const float* Wh, int heads, const float* a_src, const float* a_dst, const float* bias,
                              const float* labels, const int32_t* seg_off, int nseg, int n, int F, float alpha,
                              int mask_mode, int epilogue, int max_seg, float* hp, float* y, int ldy, void* stream) {
  return gat_fwd_launch("sgg_gat_fwd_ex", Wh, heads, a_src, a_dst, F, bias, labels, seg_off, nseg, n, F, alpha,
                        mask_mode, epilogue, max_seg, hp, y, ldy, stream);
}

extern "C" int sgg_gat_bwd_ex(const float* Wh, int heads, const float* a_src, const float* a_dst, const float* labels,
                              const int32_t* seg_off, int nseg, int n, int F, float alpha, int mask_mode, int epilogue,
                              int max_seg, const float* hp, const float* y, const float* dy, int lddy, float* dWh,
                              float* da_src, float* da_dst, float* dbias, void* work, void* stream) {
  SGG_CHECK_ARG(da_src && da_dst && work, "sgg_gat_bwd_ex: null pointer");
  SGG_CHECK_ARG(((uintptr_t)work & 15) == 0, "sgg_gat_bwd_ex: work must be 16-byte aligned");
  float* pda = reinterpret_cast<float*>(work);
  double* pdb = dbias ? reinterpret_cast<double*>(reinterpret_cast<char*>(work) + gat_pda_bytes(nseg, heads, F))
                      : nullptr;
  int rc = gat_bwd_launch("sgg_gat_bwd_ex", Wh, heads, a_src, a_dst, F, labels, seg_off, nseg, n, F, alpha, mask_mode,
                          epilogue, max_seg, hp, y, dy, lddy, dWh, nullptr, nullptr, pda, pdb, stream);
  if (rc) return rc;
  // (no segments: the reduce writes zero gradients)
  hipLaunchKernelGGL(gat_param_reduce_kernel, dim3(heads * 2 * F + (dbias ? F : 0)), dim3(256), 0,
                     (hipStream_t)stream, pda, pdb, nseg, heads, F, da_src, da_dst, dbias);
  SGG_RETURN_LAUNCH("sgg_gat_bwd_ex");
}

extern "C" size_t sgg_gat_layer_lds_bytes(int K, int F, int max_seg) {
  if (K < 1 || F < 1 || max_seg < 1) return 0;
  return gat_layer_lds(K, F, max_seg);
}

static int gat_layer_set_check(const SggGatLayerSet& s, int K, int HF, char which) {
  SGG_CHECK_ARG(s.x1 && s.seg_off && s.y && s.K1 >= 1 && s.ld1 >= s.K1 && (!s.x2 || (s.K2 >= 1 && s.ld2 >= s.K2)) &&
                    s.K1 + (s.x2 ? s.K2 : 0) == K && s.ldy >= HF && s.nseg >= 0 && s.n >= 0,
                "sgg_gat_layer_fwd2: bad set %c", which);
  SGG_CHECK_ARG(s.max_seg >= 1 && s.max_seg <= SGG_GAT_MAX_NODES, "sgg_gat_layer_fwd2: set %c max segment %d",
                which, s.max_seg);
  SGG_CHECK_ARG(!s.wh || (s.xn && s.rstd), "sgg_gat_layer_fwd2: set %c saves without xn / rstd", which);
  return 0;
}

extern "C" int sgg_gat_layer_fwd2(const SggGatLayerSet* sa, const SggGatLayerSet* sb, const float* w,
                                  const float* a_src, const float* a_dst, const float* bias, int heads, int F,
                                  float alpha, float eps, int epilogue, int bf16, void* stream) {
  SGG_CHECK_ARG(sa && sb && w && a_src && a_dst, "sgg_gat_layer_fwd2: null pointer");
  SGG_CHECK_ARG(F >= 1 && F <= 128 && heads >= 1 && heads <= 64, "sgg_gat_layer_fwd2: F=%d heads=%d", F, heads);
  SGG_CHECK_ARG(epilogue == 0 || epilogue == 1, "sgg_gat_layer_fwd2: epilogue must be 0 or 1");
  const int K = sa->K1 + (sa->x2 ? sa->K2 : 0);
  SGG_CHECK_ARG(K >= 1 && K <= 256, "sgg_gat_layer_fwd2: K=%d", K);
  if (int rc = gat_layer_set_check(*sa, K, heads * F, 'a')) return rc;
  if (int rc = gat_layer_set_check(*sb, K, heads * F, 'b')) return rc;
  SGG_CHECK_ARG(epilogue == 0 || (sa->hp && sb->hp), "sgg_gat_layer_fwd2: the ELU epilogue needs hp");
  // one LDS plan for both sets: the larger segment bound
  const int max_seg = sa->max_seg > sb->max_seg ? sa->max_seg : sb->max_seg;
  const size_t lds = gat_layer_lds(K, F, max_seg);
  SGG_CHECK_ARG(lds <= 160 * 1024, "sgg_gat_layer_fwd2: K %d, F %d, %d nodes need %zu B of LDS", K, F, max_seg, lds);
  auto args = [&](const SggGatLayerSet& s) {
    return GatLayerArgs{s.x1, s.x2, s.ld1, s.K1, s.ld2, s.x2 ? s.K2 : 0, w, a_src, a_dst, bias, s.seg_off, s.nseg,
                        s.n, heads, F, epilogue, max_seg, alpha, eps, s.xn, s.rstd, s.wh, s.hp, s.y, s.ldy};
  };
  const int g1 = gat_grid(sa->nseg, heads), g2 = gat_grid(sb->nseg, heads);
  auto k = bf16 ? (max_seg <= 32 ? gat_layer_fwd2_kernel<8, true> : max_seg <= 64 ? gat_layer_fwd2_kernel<16, true>
                                                                                   : gat_layer_fwd2_kernel<32, true>)
                : (max_seg <= 32 ? gat_layer_fwd2_kernel<8, false> : max_seg <= 64 ? gat_layer_fwd2_kernel<16, false>
                                                                                    : gat_layer_fwd2_kernel<32, false>);
  hipLaunchKernelGGL(k, dim3(g1 + g2), dim3(kGatThreads), lds, (hipStream_t)stream, args(*sa), args(*sb), g1);
  SGG_RETURN_LAUNCH("sgg_gat_layer_fwd2");
}

extern "C" int sgg_gat_layer_fwd(const float* x1, int ld1, int K1, const float* x2, int ld2, int K2, const float* w,
                                 const float* a_src, const float* a_dst, const float* bias, const int32_t* seg_off,
                                 int nseg, int n, int heads, int F, float alpha, float eps, int epilogue, int max_seg,
                                 int bf16, float* xn, float* rstd, float* wh, float* hp, float* y, int ldy,
                                 void* stream) {
  const int K = K1 + (x2 ? K2 : 0);
  SGG_CHECK_ARG(x1 && w && a_src && a_dst && seg_off && y, "sgg_gat_layer_fwd: null pointer");
  SGG_CHECK_ARG(K1 >= 1 && ld1 >= K1 && (!x2 || (K2 >= 1 && ld2 >= K2)), "sgg_gat_layer_fwd: bad input blocks");
  SGG_CHECK_ARG(K <= 256, "sgg_gat_layer_fwd: K=%d > 256", K);
  SGG_CHECK_ARG(F >= 1 && F <= 128 && heads >= 1 && heads <= 64, "sgg_gat_layer_fwd: F=%d heads=%d", F, heads);
  SGG_CHECK_ARG(epilogue == 0 || epilogue == 1, "sgg_gat_layer_fwd: epilogue must be 0 or 1");
  SGG_CHECK_ARG(epilogue == 0 || hp, "sgg_gat_layer_fwd: the ELU epilogue needs hp");
  SGG_CHECK_ARG(!wh || (xn && rstd), "sgg_gat_layer_fwd: saving needs xn, rstd and wh");
  SGG_CHECK_ARG(ldy >= heads * F && nseg >= 0 && n >= 0, "sgg_gat_layer_fwd: bad sizes");
  SGG_CHECK_ARG(max_seg >= 1 && max_seg <= SGG_GAT_MAX_NODES, "sgg_gat_layer_fwd: max segment %d outside [1, %d]",
                max_seg, SGG_GAT_MAX_NODES);
  const size_t lds = gat_layer_lds(K, F, max_seg);
  SGG_CHECK_ARG(lds <= 160 * 1024, "sgg_gat_layer_fwd: K %d, F %d, %d nodes need %zu B of LDS", K, F, max_seg, lds);
  if (nseg == 0 && n == 0) return 0;
  GatLayerArgs p{x1, x2, ld1, K1, ld2, x2 ? K2 : 0, w, a_src, a_dst, bias, seg_off, nseg, n, heads, F, epilogue,
                 max_seg, alpha, eps, xn, rstd, wh, hp, y, ldy};
  auto k = bf16 ? (max_seg <= 32 ? gat_layer_fwd_kernel<8, true> : max_seg <= 64 ? gat_layer_fwd_kernel<16, true>
                                                                                  : gat_layer_fwd_kernel<32, true>)
                : (max_seg <= 32 ? gat_layer_fwd_kernel<8, false> : max_seg <= 64 ? gat_layer_fwd_kernel<16, false>
                                                                                   : gat_layer_fwd_kernel<32, false>);
  hipLaunchKernelGGL(k, dim3(gat_grid(nseg, heads)), dim3(kGatThreads), lds, (hipStream_t)stream, p);
  SGG_RETURN_LAUNCH("sgg_gat_layer_fwd");
}
