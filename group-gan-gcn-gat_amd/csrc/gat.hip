// Graph attention over the nodes of each segment (GraphAttentionLayer,
// reference sgan/models.py:184-220; ELU / log_softmax of GAT.forward :236-237).
//
// The reference builds the (N, N, 2F) concatenation [Wh_i || Wh_j] and
// multiplies it by `a` (models.py:212-220): e_ij = a1.Wh_i + a2.Wh_j.  We use
// that decomposition directly (s_i + t_j, 2NF MACs instead of 2N^2F), which
// is exact up to fp32 reassociation.  One workgroup (4 waves) per segment
// (scene for the intra-group graph, the scene's groups for the inter-group
// graph); Wh is LDS-resident with an odd row stride (F | 1) so column walks
// across rows are bank-conflict free; one wave per attention row with lanes
// over j: row max / row sum are wave shuffles (__shfl_xor over 64 lanes).
//
// Multi-head (the batched GAT of the sgangat family, sgan/GAT.py:6-55 text):
// Wh holds all heads side by side (n x heads*F, the output of one X @ [w_0 |
// .. | w_{H-1}] transform), `a` is heads x [a_src | a_dst], and the workgroup
// grid runs over (segment, head) pairs; head h writes columns [hF, hF + F) of
// y, so the concatenation of heads (GAT.py:86) is free.  `bias` (F, shared by
// the heads, GAT.py:41) is added to the aggregate before the epilogue.
#include "sgg_common.h"

namespace sgg {

constexpr int kGatThreads = 256;
constexpr int kGatWaves = kGatThreads / 64;

__device__ __forceinline__ bool gat_edge(int mode, const float* lab, int i, int j) {
  if (mode == 1 || i == j) return true;
  const float li = lab[i];
  return li != 0.f && li == lab[j];
}

__device__ __forceinline__ float lrelu(float x, float alpha) { return x > 0.f ? x : alpha * x; }

// softmax row i over j into att[0..n) (one wave); returns nothing, writes LDS
__device__ __forceinline__ void gat_row(int i, int n, int mode, const float* lab, const float* ss,
                                        const float* ts, float alpha, float* att, int lane) {
  const float si = ss[i];
  float m = -INFINITY;
  for (int j = lane; j < n; j += 64) {
    if (gat_edge(mode, lab, i, j)) m = fmaxf(m, lrelu(si + ts[j], alpha));
  }
  m = wave_max(m);
  float sum = 0.f;
  for (int j = lane; j < n; j += 64) {
    float p = 0.f;
    if (gat_edge(mode, lab, i, j)) p = expf(lrelu(si + ts[j], alpha) - m);
    att[j] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  for (int j = lane; j < n; j += 64) att[j] *= inv;
}

__global__ void __launch_bounds__(kGatThreads) gat_fwd_kernel(
    const float* __restrict__ Wh, int heads, const float* __restrict__ a_all, const float* __restrict__ bias,
    const float* __restrict__ labels, const int32_t* __restrict__ seg_off, int nseg, int F, float alpha, int mode,
    int epi, int max_seg, float* __restrict__ hp, float* __restrict__ y, int ldy) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Fp = F | 1;
  float* Ws = reinterpret_cast<float*>(smem);       // max_seg x Fp
  float* ss = Ws + max_seg * Fp;                    // max_seg
  float* ts = ss + max_seg;                         // max_seg
  float* lab = ts + max_seg;                        // max_seg
  float* att = lab + max_seg;                       // kGatWaves x max_seg
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HF = heads * F;
  for (int gh = blockIdx.x; gh < nseg * heads; gh += gridDim.x) {
    const int g = gh / heads, hd = gh - g * heads;
    const int o = seg_off[g];
    const int n = seg_off[g + 1] - o;
    const float* a = a_all + 2 * F * hd;
    const int c0 = hd * F;
    for (int q = threadIdx.x; q < n * F; q += blockDim.x) {
      const int r = q / F, f = q - r * F;
      Ws[r * Fp + f] = Wh[(size_t)(o + r) * HF + c0 + f];
    }
    __syncthreads();
    for (int r = threadIdx.x; r < n; r += blockDim.x) {
      float s = 0.f, t = 0.f;
      for (int f = 0; f < F; ++f) {
        const float w = Ws[r * Fp + f];
        s = fmaf(w, a[f], s);
        t = fmaf(w, a[F + f], t);
      }
      ss[r] = s;
      ts[r] = t;
      lab[r] = mode == 0 ? labels[o + r] : 0.f;
    }
    __syncthreads();
    float* arow = att + wave * max_seg;
    for (int i = wave; i < n; i += kGatWaves) {
      gat_row(i, n, mode, lab, ss, ts, alpha, arow, lane);
      // the att row is written and read by this wave only: order its LDS
      // writes before the cross-lane reads below
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // aggregate: lanes over features
      float hv[2], zv[2];
      float zmax = -INFINITY;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int f = lane + 64 * c;
        float acc = 0.f;
        if (f < F) {
          for (int j = 0; j < n; ++j) acc = fmaf(arow[j], Ws[j * Fp + f], acc);
          if (bias) acc += bias[f];
        }
        hv[c] = acc;
        zv[c] = epi ? elu(acc) : acc;
        if (f < F) zmax = fmaxf(zmax, zv[c]);
      }
      float lse = 0.f;
      if (epi == 2) {
        zmax = wave_max(zmax);
        float se = 0.f;
#pragma unroll
        for (int c = 0; c < 2; ++c)
          if (lane + 64 * c < F) se += expf(zv[c] - zmax);
        se = wave_sum(se);
        lse = zmax + logf(se);
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int f = lane + 64 * c;
        if (f < F) {
          if (epi) hp[(size_t)(o + i) * HF + c0 + f] = hv[c];
          y[(size_t)(o + i) * ldy + c0 + f] = epi == 2 ? zv[c] - lse : zv[c];
        }
      }
    }
    __syncthreads();  // LDS reused by the next segment
  }
}

__global__ void __launch_bounds__(kGatThreads) gat_bwd_kernel(
    const float* __restrict__ Wh, int heads, const float* __restrict__ a_all, const float* __restrict__ labels,
    const int32_t* __restrict__ seg_off, int nseg, int F, float alpha, int mode, int epi, int max_seg,
    const float* __restrict__ hp, const float* __restrict__ y, const float* __restrict__ dy, int lddy,
    float* __restrict__ dWh, float* __restrict__ ds_out, float* __restrict__ dt_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Fp = F | 1;
  const int Np = max_seg | 1;
  float* Ws = reinterpret_cast<float*>(smem);  // max_seg x Fp
  float* Ds = Ws + max_seg * Fp;               // max_seg x Fp  (d hp)
  float* At = Ds + max_seg * Fp;               // max_seg x Np  (att, then dz)
  float* ss = At + max_seg * Np;
  float* ts = ss + max_seg;
  float* lab = ts + max_seg;
  float* dss = lab + max_seg;
  float* dts = dss + max_seg;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int HF = heads * F;
  for (int gh = blockIdx.x; gh < nseg * heads; gh += gridDim.x) {
    const int g = gh / heads, hd = gh - g * heads;
    const int o = seg_off[g];
    const int n = seg_off[g + 1] - o;
    const float* a = a_all + 2 * F * hd;
    const int c0 = hd * F;
    for (int q = threadIdx.x; q < n * F; q += blockDim.x) {
      const int r = q / F, f = q - r * F;
      Ws[r * Fp + f] = Wh[(size_t)(o + r) * HF + c0 + f];
    }
    __syncthreads();
    for (int r = threadIdx.x; r < n; r += blockDim.x) {
      float s = 0.f, t = 0.f;
      for (int f = 0; f < F; ++f) {
        const float w = Ws[r * Fp + f];
        s = fmaf(w, a[f], s);
        t = fmaf(w, a[F + f], t);
      }
      ss[r] = s;
      ts[r] = t;
      lab[r] = mode == 0 ? labels[o + r] : 0.f;
    }
    // d hp through the epilogue, one wave per row
    for (int i = wave; i < n; i += kGatWaves) {
      float d[2], h[2], sm[2];
      float sdy = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int f = lane + 64 * c;
        d[c] = 0.f; h[c] = 0.f; sm[c] = 0.f;
        if (f < F) {
          d[c] = dy[(size_t)(o + i) * lddy + c0 + f];
          if (epi) h[c] = hp[(size_t)(o + i) * HF + c0 + f];
          if (epi == 2) sm[c] = expf(y[(size_t)(o + i) * F + f]);
          sdy += d[c];
        }
      }
      if (epi == 2) sdy = wave_sum(sdy);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int f = lane + 64 * c;
        if (f < F) {
          float v = d[c];
          if (epi == 2) v = v - sm[c] * sdy;
          if (epi) v *= elu_grad(h[c]);
          Ds[i * Fp + f] = v;
        }
      }
    }
    __syncthreads();
    for (int i = wave; i < n; i += kGatWaves) gat_row(i, n, mode, lab, ss, ts, alpha, At + i * Np, lane);
    __syncthreads();
    // dWh_j (attention-weighted part) = sum_i att_ij dhp_i
    for (int q = threadIdx.x; q < n * F; q += blockDim.x) {
      const int j = q / F, f = q - j * F;
      float acc = 0.f;
      for (int i = 0; i < n; ++i) acc = fmaf(At[i * Np + j], Ds[i * Fp + f], acc);
      dWh[(size_t)(o + j) * HF + c0 + f] = acc;
    }
    __syncthreads();
    // per row: datt_ij = dhp_i . Wh_j ; softmax + LeakyReLU backward -> dz (in place of att)
    for (int i = wave; i < n; i += kGatWaves) {
      float* arow = At + i * Np;
      const float si = ss[i];
      float dot = 0.f;
      float datt[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = lane + 64 * c;
        datt[c] = 0.f;
        if (j < n) {
          float acc = 0.f;
          for (int f = 0; f < F; ++f) acc = fmaf(Ds[i * Fp + f], Ws[j * Fp + f], acc);
          datt[c] = acc;
          dot = fmaf(arow[j], acc, dot);
        }
      }
      dot = wave_sum(dot);
      float dsum = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = lane + 64 * c;
        if (j < n) {
          const float at = arow[j];
          const float de = at * (datt[c] - dot);
          const float dz = (si + ts[j]) > 0.f ? de : alpha * de;
          arow[j] = dz;
          dsum += dz;
        }
      }
      dsum = wave_sum(dsum);
      if (lane == 0) dss[i] = dsum;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
      float acc = 0.f;
      for (int i = 0; i < n; ++i) acc += At[i * Np + j];
      dts[j] = acc;
      ds_out[(size_t)(o + j) * heads + hd] = dss[j];
      dt_out[(size_t)(o + j) * heads + hd] = acc;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < n * F; q += blockDim.x) {
      const int j = q / F, f = q - j * F;
      dWh[(size_t)(o + j) * HF + c0 + f] += dss[j] * a[f] + dts[j] * a[F + f];
    }
    __syncthreads();
  }
}

static size_t gat_fwd_lds(int F, int max_seg) {
  return sizeof(float) * ((size_t)max_seg * (F | 1) + 3 * (size_t)max_seg + (size_t)kGatWaves * max_seg) + 16;
}
static size_t gat_bwd_lds(int F, int max_seg) {
  return sizeof(float) * (2 * (size_t)max_seg * (F | 1) + (size_t)max_seg * (max_seg | 1) + 5 * (size_t)max_seg) + 16;
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
  return w < 16384 ? (int)w : 16384;
}

extern "C" int sgg_gat_fwd(const float* Wh, int heads, const float* a, const float* bias, const float* labels,
                           const int32_t* seg_off, int nseg, int n, int F, float alpha, int mask_mode, int epilogue,
                           int max_seg, float* hp, float* y, int ldy, void* stream) {
  int rc = gat_args_ok("sgg_gat_fwd", Wh, heads, a, labels, seg_off, nseg, n, F, mask_mode, epilogue, max_seg);
  if (rc) return rc;
  SGG_CHECK_ARG(y && (epilogue == 0 || hp), "sgg_gat_fwd: null output");
  SGG_CHECK_ARG(ldy >= heads * F, "sgg_gat_fwd: ldy < heads * F");
  SGG_CHECK_ARG(epilogue != 2 || ldy == F, "sgg_gat_fwd: log_softmax epilogue needs a dense y (ldy == F)");
  if (nseg == 0) return 0;
  hipLaunchKernelGGL(gat_fwd_kernel, dim3(gat_grid(nseg, heads)), dim3(kGatThreads), gat_fwd_lds(F, max_seg),
                     (hipStream_t)stream, Wh, heads, a, bias, labels, seg_off, nseg, F, alpha, mask_mode, epilogue,
                     max_seg, hp, y, ldy);
  SGG_RETURN_LAUNCH("sgg_gat_fwd");
}

extern "C" int sgg_gat_bwd(const float* Wh, int heads, const float* a, const float* labels, const int32_t* seg_off,
                           int nseg, int n, int F, float alpha, int mask_mode, int epilogue, int max_seg,
                           const float* hp, const float* y, const float* dy, int lddy, float* dWh, float* ds,
                           float* dt, void* stream) {
  int rc = gat_args_ok("sgg_gat_bwd", Wh, heads, a, labels, seg_off, nseg, n, F, mask_mode, epilogue, max_seg);
  if (rc) return rc;
  SGG_CHECK_ARG(dy && dWh && ds && dt, "sgg_gat_bwd: null pointer");
  SGG_CHECK_ARG(epilogue == 0 || hp, "sgg_gat_bwd: epilogue needs hp");
  SGG_CHECK_ARG(epilogue != 2 || y, "sgg_gat_bwd: log_softmax epilogue needs y");
  SGG_CHECK_ARG(lddy >= heads * F, "sgg_gat_bwd: lddy < heads * F");
  if (nseg == 0) return 0;
  const size_t lds = gat_bwd_lds(F, max_seg);
  SGG_CHECK_ARG(lds <= 160 * 1024, "sgg_gat_bwd: segment %d x F %d needs %zu B of LDS", max_seg, F, lds);
  hipLaunchKernelGGL(gat_bwd_kernel, dim3(gat_grid(nseg, heads)), dim3(kGatThreads), lds, (hipStream_t)stream, Wh,
                     heads, a, labels, seg_off, nseg, F, alpha, mask_mode, epilogue, max_seg, hp, y, dy, lddy, dWh,
                     ds, dt);
  SGG_RETURN_LAUNCH("sgg_gat_bwd");
}
