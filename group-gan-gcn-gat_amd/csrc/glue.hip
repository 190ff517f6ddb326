// The small data-movement and loss steps around the G / D modules of a
// training iteration (reference scripts/train.py:395-484, sgan/losses.py,
// sgan/models.py:814-850), one launch each instead of the 3..15 elementwise /
// index / reduction launches the reference's torch expressions take:
//
//   sgg_traj_cat      the discriminator input traj_rel = cat(obs_rel, pred)
//                     (train.py:409-415, 468-470), fake and real halves side
//                     by side in one call (no relative_to_abs: the
//                     discriminator reads only traj[0] and traj_rel)
//   sgg_decoder_init  add_noise (models.py:814-850, 'global' mix) for
//                     `copies` samples of the batch: h0 = [ctx | z_scene],
//                     plus the decoder's first input (the last observed
//                     displacement), replicated sample-major
//   sgg_l2_select     best-of-k (train.py:443-464): per scene the sample
//                     with the smallest sum over its peds of l2_loss(raw)
//   sgg_l2_loss_fwd/bwd  sum over scenes of  l2_loss(raw) summed over the
//                     scene's peds / sum(loss_mask) (train.py:459-464)
// All sums run in a fixed order (deterministic).
#include "sgg_common.h"

namespace sgg {

namespace {

__global__ void __launch_bounds__(256) traj_cat_kernel(const float* __restrict__ head, int ldh, int T0,
                                                       const float* __restrict__ a, int lda,
                                                       const float* __restrict__ b, int ldb, int T1, int B,
                                                       float* __restrict__ out, const float* __restrict__ pos0,
                                                       float* __restrict__ start) {
  const int NB = b ? 2 * B : B;
  const int total = (T0 + T1) * NB;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total + (start ? NB : 0); e += gridDim.x * blockDim.x) {
    if (e >= total) {   // the start positions of every column: pos0 of its ped
      const int p = e - total;
      reinterpret_cast<float2*>(start)[p] = reinterpret_cast<const float2*>(pos0)[p < B ? p : p - B];
      continue;
    }
    const int t = e / NB, p = e - t * NB;
    const float* src;
    if (t < T0) {
      src = head + (size_t)t * ldh + 2 * (p < B ? p : p - B);
    } else if (p < B) {
      src = a + (size_t)(t - T0) * lda + 2 * p;
    } else {
      src = b + (size_t)(t - T0) * ldb + 2 * (p - B);
    }
    reinterpret_cast<float2*>(out)[e] = *reinterpret_cast<const float2*>(src);
  }
}

__global__ void __launch_bounds__(256) decoder_init_kernel(const float* __restrict__ ctx, int ldc, int Dc,
                                                           const float* __restrict__ z, int nz,
                                                           const int64_t* __restrict__ best, int first_k,
                                                           int copies, const int32_t* __restrict__ ped_scene,
                                                           int S, int B, const float* __restrict__ last_rel,
                                                           float* __restrict__ h0, float* __restrict__ rel0) {
  const int D = Dc + nz;
  const int total = copies * B * D;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int row = e / D, c = e - row * D;
    const int r = row / B, p = row - r * B;
    float v;
    if (c < Dc) {
      v = ctx[(size_t)p * ldc + c];
    } else {
      const int s = ped_scene[p];
      const int k = (best && r == 0) ? (int)best[s] : first_k + r - (best ? 1 : 0);
      v = z[((size_t)k * S + s) * nz + (c - Dc)];
    }
    h0[e] = v;
    if (c < 2) rel0[(size_t)row * 2 + c] = last_rel[(size_t)p * 2 + c];
  }
}

// Both L2 kernels walk a scene's (step, ped) elements PED-FASTEST, so the gt
// and pred reads of a wave are contiguous runs (gt / pred are step-major:
// [T][B][2]); the scene's loss-mask block (ped-major, [B][ldm]) is first
// staged in LDS with coalesced reads and then read at (ped, step).
constexpr int kL2MaxElems = SGG_POOL_MAX_PEDS * 32;   // n * T staged per scene (larger: read in place)

// the scene's mask block -> msk[i * T + t] (coalesced: t fastest)
__device__ __forceinline__ void stage_mask(float* msk, const float* __restrict__ mask, int ldm, int o, int n, int T,
                                           int t0, int nt) {
  for (int e = t0; e < n * T; e += nt) {
    const int i = e / T, t = e - i * T;
    msk[e] = mask[(size_t)(o + i) * ldm + t];
  }
}

// one workgroup (8 waves) per scene: wave w takes samples w, w + 8, ...
// (their loads together); lane = element, the scene sum by a wave shuffle;
// argmin over the k samples (first minimum, as torch.argmin)
__global__ void __launch_bounds__(512) l2_select_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                        const float* __restrict__ mask, int ldm,
                                                        const int32_t* __restrict__ scene_off, int T, int B, int k,
                                                        int64_t* __restrict__ best) {
  __shared__ float part[256];   // k <= 256
  __shared__ float msk[kL2MaxElems];
  const int s = blockIdx.x;
  const int o = scene_off[s], n = scene_off[s + 1] - o;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float2* g2 = reinterpret_cast<const float2*>(gt);
  const float2* p2 = reinterpret_cast<const float2*>(pred);
  const int tot = n * T;
  const bool staged = tot <= kL2MaxElems;   // uniform
  if (staged) stage_mask(msk, mask, ldm, o, n, T, threadIdx.x, blockDim.x);
  __syncthreads();
  constexpr int kRS = 4;
  for (int r0 = wave; r0 < k; r0 += 8 * kRS) {
    float acc[kRS];
#pragma unroll
    for (int j = 0; j < kRS; ++j) acc[j] = 0.f;
    // four elements per lane in flight (a 20-ped scene's 240 in one round trip);
    // the sum runs over e = lane, lane + 64, ... in order, as with any unroll
    for (int e0 = lane; e0 < tot; e0 += 256) {
      float mk[4];
      float2 g[4], q[kRS][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = min(e0 + 64 * u, tot - 1);
        const int t = e / n, i = e - t * n, p = o + i;
        mk[u] = staged ? msk[i * T + t] : mask[(size_t)p * ldm + t];
        g[u] = g2[(size_t)t * B + p];
#pragma unroll
        for (int j = 0; j < kRS; ++j) {
          const int r = min(r0 + 8 * j, k - 1);
          q[j][u] = p2[((size_t)t * k + r) * B + p];
        }
      }
#pragma unroll
      for (int j = 0; j < kRS; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (e0 + 64 * u < tot) {
            const float dx = g[u].x - q[j][u].x, dy = g[u].y - q[j][u].y;
            acc[j] = fmaf(mk[u], fmaf(dx, dx, dy * dy), acc[j]);
          }
    }
#pragma unroll
    for (int j = 0; j < kRS; ++j) {
      const float a = wave_sum(acc[j]);
      if (lane == 0 && r0 + 8 * j < k) part[r0 + 8 * j] = a;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int bi = 0;
    float bv = part[0];
    for (int r = 1; r < k; ++r)
      if (part[r] < bv) {
        bv = part[r];
        bi = r;
      }
    best[s] = bi;
  }
}

// loss = sum_s w * (sum_{i in s, t} m (gt - pred)^2) / (sum_{i in s, t} m)
// (losses.py:52-71, mode 'raw' summed per scene): one wave per scene writes
// its term and mask sum (kept for the backward), then l2_sum_kernel adds the
// terms in scene order (lane-strided partials, a fixed shuffle tree).  A
// scene without a masked step (only the padding scenes of a fixed-capacity
// batch, PaddedScenes: real scenes always have one) adds 0 instead of 0 / 0.
// one wave: the (masked squared error, mask) sums of scene [o, o + n); msk is
// the wave's own LDS staging buffer (kL2MaxElems)
__device__ __forceinline__ void l2_scene(const float* __restrict__ pred, int ldp, const float2* __restrict__ g2,
                                         const float* __restrict__ mask, int ldm, int o, int n, int T, int B,
                                         float* msk, int lane, float& acc_out, float& ms_out) {
  const int tot = n * T;
  const bool staged = tot <= kL2MaxElems;   // uniform
  if (staged) stage_mask(msk, mask, ldm, o, n, T, lane, 64);
  // lanes read entries other lanes wrote: a wavefront-scope release / acquire
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float acc = 0.f, ms = 0.f;
  for (int e0 = lane; e0 < tot; e0 += 256) {
    float mk[4];
    float2 g[4], q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + 64 * u, tot - 1);
      const int t = e / n, i = e - t * n, p = o + i;
      mk[u] = staged ? msk[i * T + t] : mask[(size_t)p * ldm + t];
      g[u] = g2[(size_t)t * B + p];
      q[u] = *reinterpret_cast<const float2*>(pred + (size_t)t * ldp + 2 * p);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (e0 + 64 * u < tot) {
        const float dx = g[u].x - q[u].x, dy = g[u].y - q[u].y;
        acc = fmaf(mk[u], fmaf(dx, dx, dy * dy), acc);
        ms += mk[u];
      }
  }
  acc_out = wave_sum(acc);
  ms_out = wave_sum(ms);
  // the staging buffer is rewritten by the wave's next scene: every lane's
  // reads of it are done (wave_sum consumed them) before the next stores
  __builtin_amdgcn_wave_barrier();
}

__global__ void __launch_bounds__(64) l2_terms_kernel(const float* __restrict__ pred, int ldp,
                                                      const float* __restrict__ gt, const float* __restrict__ mask,
                                                      int ldm, const int32_t* __restrict__ scene_off, int T, int B,
                                                      float w, float* __restrict__ msum_out,
                                                      float* __restrict__ term) {
  __shared__ float msk[kL2MaxElems];
  const int lane = threadIdx.x, s = blockIdx.x;
  const int o = scene_off[s], n = scene_off[s + 1] - o;
  float acc, ms;
  l2_scene(pred, ldp, reinterpret_cast<const float2*>(gt), mask, ldm, o, n, T, B, msk, lane, acc, ms);
  if (lane == 0) {
    msum_out[s] = ms;
    term[s] = ms > 0.f ? (w * acc) / ms : 0.f;
  }
}

__global__ void __launch_bounds__(64) l2_sum_kernel(const float* __restrict__ term, int S, float* __restrict__ loss) {
  float a = 0.f;
  for (int s = threadIdx.x; s < S; s += 64) a += term[s];
  a = wave_sum(a);
  if (threadIdx.x == 0) *loss = a;
}

__global__ void __launch_bounds__(256) l2_loss_bwd_kernel(const float* __restrict__ pred, int ldp,
                                                          const float* __restrict__ gt,
                                                          const float* __restrict__ mask, int ldm,
                                                          const int32_t* __restrict__ ped_scene,
                                                          const float* __restrict__ msum, int T, int B, float w,
                                                          const float* __restrict__ gout, float* __restrict__ dpred,
                                                          int ldd) {
  const float g = *gout * w * -2.f;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < T * B; e += gridDim.x * blockDim.x) {
    const int t = e / B, p = e - t * B;
    const float m = mask[(size_t)p * ldm + t];
    const float2 gv = reinterpret_cast<const float2*>(gt)[e];
    const float2 q = *reinterpret_cast<const float2*>(pred + (size_t)t * ldp + 2 * p);
    const float ms = msum[ped_scene[p]];
    const float c = ms > 0.f ? g * m / ms : 0.f;
    *reinterpret_cast<float2*>(dpred + (size_t)t * ldd + 2 * p) = make_float2(c * (gv.x - q.x), c * (gv.y - q.y));
  }
}

// sgg_l2_loss_bwd_scenes: one 64-lane workgroup per scene forms the scene's
// mask sum as l2_terms_kernel does (same per-lane order, the same bits as the
// forward's msum), then the scene's rows of dpred with l2_loss_bwd_kernel's
// expression
__global__ void __launch_bounds__(64) l2_loss_bwd_scenes_kernel(const float* __restrict__ pred, int ldp,
                                                                const float* __restrict__ gt,
                                                                const float* __restrict__ mask, int ldm,
                                                                const int32_t* __restrict__ scene_off, int T, int B,
                                                                float w, const float* __restrict__ gout,
                                                                float* __restrict__ dpred, int ldd,
                                                                float* __restrict__ term) {
  __shared__ float msk[kL2MaxElems];
  const int lane = threadIdx.x, s = blockIdx.x;
  const int o = scene_off[s], n = scene_off[s + 1] - o;
  float acc, ms;
  l2_scene(pred, ldp, reinterpret_cast<const float2*>(gt), mask, ldm, o, n, T, B, msk, lane, acc, ms);
  if (term && lane == 0) term[s] = ms > 0.f ? (w * acc) / ms : 0.f;   // (l2_terms_kernel's value)
  const float g = *gout * w * -2.f;
  const float2* g2 = reinterpret_cast<const float2*>(gt);
  for (int e = lane; e < n * T; e += 64) {
    const int t = e / n, p = o + (e - t * n);
    const float m = mask[(size_t)p * ldm + t];
    const float2 gv = g2[(size_t)t * B + p];
    const float2 q = *reinterpret_cast<const float2*>(pred + (size_t)t * ldp + 2 * p);
    const float c = ms > 0.f ? g * m / ms : 0.f;
    *reinterpret_cast<float2*>(dpred + (size_t)t * ldd + 2 * p) = make_float2(c * (gv.x - q.x), c * (gv.y - q.y));
  }
}

int grid_for(long long n, int per) {
  const long long g = (n + per - 1) / per;
  return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_traj_cat(const float* head, int ldh, int T0, const float* a, int lda, const float* b, int ldb,
                            int T1, int B, float* out, const float* pos0, float* start, void* stream) {
  SGG_CHECK_ARG(head && a && out, "sgg_traj_cat: null pointer");
  SGG_CHECK_ARG(!start || pos0, "sgg_traj_cat: start positions need pos0");
  SGG_CHECK_ARG(T0 >= 0 && T1 >= 0 && B >= 0 && ldh >= 2 * B && lda >= 2 * B && (!b || ldb >= 2 * B),
                "sgg_traj_cat: bad sizes");
  const long long total = (long long)(T0 + T1 + (start ? 1 : 0)) * (b ? 2 * B : B);
  if (total == 0) return 0;
  hipLaunchKernelGGL(traj_cat_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, head, ldh, T0, a,
                     lda, b, ldb, T1, B, out, pos0, start);
  SGG_RETURN_LAUNCH("sgg_traj_cat");
}

extern "C" int sgg_decoder_init(const float* ctx, int ldc, int Dc, const float* z, int nz, const int64_t* best,
                                int first_k, int copies, const int32_t* ped_scene, int S, int B,
                                const float* last_rel, float* h0, float* rel0, void* stream) {
  SGG_CHECK_ARG(ctx && ped_scene && last_rel && h0 && rel0 && (nz == 0 || z), "sgg_decoder_init: null pointer");
  SGG_CHECK_ARG(Dc > 0 && nz >= 0 && ldc >= Dc && copies >= 1 && S >= 0 && B >= 0 && Dc + nz >= 2,
                "sgg_decoder_init: bad sizes");
  const long long total = (long long)copies * B * (Dc + nz);
  if (total == 0) return 0;
  hipLaunchKernelGGL(decoder_init_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, ctx, ldc, Dc,
                     z, nz, best, first_k, copies, ped_scene, S, B, last_rel, h0, rel0);
  SGG_RETURN_LAUNCH("sgg_decoder_init");
}

extern "C" int sgg_l2_select(const float* pred, const float* gt, const float* mask, int ldm, const int32_t* scene_off,
                             int S, int T, int B, int k, int64_t* best, void* stream) {
  SGG_CHECK_ARG(pred && gt && mask && scene_off && best, "sgg_l2_select: null pointer");
  SGG_CHECK_ARG(S >= 0 && T >= 1 && B >= 0 && k >= 1 && k <= 256 && ldm >= T, "sgg_l2_select: bad sizes");
  if (S == 0) return 0;
  hipLaunchKernelGGL(l2_select_kernel, dim3(S), dim3(512), 0, (hipStream_t)stream, pred, gt, mask, ldm, scene_off, T,
                     B, k, best);
  SGG_RETURN_LAUNCH("sgg_l2_select");
}

extern "C" int sgg_l2_loss_fwd(const float* pred, int ldp, const float* gt, const float* mask, int ldm,
                               const int32_t* scene_off, int S, int T, int B, float w, float* loss, float* msum,
                               float* term_ws, void* stream) {
  SGG_CHECK_ARG(pred && gt && mask && scene_off && loss && msum && term_ws, "sgg_l2_loss_fwd: null pointer");
  SGG_CHECK_ARG(S >= 0 && T >= 1 && B >= 0 && ldm >= T && ldp >= 2 * B, "sgg_l2_loss_fwd: bad sizes");
  // (one workgroup looping over the scenes in a single launch measured slower:
  // its per-scene load latencies add up, ~50 us at 64 scenes vs ~10 us here)
  if (S > 0)
    hipLaunchKernelGGL(l2_terms_kernel, dim3(S), dim3(64), 0, (hipStream_t)stream, pred, ldp, gt, mask, ldm, scene_off,
                     T, B, w, msum, term_ws);
  hipLaunchKernelGGL(l2_sum_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, term_ws, S, loss);
  SGG_RETURN_LAUNCH("sgg_l2_loss_fwd");
}

extern "C" int sgg_l2_loss_bwd(const float* pred, int ldp, const float* gt, const float* mask, int ldm,
                               const int32_t* ped_scene, const float* msum, int T, int B, float w, const float* gout,
                               float* dpred, int ldd, void* stream) {
  SGG_CHECK_ARG(pred && gt && mask && ped_scene && msum && gout && dpred, "sgg_l2_loss_bwd: null pointer");
  SGG_CHECK_ARG(T >= 1 && B >= 0 && ldm >= T && ldp >= 2 * B && ldd >= 2 * B, "sgg_l2_loss_bwd: bad sizes");
  if (B == 0) return 0;
  hipLaunchKernelGGL(l2_loss_bwd_kernel, dim3(grid_for((long long)T * B, 256)), dim3(256), 0, (hipStream_t)stream,
                     pred, ldp, gt, mask, ldm, ped_scene, msum, T, B, w, gout, dpred, ldd);
  SGG_RETURN_LAUNCH("sgg_l2_loss_bwd");
}

extern "C" int sgg_l2_loss_bwd_scenes(const float* pred, int ldp, const float* gt, const float* mask, int ldm,
                                      const int32_t* scene_off, int S, int T, int B, float w, const float* gout,
                                      float* dpred, int ldd, float* term, void* stream) {
  SGG_CHECK_ARG(pred && gt && mask && scene_off && gout && dpred, "sgg_l2_loss_bwd_scenes: null pointer");
  SGG_CHECK_ARG(S >= 0 && T >= 1 && B >= 0 && ldm >= T && ldp >= 2 * B && ldd >= 2 * B,
                "sgg_l2_loss_bwd_scenes: bad sizes");
  if (S == 0) return 0;
  hipLaunchKernelGGL(l2_loss_bwd_scenes_kernel, dim3(S), dim3(64), 0, (hipStream_t)stream, pred, ldp, gt, mask, ldm,
                     scene_off, T, B, w, gout, dpred, ldd, term);
  SGG_RETURN_LAUNCH("sgg_l2_loss_bwd_scenes");
}
