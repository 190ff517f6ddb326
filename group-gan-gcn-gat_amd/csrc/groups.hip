// Group structure and segmented reduce / gather (reference sgan/models.py
// :263-286 and :654-699: M_intra from labels, torch.unique rows -> R,
// R-normalised mean-pool, R^T un-pool).
//
// A scene's groups are its distinct non-zero labels plus one singleton per
// label-0 ped (that is exactly the set of distinct rows of M_intra).  We
// number them scene by scene in order of first member; the reference's row
// order (torch.unique + reversal) differs, which only permutes the inter-group
// graph -- the GAT/GCN over a complete graph is permutation-equivariant.
#include "sgg_common.h"

namespace sgg {

constexpr int kGroupMaxPeds = 1024;

// one workgroup per scene: leader of each ped = first ped with its (non-zero)
// label; local group id = rank of the leader among the scene's leaders.
__global__ void __launch_bounds__(256) group_local_kernel(const float* __restrict__ labels,
                                                          const int32_t* __restrict__ off, int S,
                                                          int32_t* __restrict__ ped_gid, int32_t* __restrict__ ped_scene,
                                                          int32_t* __restrict__ ngroups, int32_t* __restrict__ ped_cnt) {
  __shared__ float lab[kGroupMaxPeds];
  __shared__ int lead[kGroupMaxPeds];
  __shared__ int rank[kGroupMaxPeds];
  for (int s = blockIdx.x; s < S; s += gridDim.x) {
    const int o = off[s];
    const int n = off[s + 1] - o;
    for (int i = threadIdx.x; i < n; i += blockDim.x) lab[i] = labels[o + i];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const float li = lab[i];
      int l = i;
      if (li != 0.f)
        for (int j = 0; j < i; ++j)
          if (lab[j] == li) { l = j; break; }
      lead[i] = l;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan of the leader flags (n <= 1024, serial is fine)
      int c = 0;
      for (int i = 0; i < n; ++i) { rank[i] = c; c += (lead[i] == i); }
      ngroups[s] = c;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int l = lead[i];
      int cnt = 0;
      for (int j = l; j < n; ++j) cnt += (lead[j] == l);
      ped_gid[o + i] = rank[l];
      ped_scene[o + i] = s;
      ped_cnt[o + i] = (l == i) ? cnt : -1;  // member count, recorded at the leader
    }
    __syncthreads();
  }
}

// exclusive scan of ngroups[S] -> group_off[S+1], single workgroup
__global__ void __launch_bounds__(1024) group_scan_kernel(const int32_t* __restrict__ ngroups, int S,
                                                          int32_t* __restrict__ group_off) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (S + 1023) / 1024;
  const int b = t * per, e = min(S, b + per);
  int sum = 0;
  for (int i = b; i < e; ++i) sum += ngroups[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = t ? part[t - 1] : 0;
  for (int i = b; i < e; ++i) { group_off[i] = run; run += ngroups[i]; }
  if (t == 1023) group_off[S] = part[1023];
}

__global__ void group_global_kernel(int B, const int32_t* __restrict__ group_off, int32_t* __restrict__ ped_gid,
                                    const int32_t* __restrict__ ped_scene, const int32_t* __restrict__ ped_cnt,
                                    int32_t* __restrict__ group_scene, int32_t* __restrict__ group_count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const int s = ped_scene[i];
  const int g = group_off[s] + ped_gid[i];
  ped_gid[i] = g;
  const int c = ped_cnt[i];
  if (c >= 0) { group_scene[g] = s; group_count[g] = c; }
}

__global__ void seg_reduce_kernel(const float* __restrict__ x, int ldx, int F, const int32_t* __restrict__ seg_of_row,
                                  const float* __restrict__ row_scale, const int32_t* __restrict__ range_off,
                                  const int32_t* __restrict__ seg_range, const int32_t* __restrict__ nseg_dev,
                                  int nseg_cap, int mean, float* __restrict__ out, int ldo) {
  const int nvalid = nseg_dev ? *nseg_dev : nseg_cap;
  const long total = (long)nseg_cap * F;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int k = (int)(e / F), f = (int)(e - (long)k * F);
    float acc = 0.f;
    if (k < nvalid) {
      const int r = seg_range ? seg_range[k] : k;
      const int lo = range_off[r], hi = range_off[r + 1];
      int cnt = 0;
      for (int i = lo; i < hi; ++i) {
        if (seg_of_row[i] == k) {
          const float v = x[(size_t)i * ldx + f];
          acc = row_scale ? fmaf(row_scale[i], v, acc) : acc + v;
          ++cnt;
        }
      }
      if (mean && cnt) acc = acc / (float)cnt;
    }
    out[(size_t)k * ldo + f] = acc;
  }
}

__global__ void seg_gather_kernel(const float* __restrict__ src, int lds, int F, const int32_t* __restrict__ seg_of_row,
                                  const float* __restrict__ row_scale, const int32_t* __restrict__ nrow_dev, int n,
                                  float* __restrict__ out, int ldo) {
  const int nvalid = nrow_dev ? *nrow_dev : n;
  const long total = (long)n * F;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int i = (int)(e / F), f = (int)(e - (long)i * F);
    float v = 0.f;
    if (i < nvalid) {
      v = src[(size_t)seg_of_row[i] * lds + f];
      if (row_scale) v *= row_scale[i];
    }
    out[(size_t)i * ldo + f] = v;
  }
}

static int grid_for(long total) {
  long g = (total + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace sgg

using namespace sgg;

extern "C" size_t sgg_group_index_ws(int S, int B) { return sizeof(int32_t) * ((size_t)S + (size_t)B) + 256; }

extern "C" int sgg_group_index(const float* labels, const int32_t* scene_off, int S, int B, int max_n,
                               int32_t* ped_gid, int32_t* ped_scene, int32_t* group_off, int32_t* group_scene,
                               int32_t* group_count, void* workspace, void* stream) {
  SGG_CHECK_ARG(labels && scene_off && ped_gid && ped_scene && group_off && group_scene && group_count && workspace,
                "sgg_group_index: null pointer");
  SGG_CHECK_ARG(S >= 1 && B >= 0, "sgg_group_index: bad sizes S=%d B=%d", S, B);
  SGG_CHECK_ARG(max_n <= kGroupMaxPeds, "sgg_group_index: scene of %d peds > %d", max_n, kGroupMaxPeds);
  hipStream_t st = (hipStream_t)stream;
  int32_t* ngroups = reinterpret_cast<int32_t*>(workspace);
  int32_t* ped_cnt = ngroups + ((S + 63) & ~63);
  const int g1 = S < 8192 ? S : 8192;
  hipLaunchKernelGGL(group_local_kernel, dim3(g1), dim3(256), 0, st, labels, scene_off, S, ped_gid, ped_scene,
                     ngroups, ped_cnt);
  hipLaunchKernelGGL(group_scan_kernel, dim3(1), dim3(1024), 0, st, ngroups, S, group_off);
  if (B > 0)
    hipLaunchKernelGGL(group_global_kernel, dim3((B + 255) / 256), dim3(256), 0, st, B, group_off, ped_gid, ped_scene,
                       ped_cnt, group_scene, group_count);
  SGG_RETURN_LAUNCH("sgg_group_index");
}

extern "C" int sgg_seg_reduce(const float* x, int ldx, int F, const int32_t* seg_of_row, const float* row_scale,
                              const int32_t* range_off, const int32_t* seg_range, const int32_t* nseg_dev,
                              int nseg_cap, int mean, float* out, int ldo, void* stream) {
  SGG_CHECK_ARG(x && seg_of_row && range_off && out, "sgg_seg_reduce: null pointer");
  SGG_CHECK_ARG(F >= 1 && ldx >= F && ldo >= F && nseg_cap >= 0, "sgg_seg_reduce: bad sizes");
  if (nseg_cap == 0) return 0;
  hipLaunchKernelGGL(seg_reduce_kernel, dim3(grid_for((long)nseg_cap * F)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     F, seg_of_row, row_scale, range_off, seg_range, nseg_dev, nseg_cap, mean, out, ldo);
  SGG_RETURN_LAUNCH("sgg_seg_reduce");
}

extern "C" int sgg_seg_gather(const float* src, int lds, int F, const int32_t* seg_of_row, const float* row_scale,
                              const int32_t* nrow_dev, int n, float* out, int ldo, void* stream) {
  SGG_CHECK_ARG(src && seg_of_row && out, "sgg_seg_gather: null pointer");
  SGG_CHECK_ARG(F >= 1 && lds >= F && ldo >= F && n >= 0, "sgg_seg_gather: bad sizes");
  if (n == 0) return 0;
  hipLaunchKernelGGL(seg_gather_kernel, dim3(grid_for((long)n * F)), dim3(256), 0, (hipStream_t)stream, src, lds, F,
                     seg_of_row, row_scale, nrow_dev, n, out, ldo);
  SGG_RETURN_LAUNCH("sgg_seg_gather");
}
