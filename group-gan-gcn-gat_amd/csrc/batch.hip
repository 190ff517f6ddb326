// Device-resident data path: one launch assembles a training batch (the
// 11-tuple of seq_collate, reference sgan/data/trajectories_GCN.py:15-42)
// from a split's ped table held in HBM for the whole run.
//
// The host picks the batch's scenes (the reference's RandomSampler order)
// and uploads the list of ped rows; each thread writes one (ped, step) of
// every time-major output: positions, displacements, velocities (2.5 x the
// displacement: the 0.4 s frame step), group labels, the loss mask, and the
// non-linearity flag at step 0.  A negative row is a padding ped (the
// fixed-capacity batches of the graph-replayed path, PaddedScenes): zeros
// everywhere, loss mask included.  Table record per ped (floats):
//   [abs x, y (T x 2) | rel x, y (T x 2) | group (T) | loss mask (T) | non_linear]
#include "sgg_common.h"

namespace sgg {

namespace {

__global__ void __launch_bounds__(256) gather_batch_kernel(const float* __restrict__ table, int rec,
                                                           const int32_t* __restrict__ rows, int B, int To, int Tp,
                                                           float* __restrict__ out) {
  const int T = To + Tp;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * T) return;
  const int b = e / T, t = e - b * T;
  const int row = rows[b];
  const bool pad = row < 0;
  const float* r = table + (size_t)(pad ? 0 : row) * rec;
  const float ax = keep_if(r[2 * t], !pad), ay = keep_if(r[2 * t + 1], !pad);
  const float rx = keep_if(r[2 * T + 2 * t], !pad), ry = keep_if(r[2 * T + 2 * t + 1], !pad);
  const float g = keep_if(r[4 * T + t], !pad);
  const size_t oB = (size_t)B;
  const size_t o_obs = 0, o_pred = o_obs + To * oB * 2, o_orel = o_pred + Tp * oB * 2, o_prel = o_orel + To * oB * 2;
  const size_t o_ovel = o_prel + Tp * oB * 2, o_pvel = o_ovel + To * oB * 2, o_og = o_pvel + Tp * oB * 2;
  const size_t o_pg = o_og + To * oB, o_nl = o_pg + Tp * oB, o_mask = o_nl + oB;
  const bool obs = t < To;
  const int tt = obs ? t : t - To;
  const size_t p2 = ((size_t)tt * B + b) * 2, p1 = (size_t)tt * B + b;
  *reinterpret_cast<float2*>(out + (obs ? o_obs : o_pred) + p2) = make_float2(ax, ay);
  *reinterpret_cast<float2*>(out + (obs ? o_orel : o_prel) + p2) = make_float2(rx, ry);
  *reinterpret_cast<float2*>(out + (obs ? o_ovel : o_pvel) + p2) = make_float2(rx * 2.5f, ry * 2.5f);
  out[(obs ? o_og : o_pg) + p1] = g;
  out[o_mask + (size_t)b * T + t] = keep_if(r[5 * T + t], !pad);
  if (t == 0) out[o_nl + b] = keep_if(r[6 * T], !pad);
}

}  // namespace

}  // namespace sgg

extern "C" long long sgg_gather_batch_floats(int B, int obs_len, int pred_len) {
  const long long T = obs_len + pred_len;
  return (long long)B * (T * 2 * 3 + T + 1 + T);
}

extern "C" int sgg_gather_batch(const float* table, int rec, const int32_t* rows, int B, int obs_len, int pred_len,
                                float* out, void* stream) {
  SGG_CHECK_ARG(table && rows && out, "sgg_gather_batch: null pointer");
  SGG_CHECK_ARG(B >= 0 && obs_len >= 1 && pred_len >= 1 && rec >= 6 * (obs_len + pred_len) + 1,
                "sgg_gather_batch: bad sizes B=%d obs=%d pred=%d rec=%d", B, obs_len, pred_len, rec);
  if (B == 0) return 0;
  const int n = B * (obs_len + pred_len);
  hipLaunchKernelGGL(sgg::gather_batch_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, table, rec,
                     rows, B, obs_len, pred_len, out);
  SGG_RETURN_LAUNCH("sgg_gather_batch");
}
