// Shared helpers for the gfx950 kernels of libsgg.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include "../../include/sgg.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace sgg {

constexpr int kWave = 64;      // CDNA wavefront
constexpr int kGatEncMaxHeads = SGG_GATENC_MAX_HEADS;
using GatEncArgs = SggGatEncArgs;
constexpr int kHidden = 512;   // pooling MLP hidden width (hard-coded, models.py:473)

// last error, per calling host thread
void set_error(const char* fmt, ...);

#define SGG_CHECK_ARG(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::sgg::set_error(__VA_ARGS__);        \
      return SGG_E_ARG;                     \
    }                                       \
  } while (0)

#define SGG_RETURN_LAUNCH(name)                                          \
  do {                                                                   \
    hipError_t e_ = hipGetLastError();                                   \
    if (e_ != hipSuccess) {                                              \
      ::sgg::set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
      return (int)e_;                                                    \
    }                                                                    \
    return 0;                                                            \
  } while (0)

// Workgroup barrier for kernels whose waves exchange data through LDS only:
// waits for the wave's own LDS operations (lgkmcnt) but not for its
// outstanding global stores, which __syncthreads()' workgroup-scope release
// drains (vmcnt(0)) -- in a per-step recurrence that puts a store round trip
// on every step.  Global data written by other waves of the workgroup is NOT
// ordered by it.
__device__ __forceinline__ void lds_barrier() { __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// lstm_mfma.hip: MFMA form of the LSTM sequence forward for large batches,
// dispatched by sgg_lstm_fwd (lstm.hip); internal, not part of the C ABI
constexpr int kLstmMfmaMinPeds = 4096;
__attribute__((visibility("hidden"))) bool lstm_fwd_mfma_ok(int H, int B);
__attribute__((visibility("hidden"))) int lstm_fwd_mfma(const float* rel, const float* A, const float* Whh,
                                                        const float* bias, const float* h0, const float* c0,
                                                        const float* Wp, const float* bp, int T, int B, int H,
                                                        int decoder, float* h_all, float* c_all, float* act_all,
                                                        float* rel_out, hipStream_t st,
                                                        const SggDecInit* di = nullptr);

// the rollout with a second no-grad decoder segment (+ its discriminator input) in one launch
__attribute__((visibility("hidden"))) int lstm_fwd_mfma_dec2(const SggDecInit* di, const SggDecInit* di2,
                                                             const float* A, const float* Whh, const float* bias,
                                                             const float* Wp, const float* bp, int T, int B, int B2,
                                                             int H, float* rel_out, float* rel_out2,
                                                             const SggTrajOut* to2, hipStream_t st);

// lstm_unit.hip: unit-per-thread LSTM sequence kernels (one barrier per
// step), dispatched by sgg_lstm_fwd / sgg_lstm_bwd; internal
__attribute__((visibility("hidden"))) bool lstm_unit_ok(int H, int decoder);
__attribute__((visibility("hidden"))) int lstm_unit_fwd(const float* rel, const float* A, const float* Whh,
                                                        const float* bias, const float* h0, const float* c0,
                                                        const float* Wp, const float* bp, int T, int B, int H,
                                                        int decoder, float* h_all, float* c_all, float* act_all,
                                                        float* rel_out, hipStream_t st);
__attribute__((visibility("hidden"))) int lstm_unit_bwd(const float* A, const float* Whh, const float* Wp,
                                                        const float* c_all, const float* act_all, const float* dh_last,
                                                        const float* dout, int T, int B, int H, int decoder, float* dG,
                                                        float* dh0, float* drel_in, float* drel_tot, hipStream_t st);

// lstm_mw.hip: MFMA LSTM sequence kernels, one workgroup of four waves (one
// per gate block) per 16 peds, tile-native saved states, weight gradients
// accumulated in the backward kernel; dispatched first by sgg_lstm_fwd /
// _bwd; internal
__attribute__((visibility("hidden"))) bool lstm_mw_ok(int H, int B);
__attribute__((visibility("hidden"))) long long lstm_mw_state_floats(int T, int B, int H, int which);
__attribute__((visibility("hidden"))) int lstm_mw_wpart_rows(int H, int B);
__attribute__((visibility("hidden"))) int lstm_mw_fwd(const float* rel, const float* A, const float* Whh,
                                                      const float* bias, const float* h0, const float* c0,
                                                      const float* Wp, const float* bp, int T, int B, int H,
                                                      int decoder, float* h_all, float* c_all, float* act_all,
                                                      float* rel_out, hipStream_t st, const float* Wu = nullptr,
                                                      int ldwu = 0, const float* cu = nullptr, int NU = 0,
                                                      float* U = nullptr, const SggDecInit* di = nullptr,
                                                      float* rel0_out = nullptr, const SggTrajOut* to = nullptr);
__attribute__((visibility("hidden"))) int lstm_mw_bwd(const float* A, const float* Whh, const float* Wp,
                                                      const float* h_all, const float* c_all, const float* act_all,
                                                      const float* rel, const float* rel_out, const float* dh_last,
                                                      const float* dout, int T, int B, int H, int decoder,
                                                      float* dh0, float* drel_in, float* drel_tot, float* wpart,
                                                      hipStream_t st, const float* dout2 = nullptr,
                                                      int bsplit = 0, int t_stop = 0, int t_sh = 0, int Bsrc = 0);
// one encoder / decoder sequence segment of the four-wave forward (lstm_mw.hip)
struct MwSeg {
  const float *rel, *A, *Whh, *bias, *h0, *c0, *Wp, *bp;
  int T, B, Bl, t0, Tl, Bsrc;
  float *h_all, *c_tile, *act_tile, *rel_out;
  const float* Wu;
  int ldwu;
  const float* cu;
  int NU;
  float* U;
  SggDecInit di;      // decoder: di.ctx != NULL builds h0 / rel0 in the prologue (sgg_lstm_fwd_dec)
  float* rel0_out;    // (with di) receives rel0 when saving
  SggTrajOut to;      // decoder: to.out != NULL writes the discriminator input (sgg_lstm_fwd_dec)
};
// h0[p][u] and rel0[p][k] of a SggDecInit (sgg_decoder_init's values)
__device__ __forceinline__ float dec_h0(const SggDecInit& d, int p, int u) {
  const int r = p / d.Bper, i = p - r * d.Bper;
  if (u < d.Dc) return d.ctx[(size_t)i * d.ldc + u];
  const int s = d.ped_scene[i];
  const int k = (d.best && r == 0) ? (int)d.best[s] : d.first_k + r - (d.best ? 1 : 0);
  return d.z[((size_t)k * d.S + s) * d.nz + (u - d.Dc)];
}
__device__ __forceinline__ float dec_rel0(const SggDecInit& d, int p, int k) {
  return d.last_rel[(size_t)(p % d.Bper) * 2 + k];
}
__attribute__((visibility("hidden"))) int lstm_mw_fwd_seg(const MwSeg& s, int H, hipStream_t st);
__attribute__((visibility("hidden"))) int lstm_mw_fwd_seg2(const MwSeg& a, int Ha, const MwSeg& b, int Hb,
                                                           hipStream_t st);
__attribute__((visibility("hidden"))) int lstm_mw_fwd_dec_seg(const float* A, const float* Whh, const float* bias,
                                                              const float* Wp, const float* bp, int T, int B, int H,
                                                              float* h_all, float* c_all, float* act_all,
                                                              float* rel_out, const SggDecInit* di, float* rel0_out,
                                                              const SggTrajOut* to, const MwSeg& b, int Hb,
                                                              hipStream_t st);
__attribute__((visibility("hidden"))) int lstm_mw_fwd_seg3(const MwSeg& a, int Ha, const MwSeg& b, int Hb,
                                                           const MwSeg& c, int Hc, hipStream_t st);

// fold.hip: the fold backwards of one sgg_grad_finish in one launch (a
// workgroup each; dA_src / db_src point at the summed (dA, dbias)); internal
__attribute__((visibility("hidden"))) void fold_bwd_multi(const SggFoldBwd* folds, int n, hipStream_t st);

// v if keep else +0.f, as a bit mask: a plain `keep ? v : 0` lets the
// compiler sink the load of v into an exec-masked branch that waits for it
// (one memory latency per load); the mask keeps every load unconditional
__device__ __forceinline__ float keep_if(float v, bool keep) {
  return __int_as_float(__float_as_int(v) & (keep ? -1 : 0));
}

__device__ __forceinline__ float elu(float x) { return x > 0.f ? x : expm1f(x); }
// derivative of ELU(alpha = 1) from its input
__device__ __forceinline__ float elu_grad(float x) { return x > 0.f ? 1.f : expf(x); }

}  // namespace sgg
