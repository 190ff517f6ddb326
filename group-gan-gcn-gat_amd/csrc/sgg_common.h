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

// --- split-bf16 fp32 products (the LSTM gate GEMMs) ---------------------
// An fp32 value x is the exact sum of three bf16 values: hi = x with its low
// 16 bits cleared, mid = the same of x - hi, lo = x - hi - mid (at most 8
// significant bits remain: a bf16 value).  A K = 32 fp32 dot product then
// runs on v_mfma_f32_16x16x32_bf16 (bf16 products exact in fp32, fp32
// accumulation) as the six products of the pieces down to 2^-24:
//   a.b = al.bh + am.bm + ah.bl + am.bh + ah.bm + ah.bh   (am.bl, al.bm, al.bl
// dropped), 6 x 16 cycles of the matrix pipe per 16x16 tile against 8 x 32 for
// the fp32 16x16x4 MFMAs, and this shape leaves half of its cycles to the VALU
// (MI355X_MICROARCH.md).  Not bitwise the fp32 MFMA's sum: within a few fp32
// roundings of it.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned sgg_uint4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_trunc(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }
// two bf16 values (the top halves of a and b) in one register, a in the low half
__device__ __forceinline__ unsigned bf16_pack_top(float a, float b) {
  return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}
// the pieces of x as fp32 values whose low 16 bits are zero.  No FMA
// contraction here: with x = a * b inlined from the caller, -ffp-contract=fast
// would form x - h as fma(a, b, -h) from the UNROUNDED product, so the pieces
// would sum to a * b rather than to the fp32 value x that the caller stores --
// and a recurrence restarted from the stored x (a segment from step t0)
// would see other pieces than the one that continued in registers
__device__ __forceinline__ void split3(float x, float& h, float& m, float& l) {
#pragma clang fp contract(off)
  h = bf16_trunc(x);
  const float r = x - h;
  m = bf16_trunc(r);
  l = r - m;
}
// the three bf16x8 operands (hi, mid, lo) of eight fp32 values
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8 (&o)[3]) {
  sgg_uint4v u[3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float h0, m0, l0, h1, m1, l1;
    split3(v[2 * i], h0, m0, l0);
    split3(v[2 * i + 1], h1, m1, l1);
    u[0][i] = bf16_pack_top(h0, h1);
    u[1][i] = bf16_pack_top(m0, m1);
    u[2][i] = bf16_pack_top(l0, l1);
  }
#pragma unroll
  for (int p = 0; p < 3; ++p) o[p] = __builtin_bit_cast(bf16x8, u[p]);
}
// c + a.b over one K = 32 chunk from the pieces (small terms first)
__device__ __forceinline__ floatx4 mfma_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
}

__device__ __forceinline__ float elu(float x) { return x > 0.f ? x : expm1f(x); }
// derivative of ELU(alpha = 1) from its input
__device__ __forceinline__ float elu_grad(float x) { return x > 0.f ? 1.f : expf(x); }

}  // namespace sgg
