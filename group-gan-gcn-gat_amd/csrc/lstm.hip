// Fused LSTM sequences: the Encoder (reference sgan/models.py:32-92) and the
// autoregressive Decoder rollout (models.py:142-178), forward and backward,
// one launch each instead of one MIOpen RNN call (plus Linear/cat kernels)
// per time step.
//
// Folding (exact up to fp32 reassociation): the input of every step is a
// 2-d relative displacement r embedded by Linear(2, E), so
//   W_ih (We r + be) + b_ih + b_hh = A r + b'    with A = W_ih We (4H x 2),
//                                                b' = W_ih be + b_ih + b_hh
// (A and b' are formed by the caller with torch ops, so autograd carries
// their gradients back to W_ih, We, be, b_ih, b_hh).  Decoder: r_0 is the
// last observed displacement, r_t = Wp h_t + bp (hidden2pos) feeds step t+1.
//
// Layout: one workgroup = P = 4 peds x 4H gate rows (16 H threads); thread
// (ped, r) owns gate row r: its W_hh row lives in registers, h_{t-1} is read
// from LDS as a per-ped broadcast, so a step is H register FMAs per thread +
// one LDS exchange of the gate activations; the H "cell" threads of a ped
// keep c_t in a register.  The backward uses the column layout (thread
// (ped, g, k) owns column k of gate block g of W_hh) so dh_{t-1} = W_hh^T dG_t
// is H register FMAs + a 4-way LDS reduction.  Parameter gradients are sums
// over (t, ped) of outer products -> the caller's GEMMs on the saved dG.
#include <stdlib.h>
#include <string.h>

#include "sgg_common.h"

namespace sgg {

constexpr int kLstmPeds = 4;
constexpr int kLstmMaxT = 32;   // encoder inputs of up to this many steps are staged in LDS up front

// v_exp_f32 / v_rcp_f32 forms (~2 ulp), as in lstm_mfma.hip: the gate
// activations sit on the serial critical path of every step
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
// (exp(-2x) as v_exp_f32(x * -2 log2(e)): -2 log2(e) is exact, so the same bits as
// __expf(-2x)'s (-2x) * log2(e) with one multiply less)
__device__ __forceinline__ float tanh_f(float x) {
  return fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -2.8853900817779268f)), -1.f);
}

template <int H>
__global__ void __launch_bounds__(16 * H) lstm_fwd_kernel(
    const float* __restrict__ rel, const float* __restrict__ A, const float* __restrict__ Whh,
    const float* __restrict__ bias, const float* __restrict__ h0, const float* __restrict__ c0,
    const float* __restrict__ Wp, const float* __restrict__ bp, int T, int B, int decoder,
    float* __restrict__ h_all, float* __restrict__ c_all, float* __restrict__ act_all, float* __restrict__ rel_out) {
  const bool save_states = act_all != nullptr;  // inference: only the final state is stored
  constexpr int G4 = 4 * H;
  __shared__ __attribute__((aligned(16))) float hbuf[kLstmPeds][H];
  __shared__ float gbuf[kLstmPeds][G4];
  __shared__ float relb[kLstmPeds][2];
  __shared__ float redb[kLstmPeds][2][H];
  __shared__ float relseq[kLstmPeds][kLstmMaxT][2];
  const int pl = threadIdx.x / G4, r = threadIdx.x - pl * G4;
  const int ped = blockIdx.x * kLstmPeds + pl;
  const bool valid = ped < B;
  float w[H];
#pragma unroll
  for (int k = 0; k < H; ++k) w[k] = Whh[r * H + k];
  const float a0 = A[2 * r], a1 = A[2 * r + 1], bb = bias[r];
  const bool is_g = r >= 2 * H && r < 3 * H;
  const float wp0 = (decoder && r < H) ? Wp[r] : 0.f, wp1 = (decoder && r < H) ? Wp[H + r] : 0.f;
  const float bp0 = decoder ? bp[0] : 0.f, bp1 = decoder ? bp[1] : 0.f;
  float c = 0.f;
  if (r < H) {
    const float hv = (valid && h0) ? h0[(size_t)ped * H + r] : 0.f;
    c = (valid && c0) ? c0[(size_t)ped * H + r] : 0.f;
    hbuf[pl][r] = hv;
    if (valid && save_states) {
      h_all[(size_t)ped * H + r] = hv;
      c_all[(size_t)ped * H + r] = c;
    }
  }
  if (decoder && r < 2) relb[pl][r] = valid ? rel[(size_t)ped * 2 + r] : 0.f;
  // encoder: the whole input sequence of the ped is loaded once, so no step
  // waits on a global load
  const bool staged = !decoder && T <= kLstmMaxT;
  if (staged && r < 2 * T) relseq[pl][r >> 1][r & 1] = valid ? rel[((size_t)(r >> 1) * B + ped) * 2 + (r & 1)] : 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    float x0, x1;
    if (decoder) {
      x0 = relb[pl][0];
      x1 = relb[pl][1];
    } else if (staged) {
      x0 = relseq[pl][t][0];
      x1 = relseq[pl][t][1];
    } else {
      x0 = valid ? rel[((size_t)t * B + ped) * 2] : 0.f;
      x1 = valid ? rel[((size_t)t * B + ped) * 2 + 1] : 0.f;
    }
    // four independent partial sums: the H-long FMA chain is the step's latency
    float p0 = fmaf(a1, x1, fmaf(a0, x0, bb)), p1 = 0.f, p2 = 0.f, p3 = 0.f;
#pragma unroll
    for (int k = 0; k < H; k += 4) {
      const float4 hv = *reinterpret_cast<const float4*>(&hbuf[pl][k]);
      p0 = fmaf(w[k], hv.x, p0);
      p1 = fmaf(w[k + 1], hv.y, p1);
      p2 = fmaf(w[k + 2], hv.z, p2);
      p3 = fmaf(w[k + 3], hv.w, p3);
    }
    const float acc = (p0 + p1) + (p2 + p3);
    const float act = is_g ? tanh_f(acc) : sigm(acc);
    if (act_all && valid) act_all[((size_t)t * B + ped) * G4 + r] = act;
    gbuf[pl][r] = act;
    __syncthreads();
    if (r < H) {
      const float ig = gbuf[pl][r], fg = gbuf[pl][H + r], gg = gbuf[pl][2 * H + r], og = gbuf[pl][3 * H + r];
      c = fmaf(fg, c, ig * gg);
      const float h = og * tanh_f(c);
      hbuf[pl][r] = h;
      if (decoder) {
        redb[pl][0][r] = wp0 * h;
        redb[pl][1][r] = wp1 * h;
      }
      if (valid && (save_states || t == T - 1)) {
        const size_t o = ((size_t)(save_states ? t + 1 : T) * B + ped) * H + r;
        h_all[o] = h;
        c_all[o] = c;
      }
    }
    __syncthreads();
    if (decoder) {
      if (r < 2) {  // rel_t = Wp h_t + bp  (H-term sum from LDS, same order for every ped)
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < H; ++k) s += redb[pl][r][k];
        s += r ? bp1 : bp0;
        relb[pl][r] = s;
        if (valid) rel_out[((size_t)t * B + ped) * 2 + r] = s;
      }
      __syncthreads();
    }
  }
}

template <int H>
__global__ void __launch_bounds__(16 * H) lstm_bwd_kernel(
    const float* __restrict__ A, const float* __restrict__ Whh, const float* __restrict__ Wp,
    const float* __restrict__ c_all, const float* __restrict__ act_all, const float* __restrict__ dh_last,
    const float* __restrict__ dout, int T, int B, int decoder, float* __restrict__ dG, float* __restrict__ dh0,
    float* __restrict__ drel_in, float* __restrict__ drel_tot) {
  constexpr int G4 = 4 * H;
  __shared__ __attribute__((aligned(16))) float dgb[kLstmPeds][G4];
  __shared__ float pb[kLstmPeds][4][H];
  __shared__ float drelb[kLstmPeds][2];
  __shared__ float fbp[kLstmPeds][2][G4 / 64 > 0 ? G4 / 64 : 1];
  const int pl = threadIdx.x / G4, q = threadIdx.x - pl * G4;
  const int g = q / H, k = q - g * H;
  const int ped = blockIdx.x * kLstmPeds + pl;
  const bool valid = ped < B;
  float wcol[H];
#pragma unroll
  for (int j = 0; j < H; ++j) wcol[j] = Whh[(g * H + j) * H + k];
  const float aq0 = A[2 * q], aq1 = A[2 * q + 1];   // row q of A (gate q of this thread)
  const int lane = threadIdx.x & 63;
  const int wq = q >> 6;                             // wave index within the ped (G4 is a multiple of 64)
  float dh = 0.f, dc = 0.f, fb = 0.f;
  const float wp0 = decoder ? Wp[q < H ? q : 0] : 0.f;
  const float wp1 = decoder ? Wp[H + (q < H ? q : 0)] : 0.f;
  if (q < H && !decoder && valid && dh_last) dh = dh_last[(size_t)ped * H + q];
  // the saved activations of step t are loaded one step ahead (registers)
  float nig = 0.f, nfg = 0.f, ngg = 0.f, nog = 0.f, nct = 0.f, ncp = 0.f;
  auto load_step = [&](int t) {
    if (q < H && valid) {
      const size_t ab = ((size_t)t * B + ped) * G4;
      nig = act_all[ab + q];
      nfg = act_all[ab + H + q];
      ngg = act_all[ab + 2 * H + q];
      nog = act_all[ab + 3 * H + q];
      nct = c_all[((size_t)(t + 1) * B + ped) * H + q];
      ncp = c_all[((size_t)t * B + ped) * H + q];
    }
  };
  load_step(T - 1);
  for (int t = T - 1; t >= 0; --t) {
    if (decoder) {
      if (q < 2) {
        const float v = (valid ? dout[((size_t)t * B + ped) * 2 + q] : 0.f) + fb;
        drelb[pl][q] = v;
        if (valid) drel_tot[((size_t)t * B + ped) * 2 + q] = v;
      }
      __syncthreads();
      if (q < H) dh = fmaf(wp0, drelb[pl][0], fmaf(wp1, drelb[pl][1], dh));
    }
    if (q < H) {
      const float ig = nig, fg = nfg, gg = ngg, og = nog, ct = nct, cp = ncp;
      if (t > 0) load_step(t - 1);   // in flight while this step computes
      const float tc = tanh_f(ct);
      const float d_o = dh * tc;
      const float dct = fmaf(dh * og, 1.f - tc * tc, dc);
      const float di = dct * gg, dgg = dct * ig, df = dct * cp;
      dc = dct * fg;
      const float vi = di * ig * (1.f - ig), vf = df * fg * (1.f - fg);
      const float vg = dgg * (1.f - gg * gg), vo = d_o * og * (1.f - og);
      dgb[pl][q] = vi;
      dgb[pl][H + q] = vf;
      dgb[pl][2 * H + q] = vg;
      dgb[pl][3 * H + q] = vo;
      if (valid) {
        const size_t ob = ((size_t)t * B + ped) * G4;
        dG[ob + q] = vi;
        dG[ob + H + q] = vf;
        dG[ob + 2 * H + q] = vg;
        dG[ob + 3 * H + q] = vo;
      }
    }
    __syncthreads();
    float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
#pragma unroll
    for (int j = 0; j < H; j += 4) {
      const float4 d4 = *reinterpret_cast<const float4*>(&dgb[pl][g * H + j]);
      p0 = fmaf(wcol[j], d4.x, p0);
      p1 = fmaf(wcol[j + 1], d4.y, p1);
      p2 = fmaf(wcol[j + 2], d4.z, p2);
      p3 = fmaf(wcol[j + 3], d4.w, p3);
    }
    pb[pl][g][k] = (p0 + p1) + (p2 + p3);
    {  // drel_t = A^T dG_t: one product per gate thread, wave shuffle + LDS combine
      const float dgq = dgb[pl][q];
      const float r0 = wave_sum(aq0 * dgq), r1 = wave_sum(aq1 * dgq);
      if (lane == 0) {
        fbp[pl][0][wq] = r0;
        fbp[pl][1][wq] = r1;
      }
    }
    __syncthreads();
    if (q < H) dh = pb[pl][0][q] + pb[pl][1][q] + pb[pl][2][q] + pb[pl][3][q];
    if (q < 2) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < G4 / 64; ++w) s += fbp[pl][q][w];
      fb = s;
      if (valid) drel_in[((size_t)t * B + ped) * 2 + q] = s;
    }
    __syncthreads();
  }
  if (q < H && valid && dh0) dh0[(size_t)ped * H + q] = dh;
}

template <int H>
static int launch_lstm_fwd(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0,
                           const float* c0, const float* Wp, const float* bp, int T, int B, int decoder, float* h_all, float* c_all,
                           float* act_all, float* rel_out, hipStream_t st) {
  const int grid = (B + kLstmPeds - 1) / kLstmPeds;
  hipLaunchKernelGGL(lstm_fwd_kernel<H>, dim3(grid), dim3(16 * H), 0, st, rel, A, Whh, bias, h0, c0, Wp, bp, T,
                     B, decoder, h_all, c_all, act_all, rel_out);
  SGG_RETURN_LAUNCH("sgg_lstm_fwd");
}

template <int H>
static int launch_lstm_bwd(const float* A, const float* Whh, const float* Wp, const float* c_all,
                           const float* act_all, const float* dh_last, const float* dout, int T, int B, int decoder,
                           float* dG, float* dh0, float* drel_in, float* drel_tot, hipStream_t st) {
  const int grid = (B + kLstmPeds - 1) / kLstmPeds;
  hipLaunchKernelGGL(lstm_bwd_kernel<H>, dim3(grid), dim3(16 * H), 0, st, A, Whh, Wp, c_all, act_all, dh_last, dout,
                     T, B, decoder, dG, dh0, drel_in, drel_tot);
  SGG_RETURN_LAUNCH("sgg_lstm_bwd");
}

}  // namespace sgg

using namespace sgg;

extern "C" long long sgg_lstm_state_floats(int T, int B, int H, int which) {
  if (T < 1 || B < 0 || (which != 0 && which != 1)) return -1;
  if (lstm_mw_ok(H, B)) return lstm_mw_state_floats(T, B, H, which);
  return which == 0 ? (long long)T * B * 4 * H : (long long)(T + 1) * B * H;
}

extern "C" const char* sgg_lstm_kernel_name(int H, int B, int decoder, int save, int bwd) {
  // mirrors the dispatch of sgg_lstm_fwd / sgg_lstm_bwd below (save = act_all
  // != NULL for the forward, = weight gradients in the kernel for the backward)
  static char buf[96];
  const int h = H == 16 ? 0 : H == 32 ? 1 : H == 48 ? 2 : H == 64 ? 3 : -1;
  if (h < 0 || B <= 0) return "";
  const bool mw = lstm_mw_ok(H, B);
  const char* tf[2] = {"false", "true"};
  if (bwd) {
    if (mw) snprintf(buf, sizeof buf, "sgg::lstm_mw_bwd_kernel<%d, %s, %s>", H, tf[decoder != 0], tf[save != 0]);
    else if (H <= 32) snprintf(buf, sizeof buf, "sgg::lstm_unit_bwd_kernel<%d>", H);
    else snprintf(buf, sizeof buf, "sgg::lstm_bwd_kernel<%d>", H);
    return buf;
  }
  if (save && mw) snprintf(buf, sizeof buf, "sgg::lstm_mw_fwd_kernel<%d, %s, true>", H, tf[decoder != 0]);
  else if (!save && lstm_fwd_mfma_ok(H, B) && !getenv("SGG_LSTM_NO_MFMA")) {
    // (lstm_mfma.hip: the split-bf16 gate GEMM for H = 32 unless SGG_LSTM_X3=0)
    const char* x3e = getenv("SGG_LSTM_X3");
    const bool x3 = H == 32 && !(x3e && strcmp(x3e, "0") == 0);
    snprintf(buf, sizeof buf, "sgg::lstm_fwd_mfma_kernel<%d, %s, %s>", H, tf[x3], tf[decoder != 0]);
  }
  else if (mw) snprintf(buf, sizeof buf, "sgg::lstm_mw_fwd_kernel<%d, %s, %s>", H, tf[decoder != 0], tf[save != 0]);
  else if (H <= 32) snprintf(buf, sizeof buf, "sgg::lstm_unit_fwd_kernel<%d>", H);
  else snprintf(buf, sizeof buf, "sgg::lstm_fwd_kernel<%d>", H);
  return buf;
}

// the family sgg_lstm_fwd picks for these sizes is the four-wave one
static bool fwd_picks_mw(int H, int B, bool save) {
  const bool mw = lstm_mw_ok(H, B);
  if (save) return mw;
  return mw && !(lstm_fwd_mfma_ok(H, B) && !getenv("SGG_LSTM_NO_MFMA"));
}

extern "C" int sgg_lstm_u_ok(int T, int B, int H, int decoder, int save, int NU) {
  return !decoder && B > 0 && T >= 1 && NU >= 16 && NU % 16 == 0 && fwd_picks_mw(H, B, save != 0);
}

extern "C" int sgg_lstm_fwd_u(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0,
                              const float* c0, int T, int B, int H, float* h_all, float* c_all, float* act_all,
                              const float* Wu, int ldwu, const float* cu, int NU, float* U, void* stream) {
  SGG_CHECK_ARG(rel && A && Whh && bias && h_all && c_all && Wu && cu && U, "sgg_lstm_fwd_u: null pointer");
  SGG_CHECK_ARG(sgg_lstm_u_ok(T, B, H, 0, act_all != nullptr, NU) && ldwu >= H,
                "sgg_lstm_fwd_u: no projection epilogue for T=%d B=%d H=%d NU=%d ldwu=%d (sgg_lstm_u_ok)", T, B, H, NU,
                ldwu);
  return lstm_mw_fwd(rel, A, Whh, bias, h0, c0, nullptr, nullptr, T, B, H, 0, h_all, c_all, act_all, nullptr,
                     (hipStream_t)stream, Wu, ldwu, cu, NU, U);
}

extern "C" int sgg_lstm_bwd_split(const float* A, const float* Whh, const float* Wp, const float* h_all,
                                  const float* c_all, const float* act_all, const float* rel, const float* rel_out,
                                  const float* dout, const float* dout2, int bsplit, int T, int B, int H, float* dh0,
                                  float* drel_in, float* drel_tot, float* wpart, void* stream) {
  SGG_CHECK_ARG(A && Whh && Wp && h_all && c_all && act_all && rel && rel_out && dout && dout2 && drel_in && drel_tot,
                "sgg_lstm_bwd_split: null pointer");
  SGG_CHECK_ARG(T >= 1 && B >= 1 && bsplit >= 0 && bsplit <= B && lstm_mw_ok(H, B),
                "sgg_lstm_bwd_split: bad sizes or no four-wave kernel (T=%d B=%d H=%d bsplit=%d)", T, B, H, bsplit);
  return lstm_mw_bwd(A, Whh, Wp, h_all, c_all, act_all, rel, rel_out, nullptr, dout, T, B, H, 1, dh0, drel_in,
                     drel_tot, wpart, (hipStream_t)stream, dout2, bsplit);
}

extern "C" int sgg_lstm_bwd_tail(const float* A, const float* Whh, const float* h_all, const float* c_all,
                                 const float* act_all, const float* rel, const float* dh_last, int T, int B, int H,
                                 int t_stop, float* drel_in, void* stream) {
  SGG_CHECK_ARG(A && Whh && h_all && c_all && act_all && rel && drel_in, "sgg_lstm_bwd_tail: null pointer");
  SGG_CHECK_ARG(T >= 1 && B >= 1 && t_stop >= 0 && t_stop < T && lstm_mw_ok(H, B),
                "sgg_lstm_bwd_tail: bad sizes or no four-wave kernel (T=%d B=%d H=%d t_stop=%d)", T, B, H, t_stop);
  return lstm_mw_bwd(A, Whh, nullptr, h_all, c_all, act_all, rel, nullptr, dh_last, nullptr, T, B, H, 0, nullptr,
                     drel_in, nullptr, nullptr, (hipStream_t)stream, nullptr, 0, t_stop);
}

static MwSeg to_mw(const SggLstmSeg& s) {
  return MwSeg{s.rel, s.A, s.Whh, s.bias, s.h0, s.c0, nullptr, nullptr, s.T, s.B, s.Bl, s.t0, s.Tl, s.Bsrc,
               s.h_all, s.c_all, s.act_all, nullptr, s.Wu, s.ldwu, s.cu, s.NU, s.U};
}

extern "C" int sgg_lstm_fwd_seg(const SggLstmSeg* seg, int H, void* stream) {
  SGG_CHECK_ARG(seg, "sgg_lstm_fwd_seg: null segment");
  SGG_CHECK_ARG(lstm_mw_ok(H, seg->B), "sgg_lstm_fwd_seg: no four-wave kernel for H=%d", H);
  return lstm_mw_fwd_seg(to_mw(*seg), H, (hipStream_t)stream);
}

extern "C" int sgg_lstm_fwd_seg2(const SggLstmSeg* a, int Ha, const SggLstmSeg* b, int Hb, void* stream) {
  SGG_CHECK_ARG(a && b, "sgg_lstm_fwd_seg2: null segment");
  SGG_CHECK_ARG(lstm_mw_ok(Ha, a->B) && lstm_mw_ok(Hb, b->B), "sgg_lstm_fwd_seg2: no four-wave kernel (Ha=%d Hb=%d)",
                Ha, Hb);
  return lstm_mw_fwd_seg2(to_mw(*a), Ha, to_mw(*b), Hb, (hipStream_t)stream);
}

extern "C" int sgg_lstm_fwd_seg3(const SggLstmSeg* a, int Ha, const SggLstmSeg* b, int Hb, const SggLstmSeg* c, int Hc,
                                 void* stream) {
  SGG_CHECK_ARG(a && b && c, "sgg_lstm_fwd_seg3: null segment");
  SGG_CHECK_ARG(lstm_mw_ok(Ha, a->B) && lstm_mw_ok(Hb, b->B) && lstm_mw_ok(Hc, c->B),
                "sgg_lstm_fwd_seg3: no four-wave kernel (Ha=%d Hb=%d Hc=%d)", Ha, Hb, Hc);
  return lstm_mw_fwd_seg3(to_mw(*a), Ha, to_mw(*b), Hb, to_mw(*c), Hc, (hipStream_t)stream);
}

extern "C" int sgg_lstm_bwd_shared(const float* A, const float* Whh, const float* h_all, const float* c_all,
                                   const float* act_all, const float* rel, const float* dh_last, int T, int B, int H,
                                   int t_sh, int Bsrc, float* drel_in, float* wpart, void* stream) {
  SGG_CHECK_ARG(A && Whh && h_all && c_all && act_all && rel && drel_in, "sgg_lstm_bwd_shared: null pointer");
  SGG_CHECK_ARG(T >= 1 && B >= 1 && t_sh >= 1 && lstm_mw_ok(H, B),
                "sgg_lstm_bwd_shared: bad sizes or no four-wave kernel (T=%d B=%d H=%d t_sh=%d)", T, B, H, t_sh);
  return lstm_mw_bwd(A, Whh, nullptr, h_all, c_all, act_all, rel, nullptr, dh_last, nullptr, T, B, H, 0, nullptr,
                     drel_in, nullptr, wpart, (hipStream_t)stream, nullptr, 0, 0, t_sh, Bsrc);
}

extern "C" int sgg_lstm_wpart_rows(int H, int B) {
  if (B < 0) return -1;
  return lstm_mw_ok(H, B) ? lstm_mw_wpart_rows(H, B) : 0;
}

extern "C" int sgg_lstm_fwd(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0,
                            const float* c0, const float* Wp, const float* bp, int T, int B, int H, int decoder, float* h_all,
                            float* c_all, float* act_all, float* rel_out, void* stream) {
  SGG_CHECK_ARG(rel && A && Whh && bias && h_all && c_all, "sgg_lstm_fwd: null pointer");
  SGG_CHECK_ARG(!decoder || (Wp && bp && rel_out), "sgg_lstm_fwd: decoder needs Wp, bp, rel_out");
  SGG_CHECK_ARG(T >= 1 && B >= 0, "sgg_lstm_fwd: bad sizes T=%d B=%d", T, B);
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  // saved states are read back by the backward of the same family
  // (sgg_lstm_state_floats): the four-wave family whenever lstm_mw_ok; the
  // MFMA rollout only without saved states (inference / no-grad samples)
  const bool mw = lstm_mw_ok(H, B);
  if (act_all && mw)
    return lstm_mw_fwd(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, H, decoder, h_all, c_all, act_all, rel_out, st);
  if (!act_all && lstm_fwd_mfma_ok(H, B) && !getenv("SGG_LSTM_NO_MFMA"))
    return lstm_fwd_mfma(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, H, decoder, h_all, c_all, nullptr, rel_out, st);
  if (mw)
    return lstm_mw_fwd(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, H, decoder, h_all, c_all, act_all, rel_out, st);
  if (lstm_unit_ok(H, decoder) && !getenv("SGG_LSTM_ROWS"))
    return lstm_unit_fwd(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, H, decoder, h_all, c_all, act_all, rel_out, st);
  switch (H) {
    case 16: return launch_lstm_fwd<16>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st);
    case 32: return launch_lstm_fwd<32>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st);
    case 48: return launch_lstm_fwd<48>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st);
    case 64: return launch_lstm_fwd<64>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st);
    default: SGG_CHECK_ARG(false, "sgg_lstm_fwd: hidden size %d not built (16/32/48/64)", H);
  }
}

static int dec_check(const SggDecInit* di, const float* A, const float* Whh, const float* bias, const float* Wp,
                     const float* bp, int T, int B, int H, float* h_all, float* c_all, float* act_all, float* rel_out,
                     const SggTrajOut* to) {
  SGG_CHECK_ARG(di && di->ctx && di->ped_scene && di->last_rel && (di->nz == 0 || di->z) && A && Whh && bias &&
                    ((h_all && c_all) || (!h_all && !c_all && !act_all)) && Wp && bp && rel_out,
                "sgg_lstm_fwd_dec: null pointer");
  SGG_CHECK_ARG(T >= 1 && B >= 0 && di->Bper >= 1 && B % di->Bper == 0 && di->Dc >= 1 && di->nz >= 0 &&
                    di->Dc + di->nz == H && di->ldc >= di->Dc && di->S >= 1,
                "sgg_lstm_fwd_dec: bad sizes (T=%d B=%d Bper=%d Dc=%d nz=%d H=%d)", T, B, di->Bper, di->Dc, di->nz, H);
  if (to) {
    SGG_CHECK_ARG(to->out && to->head && (!to->start || to->pos0), "sgg_lstm_fwd_dec: null pointer in SggTrajOut");
    SGG_CHECK_ARG(to->T0 >= 0 && to->ncol >= 1 && to->col0 >= 0 && to->col0 + to->ncol <= B &&
                      to->NB == (to->b ? 2 : 1) * to->ncol && to->ldh >= 2 * to->ncol &&
                      (!to->b || to->ldb >= 2 * to->ncol),
                  "sgg_lstm_fwd_dec: bad SggTrajOut sizes (NB=%d T0=%d col0=%d ncol=%d B=%d)", to->NB, to->T0,
                  to->col0, to->ncol, B);
  }
  return 0;
}

extern "C" int sgg_lstm_fwd_dec_seg(const SggDecInit* di, const float* A, const float* Whh, const float* bias,
                                    const float* Wp, const float* bp, int T, int B, int H, float* h_all, float* c_all,
                                    float* act_all, float* rel_out, float* rel0_out, const SggTrajOut* to,
                                    const SggLstmSeg* pre, int Hp, void* stream) {
  if (int rc = dec_check(di, A, Whh, bias, Wp, bp, T, B, H, h_all, c_all, act_all, rel_out, to)) return rc;
  SGG_CHECK_ARG(pre && B >= 1 && act_all && lstm_mw_ok(H, B) && lstm_mw_ok(Hp, pre->B),
                "sgg_lstm_fwd_dec_seg: needs a saving four-wave decoder and a prefix segment (H=%d B=%d Hp=%d)", H, B,
                Hp);
  return lstm_mw_fwd_dec_seg(A, Whh, bias, Wp, bp, T, B, H, h_all, c_all, act_all, rel_out, di, rel0_out, to,
                             to_mw(*pre), Hp, (hipStream_t)stream);
}

extern "C" int sgg_lstm_fwd_dec2(const SggDecInit* di, const SggDecInit* di2, const float* A, const float* Whh,
                                 const float* bias, const float* Wp, const float* bp, int T, int B, int B2, int H,
                                 float* rel_out, float* rel_out2, const SggTrajOut* to2, void* stream) {
  if (int rc = dec_check(di, A, Whh, bias, Wp, bp, T, B, H, nullptr, nullptr, nullptr, rel_out, nullptr)) return rc;
  if (int rc = dec_check(di2, A, Whh, bias, Wp, bp, T, B2, H, nullptr, nullptr, nullptr, rel_out2, to2)) return rc;
  SGG_CHECK_ARG(B >= 1 && B2 >= 1 && lstm_fwd_mfma_ok(H, B) && !getenv("SGG_LSTM_NO_MFMA"),
                "sgg_lstm_fwd_dec2: the batch-MFMA rollout family only (H=%d B=%d)", H, B);
  return lstm_fwd_mfma_dec2(di, di2, A, Whh, bias, Wp, bp, T, B, B2, H, rel_out, rel_out2, to2, (hipStream_t)stream);
}

extern "C" int sgg_lstm_fwd_dec(const SggDecInit* di, const float* A, const float* Whh, const float* bias,
                                const float* Wp, const float* bp, int T, int B, int H, float* h_all, float* c_all,
                                float* act_all, float* rel_out, float* rel0_out, const SggTrajOut* to,
                                void* stream) {
  if (int rc = dec_check(di, A, Whh, bias, Wp, bp, T, B, H, h_all, c_all, act_all, rel_out, to)) return rc;
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const bool mw = lstm_mw_ok(H, B);
  if (act_all && mw)
    return lstm_mw_fwd(nullptr, A, Whh, bias, nullptr, nullptr, Wp, bp, T, B, H, 1, h_all, c_all, act_all, rel_out,
                       st, nullptr, 0, nullptr, 0, nullptr, di, rel0_out, to);
  if (!act_all && lstm_fwd_mfma_ok(H, B) && !getenv("SGG_LSTM_NO_MFMA")) {
    if (to) {   // the batch-MFMA family writes the discriminator input as a second segment (alone here)
      SGG_CHECK_ARG(!h_all, "sgg_lstm_fwd_dec: the batch-MFMA family writes the discriminator input without a "
                            "final state (h_all NULL)");
      return lstm_fwd_mfma_dec2(di, di, A, Whh, bias, Wp, bp, T, 0, B, H, nullptr, rel_out, to, st);
    }
    return lstm_fwd_mfma(nullptr, A, Whh, bias, nullptr, nullptr, Wp, bp, T, B, H, 1, h_all, c_all, nullptr, rel_out,
                         st, di);
  }
  SGG_CHECK_ARG(!to || mw, "sgg_lstm_fwd_dec: no family writes the discriminator input for H=%d B=%d", H, B);
  if (!act_all && mw)
    return lstm_mw_fwd(nullptr, A, Whh, bias, nullptr, nullptr, Wp, bp, T, B, H, 1, h_all, c_all, nullptr, rel_out, st,
                       nullptr, 0, nullptr, 0, nullptr, di, nullptr, to);
  SGG_CHECK_ARG(false, "sgg_lstm_fwd_dec: no fused decoder start for H=%d B=%d (use sgg_decoder_init)", H, B);
}

extern "C" int sgg_lstm_bwd(const float* A, const float* Whh, const float* Wp, const float* h_all, const float* c_all,
                            const float* act_all, const float* rel, const float* rel_out, const float* dh_last,
                            const float* dout, int T, int B, int H, int decoder, float* dG, float* dh0,
                            float* drel_in, float* drel_tot, float* wpart, void* stream) {
  SGG_CHECK_ARG(A && Whh && c_all && act_all && drel_in, "sgg_lstm_bwd: null pointer");
  SGG_CHECK_ARG(!decoder || (Wp && dout && drel_tot), "sgg_lstm_bwd: decoder needs Wp, dout, drel_tot");
  SGG_CHECK_ARG(T >= 1 && B >= 0, "sgg_lstm_bwd: bad sizes");
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (lstm_mw_ok(H, B)) {
    SGG_CHECK_ARG(!wpart || (h_all && rel && (!decoder || rel_out)),
                  "sgg_lstm_bwd: weight gradients need h_all, rel (and rel_out for the decoder)");
    return lstm_mw_bwd(A, Whh, Wp, h_all, c_all, act_all, rel, rel_out, dh_last, dout, T, B, H, decoder, dh0, drel_in,
                       drel_tot, wpart, st);
  }
  SGG_CHECK_ARG(!wpart, "sgg_lstm_bwd: this (H=%d, B=%d) has no in-kernel weight gradient (sgg_lstm_wpart_rows = 0)", H, B);
  SGG_CHECK_ARG(dG, "sgg_lstm_bwd: dG is required unless the in-kernel form is used");
  if (lstm_unit_ok(H, decoder) && !getenv("SGG_LSTM_ROWS"))
    return lstm_unit_bwd(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, H, decoder, dG, dh0, drel_in, drel_tot, st);
  switch (H) {
    case 16: return launch_lstm_bwd<16>(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot, st);
    case 32: return launch_lstm_bwd<32>(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot, st);
    case 48: return launch_lstm_bwd<48>(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot, st);
    case 64: return launch_lstm_bwd<64>(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot, st);
    default: SGG_CHECK_ARG(false, "sgg_lstm_bwd: hidden size %d not built (16/32/48/64)", H);
  }
}
