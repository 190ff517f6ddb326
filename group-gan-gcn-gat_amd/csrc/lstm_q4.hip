// LSTM encoder segments with FOUR peds per workgroup on
// v_mfma_f32_4x4x1_16b_f32 (reference sgan/models.py:62-92, Encoder.forward).
//
// The four-wave family (lstm_mw.hip) gives a workgroup 16 peds -- the width
// of a 16x16x4 MFMA -- so the discriminator's H = 48 sequences of 1280 /
// 2560 peds run 80 / 160 workgroups: a third / two thirds of the CUs, each
// step a chain of 39 MFMAs per SIMD.  A 4x4x1 MFMA is sixteen independent
// 4 x 4 blocks: block b of wave w takes unit u = 16 w + b, its rows are the
// unit's four gates (i, f, g, o) and its columns the workgroup's four peds,
// so after the k loop lane (b, j) holds the four gates of (unit u, ped j):
//   G_b (4 gates x 4 peds) += W_hh[gate rows of u][k] (A, per lane) x h[k][peds] (B)
// over k = 0 .. H - 1 plus the input rows (A r_x, A r_y, bias) -- H + 3
// MFMAs per wave and step, two accumulators alternating over k.  H / 16
// waves per workgroup, B / 4 workgroups: four times the workgroups of the
// 16-ped form and a third of its per-SIMD step chain (measured on the
// recurrence alone, tools/lstm_q4_probe.hip: 12 steps of 1280 peds 12.6 us
// vs 24.5 us).  Activations and the cell update run on the lane's own four
// gate values; h goes to LDS (ped-major, read back as the next step's B
// operand with 16-byte reads) -- one barrier per step.
//
// Saved states are written in the four-wave family's TILE-NATIVE layout
// (lstm_mw.hip header: act float4 per (16-ped block, step, slot, lane), the
// cells per (block, step, wave, lane, slot)), so the four-wave backward
// consumes them unchanged and a segment may continue from a prefix the
// four-wave kernels ran (t0 > 0: the state of ped p mod Bsrc at step t0).
// The projection epilogue U = h_T Wu^T + cu (the pooling MLP's h half,
// models.py:538) runs on the same MFMA: rows = 64 output features per
// instruction group, columns = the four peds.
//
// Rounding: each MFMA adds one product (fma order: input rows, then k
// ascending, even k into one accumulator and odd k into the other, summed at
// the end) -- the same function as the 16-ped kernels up to fp32
// reassociation, not bitwise equal to them.
#include <stdlib.h>

#include "sgg_common.h"

namespace sgg {

namespace {

constexpr float kQ4NegLog2e = -1.4426950408889634f;
__device__ __forceinline__ float q4_gate(float x, float s, float nsl) {
  return fmaf(s, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * nsl)), 1.f - s);
}
__device__ __forceinline__ float q4_tanh(float x) {
  return fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * (2.f * kQ4NegLog2e))), -1.f);
}

constexpr int kQ4Peds = 4;

template <int H>
struct Q4Cfg {
  static constexpr int NW = H / 16;          // waves (16 units each)
  static constexpr int HP = H + 4;           // LDS row pitch of h (ped-major; 16-byte rows)
  static constexpr int MU = H / 16, KS = H / 4;   // the four-wave family's tile parameters
};

// the four-wave family's tile-native positions of (unit u, ped p)
struct MwPos {
  int b16, lane16, j16, g16, i16;
};
template <int H>
__device__ __forceinline__ MwPos mw_pos(int u, int p) {
  constexpr int MU = Q4Cfg<H>::MU;
  MwPos r;
  r.b16 = p >> 4;
  const int q16 = (u & 15) >> 2;
  r.lane16 = q16 * 16 + (p & 15);
  r.j16 = 4 * (u >> 4) + (u & 3);   // slot_unit(j16, q16) = u
  r.g16 = r.j16 / MU;
  r.i16 = r.j16 - r.g16 * MU;
  return r;
}

// One segment on workgroup blk.  NWT = the launch's waves per workgroup (a
// multi-segment launch sizes it for its widest H): waves w >= H / 16 only
// pass the barriers.  DEC: the decoder (models.py:142-178) -- h0 / rel0 from
// the SggDecInit, the hidden2pos feedback r_t = Wp h_t + bp folded into the
// weights from step 1 on (W_hh + A Wp, bias + A bp: the four-wave kernels'
// fold, the same fmaf expressions), r_t formed off the critical path (each
// wave's unit partials by lane shuffles, the waves' sums after the step's
// barrier) into rel_out and the discriminator input (SggTrajOut).
template <int H, int NWT, bool DEC, bool SAVE>
__device__ __forceinline__ void q4_fwd_body(const MwSeg& sg, int blk) {
  constexpr int NW = Q4Cfg<H>::NW, HP = Q4Cfg<H>::HP, MU = Q4Cfg<H>::MU, KS = Q4Cfg<H>::KS;
  __shared__ __attribute__((aligned(16))) float hs[2][kQ4Peds][HP];
  __shared__ float2 rpart[2][NW][kQ4Peds];
  const int w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (NWT > NW && w0 >= NW) {   // (uniform per wave) an idle wave: the body's barriers only
    __syncthreads();
    for (int t = 0; t < sg.T; ++t) __syncthreads();
    return;
  }
  const float* __restrict__ rel = sg.rel;
  const float* __restrict__ Whh = sg.Whh;
  float* __restrict__ h_all = sg.h_all;
  float* __restrict__ c_tile = sg.c_tile;
  float* __restrict__ act_tile = sg.act_tile;
  const int T = sg.T, B = sg.B, Bl = sg.Bl, t0 = sg.t0, Tl = sg.Tl;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int b = lane >> 2, j = lane & 3;
  const int u = 16 * w + b;
  const int ped = blk * kQ4Peds + j;
  const int pc = ped < B ? ped : B - 1;   // padded lanes: the clamped ped's values, benign duplicate stores
  // A operand: lane (b, i = j) supplies the rows of gate j of unit u
  const int row = j * H + u;
  float wk[H];
#pragma unroll
  for (int k = 0; k < H; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(Whh + (size_t)row * H + k);
    wk[k] = v.x;
    wk[k + 1] = v.y;
    wk[k + 2] = v.z;
    wk[k + 3] = v.w;
  }
  const float a0 = sg.A[2 * row], a1 = sg.A[2 * row + 1];
  float bb = sg.bias[row];
  const MwPos mp = mw_pos<H>(u, pc);
  // the state entering step t0
  float h, c;
  if (t0 > 0) {
    const int spc = pc % sg.Bsrc;
    const MwPos sp = mw_pos<H>(u, spc);
    h = h_all[((size_t)t0 * Bl + spc) * H + u];
    c = c_tile[((((size_t)sp.b16 * (Tl + 1) + t0) * 4 + sp.g16) * 64 + sp.lane16) * MU + sp.i16];
  } else {
    h = (DEC && sg.di.ctx) ? dec_h0(sg.di, pc, u) : sg.h0 ? sg.h0[(size_t)pc * H + u] : 0.f;
    c = sg.c0 ? sg.c0[(size_t)pc * H + u] : 0.f;
    if (SAVE) {
      h_all[(size_t)pc * H + u] = h;
      c_tile[((((size_t)mp.b16 * (Tl + 1)) * 4 + mp.g16) * 64 + mp.lane16) * MU + mp.i16] = c;
    }
  }
  hs[0][j][u] = h;
  const float wp0 = DEC ? sg.Wp[u] : 0.f, wp1 = DEC ? sg.Wp[H + u] : 0.f;
  const float bp0 = DEC ? sg.bp[0] : 0.f, bp1 = DEC ? sg.bp[1] : 0.f;
  const float2* __restrict__ rel2 = reinterpret_cast<const float2*>(rel);
  float2 xn;
  if (DEC)   // the first input: rel0 (the decoder's later inputs are its own outputs, folded)
    xn = sg.di.ctx ? make_float2(dec_rel0(sg.di, pc, 0), dec_rel0(sg.di, pc, 1)) : rel2[pc];
  else
    xn = rel2[(size_t)t0 * B + pc];
  const SggTrajOut& to = sg.to;
  const int tcol = pc - to.col0;   // this lane's column of the discriminator input
  const bool tlive = DEC && to.out != nullptr && tcol >= 0 && tcol < to.ncol;
  if (DEC) {
    if (sg.rel0_out && w == 0 && b == 0) reinterpret_cast<float2*>(sg.rel0_out)[pc] = xn;   // (the backward's x_0)
    if (to.out != nullptr) {
      // the discriminator input's entries that do not come from the
      // recurrence (head steps, the b half, start positions), for this
      // workgroup's peds (the four-wave kernels' SggTrajOut prologue)
      const int dup = to.b ? 2 : 1;
      const int nh = to.T0 * dup, nb = to.b ? T : 0, ns = to.start ? dup : 0;
      const int nto = kQ4Peds * (nh + nb + ns);
      float2* o2 = reinterpret_cast<float2*>(to.out);
      for (int e = threadIdx.x; e < nto; e += 64 * NW) {
        const int i = e % kQ4Peds, ww = e / kQ4Peds;
        const int col = min(blk * kQ4Peds + i, B - 1) - to.col0;
        if (col < 0 || col >= to.ncol) continue;
        if (ww < nh) {   // head step t (either half)
          const int t = ww / dup, half = ww - t * dup;
          o2[(size_t)t * to.NB + col + half * to.ncol] = reinterpret_cast<const float2*>(to.head + (size_t)t * to.ldh)[col];
        } else if (ww < nh + nb) {   // the b half's step T0 + t
          const int t = ww - nh;
          o2[(size_t)(to.T0 + t) * to.NB + to.ncol + col] = reinterpret_cast<const float2*>(to.b + (size_t)t * to.ldb)[col];
        } else {
          reinterpret_cast<float2*>(to.start)[col + (ww - nh - nb) * to.ncol] =
              reinterpret_cast<const float2*>(to.pos0)[col];
        }
      }
    }
  }
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const int rb = t & 1;
    if (DEC && t == 1) {
      // fold the hidden2pos feedback into the recurrence (W_hh + A Wp, bias + A bp)
#pragma unroll
      for (int k = 0; k < H; ++k) wk[k] = fmaf(a1, sg.Wp[H + k], fmaf(a0, sg.Wp[k], wk[k]));
      bb = fmaf(a1, bp1, fmaf(a0, bp0, bb));
    }
    const float2 x = xn;   // (loaded a step ahead)
    if (!DEC && t + 1 < T) xn = rel2[(size_t)(t0 + t + 1) * B + pc];
    floatx4 acc0 = floatx4{0.f, 0.f, 0.f, 0.f}, acc1 = floatx4{0.f, 0.f, 0.f, 0.f};
    if (!DEC || t == 0) {
      acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a0, x.x, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a1, x.y, acc1, 0, 0, 0);
    }
    acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(bb, 1.f, acc0, 0, 0, 0);
    const float* hr = &hs[rb][j][0];
#pragma unroll
    for (int k = 0; k < H; k += 4) {
      const float4 hv = *reinterpret_cast<const float4*>(hr + k);
      acc1 = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[k], hv.x, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[k + 1], hv.y, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[k + 2], hv.z, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[k + 3], hv.w, acc0, 0, 0, 0);
    }
    const floatx4 g = acc0 + acc1;
    float a[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = r == 2 ? 2.f : 1.f;
      a[r] = q4_gate(g[r], s, s * kQ4NegLog2e);
    }
    c = fmaf(a[1], c, a[0] * a[2]);
    h = a[3] * q4_tanh(c);
    hs[rb ^ 1][j][u] = h;
    if (SAVE) {
      reinterpret_cast<float4*>(act_tile)[(((size_t)mp.b16 * Tl + t0 + t) * KS + mp.j16) * 64 + mp.lane16] =
          make_float4(a[0], a[1], a[2], a[3]);
      c_tile[((((size_t)mp.b16 * (Tl + 1) + t0 + t + 1) * 4 + mp.g16) * 64 + mp.lane16) * MU + mp.i16] = c;
    }
    if (SAVE || (t == T - 1 && h_all)) h_all[((size_t)(t0 + (SAVE ? t + 1 : T)) * Bl + pc) * H + u] = h;
    if (DEC) {   // this wave's units' share of r_t = Wp h_t (the 16 lanes of ped j)
      float px = wp0 * h, py = wp1 * h;
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) {
        px += __shfl_xor(px, o);
        py += __shfl_xor(py, o);
      }
      if (b == 0) rpart[rb][w][j] = make_float2(px, py);
    }
    __syncthreads();
    if (DEC && w == 0 && b == 0) {   // r_t = sum of the waves' shares + bp
      float2 r = rpart[rb][0][j];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) {
        const float2 q = rpart[rb][ww][j];
        r.x += q.x;
        r.y += q.y;
      }
      r.x += bp0;
      r.y += bp1;
      reinterpret_cast<float2*>(sg.rel_out)[(size_t)t * B + pc] = r;
      if (tlive) reinterpret_cast<float2*>(to.out)[(size_t)(to.T0 + t) * to.NB + tcol] = r;
    }
  }

  // projection epilogue: U[p][n] = sum_k h_T[p][k] Wu[n][k] + cu[n]; group m
  // = output rows 64 m .. 64 m + 63 (block b: rows 64 m + 4 b + i), waves
  // take groups w, w + NW, ...
  float* __restrict__ U = sg.U;
  if (U) {
    const float* __restrict__ Wu = sg.Wu;
    const int ldwu = sg.ldwu, NU = sg.NU;
    const bool vec = ((reinterpret_cast<uintptr_t>(Wu) | ((uintptr_t)ldwu * 4)) & 15) == 0;
    const float* hr = &hs[T & 1][j][0];
    float hk[H];
#pragma unroll
    for (int k = 0; k < H; k += 4) {
      const float4 hv = *reinterpret_cast<const float4*>(hr + k);
      hk[k] = hv.x;
      hk[k + 1] = hv.y;
      hk[k + 2] = hv.z;
      hk[k + 3] = hv.w;
    }
    for (int m = w; 64 * m < NU; m += NW) {
      const int n = 64 * m + 4 * b + j;   // this lane's A row
      const bool live = n < NU;
      const float* wr = Wu + (size_t)(live ? n : 0) * ldwu;
      float wv[H];
      if (vec) {
#pragma unroll
        for (int k = 0; k < H; k += 4) {
          const float4 v = *reinterpret_cast<const float4*>(wr + k);
          wv[k] = keep_if(v.x, live);
          wv[k + 1] = keep_if(v.y, live);
          wv[k + 2] = keep_if(v.z, live);
          wv[k + 3] = keep_if(v.w, live);
        }
      } else {
#pragma unroll
        for (int k = 0; k < H; ++k) wv[k] = keep_if(wr[k], live);
      }
      floatx4 e0 = floatx4{0.f, 0.f, 0.f, 0.f}, e1 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < H; k += 2) {
        e0 = __builtin_amdgcn_mfma_f32_4x4x1f32(wv[k], hk[k], e0, 0, 0, 0);
        e1 = __builtin_amdgcn_mfma_f32_4x4x1f32(wv[k + 1], hk[k + 1], e1, 0, 0, 0);
      }
      const floatx4 e = e0 + e1;
      const int n0 = 64 * m + 4 * b;   // lane (b, j): rows n0 .. n0 + 3 of ped j
      if (n0 < NU) {
        const float4 cv = *reinterpret_cast<const float4*>(sg.cu + n0);
        *reinterpret_cast<float4*>(U + (size_t)pc * NU + n0) =
            make_float4(e[0] + cv.x, e[1] + cv.y, e[2] + cv.z, e[3] + cv.w);
      }
    }
  }
}

// Encoder backward (sgg_lstm_bwd / _shared / _tail for encoders) on the
// four-wave family's tile-native saved states.  Lane (b, j) = (unit u =
// 16 w + b, ped j) turns dh_t (the waves' partials of W^T dG_{t+1} from LDS,
// + dh_last at t = T - 1) into its four gate gradients with the saved
// activations and cells (loaded a step ahead) -- the four-wave backward's
// expressions -- and the wave runs its rows' share of
//   dh_{t-1}[k][peds] = sum over (unit u' of the wave, gate r) W_hh[r H + u'][k] dG[r H + u'][peds]
// on the 4x4x1 MFMA: block b = output rows k = 4 b .. 4 b + 3, one MFMA per
// (u', r) (64 per wave and step), the A operand this lane's W_hh^T entries
// (registers), the B operand the wave's dG read back from LDS.  drel_in[t] =
// A^T dG_t: lane partials reduced by shuffles, the waves' sums after the
// step's barrier.  t_sh > 0: the states of steps < t_sh are ped (p mod
// Bsrc)'s (a shared prefix, as in the four-wave backward).  t_stop > 0:
// input gradients of steps >= t_stop only (no weight gradients).
// WGRAD: the workgroup's slab row [dW_hh (4H x H) | db (4H) | dA (4H x 2)]
// over its four peds -- dW_hh += dG_t h_{t-1}^T on the same MFMA (block b =
// unit u's four gate rows, columns k = 4 s + c, K = the four peds; 12 / 8
// column sets per wave and step for H = 48 / 32), h_{t-1} staged in LDS a
// step ahead; db, dA on the VALU.  Sums over the peds in a fixed order.
template <int H, bool WGRAD>
__global__ void __launch_bounds__(64 * (H / 16)) q4_bwd_kernel(
    const float* __restrict__ A, const float* __restrict__ Whh, const float* __restrict__ h_all,
    const float* __restrict__ c_tile, const float* __restrict__ act_tile, const float* __restrict__ rel,
    const float* __restrict__ dh_last, int T, int B, int t_stop, int t_sh, int Bsrc, float* __restrict__ dh0,
    float* __restrict__ drel_in, float* __restrict__ wpart) {
  constexpr int NW = Q4Cfg<H>::NW, MU = Q4Cfg<H>::MU, KS = Q4Cfg<H>::KS, G4 = 4 * H;
  constexpr int NB = H / 4;   // output blocks of dh (k = 4 b + i); column sets of dW_hh
  __shared__ __attribute__((aligned(16))) float dgl[NW][kQ4Peds][16][4];      // dG of the wave's (unit, gate), per ped
  __shared__ __attribute__((aligned(16))) float part[2][NW][kQ4Peds][H];      // the waves' dh partials
  __shared__ __attribute__((aligned(16))) float hst[WGRAD ? 2 : 1][kQ4Peds][4][NB];   // h_{t-1}[4 s + c] at [p][c][s]
  __shared__ float2 fbp[2][NW][kQ4Peds];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int b = lane >> 2, j = lane & 3;
  const int u = 16 * w + b;
  const int ped = blockIdx.x * kQ4Peds + j;
  const bool valid = ped < B;
  const int pc = valid ? ped : B - 1;
  // A operand of term (u', r): W_hh[r H + 16 w + u'][4 b + i], i = j (blocks b >= NB: zero)
  float wt[16][4];
#pragma unroll
  for (int up = 0; up < 16; ++up)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      wt[up][r] = b < NB ? Whh[(size_t)(r * H + 16 * w + up) * H + 4 * (b < NB ? b : 0) + j] : 0.f;
  float aa0[4], aa1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    aa0[r] = A[2 * (r * H + u)];
    aa1[r] = A[2 * (r * H + u) + 1];
  }
  float dc = 0.f;
  const float dhl = dh_last ? dh_last[(size_t)pc * H + u] : 0.f;
  const MwPos mp = mw_pos<H>(u, pc);
  const int spc = t_sh > 0 ? pc % Bsrc : pc;
  const MwPos ms = mw_pos<H>(u, spc);   // a shared prefix's source ped
  // saved states of step t, one step ahead: the gates' activations, c_t,
  // c_{t-1}; WGRAD: the step input r_t and h_{t-1} = h_all[t]
  float4 nact;
  float nc, ncp, nh = 0.f;
  float2 nr = make_float2(0.f, 0.f);
  auto load_step = [&](int t) {
    const MwPos& pa = t < t_sh ? ms : mp;
    nact = reinterpret_cast<const float4*>(act_tile)[(((size_t)pa.b16 * T + t) * KS + pa.j16) * 64 + pa.lane16];
    const MwPos& p1 = t + 1 <= t_sh ? ms : mp;
    nc = c_tile[((((size_t)p1.b16 * (T + 1) + t + 1) * 4 + p1.g16) * 64 + p1.lane16) * MU + p1.i16];
    const MwPos& p0 = t <= t_sh ? ms : mp;
    ncp = c_tile[((((size_t)p0.b16 * (T + 1) + t) * 4 + p0.g16) * 64 + p0.lane16) * MU + p0.i16];
    if (WGRAD) {
      nr = reinterpret_cast<const float2*>(rel)[(size_t)t * B + pc];
      nh = h_all[((size_t)t * B + (t <= t_sh ? spc : pc)) * H + u];
    }
  };
  floatx4 dw[WGRAD ? NB : 1];
  float db[4], dax[4], day[4];
#pragma unroll
  for (int s = 0; s < (WGRAD ? NB : 1); ++s) dw[s] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) db[r] = dax[r] = day[r] = 0.f;
  load_step(T - 1);
  if (WGRAD) {   // h_{T-2} of step T - 1 into its buffer (read by every wave)
    hst[(T - 1) & 1][j][u & 3][u >> 2] = nh;
    __syncthreads();
  }
  for (int t = T - 1; t >= t_stop; --t) {
    const int cur = t & 1;
    const float4 ac = nact;
    const float cc = nc, ccp = ncp;
    const float2 rin = nr;
    if (t > t_stop) load_step(t - 1);   // in flight while this step computes
    float dhv = dhl;
    if (t < T - 1) {
      dhv = part[cur ^ 1][0][j][u];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) dhv += part[cur ^ 1][ww][j][u];
    }
    const float ig = ac.x, fg = ac.y, gg = ac.z, og = ac.w;
    const float tc = q4_tanh(cc);
    const float d_o = dhv * tc;
    const float dct = fmaf(dhv * og, 1.f - tc * tc, dc);
    dc = dct * fg;
    const float vv[4] = {keep_if(dct * gg * ig * (1.f - ig), valid), keep_if(dct * ccp * fg * (1.f - fg), valid),
                         keep_if(dct * ig * (1.f - gg * gg), valid), keep_if(d_o * og * (1.f - og), valid)};
    if (WGRAD) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        db[r] += vv[r];
        dax[r] = fmaf(vv[r], rin.x, dax[r]);
        day[r] = fmaf(vv[r], rin.y, day[r]);
      }
    }
    // drel_in[t]: this lane's A^T dG terms, summed over the wave's units of ped j
    float f0 = fmaf(aa0[3], vv[3], fmaf(aa0[2], vv[2], fmaf(aa0[1], vv[1], aa0[0] * vv[0])));
    float f1 = fmaf(aa1[3], vv[3], fmaf(aa1[2], vv[2], fmaf(aa1[1], vv[1], aa1[0] * vv[0])));
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) {
      f0 += __shfl_xor(f0, o);
      f1 += __shfl_xor(f1, o);
    }
    if (b == 0) fbp[cur][w][j] = make_float2(f0, f1);
    // the wave's dG to LDS, read back as the MFMA operands (wave-local)
    *reinterpret_cast<float4*>(&dgl[w][j][b][0]) = make_float4(vv[0], vv[1], vv[2], vv[3]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    floatx4 acc0 = floatx4{0.f, 0.f, 0.f, 0.f}, acc1 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int up = 0; up < 16; ++up) {
      const float4 g4 = *reinterpret_cast<const float4*>(&dgl[w][j][up][0]);
      acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt[up][0], g4.x, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt[up][1], g4.y, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt[up][2], g4.z, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_4x4x1f32(wt[up][3], g4.w, acc1, 0, 0, 0);
    }
    const floatx4 dp = acc0 + acc1;   // rows 4 b .. 4 b + 3 of ped j
    if (b < NB) *reinterpret_cast<float4*>(&part[cur][w][j][4 * b]) = make_float4(dp[0], dp[1], dp[2], dp[3]);
    if (WGRAD) {
      // dW_hh[gate i][u][4 s + c] += sum over peds p of dG[i][u][p] h_{t-1}[4 s + c][p]:
      // A = dG of (unit u, gate i = j) for ped p, B = h_{t-1}[4 s + c = j][p]
#pragma unroll
      for (int p = 0; p < kQ4Peds; ++p) {
        const float ga = dgl[w][p][b][j];
#pragma unroll
        for (int s4 = 0; s4 < NB; s4 += 4) {
          const float4 hb = *reinterpret_cast<const float4*>(&hst[cur][p][j][s4]);
          dw[s4] = __builtin_amdgcn_mfma_f32_4x4x1f32(ga, hb.x, dw[s4], 0, 0, 0);
          dw[s4 + 1] = __builtin_amdgcn_mfma_f32_4x4x1f32(ga, hb.y, dw[s4 + 1], 0, 0, 0);
          dw[s4 + 2] = __builtin_amdgcn_mfma_f32_4x4x1f32(ga, hb.z, dw[s4 + 2], 0, 0, 0);
          dw[s4 + 3] = __builtin_amdgcn_mfma_f32_4x4x1f32(ga, hb.w, dw[s4 + 3], 0, 0, 0);
        }
      }
      if (t > 0) hst[cur ^ 1][j][u & 3][u >> 2] = nh;   // h_{t-2} of step t - 1 (read after the barrier)
    }
    __syncthreads();
    if (w == 0 && b == 0 && valid) {
      float2 r = fbp[cur][0][j];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) {
        const float2 q = fbp[cur][ww][j];
        r.x += q.x;
        r.y += q.y;
      }
      reinterpret_cast<float2*>(drel_in)[(size_t)t * B + ped] = r;
    }
  }
  if (t_stop > 0 && w == 0 && b == 0 && valid)   // the skipped steps' input gradients are defined as zero
    for (int t = 0; t < t_stop; ++t) reinterpret_cast<float2*>(drel_in)[(size_t)t * B + ped] = make_float2(0.f, 0.f);
  if (dh0 && valid) {   // dh0 = W_hh^T dG_0 (the waves' partials of the last step, t = 0)
    float v = part[0][0][j][u];
#pragma unroll
    for (int ww = 1; ww < NW; ++ww) v += part[0][ww][j][u];
    dh0[(size_t)ped * H + u] = v;
  }
  if (WGRAD) {
    float* row = wpart + (size_t)blockIdx.x * (G4 * H + G4 + 2 * G4);
    // dW_hh: lane (b, c) holds rows (gate i, unit u), columns 4 s + c
#pragma unroll
    for (int s = 0; s < NB; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) row[(size_t)(i * H + u) * H + 4 * s + j] = dw[s][i];
    // db, dA of (gate r, unit u): sums over the four peds (lanes j of the quad)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = db[r], x = dax[r], y = day[r];
#pragma unroll
      for (int o = 1; o < 4; o <<= 1) {
        a += __shfl_xor(a, o);
        x += __shfl_xor(x, o);
        y += __shfl_xor(y, o);
      }
      if (j == 0) {
        row[G4 * H + r * H + u] = a;
        row[G4 * H + G4 + 2 * (r * H + u)] = x;
        row[G4 * H + G4 + 2 * (r * H + u) + 1] = y;
      }
    }
  }
}

template <int H, bool SAVE>
__global__ void __launch_bounds__(64 * (H / 16)) q4_fwd_seg_kernel(const MwSeg sg) {
  q4_fwd_body<H, H / 16, false, SAVE>(sg, blockIdx.x);
}

constexpr int q4_max(int a, int b) { return a > b ? a : b; }

// two / three independent encoder segments in one launch (the workgroups of
// a, then b, then c), e.g. the generator's encoders of two batches beside the
// discriminator's observed-steps prefix (sgg_lstm_fwd_seg3)
template <int HA, bool SA, int HB, bool SB>
__global__ void __launch_bounds__(64 * q4_max(HA, HB) / 16) q4_fwd2_kernel(const MwSeg a, const MwSeg b, int na) {
  constexpr int NWT = q4_max(HA, HB) / 16;
  const int blk = blockIdx.x;
  if (blk < na)
    q4_fwd_body<HA, NWT, false, SA>(a, blk);
  else
    q4_fwd_body<HB, NWT, false, SB>(b, blk - na);
}

// a decoder segment (a) beside an encoder segment (b): the generator step's
// decoder with the discriminator's observed-steps prefix (sgg_lstm_fwd_dec_seg)
template <int HA, bool SA, int HB, bool SB>
__global__ void __launch_bounds__(64 * q4_max(HA, HB) / 16) q4_fwd2d_kernel(const MwSeg a, const MwSeg b, int na) {
  constexpr int NWT = q4_max(HA, HB) / 16;
  const int blk = blockIdx.x;
  if (blk < na)
    q4_fwd_body<HA, NWT, true, SA>(a, blk);
  else
    q4_fwd_body<HB, NWT, false, SB>(b, blk - na);
}

template <int HA, bool SA, int HB, bool SB, int HC, bool SC>
__global__ void __launch_bounds__(64 * q4_max(q4_max(HA, HB), HC) / 16)
    q4_fwd3_kernel(const MwSeg a, const MwSeg b, const MwSeg c, int na, int nb) {
  constexpr int NWT = q4_max(q4_max(HA, HB), HC) / 16;
  const int blk = blockIdx.x;
  if (blk < na)
    q4_fwd_body<HA, NWT, false, SA>(a, blk);
  else if (blk < na + nb)
    q4_fwd_body<HB, NWT, false, SB>(b, blk - na);
  else
    q4_fwd_body<HC, NWT, false, SC>(c, blk - na - nb);
}

int q4_blocks(const MwSeg& s) { return (s.B + kQ4Peds - 1) / kQ4Peds; }

template <int H>
int launch_q4(const MwSeg& s, hipStream_t st) {
  const dim3 grid(q4_blocks(s)), blk(64 * (H / 16));
  if (s.act_tile)
    hipLaunchKernelGGL((q4_fwd_seg_kernel<H, true>), grid, blk, 0, st, s);
  else
    hipLaunchKernelGGL((q4_fwd_seg_kernel<H, false>), grid, blk, 0, st, s);
  SGG_RETURN_LAUNCH("sgg_lstm_fwd_seg (q4)");
}

}  // namespace

// SGG_LSTM_Q4=1 (or sgg_lstm_q4_enable(1)) routes encoder sequences to the
// four-peds kernels; otherwise they stay on the four-wave kernels
static int g_q4_on = -1;

bool lstm_q4_ok(int H, int B) {
  if (g_q4_on < 0) {
    const char* e = getenv("SGG_LSTM_Q4");
    g_q4_on = e && e[0] == '1';
  }
  return g_q4_on && (H == 32 || H == 48) && B >= 1;
}

int lstm_q4_enable(int on) {
  const int prev = lstm_q4_ok(32, 1) ? 1 : 0;
  g_q4_on = on ? 1 : 0;
  return prev;
}

static int q4_seg_check(const MwSeg& s, const char* fn) {
  SGG_CHECK_ARG(!s.U || (s.cu && (reinterpret_cast<uintptr_t>(s.cu) & 15) == 0 && s.NU % 16 == 0),
                "%s (q4): cu must be 16-byte aligned, NU %% 16 == 0", fn);
  SGG_CHECK_ARG((reinterpret_cast<uintptr_t>(s.Whh) & 15) == 0, "%s (q4): W_hh must be 16-byte aligned", fn);
  return 0;
}

// the pairs / triples the training step launches; 0 = no such kernel here
int lstm_q4_fwd_seg2(const MwSeg& a, int Ha, const MwSeg& b, int Hb, hipStream_t st) {
  if (!(Ha == 32 && Hb == 48 && b.act_tile)) return 1;
  if (int rc = q4_seg_check(a, "sgg_lstm_fwd_seg2")) return rc;
  if (int rc = q4_seg_check(b, "sgg_lstm_fwd_seg2")) return rc;
  const int na = q4_blocks(a), nb = q4_blocks(b);
  if (a.act_tile)
    hipLaunchKernelGGL((q4_fwd2_kernel<32, true, 48, true>), dim3(na + nb), dim3(192), 0, st, a, b, na);
  else
    hipLaunchKernelGGL((q4_fwd2_kernel<32, false, 48, true>), dim3(na + nb), dim3(192), 0, st, a, b, na);
  SGG_RETURN_LAUNCH("sgg_lstm_fwd_seg2 (q4)");
}

int lstm_q4_fwd_seg3(const MwSeg& a, int Ha, const MwSeg& b, int Hb, const MwSeg& c, int Hc, hipStream_t st) {
  if (!(Ha == 32 && Hb == 48 && Hc == 32 && !a.act_tile && b.act_tile && c.act_tile)) return 1;
  for (const MwSeg* p : {&a, &b, &c})
    if (int rc = q4_seg_check(*p, "sgg_lstm_fwd_seg3")) return rc;
  const int na = q4_blocks(a), nb = q4_blocks(b), nc = q4_blocks(c);
  hipLaunchKernelGGL((q4_fwd3_kernel<32, false, 48, true, 32, true>), dim3(na + nb + nc), dim3(192), 0, st, a, b, c,
                     na, nb);
  SGG_RETURN_LAUNCH("sgg_lstm_fwd_seg3 (q4)");
}

int lstm_q4_fwd_dec_seg(const MwSeg& a, int Ha, const MwSeg& b, int Hb, hipStream_t st) {
  if (!(Ha == 32 && Hb == 48 && a.act_tile && b.act_tile)) return 1;
  if (int rc = q4_seg_check(a, "sgg_lstm_fwd_dec_seg")) return rc;
  if (int rc = q4_seg_check(b, "sgg_lstm_fwd_dec_seg")) return rc;
  const int na = q4_blocks(a), nb = q4_blocks(b);
  hipLaunchKernelGGL((q4_fwd2d_kernel<32, true, 48, true>), dim3(na + nb), dim3(192), 0, st, a, b, na);
  SGG_RETURN_LAUNCH("sgg_lstm_fwd_dec_seg (q4)");
}

int lstm_q4_wpart_rows(int B) { return (B + kQ4Peds - 1) / kQ4Peds; }

int lstm_q4_bwd(const float* A, const float* Whh, const float* h_all, const float* c_all, const float* act_all,
                const float* rel, const float* dh_last, int T, int B, int H, int t_stop, int t_sh, int Bsrc,
                float* dh0, float* drel_in, float* wpart, hipStream_t st) {
  SGG_CHECK_ARG(t_sh == 0 || (Bsrc >= 1 && B % Bsrc == 0 && t_sh < T),
                "sgg_lstm_bwd (q4): Bsrc %d must divide B %d, t_sh %d < T %d", Bsrc, B, t_sh, T);
  SGG_CHECK_ARG(!wpart || (t_stop == 0 && h_all && rel), "sgg_lstm_bwd (q4): weight gradients need every step, h_all, rel");
  const dim3 grid((B + kQ4Peds - 1) / kQ4Peds);
#define SGG_Q4B(HH, W)                                                                                       \
  hipLaunchKernelGGL((q4_bwd_kernel<HH, W>), grid, dim3(64 * (HH / 16)), 0, st, A, Whh, h_all, c_all, act_all, \
                     rel, dh_last, T, B, t_stop, t_sh, Bsrc, dh0, drel_in, wpart)
  if (H == 32) {
    if (wpart) SGG_Q4B(32, true); else SGG_Q4B(32, false);
  } else {
    if (wpart) SGG_Q4B(48, true); else SGG_Q4B(48, false);
  }
#undef SGG_Q4B
  SGG_RETURN_LAUNCH("sgg_lstm_bwd (q4)");
}

int lstm_q4_fwd_seg(const MwSeg& s, int H, hipStream_t st) {
  if (int rc = q4_seg_check(s, "sgg_lstm_fwd_seg")) return rc;
  return H == 32 ? launch_q4<32>(s, st) : launch_q4<48>(s, st);
}

}  // namespace sgg
