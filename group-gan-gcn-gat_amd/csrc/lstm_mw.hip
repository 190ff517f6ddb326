// Fused LSTM sequences on v_mfma_f32_16x16x4_f32, one workgroup of four
// waves per 16 peds (Encoder, reference sgan/models.py:62-92; Decoder
// rollout :142-178).  Same contract as sgg_lstm_fwd / sgg_lstm_bwd
// (include/sgg.h), dispatched by lstm.hip for the discriminator's H = 48
// sequences (and every H with SGG_LSTM_MW=all): each step of the recurrence
// is latency-bound and the per-ped gate GEMM (4H x H) is spread over all four
// SIMDs of a CU.
//
// "Slot" j of lane (q, c16) is unit slot_unit(j, q) = 16 (j >> 2) + 4 q +
// (j & 3) of ped c16; wave w owns slots w MU .. w MU + MU - 1 (MU = H / 16).
// Forward step: wave w's tile mu holds the four gates of its slot j = w MU +
// mu, gate-interleaved -- D row 4 q + r is (gate r, unit slot_unit(j, q)):
//   G^T (H rows x 16 peds) = [W_hh | A b] (those rows) . [h_{t-1} | r_x r_y 1 0]^T
// = MU tiles x (H / 4 + 1) k-steps of 16x16x4 per wave, so a lane ends the
// MFMAs holding i, f, g, o of its own slots: activations and the cell update
// run in registers (c too) and h goes to hb[t & 1][j][lane].  The next step's
// B operand for k-step ks is h of unit slot_unit(ks, q) -- exactly
// hb[.][ks][lane], because W_hh's columns are loaded in that permuted order.
// ONE barrier per step (hb double-buffered); every LDS access is lane-linear.
// Decoder: the hidden2pos feedback r_t = Wp h_t + bp into step t+1 is folded
// into the weights before step 1 (W_hh + A Wp, b' + A bp; lstm_unit.hip), so
// r_t is off the critical path: wave partials in LDS, summed by wave 0 after
// the step's second barrier.
//
// Saved states for the backward are TILE-NATIVE (this family's private
// layout, sized by sgg_lstm_state_floats): the four gate activations of
// block b, step t, slot j are one float4 per lane, act[(b T + t) KS + j][lane],
// and the cells of wave g's MU slots MU consecutive floats per lane,
// c[((b (T+1) + t) 4 + g)][lane][MU] -- one vector store per slot (act) and
// per wave (c) and step, read back by the slot's owner in the backward with
// the same instruction count.  h_all stays in the public (T+1) x B x H
// layout (it is the encoder's output).
//
// Backward step t (reverse): the slot owners turn dh_t (four wave partials of
// W^T dG_{t+1} from LDS, + Wp^T dout_t for the decoder) into dG_t with the
// saved activations (loaded a step ahead), and straight from registers run
// their slots' share of dh_{t-1}:
//   P_w (H x 16) = sum over the wave's slots j and gates r of
//                  W_hh[r H + slot_unit(j, q)]^T . dG_r,j     (MU tiles x 4 MU k-steps)
// -- k-step (j, r) takes lane quarter q's own dG value of gate r -- written
// to LDS part[t & 1] for the next step's owners: ONE barrier per step.  The
// decoder uses the folded W' for t >= 1 (its input r_{t-1} depends on
// h_{t-1}) and plain W_hh at t = 0 (dh0).  drel_in = A^T dG_t is a slot
// partial reduced over the q lanes and the waves off the critical path.
//
// Weight gradients in the kernel (wpart != NULL): wave g accumulates, on the
// MFMA, its gate block's
//   dW_hh,g += dG_g^T (H x 16 peds) . h_{t-1}
// (MU x MU tiles, K = the block's 16 peds = 4 k-steps) in four helper waves,
// the A operand read from the double-buffered dG image the owners leave in
// LDS, h_{t-1} staged from h_all one step ahead; the helpers pass the owners'
// one barrier per step, so they run beside the next step's owners.  The slot owners sum db += dG and
// dA += dG r_in^T on the VALU (3 FMA per gate value; reduced over the 16 peds
// by lane shuffles at the end).  dG never reaches HBM: the workgroup writes
// one slab row [dW_hh (4H x H) | db (4H) | dA (4H x 2)] that sgg_slab_reduce
// sums (fixed order).
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "sgg_common.h"

namespace sgg {

namespace {

constexpr int kMwThreads = 256;   // four waves: one per gate block, one per SIMD
constexpr int kMwPeds = 16;       // MFMA columns
constexpr int kMwMaxT = 64;       // encoder inputs (all T steps) are staged in LDS: T <= this
constexpr int kDgPitch = 68;      // dG image row pitch: conflict-free for the transposed A-operand read

// v_exp_f32 / v_rcp_f32 forms (~2 ulp), as the other LSTM kernels.
// s = 1: sigmoid(x); s = 2: tanh(x) = 2 sigmoid(2x) - 1 (the same
// expressions as lstm_unit.hip's sigm_u / tanh_u).  exp(-s x) is taken as
// v_exp_f32(x * nsl), nsl = -s log2(e): s is a power of two, so nsl is exact
// and the argument rounds exactly as __expf's (-(s x)) * log2(e) -- the same
// bits with one multiply less per gate value
constexpr float kNegLog2e = -1.4426950408889634f;
__device__ __forceinline__ float gate_act(float x, float s, float nsl) {
  return fmaf(s, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * nsl)), 1.f - s);
}
__device__ __forceinline__ float tanh_m(float x) {
  return fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * (2.f * kNegLog2e))), -1.f);
}

// MU consecutive floats in one vector access (the cell layout of a lane)
template <int MU>
__device__ __forceinline__ void store_vec(float* p, const float (&v)[MU]) {
  if constexpr (MU == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (MU == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else if constexpr (MU == 3) {
    typedef float f3 __attribute__((ext_vector_type(3)));
    f3 x = {v[0], v[1], v[2]};
    __builtin_memcpy(p, &x, 12);
  } else {
#pragma unroll
    for (int i = 0; i < MU; ++i) p[i] = v[i];
  }
}
template <int MU>
__device__ __forceinline__ void load_vec(const float* p, float (&v)[MU]) {
  if constexpr (MU == 4) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else if constexpr (MU == 2) {
    const float2 x = *reinterpret_cast<const float2*>(p);
    v[0] = x.x; v[1] = x.y;
  } else if constexpr (MU == 3) {
    typedef float f3 __attribute__((ext_vector_type(3)));
    f3 x;
    __builtin_memcpy(&x, p, 12);
    v[0] = x.x; v[1] = x.y; v[2] = x.z;
  } else {
#pragma unroll
    for (int i = 0; i < MU; ++i) v[i] = p[i];
  }
}

// unit held by slot j of lane quarter q
__device__ __forceinline__ int slot_unit(int j, int q) { return 16 * (j >> 2) + 4 * q + (j & 3); }

// c + a.b over two K = 32 chunks from the pieces (sgg_common.h mfma_x3): the
// six product kinds smallest first, each over both chunks, on one
// accumulator (16x16x32 bf16 MFMAs issue back to back on one chain)
__device__ __forceinline__ floatx4 mfma_x3x2(const bf16x8 (&a)[2][3], const bf16x8 (&b)[2][3], floatx4 c) {
  constexpr int pa[6] = {2, 1, 0, 1, 0, 0}, pb[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][pa[k]], b[0][pb[k]], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][pa[k]], b[1][pb[k]], c, 0, 0, 0);
  }
  return c;
}

// h staging pitch: q * pitch mod 64 in {0, 16, 32, 48} keeps the B-operand
// read (4 peds x 16 consecutive units) on distinct banks
template <int H>
struct MwCfg {
  static constexpr int MU = H / 16, KS = H / 4, G4 = 4 * H;
  static constexpr int HP = H <= 16 ? 16 : 80;
  static constexpr int NHS = (kMwPeds * H + kMwThreads - 1) / kMwThreads;   // staged h floats per thread
  static constexpr int P = G4 * H + G4 + 2 * G4;                           // slab row floats
};

}  // namespace

// One sequence segment of the forward (MwSeg, sgg_common.h; sgg.h
// SggLstmSeg): steps t0 .. t0 + T - 1 of a Tl-step sequence.  rel holds B
// rows per step and is read at steps t0 + t; h_all rows are Bl apart; the
// saved states sit at their Tl-layout positions.  t0 > 0: the state entering
// step t0 is ped (p mod Bsrc)'s, read from h_all[t0] and the tile-native c
// at t0 (written by the segment that ran steps 0 .. t0 - 1 on Bsrc peds, e.g.
// the discriminator's observed-steps prefix shared by its real and fake
// halves).

#ifdef SGG_LSTM_PROF
// phase timestamps of workgroup 0 (tools/lstm_mw_probe.hip; diagnostic builds only)
__device__ long long g_lstm_prof[256];
#define LMARK(i) \
  if (threadIdx.x == 0 && blk == 0) g_lstm_prof[i] = wall_clock64();
// sub-phases of step 4, lane 0 of every wave: [64 + 8 wave + k]
#define LSUB(k) \
  if ((threadIdx.x & 63) == 0 && blk == 0 && t == 4) g_lstm_prof[64 + 8 * (threadIdx.x >> 6) + (k)] = wall_clock64();
#define LUSE(x) __asm__ volatile("" ::"v"(x));
// backward: sub-phases of the 5th step from the end, lane 0 of every wave: [96 + 8 wave + k]
#define LSUBB(k) \
  if ((threadIdx.x & 63) == 0 && blk == 0 && t == T - 5) g_lstm_prof[96 + 8 * (threadIdx.x >> 6) + (k)] = wall_clock64();
#else
#define LSUBB(k)
#define LMARK(i)
#define LSUB(k)
#define LUSE(x)
#endif

#ifndef SGG_MW_UPRE
#define SGG_MW_UPRE 1   // the projection epilogue's Wu fragments fetched in the prologue (0: probe A/B only)
#endif
#ifndef SGG_MW_FWD_X3
#define SGG_MW_FWD_X3 1   // the encoders' gate GEMM on split-bf16 MFMAs (0: the fp32 16x16x4 form; A/B builds)
#endif

namespace {

// DEC / SAVE are compile-time, so the step loop carries no per-store
// branches.  A padded lane (ped >= B, last block) runs on the clamped ped's
// inputs, so it computes bit-identical values and its stores to that ped's
// rows (h_all, rel_out) are benign duplicates: no store needs a guard.
template <int H, bool DEC, bool SAVE>
__device__ __forceinline__ void mw_fwd_body(const MwSeg& sg, int blk) {
  constexpr int MU = MwCfg<H>::MU, KS = MwCfg<H>::KS;
  constexpr bool decoder = DEC, save = SAVE;
  const float* __restrict__ rel = sg.rel;
  const float* __restrict__ A = sg.A;
  const float* __restrict__ Whh = sg.Whh;
  const float* __restrict__ bias = sg.bias;
  const float* __restrict__ Wp = sg.Wp;
  const float* __restrict__ bp = sg.bp;
  float* __restrict__ h_all = sg.h_all;
  float* __restrict__ c_tile = sg.c_tile;
  float* __restrict__ act_tile = sg.act_tile;
  float* __restrict__ rel_out = sg.rel_out;
  const int T = sg.T, B = sg.B, Bl = sg.Bl, t0 = sg.t0, Tl = sg.Tl;
  // X3 (encoders, H 48): the gate GEMM on split-bf16 MFMAs (section
  // 4a of DESIGN.md).  h_{t-1} is exchanged as its three bf16 pieces in the
  // B-operand layout of v_mfma_f32_16x16x32_bf16: lane (q, c16) holds, per
  // chunk c and piece p, the 8 values of K slots s = 8 c + i of quarter q,
  // ped c16, one 16-byte LDS read each (hx[buf][p][c][lane]).  Slot s = 4 w + m
  // is h of unit slot_unit(w MU + m, q) -- written by lane (q, c16) of wave w,
  // its m-th slot -- for m < MU, and the step input for m = 3 (w = 0: r_x,
  // 1: r_y, 2: the bias' 1, 3: 0; the weights read it in quarter 0 only);
  // each producer lane writes its 4 slots of a piece as one 8-byte store.
  // The fp32 gate tiles of the MFMA output are those of the fp32 form (the
  // same A rows), so activations, saved states and the backward are
  // unchanged.  36 MFMAs of 16 cycles per wave and step at H = 48 (fp32:
  // 39 of 32), and this MFMA shape leaves VALU issue slots beside it.
  // (H = 48 only: the discriminator's encoder, where the launches are long.
  // The generator's H = 32 encoder keeps the fp32 form -- the split form is
  // as accurate (tools/lstm_accuracy.py: 2.9e-7 vs 2.9e-7 from float64) but
  // rounds differently, and the generator's gradients downstream of the
  // pooling / GCN ReLUs are what the 64-ped error-ratio test pins)
  constexpr bool X3 = !DEC && SGG_MW_FWD_X3 && H == 48;
  __shared__ float hb[X3 ? 1 : 2][KS][64];        // fp32 form: h_{t-1}; X3: h_T for the epilogue
  __shared__ sgg_uint4v hx[X3 ? 2 : 1][3][2][64];  // X3: the pieces of h_{t-1} and the step input
  // X3 with saved states: h_t staged by (ped, unit) and written to h_all as
  // whole rows after the next barrier (the per-lane stores of the fp32 form
  // hit 16 rows x 4 units per instruction)
  constexpr int kHsP = H + 4;   // row pitch (16-byte aligned rows)
  __shared__ float hst[X3 && SAVE ? 2 : 1][kMwPeds][X3 && SAVE ? kHsP : 1];
  __shared__ float2 rpart[2][4][kMwPeds];
  __shared__ float relseq[kMwMaxT][kMwPeds][2];
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, c16 = lane & 15;
  const int ped = blk * kMwPeds + c16;
  const int pc = ped < B ? ped : B - 1;   // clamped: every load and store unconditional and in bounds
  LMARK(0);

  // [W_hh | A b] rows of tile mu in registers: A-operand row c16 is gate
  // c16 & 3 of unit slot_unit(g MU + mu, c16 >> 2); W_hh's columns in the
  // permuted k order (slot_unit(4 m + i, q) = 16 m + 4 q + i: one 16-byte load
  // per block m)
  float w[MU][KS + 1], ak0[MU], ak1[MU];
  bf16x8 wx[X3 ? MU : 1][2][3];
  if constexpr (X3) {
    // A operand of the split form: lane (q, c16) holds row c16 (gate c16 & 3
    // of unit slot_unit(g MU + mu, c16 >> 2)) at the K slots of quarter q
#pragma unroll
    for (int mu = 0; mu < MU; ++mu) {
      const int row = (c16 & 3) * H + slot_unit(g * MU + mu, c16 >> 2);
      const float a0 = A[2 * row], a1 = A[2 * row + 1], bi = bias[row];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int w2 = (8 * c + i) >> 2, m2 = (8 * c + i) & 3;
          if (m2 < MU)
            v[i] = Whh[row * H + slot_unit(w2 * MU + m2, q)];
          else if (m2 == 3)
            v[i] = q != 0 ? 0.f : w2 == 0 ? a0 : w2 == 1 ? a1 : w2 == 2 ? bi : 0.f;
          else
            v[i] = 0.f;
        }
        split8(v, wx[mu][c]);
      }
    }
  }
#pragma unroll
  for (int mu = 0; mu < (X3 ? 0 : MU); ++mu) {
    const int row = (c16 & 3) * H + slot_unit(g * MU + mu, c16 >> 2);
#pragma unroll
    for (int m = 0; m < KS / 4; ++m) {
      const float4 v = *reinterpret_cast<const float4*>(Whh + row * H + 16 * m + 4 * q);
      w[mu][4 * m] = v.x;
      w[mu][4 * m + 1] = v.y;
      w[mu][4 * m + 2] = v.z;
      w[mu][4 * m + 3] = v.w;
    }
    ak0[mu] = A[2 * row];
    ak1[mu] = A[2 * row + 1];
    w[mu][KS] = q == 0 ? ak0[mu] : q == 1 ? ak1[mu] : q == 2 ? bias[row] : 0.f;
  }
  float c[MU], wp0[MU], wp1[MU], hv0[MU];
  // t0 > 0: the source block / row of the state entering step t0
  const int nsrc = (sg.Bsrc + kMwPeds - 1) / kMwPeds;
  const int sblk = t0 > 0 ? blk % nsrc : blk;
  const int spc = t0 > 0 ? pc % sg.Bsrc : pc;
#pragma unroll
  for (int i = 0; i < MU; ++i) {
    const int j = g * MU + i, u = slot_unit(j, q);
    float hv, cv;
    if (t0 > 0) {
      hv = h_all[((size_t)t0 * Bl + spc) * H + u];
      cv = c_tile[((((size_t)sblk * (Tl + 1) + t0) * 4 + g) * 64 + lane) * MU + i];
    } else {
      hv = sg.di.ctx ? dec_h0(sg.di, pc, u) : sg.h0 ? sg.h0[(size_t)pc * H + u] : 0.f;
      cv = sg.c0 ? sg.c0[(size_t)pc * H + u] : 0.f;
      if (save) {
        h_all[(size_t)pc * H + u] = hv;
        c_tile[(((size_t)blk * (Tl + 1) * 4 + g) * 64 + lane) * MU + i] = cv;
      }
    }
    c[i] = cv;
    hv0[i] = hv;
    if constexpr (!X3) hb[0][j][lane] = hv;
    wp0[i] = decoder ? Wp[u] : 0.f;
    wp1[i] = decoder ? Wp[H + u] : 0.f;
  }
  const float bp0 = decoder ? bp[0] : 0.f, bp1 = decoder ? bp[1] : 0.f;
  // the discriminator input's entries of this workgroup's peds that do not
  // come from the recurrence (head steps, the b half, start positions;
  // SggTrajOut): loaded with the weights, stored after the prologue
  constexpr int kTo = 4;
  float2 tov[kTo];
  float2* tod[kTo];
  int nto = 0;
  if (DEC && sg.to.out != nullptr) {
    const SggTrajOut& to = sg.to;
    const int dup = to.b ? 2 : 1;
    const int nh = to.T0 * dup, nb = to.b ? T : 0, ns = to.start ? dup : 0;
    nto = kMwPeds * (nh + nb + ns);
    auto entry = [&](int e, float2*& d) -> float2 {
      const int i = e % kMwPeds, w = e / kMwPeds;
      const int col = min(blk * kMwPeds + i, B - 1) - to.col0;
      d = nullptr;
      if (col < 0 || col >= to.ncol) return make_float2(0.f, 0.f);
      float2* o2 = reinterpret_cast<float2*>(to.out);
      if (w < nh) {   // head step t (either half)
        const int t = w / dup, half = w - t * dup;
        d = o2 + (size_t)t * to.NB + col + half * to.ncol;
        return reinterpret_cast<const float2*>(to.head + (size_t)t * to.ldh)[col];
      }
      if (w < nh + nb) {   // the b half's step T0 + t
        const int t = w - nh;
        d = o2 + (size_t)(to.T0 + t) * to.NB + to.ncol + col;
        return reinterpret_cast<const float2*>(to.b + (size_t)t * to.ldb)[col];
      }
      d = reinterpret_cast<float2*>(to.start) + col + (w - nh - nb) * to.ncol;
      return reinterpret_cast<const float2*>(to.pos0)[col];
    };
#pragma unroll
    for (int m = 0; m < kTo; ++m) {
      const int e = threadIdx.x + m * kMwThreads;
      tod[m] = nullptr;
      if (e < nto) tov[m] = entry(e, tod[m]);
    }
    for (int e = threadIdx.x + kTo * kMwThreads; e < nto; e += kMwThreads) {   // (longer heads: rare)
      float2* d;
      const float2 v = entry(e, d);
      if (d) *d = v;
    }
  }

  // the encoder's inputs of all T steps: loaded into registers here, written
  // to LDS after the epilogue's prefetch below is issued (so the LDS writes
  // wait for these loads only)
  constexpr int kRelPer = 2 * kMwPeds * kMwMaxT / kMwThreads;
  float rv[kRelPer];
  if (!decoder) {
#pragma unroll
    for (int m = 0; m < kRelPer; ++m) {
      const int e = threadIdx.x + m * kMwThreads;
      if (e < 2 * kMwPeds * T) {
        const int t = e / (2 * kMwPeds), p = (e >> 1) & (kMwPeds - 1), k = e & 1;
        const int pp = min(blk * kMwPeds + p, B - 1);   // padded lanes see the clamped ped's inputs
        rv[m] = rel[((size_t)(t0 + t) * B + pp) * 2 + k];
      }
    }
  }

  // the projection epilogue's Wu fragments (see below), fetched now so their
  // latency hides under the recurrence: all of this wave's <= 8 tiles in
  // registers (NU <= 512, H <= 48, 16-byte aligned rows)
  constexpr bool kUPre = SGG_MW_UPRE && !DEC && H <= 48;
  constexpr int kUT = 8;
  const float* __restrict__ Wu = sg.Wu;
  const int ldwu = sg.ldwu, NU = sg.NU;
  const bool upre = kUPre && sg.U && NU <= 16 * 4 * kUT &&
                    ((reinterpret_cast<uintptr_t>(Wu) | ((uintptr_t)ldwu * 4)) & 15) == 0;
  // One tile per recurrence step (tile i at step i, the rest after the
  // loop): all eight at once in the prologue were ~100 loads per wave behind
  // the recurrence's operands (a wave tracks <= 63 outstanding), which held
  // the first step back ~1.7 us (tools/lstm_mw_probe.hip, SGG_MW_UPRE A/B)
  float wu[kUPre ? kUT : 1][KS];
  float cuv[kUPre ? kUT : 1][4];
  auto load_wu = [&](int i) {   // (called with compile-time i only: wu stays in registers)
    const int ntile = NU >> 4;
    const float4 v = *reinterpret_cast<const float4*>(sg.cu + 16 * min(g + 4 * i, ntile - 1) + 4 * q);
    cuv[i][0] = v.x;
    cuv[i][1] = v.y;
    cuv[i][2] = v.z;
    cuv[i][3] = v.w;
    const float* wr = Wu + (size_t)(min(g + 4 * i, ntile - 1) * 16 + c16) * ldwu;
#pragma unroll
    for (int m = 0; m < KS / 4; ++m) {
      const float4 w4 = *reinterpret_cast<const float4*>(wr + 16 * m + 4 * q);
      wu[i][4 * m] = w4.x;
      wu[i][4 * m + 1] = w4.y;
      wu[i][4 * m + 2] = w4.z;
      wu[i][4 * m + 3] = w4.w;
    }
  };

  if (!decoder) {
#pragma unroll
    for (int m = 0; m < kRelPer; ++m) {
      const int e = threadIdx.x + m * kMwThreads;
      if (e < 2 * kMwPeds * T) relseq[e / (2 * kMwPeds)][(e >> 1) & (kMwPeds - 1)][e & 1] = rv[m];
    }
  }
  if (DEC && nto > 0) {
#pragma unroll
    for (int m = 0; m < kTo; ++m)
      if (tod[m]) *tod[m] = tov[m];
  }
  // the split image of h_{-1} and the step-0 input (this wave's slots)
  auto put_x3 = [&](int buf, const float (&hv)[MU], float inv) {
    float v[4] = {0.f, 0.f, 0.f, inv};
#pragma unroll
    for (int i = 0; i < MU; ++i) v[i] = hv[i];
    unsigned wd[3][2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float h0, m0, l0, h1, m1, l1;
      split3(v[2 * k], h0, m0, l0);
      split3(v[2 * k + 1], h1, m1, l1);
      wd[0][k] = bf16_pack_top(h0, h1);
      wd[1][k] = bf16_pack_top(m0, m1);
      wd[2][k] = bf16_pack_top(l0, l1);
    }
#pragma unroll
    for (int p = 0; p < 3; ++p)
      reinterpret_cast<uint2*>(&hx[buf][p][g >> 1][lane])[g & 1] = make_uint2(wd[p][0], wd[p][1]);
  };
  // the step input of this wave's slot 3 (r_x, r_y, 1, 0)
  auto in_x3 = [&](int t) -> float {
    return g < 2 ? rel[((size_t)(t0 + t) * B + pc) * 2 + g] : (g == 2 ? 1.f : 0.f);
  };
  if constexpr (X3) put_x3(0, hv0, in_x3(0));
  // LDS only: the prologue's global stores (saved initial state) need not
  // complete before the recurrence
  lds_barrier();
  LMARK(1);

  // input k-step operand: r_x (q = 0), r_y (q = 1), 1 (q = 2), 0 (q = 3)
  // (loads unconditional, the constant lanes selected after)
  auto input = [&](int t) -> float {
    const float v = decoder ? (sg.di.ctx ? dec_rel0(sg.di, pc, q & 1) : rel[(size_t)pc * 2 + (q & 1)])
                            : relseq[t][c16][q & 1];
    return q < 2 ? v : (q == 2 ? 1.f : 0.f);
  };
  float xin = input(0);
  if (decoder && sg.rel0_out && g == 0 && q < 2) sg.rel0_out[(size_t)pc * 2 + q] = xin;   // (the backward's x_0)
  const SggTrajOut& to = sg.to;
  const int tcol = pc - to.col0;   // this lane's column of the discriminator input
  const bool tlive = decoder && to.out != nullptr && tcol >= 0 && tcol < to.ncol;
  float hl[MU];   // X3: h of the last step
  // X3 + SAVE: h_t rows of the block's peds from the staging image (after a
  // barrier), one float4 per thread (16 H / 4 <= 256 threads)
  auto put_rows = [&](int t) {
    constexpr int NQ = kMwPeds * H / 4;
    const int e = threadIdx.x;
    if (e < NQ) {
      const int p = e / (H / 4), k = e - p * (H / 4);
      const int ped_p = blk * kMwPeds + p;
      if (ped_p < B)
        *reinterpret_cast<float4*>(h_all + ((size_t)(t0 + t + 1) * Bl + ped_p) * H + 4 * k) =
            *reinterpret_cast<const float4*>(&hst[t & 1][p][4 * k]);
    }
  };
  for (int t = 0; t < T; ++t) {
    if (decoder && t == 1) {
      // fold the hidden2pos feedback into the recurrence (see header)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int u = slot_unit(ks, q);
        const float p0 = Wp[u], p1 = Wp[H + u];
#pragma unroll
        for (int mu = 0; mu < MU; ++mu) w[mu][ks] = fmaf(ak1[mu], p1, fmaf(ak0[mu], p0, w[mu][ks]));
      }
#pragma unroll
      for (int mu = 0; mu < MU; ++mu)
        if (q == 2) w[mu][KS] = fmaf(ak1[mu], bp1, fmaf(ak0[mu], bp0, w[mu][KS]));
      xin = q == 2 ? 1.f : 0.f;
    }
    const int rb = t & 1;   // h_{t-1} is in hb[rb] (hx[rb]); h_t goes to hb[rb ^ 1] (hx[rb ^ 1])
    if constexpr (X3) {
      // the split-bf16 step: tile mu + 1's MFMA chain is issued before tile
      // mu's activations, so the VALU work of one tile runs in the issue
      // slots the 16x16x32 bf16 MFMAs of the next leave free
      LSUB(0);
      if (save && t > 0) put_rows(t - 1);   // h_{t-1}, staged before the barrier just passed
      bf16x8 hbx[2][3];
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int p = 0; p < 3; ++p) hbx[cc][p] = __builtin_bit_cast(bf16x8, hx[rb][p][cc][lane]);
      const float xnext = g < 2 ? relseq[min(t + 1, T - 1)][c16][g] : (g == 2 ? 1.f : 0.f);
      LUSE(__builtin_bit_cast(sgg_uint4v, hbx[1][2])[0]);
      LSUB(1);
      if (kUPre && upre) {
#pragma unroll
        for (int i = 0; i < kUT; ++i)
          if (t == i) load_wu(i);
      }
      floatx4 acc[MU];
      acc[0] = mfma_x3x2(wx[0], hbx, floatx4{0.f, 0.f, 0.f, 0.f});
      LSUB(2);
      float hn[MU];
#pragma unroll
      for (int mu = 0; mu < MU; ++mu) {
        if (mu + 1 < MU) acc[mu + 1] = mfma_x3x2(wx[mu + 1], hbx, floatx4{0.f, 0.f, 0.f, 0.f});
        const int j = g * MU + mu;
        float a[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float s = r == 2 ? 2.f : 1.f;
          a[r] = gate_act(acc[mu][r], s, s * kNegLog2e);
        }
        if (save)
          reinterpret_cast<float4*>(act_tile)[(((size_t)blk * Tl + t0 + t) * KS + j) * 64 + lane] =
              make_float4(a[0], a[1], a[2], a[3]);
        c[mu] = fmaf(a[1], c[mu], a[0] * a[2]);
        hn[mu] = a[3] * tanh_m(c[mu]);
        hl[mu] = hn[mu];
        if (save) hst[t & 1][c16][slot_unit(j, q)] = hn[mu];
      }
      if (save)
        store_vec<MU>(c_tile + ((((size_t)blk * (Tl + 1) + t0 + t + 1) * 4 + g) * 64 + lane) * MU, c);
      LSUB(3);
      put_x3(rb ^ 1, hn, xnext);
      LSUB(4);
      lds_barrier();
      LSUB(5);
      if (t < 60) LMARK(t + 2);
      continue;
    }
    floatx4 acc[MU];
    {
#pragma unroll
      for (int mu = 0; mu < MU; ++mu)
        acc[mu] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[mu][KS], xin, floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      float hk[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) hk[ks] = hb[rb][ks][lane];
      if (!decoder && t + 1 < T) xin = input(t + 1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int mu = 0; mu < MU; ++mu)
          acc[mu] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[mu][ks], hk[ks], acc[mu], 0, 0, 0);
    }
    if (kUPre && upre) {
#pragma unroll
      for (int i = 0; i < kUT; ++i)
        if (t == i) load_wu(i);
    }

    // activations (r = 2: tanh, else sigmoid) and the cell update of this
    // wave's slots, in registers
    float px = 0.f, py = 0.f;
#pragma unroll
    for (int mu = 0; mu < MU; ++mu) {
      const int j = g * MU + mu;
      float a[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = r == 2 ? 2.f : 1.f;
        a[r] = gate_act(acc[mu][r], s, s * kNegLog2e);
      }
      if (save)   // tile-native: slot j's four gates as one 16-byte value per lane
        reinterpret_cast<float4*>(act_tile)[(((size_t)blk * Tl + t0 + t) * KS + j) * 64 + lane] =
            make_float4(a[0], a[1], a[2], a[3]);
      c[mu] = fmaf(a[1], c[mu], a[0] * a[2]);
      const float h = a[3] * tanh_m(c[mu]);
      hb[rb ^ 1][j][lane] = h;
      if (save || (t == T - 1 && h_all)) h_all[((size_t)(t0 + (save ? t + 1 : T)) * Bl + pc) * H + slot_unit(j, q)] = h;
      px = fmaf(wp0[mu], h, px);
      py = fmaf(wp1[mu], h, py);
    }
    if (save)   // the wave's MU cells of this lane, contiguous
      store_vec<MU>(c_tile + ((((size_t)blk * (Tl + 1) + t0 + t + 1) * 4 + g) * 64 + lane) * MU, c);
    if (decoder) {
      px += __shfl_xor(px, 16);
      px += __shfl_xor(px, 32);
      py += __shfl_xor(py, 16);
      py += __shfl_xor(py, 32);
      if (q == 0) rpart[t & 1][g][c16] = make_float2(px, py);
    }
    lds_barrier();
    if (t < 60) LMARK(t + 2);
    if (decoder && g == 0 && q == 0) {   // r_t = Wp h_t + bp
      const float2 r0 = rpart[t & 1][0][c16], r1 = rpart[t & 1][1][c16], r2 = rpart[t & 1][2][c16],
                   r3 = rpart[t & 1][3][c16];
      const float2 rv2 = make_float2(((r0.x + r1.x) + (r2.x + r3.x)) + bp0, ((r0.y + r1.y) + (r2.y + r3.y)) + bp1);
      *reinterpret_cast<float2*>(rel_out + ((size_t)t * B + pc) * 2) = rv2;
      if (tlive) {   // staged in LDS (the decoder's relseq is free), stored after the loop
        if (T <= kMwMaxT) {
          relseq[t][c16][0] = rv2.x;
          relseq[t][c16][1] = rv2.y;
        } else {
          reinterpret_cast<float2*>(to.out)[(size_t)(to.T0 + t) * to.NB + tcol] = rv2;
        }
      }
    }
  }
  if constexpr (X3) {   // h_T: the projection epilogue's operand (fp32, permuted k order), the output row
    if (save) put_rows(T - 1);
#pragma unroll
    for (int mu = 0; mu < MU; ++mu) {
      hb[0][g * MU + mu][lane] = hl[mu];
      if (!save && h_all) h_all[((size_t)(t0 + T) * Bl + pc) * H + slot_unit(g * MU + mu, q)] = hl[mu];
    }
    lds_barrier();
  }
  if (DEC && to.out != nullptr && T <= kMwMaxT) {   // the generated steps of the discriminator input
    lds_barrier();
    for (int e = threadIdx.x; e < T * kMwPeds; e += kMwThreads) {
      const int t = e / kMwPeds, i = e - t * kMwPeds;
      const int col = min(blk * kMwPeds + i, B - 1) - to.col0;
      if (col >= 0 && col < to.ncol)
        reinterpret_cast<float2*>(to.out)[(size_t)(to.T0 + t) * to.NB + col] =
            make_float2(relseq[t][i][0], relseq[t][i][1]);
    }
  }
  const float* __restrict__ cu = sg.cu;
  float* __restrict__ U = sg.U;
  if (kUPre && upre) {
#pragma unroll
    for (int i = 0; i < kUT; ++i)
      if (i >= T) load_wu(i);   // (a recurrence shorter than the tile count)
    // U^T tiles g + 4 i from the prefetched fragments: eight independent
    // accumulation chains
    float hk[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) hk[ks] = hb[X3 ? 0 : T & 1][ks][lane];
    const int ntile = NU >> 4;
    floatx4 acc[kUT];
#pragma unroll
    for (int i = 0; i < kUT; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < kUT; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(wu[i][ks], hk[ks], acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < kUT; ++i) {
      const int nt = g + 4 * i;
      if (nt < ntile)
        *reinterpret_cast<float4*>(U + (size_t)pc * NU + 16 * nt + 4 * q) =
            make_float4(acc[i][0] + cuv[i][0], acc[i][1] + cuv[i][1], acc[i][2] + cuv[i][2], acc[i][3] + cuv[i][3]);
    }
  } else if (!decoder && U) {
    // projection epilogue: U = h_T Wu^T + cu (B x NU; the pooling MLP's h-half
    // of its first layer, models.py:538) while h_T is still in LDS, in the
    // recurrence's own operand layout: U^T tile (16 units x 16 peds) =
    // Wu[tile rows][k] . h[k][peds] over the permuted k order of hb.  Wave g
    // takes tiles g, g + 4, ...
    float hk[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) hk[ks] = hb[X3 ? 0 : T & 1][ks][lane];
    const int ntile = NU >> 4;
    // tiles in pairs (two independent accumulation chains); the next pair's
    // Wu fragments are in flight during the current pair's MFMAs
    float wa[2][KS], wn[2][KS];
    // lane q's k values of unit block m, slot_unit(4 m + i, q) = 16 m + 4 q + i,
    // are 4 consecutive floats: one 16-byte load per block (a full 64-byte line
    // per row and wave instruction) when Wu's rows are 16-byte aligned
    const bool vec = ((reinterpret_cast<uintptr_t>(Wu) | ((uintptr_t)ldwu * 4)) & 15) == 0;
    auto load_w = [&](int nt, float (&w)[KS]) {
      const float* wr = Wu + (size_t)(min(nt, ntile - 1) * 16 + c16) * ldwu;
      if (vec) {
#pragma unroll
        for (int m = 0; m < KS / 4; ++m) {
          const float4 v = *reinterpret_cast<const float4*>(wr + 16 * m + 4 * q);
          w[4 * m] = v.x;
          w[4 * m + 1] = v.y;
          w[4 * m + 2] = v.z;
          w[4 * m + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) w[ks] = wr[slot_unit(ks, q)];
      }
    };
    load_w(g, wa[0]);
    load_w(g + 4, wa[1]);
    for (int nt = g; nt < ntile; nt += 8) {
      const bool more = nt + 8 < ntile;
      if (more) {
        load_w(nt + 8, wn[0]);
        load_w(nt + 12, wn[1]);
      }
      floatx4 acc0 = floatx4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[0][ks], hk[ks], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[1][ks], hk[ks], acc1, 0, 0, 0);
      }
      const float4 cb0 = *reinterpret_cast<const float4*>(cu + 16 * nt + 4 * q);
      *reinterpret_cast<float4*>(U + (size_t)pc * NU + 16 * nt + 4 * q) =
          make_float4(acc0[0] + cb0.x, acc0[1] + cb0.y, acc0[2] + cb0.z, acc0[3] + cb0.w);
      if (nt + 4 < ntile) {
        const float4 cb1 = *reinterpret_cast<const float4*>(cu + 16 * (nt + 4) + 4 * q);
        *reinterpret_cast<float4*>(U + (size_t)pc * NU + 16 * (nt + 4) + 4 * q) =
            make_float4(acc1[0] + cb1.x, acc1[1] + cb1.y, acc1[2] + cb1.z, acc1[3] + cb1.w);
      }
      if (more) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          wa[0][ks] = wn[0][ks];
          wa[1][ks] = wn[1][ks];
        }
      }
    }
  }
  LMARK(63);
}

template <int H, bool DEC, bool SAVE>
__global__ void __launch_bounds__(kMwThreads) lstm_mw_fwd_kernel(MwSeg sg) {
  mw_fwd_body<H, DEC, SAVE>(sg, blockIdx.x);
}

// two independent encoder segments in ONE launch: workgroups [0, nblk_a) run
// segment a, the rest segment b (e.g. the generator's encoder beside the
// discriminator's observed-steps prefix: both read only the observed steps)
template <int HA, bool SA, int HB, bool SB>
__global__ void __launch_bounds__(kMwThreads) lstm_mw_fwd2_kernel(MwSeg a, MwSeg b, int nblk_a) {
  if ((int)blockIdx.x < nblk_a)
    mw_fwd_body<HA, false, SA>(a, blockIdx.x);
  else
    mw_fwd_body<HB, false, SB>(b, blockIdx.x - nblk_a);
}

// a decoder segment (the generator step's best / last samples with saved
// states, decoder start and discriminator input built in the kernel) and an
// independent encoder segment (the discriminator's observed-steps prefix of
// the same step) in ONE launch
template <int HA, bool SA, int HB, bool SB>
__global__ void __launch_bounds__(kMwThreads) lstm_mw_fwd2d_kernel(MwSeg a, MwSeg b, int nblk_a) {
  if ((int)blockIdx.x < nblk_a)
    mw_fwd_body<HA, true, SA>(a, blockIdx.x);
  else
    mw_fwd_body<HB, false, SB>(b, blockIdx.x - nblk_a);
}

// three independent encoder segments in ONE launch: the discriminator
// step's generator encoder (a, no saved states) and the discriminator's
// observed-steps prefix (b) beside the generator step's encoder (c, saved
// states for its backward) -- G.context_pair
template <int HA, bool SA, int HB, bool SB, int HC, bool SC>
__global__ void __launch_bounds__(kMwThreads) lstm_mw_fwd3_kernel(MwSeg a, MwSeg b, MwSeg c, int nblk_a, int nblk_b) {
  const int blk = blockIdx.x;
  if (blk < nblk_a)
    mw_fwd_body<HA, false, SA>(a, blk);
  else if (blk < nblk_a + nblk_b)
    mw_fwd_body<HB, false, SB>(b, blk - nblk_a);
  else
    mw_fwd_body<HC, false, SC>(c, blk - nblk_a - nblk_b);
}

#ifndef SGG_MW_BWD_DB
#define SGG_MW_BWD_DB 1
#endif
#ifndef SGG_MW_BWD_X3
#define SGG_MW_BWD_X3 1
#endif

template <int H, bool DEC, bool WGRAD>
__global__ void __launch_bounds__(WGRAD ? 2 * kMwThreads : kMwThreads) lstm_mw_bwd_kernel(
    const float* __restrict__ A, const float* __restrict__ Whh, const float* __restrict__ Wp,
    const float* __restrict__ h_all, const float* __restrict__ c_tile, const float* __restrict__ act_tile,
    const float* __restrict__ rel, const float* __restrict__ rel_out, const float* __restrict__ dh_last,
    const float* __restrict__ dout, int T, int B, float* __restrict__ dh0, float* __restrict__ drel_in,
    float* __restrict__ drel_tot, float* __restrict__ wpart, const float* __restrict__ dout2, int bsplit,
    int t_stop, int t_sh, int Bsrc) {
  constexpr int MU = MwCfg<H>::MU, KS = MwCfg<H>::KS, G4 = MwCfg<H>::G4, HP = MwCfg<H>::HP;
  constexpr bool decoder = DEC, wgrad = WGRAD;
  constexpr bool BX3 = SGG_MW_BWD_X3 != 0;   // dh_{t-1} partials on split-bf16 MFMAs (below)
  // with weight gradients the helper waves also take the db and dA sums
  // (hsum below), and for the encoder drel_in too, so the owners' step is the
  // recurrence alone (the decoder's owners keep drel_in: their dWp / dbp
  // accumulators read it the next step)
  constexpr bool hacc = wgrad && !decoder;   // helpers: drel_in
  constexpr bool hdb = wgrad;                 // helpers: db, dA
  // decoder slab rows carry [dWp (2 x H) | dbp (2)] after [dW_hh | db | dA]
  constexpr int NHS = MwCfg<H>::NHS, P0 = MwCfg<H>::P, P = P0 + (DEC ? 2 * H + 2 : 0);
  __shared__ float dgb[2][4][KS][kDgPitch];
  __shared__ float part[2][4][KS][64];
  __shared__ float2 fbp[2][4][kMwPeds];
  __shared__ float hs[2][kMwPeds][HP];
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, c16 = lane & 15;
  const int blk = blockIdx.x;
  LMARK(0);
  const int ped = blk * kMwPeds + c16;
  const bool valid = ped < B;
  const int pc = valid ? ped : B - 1;
  // t_sh > 0: the states of steps < t_sh (cells / h up to index t_sh) of ped
  // p are ped (p mod Bsrc)'s -- a prefix shared by the halves of the batch
  // and saved once (MwSeg t0); Bsrc is a multiple of 16 there
  const int nsrc = t_sh > 0 ? Bsrc / kMwPeds : 1;
  // (t_sh == 0: no shared prefix -- every step reads its own block, the
  // initial cell c_{-1} at index 0 included)
  auto sblk = [&](bool shared_at) { return (shared_at && t_sh > 0) ? blk % nsrc : blk; };

  // weight-gradient operand of step t: h_{t-1} = h_all[t] of the block's 16
  // peds, fetched one step ahead, staged in LDS
  float hv[NHS];
  const int ht = threadIdx.x & (kMwThreads - 1);   // thread index among the four (helper) waves
  auto stage_load = [&](int t) {
#pragma unroll
    for (int m = 0; m < NHS; ++m) {
      const int e = ht + m * kMwThreads;   // < 16 H exactly (NHS = 16 H / 256)
      int r = min(blk * kMwPeds + e / H, B - 1);
      if (t <= t_sh && t_sh > 0) r %= Bsrc;
      hv[m] = h_all[((size_t)t * B + r) * H + e % H];
    }
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int m = 0; m < NHS; ++m) {
      const int e = ht + m * kMwThreads;
      hs[buf][e / H][e % H] = hv[m];
    }
  };
  if (wgrad && g >= 4) {
    // helper waves 4..7: the weight gradient of gate block hg, off the
    // recurrence's critical path.  They pass the owners' barrier of each step:
    // after barrier (t) dG_t is in dgb[t & 1] and h_{t-1} in hs[t & 1]; the
    // MFMAs run while the owners compute step t - 1, then h_{t-2} is staged
    // into the other buffer (its last readers, step t + 1, all passed barrier
    // (t)).  dgb[t & 1] is rewritten at step t - 2, after barrier (t - 1),
    // which a helper reaches only once its step-t MFMAs are issued.
    const int hg = g - 4;
    floatx4 dw[MU][MU];
#pragma unroll
    for (int mu = 0; mu < MU; ++mu)
#pragma unroll
      for (int nu = 0; nu < MU; ++nu) dw[mu][nu] = floatx4{0.f, 0.f, 0.f, 0.f};
    // dw[mu][nu] += dG_g^T (units 16 mu..) x h (units 16 nu..) over the 16 peds
    // encoder: the per-gate sums of the owners' dG image as well, off the
    // recurrence's critical path -- db and dA (= dG r_in^T) of gate hg for
    // every slot (lane-accumulated over the steps in the owners' former
    // order), and gate hg's partial of drel_in = A^T dG (reduced over the
    // lane quarters here, over the four gates by helper 4 one barrier later)
    constexpr int KH = hdb ? KS : 1, KA = hacc ? KS : 1;
    float ha0[KA], ha1[KA], sdb[KH], sdx[KH], sdy[KH];
    float hr0 = 0.f, hr1 = 0.f, nr0 = 0.f, nr1 = 0.f;
#pragma unroll
    for (int j = 0; j < KH; ++j) sdb[j] = sdx[j] = sdy[j] = 0.f;
    if (hacc) {
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        const int u = slot_unit(j, q);
        ha0[j] = A[2 * (hg * H + u)];
        ha1[j] = A[2 * (hg * H + u) + 1];
      }
    }
    // r_in(t) of the lane's ped: rel[t] (encoder); rel0, then rel_out[t - 1] (decoder)
    auto rel_load = [&](int t) {
      const float* rp = !decoder ? rel + ((size_t)t * B + pc) * 2
                                 : (t == 0 ? rel + (size_t)pc * 2 : rel_out + ((size_t)(t - 1) * B + pc) * 2);
      const float2 rv = *reinterpret_cast<const float2*>(rp);
      nr0 = rv.x;
      nr1 = rv.y;
    };
    auto hsum = [&](int buf) {
      float f0 = 0.f, f1 = 0.f;
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        const float v = dgb[buf][hg][j][lane];
        sdb[j] += v;
        sdx[j] = fmaf(v, hr0, sdx[j]);
        sdy[j] = fmaf(v, hr1, sdy[j]);
        if (hacc) {
          f0 = fmaf(ha0[j], v, f0);
          f1 = fmaf(ha1[j], v, f1);
        }
      }
      if (hacc) {
        f0 += __shfl_xor(f0, 16);
        f0 += __shfl_xor(f0, 32);
        f1 += __shfl_xor(f1, 16);
        f1 += __shfl_xor(f1, 32);
        if (q == 0) fbp[buf][hg][c16] = make_float2(f0, f1);
      }
    };
    // drel_in[t] from the four gates' partials of step t (written before the barrier just passed)
    auto drel_store = [&](int t) {
      if (hg == 0 && q == 0 && valid) {
        const int buf = t & 1;
        const float2 r0 = fbp[buf][0][c16], r1 = fbp[buf][1][c16], r2 = fbp[buf][2][c16], r3 = fbp[buf][3][c16];
        *reinterpret_cast<float2*>(drel_in + ((size_t)t * B + ped) * 2) =
            make_float2((r0.x + r1.x) + (r2.x + r3.x), (r0.y + r1.y) + (r2.y + r3.y));
      }
    };
    auto dw_accum = [&](int buf) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int p = 4 * kk + q;
        float bh[MU];
#pragma unroll
        for (int nu = 0; nu < MU; ++nu) bh[nu] = hs[buf][p][16 * nu + c16];
#pragma unroll
        for (int mu = 0; mu < MU; ++mu) {
          const float a = dgb[buf][hg][4 * mu + (c16 & 3)][((c16 >> 2) << 4) + p];
#pragma unroll
          for (int nu = 0; nu < MU; ++nu) dw[mu][nu] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bh[nu], dw[mu][nu], 0, 0, 0);
        }
      }
    };

    stage_load(T - 1);
    stage_store((T - 1) & 1);
    if (T >= 2) stage_load(T - 2);
    if (hdb) rel_load(T - 1);
    for (int t = T - 1; t >= 0; --t) {
      const int cur = t & 1;
      if (hdb) {
        hr0 = nr0;
        hr1 = nr1;
        if (t > 0) rel_load(t - 1);
      }
      lds_barrier();   // (t)
      LSUBB(0);
      dw_accum(cur);
      LUSE(dw[0][0][0]);
      LSUBB(1);
      if (hacc && t < T - 1) drel_store(t + 1);
      if (hdb) hsum(cur);
      LSUBB(2);
      if (t > 0) {
        stage_store(cur ^ 1);
        if (t > 1) stage_load(t - 2);
      }
      LSUBB(3);
    }
    if (hacc) {   // the owners' extra barrier: step 0's partials are complete
      lds_barrier();
      drel_store(0);
    }
    // slab row of this workgroup: D tile (mu, nu) holds rows hg H + 16 mu + 4 q + r, cols 16 nu + c16
    float* row = wpart + (size_t)blk * P;
#pragma unroll
    for (int mu = 0; mu < MU; ++mu)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = hg * H + 16 * mu + 4 * q + r;
#pragma unroll
        for (int nu = 0; nu < MU; ++nu) row[(size_t)gr * H + 16 * nu + c16] = dw[mu][nu][r];
      }
    if (hdb) {   // db / dA of gate hg: sums over the 16 peds (lanes c16 of each q)
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        const int u = slot_unit(j, q);
        float a = sdb[j], x = sdx[j], y = sdy[j];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          a += __shfl_xor(a, o);
          x += __shfl_xor(x, o);
          y += __shfl_xor(y, o);
        }
        if (c16 == 0) {
          row[G4 * H + hg * H + u] = a;
          row[G4 * H + G4 + 2 * (hg * H + u)] = x;
          row[G4 * H + G4 + 2 * (hg * H + u) + 1] = y;
        }
      }
    }
    return;
  }

  // the wave's rows of W_hh^T in registers, k-step (i, r) = gate r of slot
  // g MU + i: wt[mu][i][r] = W_hh[r H + slot_unit(g MU + i, q)][16 mu + c16]
  // (decoder: the folded W' = W_hh + A Wp for t >= 1, plain W_hh for t = 0 --
  // kept in registers for H <= 32, reloaded at t = 0 above that, where a
  // second copy would spill)
  constexpr bool wt0_reg = MU <= 2;
  float wt[MU][MU][4], wt0[MU][MU][4];
#pragma unroll
  for (int i = 0; i < MU; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r * H + slot_unit(g * MU + i, q);
      const float a0 = decoder ? A[2 * row] : 0.f, a1 = decoder ? A[2 * row + 1] : 0.f;
#pragma unroll
      for (int mu = 0; mu < MU; ++mu) {
        const int col = 16 * mu + c16;
        const float v = Whh[row * H + col];
        wt0[mu][i][r] = v;
        wt[mu][i][r] = decoder ? fmaf(a1, Wp[H + col], fmaf(a0, Wp[col], v)) : v;
      }
    }
  // X3: P_w on split-bf16 MFMAs (sgg_common.h mfma_x3).  The lane's 4 MU dG
  // values (slot i, gate r at index 4 i + r) are its k-elements of K = 32
  // chunks -- k = 32 ch + 8 q + j <-> index 8 ch + j of lane quarter q, zero
  // past 4 MU -- so the B operand is the lane's own values and the A operand
  // the same W_hh^T entries as wt (their pieces, built once here; the
  // decoder's plain set for step 0 beside the folded one while MU <= 2).
  constexpr int KCH = (4 * MU + 7) / 8;
  constexpr bool kWq0 = BX3 && DEC && MU <= 2;
  bf16x8 wq[BX3 ? MU : 1][BX3 ? KCH : 1][3], wq0[kWq0 ? MU : 1][kWq0 ? KCH : 1][3];
  auto build_wq = [&](const float (&w)[MU][MU][4], bf16x8 (&o)[BX3 ? MU : 1][BX3 ? KCH : 1][3]) {
    if constexpr (BX3) {
#pragma unroll
      for (int mu = 0; mu < MU; ++mu)
#pragma unroll
        for (int ch = 0; ch < KCH; ++ch) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int x = 8 * ch + j;
            v[j] = x < 4 * MU ? w[mu][x >> 2][x & 3] : 0.f;
          }
          split8(v, o[mu][ch]);
        }
    }
  };
  build_wq(wt, wq);
  if constexpr (kWq0) build_wq(wt0, wq0);
  // per owned slot: rows of A for the four gates (A^T dG), Wp columns, dc
  float aa0[MU][4], aa1[MU][4], wp0[MU], wp1[MU], dc[MU], dh[MU];
#pragma unroll
  for (int i = 0; i < MU; ++i) {
    const int u = slot_unit(g * MU + i, q);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      aa0[i][k] = A[2 * (k * H + u)];
      aa1[i][k] = A[2 * (k * H + u) + 1];
    }
    wp0[i] = decoder ? Wp[u] : 0.f;
    wp1[i] = decoder ? Wp[H + u] : 0.f;
    dc[i] = 0.f;
    dh[i] = (!decoder && dh_last) ? dh_last[(size_t)pc * H + u] : 0.f;
  }

  // saved activations and cells of the owned slots (and the decoder's output
  // gradient, the step input of the weight gradient), one step ahead;
  // tile-native, lane-linear
  // (the activations stay one 16-byte vector per slot from the load to the
  // use: split into scalars, the loop-carried copies did not line up with the
  // dwordx4 load's registers and the compiler moved two lanes of the FRESH
  // load right after issuing it -- a wait for a whole memory round trip at
  // the head of every step, ~1 us; tools/lstm_bwd_probe.hip)
  // (the two-set form keeps the cells as one native vector each: as float
  // arrays their copies were v_movs placed right after the fresh loads, and
  // each step waited vmcnt(0) for its own prefetch before its barrier)
  typedef float fvmu __attribute__((ext_vector_type(MU)));
  struct FArr {   // the one-set form's cells: plain arrays (its measured code)
    float v[MU];
    __device__ float operator[](int i) const { return v[i]; }
  };
  constexpr bool kDB = SGG_MW_BWD_DB && !(WGRAD && !DEC);
  typedef typename std::conditional<kDB, fvmu, FArr>::type CellV;
  struct StepIn {
    floatx4 a[MU];
    CellV c, cp;
    float d0, d1, r0, r1;
  };
  StepIn sa, sb;
  sa.d0 = sa.d1 = sa.r0 = sa.r1 = sb.d0 = sb.d1 = sb.r0 = sb.r1 = 0.f;
  auto load_step = [&](int t, StepIn& s) {
    if (wgrad) {   // r_in(t): rel[t] (encoder); rel0, then rel_out[t - 1] (decoder)
      const float* rp = !decoder ? rel + ((size_t)t * B + pc) * 2
                                 : (t == 0 ? rel + (size_t)pc * 2 : rel_out + ((size_t)(t - 1) * B + pc) * 2);
      const float2 rv = *reinterpret_cast<const float2*>(rp);
      s.r0 = rv.x;
      s.r1 = rv.y;
    }
    const float4* ab = reinterpret_cast<const float4*>(act_tile) + ((size_t)sblk(t < t_sh) * T + t) * KS * 64 + lane;
#pragma unroll
    for (int i = 0; i < MU; ++i) s.a[i] = *reinterpret_cast<const floatx4*>(ab + (g * MU + i) * 64);
    const float* pc1 = c_tile + ((((size_t)sblk(t + 1 <= t_sh) * (T + 1) + t + 1) * 4 + g) * 64 + lane) * MU;
    const float* pc0 = c_tile + ((((size_t)sblk(t <= t_sh) * (T + 1) + t) * 4 + g) * 64 + lane) * MU;
    if constexpr (kDB) {
      __builtin_memcpy(&s.c, pc1, MU * sizeof(float));
      __builtin_memcpy(&s.cp, pc0, MU * sizeof(float));
    } else {
      load_vec<MU>(pc1, s.c.v);
      load_vec<MU>(pc0, s.cp.v);
    }
    if (decoder) {
      // dout2: the output gradient of peds >= bsplit is a separate (T x (B - bsplit) x 2) block
      const float* dp = (dout2 && pc >= bsplit) ? dout2 + ((size_t)t * (B - bsplit) + (pc - bsplit)) * 2
                                                : dout + ((size_t)t * (dout2 ? bsplit : B) + pc) * 2;
      const float2 dv = *reinterpret_cast<const float2*>(dp);
      s.d0 = dv.x;
      s.d1 = dv.y;
    }
  };

  float db[MU][4], dax[MU][4], day[MU][4];
#pragma unroll
  for (int i = 0; i < MU; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) db[i][k] = dax[i][k] = day[i][k] = 0.f;

  load_step(T - 1, sa);
  float din_x = 0.f, din_y = 0.f;   // drel_in[t + 1] (wave 0, q = 0 lanes; every lane for the decoder's dWp)
  // decoder weight gradients of hidden2pos, lane-accumulated over the steps:
  // dWp += drel_tot[t] h_{t+1}^T (the lane's slots), dbp += drel_tot[t]
  constexpr bool pgrad = decoder && wgrad;
  float dwp0[MU], dwp1[MU], dbp0 = 0.f, dbp1 = 0.f;
#pragma unroll
  for (int i = 0; i < MU; ++i) dwp0[i] = dwp1[i] = 0.f;

  // t_stop > 0 (input gradients only, no dh0): the steps below t_stop are
  // skipped -- their input gradients are not wanted (the discriminator's
  // observed part in the generator step)
  LMARK(1);
  // (two sets (kDB, above) where the owners are the step's long pole; with
  // the encoders' weight gradients the helpers are, and the owners' earlier
  // start only took issue slots from them -- H = 48: 38.5 -> 42.8 us; the
  // G-step's H = 48 input-gradient form 18.0 -> 16.8 us, the decoder's
  // 19.1 -> 18.7 us)
  // the step's loaded operands in two register sets used in turn (the loop
  // runs two steps per iteration): a set is loaded one step ahead and read
  // where it was loaded, no loop-carried copy -- a copy of a fresh load had
  // the compiler wait for the prefetch inside the step that issued it
  auto step = [&](int t, const StepIn& si, StepIn& so) {
    if (T - 1 - t < 60) LMARK(2 + T - 1 - t);
    const int cur = t & 1;
    LSUBB(0);
    const float d0 = si.d0, d1 = si.d1, r0 = si.r0, r1 = si.r1;
    floatx4 ca[MU];
#pragma unroll
    for (int i = 0; i < MU; ++i) ca[i] = si.a[i];
    const CellV cc = si.c, ccp = si.cp;
    // in flight while this step computes; with two sets unconditional (the
    // last step re-reads a valid step): under a branch the compiler's wait
    // counts at the join assumed the loads absent and waited for them inside
    // this step
    if (kDB || t > t_stop) load_step(t > 0 ? t - 1 : 0, so);

    float f0 = 0.f, f1 = 0.f;
    // drel_tot[t] = dout[t] + drel_in[t + 1] of this lane's ped (zero for a padded ped)
    const float rtx = keep_if(d0 + din_x, valid), rty = keep_if(d1 + din_y, valid);
    if (pgrad) {
      dbp0 += rtx;
      dbp1 += rty;
    }
    if (decoder && t == 0) {
#pragma unroll
      for (int mu = 0; mu < MU; ++mu)
#pragma unroll
        for (int i = 0; i < MU; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            wt[mu][i][r] = wt0_reg ? wt0[mu][i][r] : Whh[(r * H + slot_unit(g * MU + i, q)) * H + 16 * mu + c16];
      if constexpr (BX3) {
        if constexpr (kWq0) {
#pragma unroll
          for (int mu = 0; mu < MU; ++mu)
#pragma unroll
            for (int ch = 0; ch < KCH; ++ch)
#pragma unroll
              for (int pc3 = 0; pc3 < 3; ++pc3) wq[mu][ch][pc3] = wq0[mu][ch][pc3];
        } else {
          build_wq(wt, wq);
        }
      }
    }
    floatx4 acc[MU];
#pragma unroll
    for (int mu = 0; mu < MU; ++mu) acc[mu] = floatx4{0.f, 0.f, 0.f, 0.f};
    float vall[BX3 ? 8 * KCH : 1];   // X3: the lane's dG values in k order, zero padded
#pragma unroll
    for (int x = 0; x < (BX3 ? 8 * KCH : 1); ++x) vall[x] = 0.f;
#pragma unroll
    for (int i = 0; i < MU; ++i) {
      const int j = g * MU + i;
      float dhv = dh[i];
      if (t < T - 1)
        dhv = (part[cur ^ 1][0][j][lane] + part[cur ^ 1][1][j][lane]) + (part[cur ^ 1][2][j][lane] + part[cur ^ 1][3][j][lane]);
      if (i == 0) {
        LUSE(dhv);
        LSUBB(1);
      }
      if (decoder) dhv = fmaf(wp0[i], d0, fmaf(wp1[i], d1, dhv));
      const float ig = ca[i][0], fg = ca[i][1], gg = ca[i][2], og = ca[i][3];
      const float tc = tanh_m(cc[i]);
      if (pgrad) {   // h_{t+1} of the slot = o_t tanh(c_t)
        const float hn = og * tc;
        dwp0[i] = fmaf(rtx, hn, dwp0[i]);
        dwp1[i] = fmaf(rty, hn, dwp1[i]);
      }
      const float d_o = dhv * tc;
      const float dct = fmaf(dhv * og, 1.f - tc * tc, dc[i]);
      dc[i] = dct * fg;
      // a padded ped (last block) carries no gradient: its dG is zero, so it
      // adds nothing to the weight gradients
      const float vv[4] = {keep_if(dct * gg * ig * (1.f - ig), valid), keep_if(dct * ccp[i] * fg * (1.f - fg), valid),
                           keep_if(dct * ig * (1.f - gg * gg), valid), keep_if(d_o * og * (1.f - og), valid)};
      if constexpr (BX3) {
#pragma unroll
        for (int r = 0; r < 4; ++r) vall[4 * i + r] = vv[r];
        // a chunk's MFMAs as soon as its 8 values are in (slots 0-1, then 2-3)
        if ((4 * i + 4) % 8 == 0 || i == MU - 1) {
          const int ch = (4 * i) / 8;
          float v8[8];
#pragma unroll
          for (int x = 0; x < 8; ++x) v8[x] = vall[8 * ch + x];
          bf16x8 hp[3];
          split8(v8, hp);
#pragma unroll
          for (int mu = 0; mu < MU; ++mu) acc[mu] = mfma_x3(wq[mu][ch], hp, acc[mu]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int mu = 0; mu < MU; ++mu) acc[mu] = __builtin_amdgcn_mfma_f32_16x16x4f32(wt[mu][i][r], vv[r], acc[mu], 0, 0, 0);
      }
      if (wgrad) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          dgb[cur][k][j][lane] = vv[k];
          if (!hdb) {
            db[i][k] += vv[k];
            dax[i][k] = fmaf(vv[k], r0, dax[i][k]);
            day[i][k] = fmaf(vv[k], r1, day[i][k]);
          }
        }
      }
      if (!hacc) {
        f0 = fmaf(aa0[i][3], vv[3], fmaf(aa0[i][2], vv[2], fmaf(aa0[i][1], vv[1], fmaf(aa0[i][0], vv[0], f0))));
        f1 = fmaf(aa1[i][3], vv[3], fmaf(aa1[i][2], vv[2], fmaf(aa1[i][1], vv[1], fmaf(aa1[i][0], vv[0], f1))));
      }
    }
    if (!hacc) {
      f0 += __shfl_xor(f0, 16);
      f0 += __shfl_xor(f0, 32);
      f1 += __shfl_xor(f1, 16);
      f1 += __shfl_xor(f1, 32);
      if (q == 0) fbp[cur][g][c16] = make_float2(f0, f1);
    }
    LUSE(acc[MU - 1][0]);
    LSUBB(2);
    // this wave's share of dh_{t-1}: D row 4 q + r of tile mu is unit
    // slot_unit(4 mu + r, q), i.e. slot 4 mu + r of the next step's owners
#pragma unroll
    for (int mu = 0; mu < MU; ++mu)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[cur][g][4 * mu + r][lane] = acc[mu][r];
    LSUBB(3);
    lds_barrier();
    LSUBB(4);
    if (!hacc && (pgrad || (g == 0 && q == 0))) {   // drel_in[t] = A^T dG_t; decoder: drel_tot[t] = dout[t] + drel_in[t + 1]
      const float2 r0 = fbp[cur][0][c16], r1 = fbp[cur][1][c16], r2 = fbp[cur][2][c16], r3 = fbp[cur][3][c16];
      const float sx = (r0.x + r1.x) + (r2.x + r3.x), sy = (r0.y + r1.y) + (r2.y + r3.y);
      if (valid && g == 0 && q == 0) {
        *reinterpret_cast<float2*>(drel_in + ((size_t)t * B + ped) * 2) = make_float2(sx, sy);
        if (decoder) *reinterpret_cast<float2*>(drel_tot + ((size_t)t * B + ped) * 2) = make_float2(d0 + din_x, d1 + din_y);
      }
      din_x = sx;
      din_y = sy;
    }
    };
  if constexpr (kDB) {
    for (int t = T - 1; t >= t_stop; t -= 2) {
      step(t, sa, sb);
      if (t - 1 < t_stop) break;
      step(t - 1, sb, sa);
    }
  } else {
    for (int t = T - 1; t >= t_stop; --t) {
      const StepIn si = sa;
      step(t, si, sa);
    }
  }

  if (hacc) lds_barrier();   // the helpers' last drel_in partials (helper branch)
  if (t_stop > 0 && valid && g == 0 && q == 0) {   // the skipped steps' input gradients are defined as zero
    for (int t = 0; t < t_stop; ++t) *reinterpret_cast<float2*>(drel_in + ((size_t)t * B + ped) * 2) = make_float2(0.f, 0.f);
  }
  if (dh0 && valid) {   // dh0 = W_hh^T dG_0
#pragma unroll
    for (int i = 0; i < MU; ++i) {
      const int j = g * MU + i;
      dh0[(size_t)ped * H + slot_unit(j, q)] = (part[0][0][j][lane] + part[0][1][j][lane]) + (part[0][2][j][lane] + part[0][3][j][lane]);
    }
  }
  if (wgrad) {
    float* row = wpart + (size_t)blk * P;
    // db / dA of the owned slots: sum over the 16 peds (lanes c16 of each q)
    // (with the helpers' sums, hdb, nothing here)
#pragma unroll
    for (int i = 0; i < (hdb ? 0 : MU); ++i) {
      const int u = slot_unit(g * MU + i, q);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = db[i][k], x = dax[i][k], y = day[i][k];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          a += __shfl_xor(a, o);
          x += __shfl_xor(x, o);
          y += __shfl_xor(y, o);
        }
        if (c16 == 0) {
          row[G4 * H + k * H + u] = a;
          row[G4 * H + G4 + 2 * (k * H + u)] = x;
          row[G4 * H + G4 + 2 * (k * H + u) + 1] = y;
        }
      }
    }
    if (pgrad) {   // [dWp (2 x H) | dbp (2)]: sums over the 16 peds
#pragma unroll
      for (int i = 0; i < MU; ++i) {
        float x = dwp0[i], y = dwp1[i];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          x += __shfl_xor(x, o);
          y += __shfl_xor(y, o);
        }
        const int u = slot_unit(g * MU + i, q);
        if (c16 == 0) {
          row[P0 + u] = x;
          row[P0 + H + u] = y;
        }
      }
      if (g == 0 && q == 0) {
        float x = dbp0, y = dbp1;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          x += __shfl_xor(x, o);
          y += __shfl_xor(y, o);
        }
        if (c16 == 0) {
          row[P0 + 2 * H] = x;
          row[P0 + 2 * H + 1] = y;
        }
      }
    }
  }
  LMARK(62);
}

template <int H>
int launch_seg(const MwSeg& sg, bool decoder, hipStream_t st) {
  const int grid = (sg.B + kMwPeds - 1) / kMwPeds;
  auto k = decoder ? (sg.act_tile ? lstm_mw_fwd_kernel<H, true, true> : lstm_mw_fwd_kernel<H, true, false>)
                   : (sg.act_tile ? lstm_mw_fwd_kernel<H, false, true> : lstm_mw_fwd_kernel<H, false, false>);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kMwThreads), 0, st, sg);
  SGG_RETURN_LAUNCH("sgg_lstm_fwd");
}

int launch_seg_h(const MwSeg& sg, int H, bool decoder, hipStream_t st) {
  switch (H) {
    case 16: return launch_seg<16>(sg, decoder, st);
    case 32: return launch_seg<32>(sg, decoder, st);
    case 48: return launch_seg<48>(sg, decoder, st);
    default: return launch_seg<64>(sg, decoder, st);
  }
}

template <int H>
int launch_bwd(const float* A, const float* Whh, const float* Wp, const float* h_all, const float* c_all,
               const float* act_all, const float* rel, const float* rel_out, const float* dh_last, const float* dout,
               int T, int B, int decoder, float* dh0, float* drel_in, float* drel_tot, float* wpart, hipStream_t st,
               const float* dout2, int bsplit, int t_stop, int t_sh, int Bsrc) {
  const int grid = (B + kMwPeds - 1) / kMwPeds;
  auto k = decoder ? (wpart ? lstm_mw_bwd_kernel<H, true, true> : lstm_mw_bwd_kernel<H, true, false>)
                   : (wpart ? lstm_mw_bwd_kernel<H, false, true> : lstm_mw_bwd_kernel<H, false, false>);
  hipLaunchKernelGGL(k, dim3(grid), dim3(wpart ? 2 * kMwThreads : kMwThreads), 0, st, A, Whh, Wp, h_all, c_all, act_all, rel, rel_out,
                     dh_last, dout, T, B, dh0, drel_in, drel_tot, wpart, dout2, bsplit, t_stop, t_sh, Bsrc);
  SGG_RETURN_LAUNCH("sgg_lstm_bwd");
}

}  // namespace

// Policy: every H (16 / 32 / 48 / 64).  Measured at the training shapes
// (tools/lstm_probe.py, profiles/r02_lstm_*): the generator's H = 32 encoder
// (T 8, B 1280) fwd 10.7 / bwd 18.2 us here vs 11.2 / 18.9 us + two weight-
// gradient reductions in the unit-per-thread family, its decoder (T 12,
// B 2560) 17.6 / 25.8 vs 23.1 / 35.6 us + three reductions.  SGG_LSTM_MW=0
// disables this form, SGG_LSTM_MW=big keeps it to H >= 48 (kernel
// comparisons, tools/).  The same predicate picks the forward (when it
// saves states) and the backward, so the tile-native saved layout is always
// read by the kernel that wrote it.
bool lstm_mw_ok(int H, int B) {
  (void)B;
  const char* e = getenv("SGG_LSTM_MW");
  if (e && strcmp(e, "0") == 0) return false;
  if (e && strcmp(e, "big") == 0) return H == 48 || H == 64;
  return H == 16 || H == 32 || H == 48 || H == 64;
}

long long lstm_mw_state_floats(int T, int B, int H, int which) {
  const long long padded = (long long)(B + kMwPeds - 1) / kMwPeds * kMwPeds;
  return which == 0 ? (long long)T * padded * 4 * H : (long long)(T + 1) * padded * H;
}

int lstm_mw_wpart_rows(int H, int B) {
  (void)H;
  return (B + kMwPeds - 1) / kMwPeds;
}

int lstm_mw_fwd(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0,
                const float* c0, const float* Wp, const float* bp, int T, int B, int H, int decoder, float* h_all,
                float* c_all, float* act_all, float* rel_out, hipStream_t st, const float* Wu, int ldwu,
                const float* cu, int NU, float* U, const SggDecInit* di, float* rel0_out, const SggTrajOut* to) {
  SGG_CHECK_ARG(decoder || T <= kMwMaxT, "sgg_lstm_fwd: encoder sequences of the H=%d kernels hold <= %d steps (T=%d)",
                H, kMwMaxT, T);
  MwSeg sg{rel, A, Whh, bias, h0, c0, Wp, bp, T, B, B, 0, T, B, h_all, c_all, act_all, rel_out, Wu, ldwu, cu, NU, U};
  if (di) {
    sg.di = *di;
    sg.rel0_out = rel0_out;
  }
  if (to) sg.to = *to;
  return launch_seg_h(sg, H, decoder != 0, st);
}

// checks of one encoder segment (sgg.h SggLstmSeg)
static int seg_check(const MwSeg& s, int H, const char* fn) {
  SGG_CHECK_ARG(s.rel && s.A && s.Whh && s.bias && s.h_all && (s.c_tile || !s.act_tile), "%s: null pointer", fn);
  SGG_CHECK_ARG(H == 16 || H == 32 || H == 48 || H == 64, "%s: hidden size %d (16/32/48/64)", fn, H);
  SGG_CHECK_ARG(s.T >= 1 && s.T <= kMwMaxT && s.B >= 1 && s.Bl >= s.B && s.t0 >= 0 && s.t0 + s.T <= s.Tl,
                "%s: bad sizes T=%d B=%d Bl=%d t0=%d Tl=%d", fn, s.T, s.B, s.Bl, s.t0, s.Tl);
  SGG_CHECK_ARG(s.t0 == 0 || (s.c_tile && s.Bsrc >= 1 && s.Bsrc <= s.Bl &&
                              (s.Bsrc == s.B || (s.Bsrc % kMwPeds == 0 && s.B % s.Bsrc == 0))),
                "%s: a segment from step t0=%d needs the saved cells and Bsrc = B or a multiple of 16 dividing B "
                "(B=%d Bsrc=%d)", fn, s.t0, s.B, s.Bsrc);
  SGG_CHECK_ARG(s.t0 == 0 || (!s.h0 && !s.c0), "%s: t0 > 0 takes its state from h_all / c_all, not h0 / c0", fn);
  SGG_CHECK_ARG(!s.U || (s.Wu && s.cu && s.NU >= 16 && s.NU % 16 == 0 && s.ldwu >= H), "%s: bad projection", fn);
  return 0;
}

int lstm_mw_fwd_seg(const MwSeg& s, int H, hipStream_t st) {
  if (int rc = seg_check(s, H, "sgg_lstm_fwd_seg")) return rc;
  return launch_seg_h(s, H, false, st);
}

int lstm_mw_fwd_seg2(const MwSeg& a, int Ha, const MwSeg& b, int Hb, hipStream_t st) {
  if (int rc = seg_check(a, Ha, "sgg_lstm_fwd_seg2 (a)")) return rc;
  if (int rc = seg_check(b, Hb, "sgg_lstm_fwd_seg2 (b)")) return rc;
  const int na = (a.B + kMwPeds - 1) / kMwPeds, nb = (b.B + kMwPeds - 1) / kMwPeds;
  if (Ha == 32 && Hb == 48 && b.act_tile) {   // the generator encoder + the discriminator prefix
    auto k = a.act_tile ? lstm_mw_fwd2_kernel<32, true, 48, true> : lstm_mw_fwd2_kernel<32, false, 48, true>;
    hipLaunchKernelGGL(k, dim3(na + nb), dim3(kMwThreads), 0, st, a, b, na);
    SGG_RETURN_LAUNCH("sgg_lstm_fwd_seg2");
  }
  // other hidden-size pairs: two launches
  if (int rc = launch_seg_h(a, Ha, false, st)) return rc;
  return launch_seg_h(b, Hb, false, st);
}

int lstm_mw_fwd_dec_seg(const float* A, const float* Whh, const float* bias, const float* Wp, const float* bp, int T,
                        int B, int H, float* h_all, float* c_all, float* act_all, float* rel_out, const SggDecInit* di,
                        float* rel0_out, const SggTrajOut* to, const MwSeg& b, int Hb, hipStream_t st) {
  if (int rc = seg_check(b, Hb, "sgg_lstm_fwd_dec_seg (prefix)")) return rc;
  MwSeg a{nullptr, A, Whh, bias, nullptr, nullptr, Wp, bp, T, B, B, 0, T, B, h_all, c_all, act_all, rel_out};
  a.di = *di;
  a.rel0_out = rel0_out;
  if (to) a.to = *to;
  const int na = (B + kMwPeds - 1) / kMwPeds, nb = (b.B + kMwPeds - 1) / kMwPeds;
  if (H == 32 && Hb == 48 && act_all && b.act_tile) {
    hipLaunchKernelGGL((lstm_mw_fwd2d_kernel<32, true, 48, true>), dim3(na + nb), dim3(kMwThreads), 0, st, a, b, na);
    SGG_RETURN_LAUNCH("sgg_lstm_fwd_dec_seg");
  }
  if (int rc = launch_seg_h(a, H, true, st)) return rc;   // other sizes: two launches
  return launch_seg_h(b, Hb, false, st);
}

int lstm_mw_fwd_seg3(const MwSeg& a, int Ha, const MwSeg& b, int Hb, const MwSeg& c, int Hc, hipStream_t st) {
  if (int rc = seg_check(a, Ha, "sgg_lstm_fwd_seg3 (a)")) return rc;
  if (int rc = seg_check(b, Hb, "sgg_lstm_fwd_seg3 (b)")) return rc;
  if (int rc = seg_check(c, Hc, "sgg_lstm_fwd_seg3 (c)")) return rc;
  const int na = (a.B + kMwPeds - 1) / kMwPeds, nb = (b.B + kMwPeds - 1) / kMwPeds, nc = (c.B + kMwPeds - 1) / kMwPeds;
  if (Ha == 32 && Hb == 48 && Hc == 32 && !a.act_tile && b.act_tile && c.act_tile) {
    hipLaunchKernelGGL((lstm_mw_fwd3_kernel<32, false, 48, true, 32, true>), dim3(na + nb + nc), dim3(kMwThreads), 0, st,
                       a, b, c, na, nb);
    SGG_RETURN_LAUNCH("sgg_lstm_fwd_seg3");
  }
  // other combinations: the first two in one launch where seg2 has a kernel, then the third
  if (int rc = lstm_mw_fwd_seg2(a, Ha, b, Hb, st)) return rc;
  return launch_seg_h(c, Hc, false, st);
}

int lstm_mw_bwd(const float* A, const float* Whh, const float* Wp, const float* h_all, const float* c_all,
                const float* act_all, const float* rel, const float* rel_out, const float* dh_last, const float* dout,
                int T, int B, int H, int decoder, float* dh0, float* drel_in, float* drel_tot, float* wpart,
                hipStream_t st, const float* dout2, int bsplit, int t_stop, int t_sh, int Bsrc) {
  // the helper waves pass one barrier per step of ALL T steps
  SGG_CHECK_ARG(!wpart || t_stop == 0, "sgg_lstm_bwd: weight gradients need every step (t_stop=%d)", t_stop);
  SGG_CHECK_ARG(t_sh == 0 || (!decoder && t_sh < T && Bsrc >= kMwPeds && Bsrc % kMwPeds == 0 && B % Bsrc == 0),
                "sgg_lstm_bwd: a shared prefix needs an encoder, t_sh < T and Bsrc a multiple of 16 dividing B "
                "(t_sh=%d T=%d B=%d Bsrc=%d)", t_sh, T, B, Bsrc);
  switch (H) {
    case 16: return launch_bwd<16>(A, Whh, Wp, h_all, c_all, act_all, rel, rel_out, dh_last, dout, T, B, decoder, dh0, drel_in, drel_tot, wpart, st, dout2, bsplit, t_stop, t_sh, Bsrc);
    case 32: return launch_bwd<32>(A, Whh, Wp, h_all, c_all, act_all, rel, rel_out, dh_last, dout, T, B, decoder, dh0, drel_in, drel_tot, wpart, st, dout2, bsplit, t_stop, t_sh, Bsrc);
    case 48: return launch_bwd<48>(A, Whh, Wp, h_all, c_all, act_all, rel, rel_out, dh_last, dout, T, B, decoder, dh0, drel_in, drel_tot, wpart, st, dout2, bsplit, t_stop, t_sh, Bsrc);
    default: return launch_bwd<64>(A, Whh, Wp, h_all, c_all, act_all, rel, rel_out, dh_last, dout, T, B, decoder, dh0, drel_in, drel_tot, wpart, st, dout2, bsplit, t_stop, t_sh, Bsrc);
  }
}

}  // namespace sgg
