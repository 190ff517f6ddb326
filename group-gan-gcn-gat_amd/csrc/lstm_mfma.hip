// Fused LSTM sequence forward on v_mfma_f32_16x16x4_f32 (Encoder,
// reference sgan/models.py:62-92; Decoder rollout :142-178).  Same contract
// as lstm_fwd_kernel (lstm.hip, sgg_lstm_fwd in include/sgg.h); used for the
// large batches of the training step, where the per-step gate GEMM
// (4H x H per ped) dominates and the VALU form is FMA-bound.
//
// One wave = 16 peds and the whole recurrence stays in its registers:
//   G^T (4H x 16 peds) = W_ext (4H x (H + 4)) . X^T ((H + 4) x 16 peds)
// with X = [h_{t-1} | r_x r_y 1 0]: the folded input projection A r + b'
// rides along as one extra 4-deep k-step.  16x16x4 lane maps (A[row][k]:
// lane (k<<4 | row); B[k][col]: lane (k<<4 | col); D[row][col]: lane
// (row>>2 << 4 | col), register row & 3), so lane l = (q = l >> 4, ped = l & 15)
// ends a step holding gate rows 16 mt + 4q + r of its ped: the i, f, g and o
// rows of unit u = 16 mu + 4q + r sit in tiles mu, mu + H/16, mu + 2H/16,
// mu + 3H/16 of the SAME lane and register, so the cell update is lane-local.
// The k order of the next step's GEMM is permuted so that k-step ks, lane q
// supplies unit 16 (ks >> 2) + 4q + (ks & 3) -- exactly the h value that lane
// just produced (h[ks]); W_ext's columns are loaded into registers in the
// same permuted order once (staged through LDS by the workgroup, one barrier
// in the prologue); the steps need no LDS and no barriers.
// Decoder: rel_t = Wp h_t + bp is a lane partial over its H/4 units plus two
// cross-q shuffles, and feeds the next step's input k-step in registers.
#include <stdlib.h>
#include <string.h>

#include "sgg_common.h"

namespace sgg {

namespace {

// v_exp_f32 / v_rcp_f32 forms (~2 ulp): the 5H transcendentals per ped and
// step are the VALU side of this kernel
__device__ __forceinline__ float sigm_fast(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
// (exp(-2x) as v_exp_f32(x * -2 log2(e)): -2 log2(e) is exact, so the same bits as
// __expf(-2x)'s (-2x) * log2(e) with one multiply less)
__device__ __forceinline__ float tanh_fast(float x) {
  return fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -2.8853900817779268f)), -1.f);
}
// the same activations of a pre-activation the weights already scaled by
// -log2(e) (sigmoid) or -2 log2(e) (tanh): v_exp_f32 takes it directly (the
// scale rides in W_ext, loaded once; one VALU multiply less per gate value)
constexpr float kNegLog2e = -1.4426950408889634f;
__device__ __forceinline__ float sigm_pre(float y) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(y)); }
__device__ __forceinline__ float tanh_pre(float y) { return fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(y)), -1.f); }

// a second no-grad decoder segment of the same decoder weights in the same
// launch (sgg_lstm_fwd_dec2): workgroups from nblk1 on run it -- the
// discriminator step's generator decoder beside the generator step's
// best-of-k rollout; its discriminator input (SggTrajOut) written here too
struct RollSeg2 {
  SggDecInit di;
  float* rel_out;
  SggTrajOut to;
  int B, nblk1;
};

__device__ __forceinline__ SggDecInit pick_di(const SggDecInit& a, const SggDecInit& b, bool two) {
  SggDecInit d;
  d.ctx = two ? b.ctx : a.ctx;
  d.ldc = two ? b.ldc : a.ldc;
  d.Dc = two ? b.Dc : a.Dc;
  d.z = two ? b.z : a.z;
  d.nz = two ? b.nz : a.nz;
  d.best = two ? b.best : a.best;
  d.first_k = two ? b.first_k : a.first_k;
  d.ped_scene = two ? b.ped_scene : a.ped_scene;
  d.S = two ? b.S : a.S;
  d.Bper = two ? b.Bper : a.Bper;
  d.last_rel = two ? b.last_rel : a.last_rel;
  return d;
}

// Sum of a value over the four 16-lane rows of the wave (the four q lanes of a
// ped), in every lane: two lane-swap moves (gfx950 v_permlane16_swap /
// v_permlane32_swap, VALU) instead of two LDS-routed shuffles; the additions
// pair (row 0 + row 1) + (row 2 + row 3) in every lane, as the xor-16 / xor-32
// shuffle tree did.
__device__ __forceinline__ float rows_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

typedef float float2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2v exp2v(float2v y) {
  return float2v{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
}
__device__ __forceinline__ float2v rcpv(float2v y) {
  return float2v{__builtin_amdgcn_rcpf(y.x), __builtin_amdgcn_rcpf(y.y)};
}
// exponent arguments are clamped where an infinite exponential would meet a
// zero (0 * inf): 2^64 keeps every product below finite range, and the
// functions it feeds are saturated there to far below fp32 resolution
constexpr float kExpArgMax = 64.f;
__device__ __forceinline__ float2v clampv(float2v y) {
  return float2v{__builtin_amdgcn_fmed3f(y.x, -kExpArgMax, kExpArgMax), __builtin_amdgcn_fmed3f(y.y, -kExpArgMax, kExpArgMax)};
}

// The cell update of two units at once from their gate pre-activations,
// pre-scaled by -log2(e) (i, f, o) and -2 log2(e) (g):  with e_x = 2^{y_x},
//   f c = c / (1 + e_f),   i g = (1 - e_g) / ((1 + e_i)(1 + e_g)),
//   h   = o tanh(c') = (1 - e_c) / ((1 + e_o)(1 + e_c)),  e_c = 2^{-2 log2(e) c'}
// -- five exponentials and three reciprocals per unit (the per-gate form
// takes five of each), the rest as packed two-unit VALU operations.
__device__ __forceinline__ void cell2(float2v yi, float2v yf, float2v yg, float2v yo, float2v& c, float2v& h) {
  const float2v one = {1.f, 1.f};
  const float2v ei = exp2v(yi), ef = exp2v(yf), eg = exp2v(clampv(yg)), eo = exp2v(yo);
  const float2v rf = rcpv(one + ef);
  const float2v rig = rcpv((one + ei) * (one + eg));
  c = __builtin_elementwise_fma(c, rf, (one - eg) * rig);
  const float2v ec = exp2v(clampv(c * float2v{-2.8853900817779268f, -2.8853900817779268f}));
  h = (one - ec) * rcpv((one + eo) * (one + ec));
}

// X3 (H = 32): the gate GEMM on split-bf16 MFMAs (sgg_common.h mfma_x3):
// per step 48 x 16 instead of 64 x 32 cycles of the matrix pipe, within a few
// fp32 roundings of the fp32 form (not bitwise).

// DEC (runtime, uniform): the decoder's output feedback folded into the
// recurrence.  The next input is rel_t = Wp h_t + bp, so for t >= 1
//   W_hh h + A rel + b = (W_hh + A Wp) h + (b + A bp):
// the lane's weight registers hold W' = W_hh + A Wp and its accumulators start
// from b' = b + A bp (the first MFMA's C operand), so a step is 4H/16 x H/4
// MFMAs with no input k-step.  Step 0 adds A (rel_0 - Wp h_0 - bp) through
// the input k-step.  The encoder (no feedback) keeps the input k-step
// [r_x r_y 0 0] every step.
// (H = 32: two waves per SIMD, pinned -- the build's -amdgpu-mfma-vgpr-form
// keeps the accumulators in VGPRs (227); without that flag the allocator
// parks them in 64 AGPRs, 292 registers in all, one wave per SIMD)
// phase probe (tools/lstm_roll_probe.hip builds its own copy with
// SGG_ROLL_PROF): wall-clock marks per step of workgroups 0 and 300, shader
// cycle marks of step 4's phases; nothing in the library build
#ifdef SGG_ROLL_PROF
__device__ long long g_roll_prof[8192 + 512];
#define RMARK(t)                                                                                      \
  if (threadIdx.x == 0 && blockIdx.x < 512 && (t) < 16) g_roll_prof[16 * blockIdx.x + (t)] = wall_clock64();
#define RSUB(k)                                                                                       \
  if ((threadIdx.x & 63) == 0 && (blockIdx.x == 0 || blockIdx.x == 300) && t == 4)                   \
    g_roll_prof[8192 + (blockIdx.x ? 64 : 0) + 8 * (threadIdx.x >> 6) + (k)] = clock64();
#define RUSE(x) __asm__ volatile("" ::"v"(x));
#else
#define RMARK(t)
#define RSUB(k)
#define RUSE(x)
#endif

#ifndef SGG_ROLL_WPE
#define SGG_ROLL_WPE 2
#endif
// (DEC a template parameter: with one step loop for both forms, the encoder's
// prefetch load made the compiler wait vmcnt(0) at the loop's back edge --
// and on gfx9 vmcnt counts stores too, so every decoder step waited for the
// acknowledgement of its own output stores)
template <int H, bool X3, bool DEC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(H <= 32 ? SGG_ROLL_WPE : 1))) lstm_fwd_mfma_kernel(
    const float* __restrict__ rel, const float* __restrict__ A, const float* __restrict__ Whh,
    const float* __restrict__ bias, const float* __restrict__ h0, const float* __restrict__ c0,
    const float* __restrict__ Wp, const float* __restrict__ bp, int T, int B1,
    float* __restrict__ h_all, float* __restrict__ c_all, float* __restrict__ rel_out1, SggDecInit di1, RollSeg2 s2) {
  constexpr bool decoder = DEC;
  constexpr int G4 = 4 * H;
  constexpr int MT = G4 / 16;     // gate-row tiles
  constexpr int MU = H / 16;      // unit tiles (i/f/g/o blocks are MU tiles apart)
  constexpr int KSH = H / 4;      // k-steps over h_{t-1}
  constexpr int NU = H / 4;       // units per lane
  const bool two = s2.B > 0 && (int)blockIdx.x >= s2.nblk1;   // uniform: the second segment's workgroup
  const SggDecInit di = pick_di(di1, s2.di, two);
  const int B = two ? s2.B : B1;
  float* __restrict__ rel_out = two ? s2.rel_out : rel_out1;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, c16 = lane & 15;
  const int ped = (((int)blockIdx.x - (two ? s2.nblk1 : 0)) * 4 + (threadIdx.x >> 6)) * 16 + c16;
  const bool valid = ped < B;
  // the second segment's discriminator input: head steps (both halves), the
  // real half's steps and the start positions of this lane's column copied
  // in the prologue; the generated steps stored as they are formed
  const SggTrajOut& to = s2.to;
  const int tcol = ped - to.col0;
  const bool tlive = two && valid && to.out != nullptr && tcol >= 0 && tcol < to.ncol;
  // (entries e = T0 head steps, T b steps, the start: the ped's four q lanes
  // take every fourth, all loads of a chunk in flight before its stores -- a
  // load-store loop per entry was a memory round trip each, ~20 in a row
  // before these workgroups' first step)
  if (tlive) {
    float2* o2 = reinterpret_cast<float2*>(to.out);
    const int dup = to.b ? 2 : 1;   // (SggTrajOut: b != NULL <-> NB = 2 ncol)
    const int nh = to.T0, nb = to.b ? T : 0, n = nh + nb + (to.start ? 1 : 0);
    constexpr int kJ = 8;
    for (int base = 0; base < n; base += 4 * kJ) {
      float2 v[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const int e = base + 4 * j + q;
        const float2* src = e < nh ? reinterpret_cast<const float2*>(to.head + (size_t)e * to.ldh)
                            : e < nh + nb ? reinterpret_cast<const float2*>(to.b + (size_t)(e - nh) * to.ldb)
                            : e < n       ? reinterpret_cast<const float2*>(to.pos0)
                                          : reinterpret_cast<const float2*>(to.head);
        v[j] = src[tcol];
      }
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const int e = base + 4 * j + q;
        float2* dst = e < nh ? o2 + (size_t)e * to.NB + tcol
                      : e < nh + nb ? o2 + (size_t)(to.T0 + e - nh) * to.NB + to.ncol + tcol
                                    : reinterpret_cast<float2*>(to.start) + tcol;
        if (e < n) dst[0] = v[j];
        if (e < n && dup == 2 && (e < nh || e >= nh + nb)) dst[to.ncol] = v[j];   // (the head / start copy of the b half)
      }
    }
  }

  RMARK(15);   // (probe: workgroup start)
  // the weights through LDS, once per workgroup: coalesced 16-byte loads
  // (read per lane they were ~50 row gathers of 16 cache lines each per wave,
  // with every workgroup of the launch in its prologue at once -- the first
  // step of a late workgroup took ~9 us, tools/lstm_roll_probe.hip)
  constexpr int WP = H + 4;   // row pitch: the lanes' 16-byte reads of 16 rows spread over the banks
  __shared__ __attribute__((aligned(16))) float sW[G4 * WP];
  __shared__ __attribute__((aligned(16))) float sA[2 * G4];
  __shared__ __attribute__((aligned(16))) float sBias[G4];
  __shared__ float sWp[2 * H];
  {
    const bool al = ((reinterpret_cast<uintptr_t>(Whh) | reinterpret_cast<uintptr_t>(A) |
                      reinterpret_cast<uintptr_t>(bias)) & 15) == 0;
    if (al) {
      for (int e = threadIdx.x; e < G4 * H / 4; e += 256) {
        const int r = e / (H / 4), c4 = e - r * (H / 4);
        *reinterpret_cast<float4*>(&sW[r * WP + 4 * c4]) = reinterpret_cast<const float4*>(Whh)[e];
      }
      for (int e = threadIdx.x; e < G4 / 2; e += 256) reinterpret_cast<float4*>(sA)[e] = reinterpret_cast<const float4*>(A)[e];
      for (int e = threadIdx.x; e < G4 / 4; e += 256)
        reinterpret_cast<float4*>(sBias)[e] = reinterpret_cast<const float4*>(bias)[e];
    } else {
      for (int e = threadIdx.x; e < G4 * H; e += 256) sW[(e / H) * WP + e % H] = Whh[e];
      for (int e = threadIdx.x; e < 2 * G4; e += 256) sA[e] = A[e];
      for (int e = threadIdx.x; e < G4; e += 256) sBias[e] = bias[e];
    }
    if (decoder)
      for (int e = threadIdx.x; e < 2 * H; e += 256) sWp[e] = Wp[e];
  }
  __syncthreads();

  // the lane's k-step units (k = 4 mu + r  <->  unit 16 mu + 4q + r, the
  // permuted k order) and the decoder's Wp columns of them
  float wp0[NU], wp1[NU];
#pragma unroll
  for (int k = 0; k < NU; ++k) {
    const int u = 16 * (k >> 2) + 4 * q + (k & 3);
    wp0[k] = decoder ? sWp[u] : 0.f;
    wp1[k] = decoder ? sWp[H + u] : 0.f;
  }
  const float bp0 = decoder ? bp[0] : 0.f, bp1 = decoder ? bp[1] : 0.f;
  // W' (or W_hh) in registers, columns in the permuted k order; the input
  // column [A_x A_y 0 0] by q; the accumulator start b' (or b) in the D layout
  // (rows 16 mt + 4q + r); all pre-scaled for v_exp_f32
  static_assert(!X3 || KSH == 8, "the split-bf16 form takes H = 32 (one K = 32 MFMA per tile)");
  constexpr int KW = X3 ? 1 : KSH + 1;
  float w[MT][KW];
  bf16x8 wb[X3 ? MT : 1][3];   // X3: the A operand (lane: row c16, k = 8q + j <-> k-step j) as hi, mid, lo
  floatx4 b0[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row = 16 * mt + c16;
    // gate of tile mt: i, f, g, o blocks of MU tiles; g (tanh) takes -2 log2(e)
    const float sc = (mt / MU == 2 ? 2.f : 1.f) * kNegLog2e;
    const float ax = sA[2 * row], ay = sA[2 * row + 1];
    float wk[KSH];
#pragma unroll
    for (int ks = 0; ks < KSH; ++ks) {
      const float wv = sW[row * WP + 16 * (ks >> 2) + 4 * q + (ks & 3)];
      wk[ks] = sc * (decoder ? fmaf(ay, wp1[ks], fmaf(ax, wp0[ks], wv)) : wv);
    }
    if constexpr (X3) {
      split8(wk, wb[mt]);
    } else {
#pragma unroll
      for (int ks = 0; ks < KSH; ++ks) w[mt][ks] = wk[ks];
    }
    w[mt][KW - 1] = q == 0 ? sc * ax : q == 1 ? sc * ay : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // (A loaded unconditionally: under the runtime `decoder` branch each
      // entry's load was followed by its own vmcnt(0) -- 4 MT round trips)
      const int brow = 16 * mt + 4 * q + r;
      const float bv = sBias[brow];
      const float bd = fmaf(sA[2 * brow + 1], bp1, fmaf(sA[2 * brow], bp0, bv));
      b0[mt][r] = sc * (decoder ? bd : bv);
    }
  }

  // state of the lane's NU units, as unit pairs (k, k + 1)
  float2v h[NU / 2], c[NU / 2];
#pragma unroll
  for (int mu = 0; mu < MU; ++mu) {
    const size_t o = (size_t)ped * H + 16 * mu + 4 * q;
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f), cv = hv;
    if (valid && di.ctx) {   // add_noise in the prologue (sgg_lstm_fwd_dec)
      const int u = 16 * mu + 4 * q;
      hv = make_float4(dec_h0(di, ped, u), dec_h0(di, ped, u + 1), dec_h0(di, ped, u + 2), dec_h0(di, ped, u + 3));
    } else if (valid && h0) {
      hv = *reinterpret_cast<const float4*>(h0 + o);
    }
    if (valid && c0) cv = *reinterpret_cast<const float4*>(c0 + o);
    h[2 * mu] = float2v{hv.x, hv.y};
    h[2 * mu + 1] = float2v{hv.z, hv.w};
    c[2 * mu] = float2v{cv.x, cv.y};
    c[2 * mu + 1] = float2v{cv.z, cv.w};
  }
  // input k-step operand: r_x (q = 0), r_y (q = 1), 0 (q = 2, 3)
  auto load_in = [&](int t) -> float {
    if (q >= 2 || !valid) return 0.f;
    if (decoder && di.ctx) return dec_rel0(di, ped, q);
    return decoder ? rel[(size_t)ped * 2 + q] : rel[((size_t)t * B + ped) * 2 + q];
  };
  float xin = load_in(0);
  if (decoder) {   // step 0's input correction rel_0 - (Wp h_0 + bp)
    float px = 0.f, py = 0.f;
#pragma unroll
    for (int k = 0; k < NU; ++k) {
      const float hk = (k & 1) ? h[k >> 1].y : h[k >> 1].x;
      px = fmaf(wp0[k], hk, px);
      py = fmaf(wp1[k], hk, py);
    }
    px = rows_sum(px) + bp0;
    py = rows_sum(py) + bp1;
    xin = q == 0 ? xin - px : q == 1 ? xin - py : 0.f;
  }

  RMARK(0);
  for (int t = 0; t < T; ++t) {
    RSUB(0);
    const float xnext = (!decoder && t + 1 < T) ? load_in(t + 1) : 0.f;   // prefetch
    floatx4 acc[MT];
    if constexpr (X3) {
      // B operand: lane (q, ped) holds k = 8q + j <-> its own h of k-step j
      const float hv[8] = {h[0].x, h[0].y, h[1].x, h[1].y, h[2].x, h[2].y, h[3].x, h[3].y};
      bf16x8 hb[3];
      split8(hv, hb);
      RUSE(hb[2]);
      RSUB(1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma_x3(wb[mt], hb, b0[mt]);
      RUSE(acc[MT - 1]);
      RSUB(2);
    } else {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[mt][0], h[0].x, b0[mt], 0, 0, 0);
#pragma unroll
      for (int ks = 1; ks < KSH; ++ks) {
        const float hk = (ks & 1) ? h[ks >> 1].y : h[ks >> 1].x;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[mt][ks], hk, acc[mt], 0, 0, 0);
      }
    }
    if (!decoder || t == 0) {   // (uniform)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[mt][KW - 1], xin, acc[mt], 0, 0, 0);
    }

    // gate activations (i, f, o sigmoid; g tanh) and the cell update, two
    // units at a time
    float px = 0.f, py = 0.f;
#pragma unroll
    for (int mu = 0; mu < MU; ++mu) {
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const int k2 = 2 * mu + (r >> 1);
        cell2(float2v{acc[mu][r], acc[mu][r + 1]}, float2v{acc[MU + mu][r], acc[MU + mu][r + 1]},
              float2v{acc[2 * MU + mu][r], acc[2 * MU + mu][r + 1]}, float2v{acc[3 * MU + mu][r], acc[3 * MU + mu][r + 1]},
              c[k2], h[k2]);
        px = fmaf(wp0[2 * k2], h[k2].x, fmaf(wp0[2 * k2 + 1], h[k2].y, px));
        py = fmaf(wp1[2 * k2], h[k2].x, fmaf(wp1[2 * k2 + 1], h[k2].y, py));
      }
      if (valid && t == T - 1 && h_all) {   // (no-grad rollout: h_all NULL, final state unwanted)
        const size_t o = ((size_t)T * B + ped) * H + 16 * mu + 4 * q;
        *reinterpret_cast<float4*>(h_all + o) = make_float4(h[2 * mu].x, h[2 * mu].y, h[2 * mu + 1].x, h[2 * mu + 1].y);
        *reinterpret_cast<float4*>(c_all + o) = make_float4(c[2 * mu].x, c[2 * mu].y, c[2 * mu + 1].x, c[2 * mu + 1].y);
      }
    }
    RUSE(h[NU / 2 - 1]);
    RSUB(3);
    if (decoder) {   // rel_t = Wp h_t + bp: sum the 4 q-lanes of the ped
      px = rows_sum(px) + bp0;
      py = rows_sum(py) + bp1;
      if (valid && q == 0) *reinterpret_cast<float2*>(rel_out + ((size_t)t * B + ped) * 2) = make_float2(px, py);
      if (tlive && q == 0)
        reinterpret_cast<float2*>(to.out)[(size_t)(to.T0 + t) * to.NB + tcol] = make_float2(px, py);
    } else {
      xin = xnext;
    }
    RSUB(4);
    RMARK(t + 1);
  }
}

template <int H>
int launch(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0, const float* c0,
           const float* Wp, const float* bp, int T, int B, int decoder, float* h_all, float* c_all, float* act_all,
           float* rel_out, hipStream_t st, const SggDecInit* di, const RollSeg2* seg2 = nullptr) {
  if (act_all) {   // (the dispatch never sends saved-state forwards here)
    sgg::set_error("sgg_lstm_fwd: the batch-MFMA rollout keeps no saved states");
    return SGG_E_ARG;
  }
  // the split-bf16 gate GEMM for H = 32 (SGG_LSTM_X3=0: the fp32 MFMA form)
  const char* x3e = getenv("SGG_LSTM_X3");
  const bool x3 = H == 32 && !(x3e && strcmp(x3e, "0") == 0);
  constexpr bool kX3 = H == 32;
  const int grid = (B + 63) / 64;
  SggDecInit d = {};
  if (di) d = *di;
  RollSeg2 s2 = {};
  if (seg2) s2 = *seg2;
  s2.nblk1 = grid;
  const int grid2 = s2.B > 0 ? (s2.B + 63) / 64 : 0;
  auto kfn = decoder ? (x3 ? lstm_fwd_mfma_kernel<H, kX3, true> : lstm_fwd_mfma_kernel<H, false, true>)
                     : (x3 ? lstm_fwd_mfma_kernel<H, kX3, false> : lstm_fwd_mfma_kernel<H, false, false>);
  hipLaunchKernelGGL(kfn, dim3(grid + grid2), dim3(256), 0, st, rel, A, Whh, bias, h0, c0, Wp, bp, T, B, h_all, c_all,
                     rel_out, d, s2);
  SGG_RETURN_LAUNCH("sgg_lstm_fwd");
}

}  // namespace

// measured crossover vs the VALU kernel (tools/bench_kernels.py lstm)
// (H = 48 at B <= 2560 -- the discriminator -- is slower than the VALU kernel:
// 156 MFMAs per step at one wave per SIMD (233 VGPRs))
bool lstm_fwd_mfma_ok(int H, int B) { return H == 32 && B >= kLstmMfmaMinPeds; }

int lstm_fwd_mfma(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0,
                  const float* c0, const float* Wp, const float* bp, int T, int B, int H, int decoder, float* h_all,
                  float* c_all, float* act_all, float* rel_out, hipStream_t st, const SggDecInit* di) {
  if (H == 32)
    return launch<32>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st, di);
  return launch<48>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st, di);
}

int lstm_fwd_mfma_dec2(const SggDecInit* di, const SggDecInit* di2, const float* A, const float* Whh,
                       const float* bias, const float* Wp, const float* bp, int T, int B, int B2, int H,
                       float* rel_out, float* rel_out2, const SggTrajOut* to2, hipStream_t st) {
  RollSeg2 s2 = {};
  s2.di = *di2;
  s2.rel_out = rel_out2;
  if (to2) s2.to = *to2;
  s2.B = B2;
  if (H == 32)
    return launch<32>(nullptr, A, Whh, bias, nullptr, nullptr, Wp, bp, T, B, 1, nullptr, nullptr, nullptr, rel_out, st,
                      di, &s2);
  return launch<48>(nullptr, A, Whh, bias, nullptr, nullptr, Wp, bp, T, B, 1, nullptr, nullptr, nullptr, rel_out, st,
                    di, &s2);
}

}  // namespace sgg
