// Fused LSTM sequences, unit-per-thread form (Encoder, reference
// sgan/models.py:62-92; Decoder rollout :142-178).  Same contract as
// sgg_lstm_fwd / sgg_lstm_bwd (include/sgg.h), dispatched by lstm.hip.
//
// Thread (ped, unit u) owns all four gate rows of its unit (i, f, g, o rows
// u, H+u, 2H+u, 3H+u of W_hh in registers), so the cell update is
// thread-local and a step needs ONE workgroup barrier: h_t goes to a
// double-buffered LDS row that every unit of the ped reads (float4
// broadcasts) for the next step.  The decoder's feedback r_t = Wp h_t + bp
// into step t+1 is folded into the recurrence once, before step 1:
//   W_hh h_t + A (Wp h_t + bp) + b'  =  (W_hh + A Wp) h_t + (A bp + b')
// (exact up to fp32 reassociation), so the rollout's critical path is the
// same as the encoder's; r_t itself is still written out (a lane-shuffle
// sum over the ped's units, off the critical path).
//
// Backward: thread (ped, u) owns column u of W_hh (4H registers):
// dh_{t-1}[u] = sum_r W_hh[r][u] dG_t[r] reads the ped's dG_t row from a
// double-buffered LDS row -- again one barrier per step.  The saved
// activations of step t-1 are loaded while step t computes.
#include "sgg_common.h"

namespace sgg {

namespace {

constexpr int kUnitMaxT = 32;   // encoder inputs of up to this many steps are staged in LDS

__device__ __forceinline__ float sigm_u(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
// (exp(-2x) as v_exp_f32(x * -2 log2(e)): -2 log2(e) is exact, so the same bits as
// __expf(-2x)'s (-2x) * log2(e) with one multiply less)
__device__ __forceinline__ float tanh_u(float x) {
  return fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -2.8853900817779268f)), -1.f);
}

// sum over the H consecutive lanes of a ped (H divides 64)
template <int H>
__device__ __forceinline__ float ped_sum(float v) {
#pragma unroll
  for (int o = H / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int H>
struct UnitCfg {
  static constexpr int TPP = 2 * H;                              // threads per ped
  static constexpr int PPW = (256 / TPP) > 0 ? 256 / TPP : 1;    // peds per workgroup
  static constexpr int NT = PPW * TPP;
  // waves per SIMD the register allocation must allow: 2560 peds x 2H
  // threads (the discriminator's batch) in one round of the chip
  static constexpr int WPE = H <= 16 ? 4 : (H <= 32 ? 4 : (H <= 48 ? 3 : 2));
};

// Thread (ped, u, half), index 2u + half within the ped: half 0 owns gate
// rows i, f of unit u, half 1 rows g, o (2H weights each); the partner
// holding the other two gates is lane ^ 1, so the cell update is a single
// pair of shuffles, done redundantly by both threads.
template <int H>
__global__ void __launch_bounds__(UnitCfg<H>::NT) __attribute__((amdgpu_waves_per_eu(UnitCfg<H>::WPE)))
lstm_unit_fwd_kernel(
    const float* __restrict__ rel, const float* __restrict__ A, const float* __restrict__ Whh,
    const float* __restrict__ bias, const float* __restrict__ h0, const float* __restrict__ c0,
    const float* __restrict__ Wp, const float* __restrict__ bp, int T, int B, int decoder,
    float* __restrict__ h_all, float* __restrict__ c_all, float* __restrict__ act_all, float* __restrict__ rel_out) {
  constexpr int PPW = UnitCfg<H>::PPW, TPP = UnitCfg<H>::TPP;
  constexpr int G4 = 4 * H;
  const bool save = act_all != nullptr;
  __shared__ __attribute__((aligned(16))) float hbuf[2][PPW][H];
  __shared__ float relseq[PPW][kUnitMaxT][2];
  // W_hh (4H x H) is read coalesced into LDS, then each thread takes its
  // two rows (in the row-major matrix the lanes' rows are H floats apart)
  __shared__ __attribute__((aligned(16))) float wst[4 * H * H];
  const int pl = threadIdx.x / TPP, q = threadIdx.x - pl * TPP;
  const int u = q >> 1, half = q & 1;
  const int ped = blockIdx.x * PPW + pl;
  const bool valid = ped < B;
  for (int e = threadIdx.x; e < H * H; e += UnitCfg<H>::NT)
    *reinterpret_cast<float4*>(wst + 4 * e) = *reinterpret_cast<const float4*>(Whh + 4 * e);
  __syncthreads();
  float w[2][H], ak0[2], ak1[2], bk[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = (2 * half + k) * H + u;
#pragma unroll
    for (int j = 0; j < H; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(wst + row * H + j);
      w[k][j] = v.x;
      w[k][j + 1] = v.y;
      w[k][j + 2] = v.z;
      w[k][j + 3] = v.w;
    }
    ak0[k] = A[2 * row];
    ak1[k] = A[2 * row + 1];
    bk[k] = bias[row];
  }
  const float wp0 = (decoder && !half) ? Wp[u] : 0.f, wp1 = (decoder && !half) ? Wp[H + u] : 0.f;
  const float bp0 = decoder ? bp[0] : 0.f, bp1 = decoder ? bp[1] : 0.f;
  float c = (valid && c0) ? c0[(size_t)ped * H + u] : 0.f;
  float h = (valid && h0) ? h0[(size_t)ped * H + u] : 0.f;
  if (!half) hbuf[0][pl][u] = h;
  if (valid && save && !half) {
    h_all[(size_t)ped * H + u] = h;
    c_all[(size_t)ped * H + u] = c;
  }
  float x0 = 0.f, x1 = 0.f;
  if (decoder && valid) {
    x0 = rel[(size_t)ped * 2];
    x1 = rel[(size_t)ped * 2 + 1];
  }
  const bool staged = !decoder && T <= kUnitMaxT;
  if (staged)
    for (int e = q; e < 2 * T; e += TPP) relseq[pl][e >> 1][e & 1] = valid ? rel[((size_t)(e >> 1) * B + ped) * 2 + (e & 1)] : 0.f;
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    if (!decoder) {
      if (staged) {
        x0 = relseq[pl][t][0];
        x1 = relseq[pl][t][1];
      } else {
        x0 = valid ? rel[((size_t)t * B + ped) * 2] : 0.f;
        x1 = valid ? rel[((size_t)t * B + ped) * 2 + 1] : 0.f;
      }
    } else if (t == 1) {
      // fold the hidden2pos feedback into the recurrence (see header)
#pragma unroll
      for (int j = 0; j < H; ++j) {
        const float p0 = Wp[j], p1 = Wp[H + j];
#pragma unroll
        for (int k = 0; k < 2; ++k) w[k][j] = fmaf(ak1[k], p1, fmaf(ak0[k], p0, w[k][j]));
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) bk[k] = fmaf(ak1[k], bp1, fmaf(ak0[k], bp0, bk[k]));
      x0 = x1 = 0.f;
    }
    float ga[2], gb[2], gc[2], gd[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      ga[k] = fmaf(ak1[k], x1, fmaf(ak0[k], x0, bk[k]));
      gb[k] = gc[k] = gd[k] = 0.f;
    }
    const float* hp = hbuf[t & 1][pl];
#pragma unroll
    for (int j = 0; j < H; j += 4) {
      const float4 hv = *reinterpret_cast<const float4*>(hp + j);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        ga[k] = fmaf(w[k][j], hv.x, ga[k]);
        gb[k] = fmaf(w[k][j + 1], hv.y, gb[k]);
        gc[k] = fmaf(w[k][j + 2], hv.z, gc[k]);
        gd[k] = fmaf(w[k][j + 3], hv.w, gd[k]);
      }
    }
    const float z0 = (ga[0] + gb[0]) + (gc[0] + gd[0]);
    const float z1 = (ga[1] + gb[1]) + (gc[1] + gd[1]);
    const float act0 = half ? tanh_u(z0) : sigm_u(z0);   // i | g
    const float act1 = sigm_u(z1);                        // f | o
    const float oth0 = __shfl_xor(act0, 1), oth1 = __shfl_xor(act1, 1);
    const float ig = half ? oth0 : act0, fg = half ? oth1 : act1;
    const float gg = half ? act0 : oth0, og = half ? act1 : oth1;
    c = fmaf(fg, c, ig * gg);
    h = og * tanh_u(c);
    if (valid && save) {
      float* ab = act_all + ((size_t)t * B + ped) * G4 + 2 * half * H + u;
      ab[0] = act0;
      ab[H] = act1;
    }
    if (!half) {
      if (valid && (save || t == T - 1)) {
        const size_t o = ((size_t)(save ? t + 1 : T) * B + ped) * H + u;
        h_all[o] = h;
        c_all[o] = c;
      }
      hbuf[(t + 1) & 1][pl][u] = h;
    }
    if (decoder) {   // r_t = Wp h_t + bp, written out (the recurrence uses the fold)
      const float r0 = ped_sum<TPP>(wp0 * h), r1 = ped_sum<TPP>(wp1 * h);
      if (q == 0 && valid) *reinterpret_cast<float2*>(rel_out + ((size_t)t * B + ped) * 2) = make_float2(r0 + bp0, r1 + bp1);
    }
    lds_barrier();
  }
}

template <int H>
__global__ void __launch_bounds__(UnitCfg<H>::NT) __attribute__((amdgpu_waves_per_eu(UnitCfg<H>::WPE)))
lstm_unit_bwd_kernel(
    const float* __restrict__ A, const float* __restrict__ Whh, const float* __restrict__ Wp,
    const float* __restrict__ c_all, const float* __restrict__ act_all, const float* __restrict__ dh_last,
    const float* __restrict__ dout, int T, int B, int decoder, float* __restrict__ dG, float* __restrict__ dh0,
    float* __restrict__ drel_in, float* __restrict__ drel_tot) {
  constexpr int PPW = UnitCfg<H>::PPW, TPP = UnitCfg<H>::TPP;
  constexpr int G4 = 4 * H;
  __shared__ __attribute__((aligned(16))) float dgb[2][PPW][G4];
  const int pl = threadIdx.x / TPP, q = threadIdx.x - pl * TPP;
  const int u = q >> 1, half = q & 1;
  const int ped = blockIdx.x * PPW + pl;
  const bool valid = ped < B;

  // column u of gate blocks 2 half, 2 half + 1 of W_hh (coalesced over u)
  float wcol[2 * H];
#pragma unroll
  for (int r = 0; r < 2 * H; ++r) wcol[r] = Whh[(2 * half * H + r) * H + u];
  float a0[2], a1[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    a0[k] = A[2 * ((2 * half + k) * H + u)];
    a1[k] = A[2 * ((2 * half + k) * H + u) + 1];
  }
  const float wp0 = decoder ? Wp[u] : 0.f, wp1 = decoder ? Wp[H + u] : 0.f;
  float dh = (!decoder && valid && dh_last) ? dh_last[(size_t)ped * H + u] : 0.f;
  float dc = 0.f, fb0 = 0.f, fb1 = 0.f;

  // saved activations of step t (all four gates of unit u), loaded one step ahead
  float n_i = 0.f, n_f = 0.f, n_g = 0.f, n_o = 0.f, n_c = 0.f, n_cp = 0.f;
  auto load_step = [&](int t) {
    if (valid) {
      const float* ab = act_all + ((size_t)t * B + ped) * G4 + u;
      n_i = ab[0];
      n_f = ab[H];
      n_g = ab[2 * H];
      n_o = ab[3 * H];
      n_c = c_all[((size_t)(t + 1) * B + ped) * H + u];
      n_cp = c_all[((size_t)t * B + ped) * H + u];
    }
  };
  load_step(T - 1);
  for (int t = T - 1; t >= 0; --t) {
    if (decoder) {   // r_t feeds the output and step t+1's input
      float d0 = fb0, d1 = fb1;
      if (valid) {
        const float2 dv = *reinterpret_cast<const float2*>(dout + ((size_t)t * B + ped) * 2);
        d0 += dv.x;
        d1 += dv.y;
      }
      if (q == 0 && valid) *reinterpret_cast<float2*>(drel_tot + ((size_t)t * B + ped) * 2) = make_float2(d0, d1);
      dh = fmaf(wp0, d0, fmaf(wp1, d1, dh));
    }
    const float ig = n_i, fg = n_f, gg = n_g, og = n_o, ct = n_c, cp = n_cp;
    if (t > 0) load_step(t - 1);
    const float tc = tanh_u(ct);
    const float d_o = dh * tc;
    const float dct = fmaf(dh * og, 1.f - tc * tc, dc);
    dc = dct * fg;
    float v[2];
    if (!half) {
      v[0] = dct * gg * ig * (1.f - ig);
      v[1] = dct * cp * fg * (1.f - fg);
    } else {
      v[0] = dct * ig * (1.f - gg * gg);
      v[1] = d_o * og * (1.f - og);
    }
    float* dgrow = dgb[t & 1][pl];
    dgrow[2 * half * H + u] = v[0];
    dgrow[(2 * half + 1) * H + u] = v[1];
    if (valid) {
      float* gr = dG + ((size_t)t * B + ped) * G4 + 2 * half * H + u;
      gr[0] = v[0];
      gr[H] = v[1];
    }
    if (decoder) {   // A^T dG_t: the input gradient of step t (feedback into r_{t-1})
      fb0 = ped_sum<TPP>(fmaf(a0[1], v[1], a0[0] * v[0]));
      fb1 = ped_sum<TPP>(fmaf(a1[1], v[1], a1[0] * v[0]));
      if (q == 0 && valid) *reinterpret_cast<float2*>(drel_in + ((size_t)t * B + ped) * 2) = make_float2(fb0, fb1);
    }
    lds_barrier();
    const float* dsrc = dgrow + 2 * half * H;
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 2 * H; r += 4) {
      const float4 d4 = *reinterpret_cast<const float4*>(dsrc + r);
      p[0] = fmaf(wcol[r], d4.x, p[0]);
      p[1] = fmaf(wcol[r + 1], d4.y, p[1]);
      p[2] = fmaf(wcol[r + 2], d4.z, p[2]);
      p[3] = fmaf(wcol[r + 3], d4.w, p[3]);
    }
    const float part = (p[0] + p[1]) + (p[2] + p[3]);
    const float other = __shfl_xor(part, 1);
    dh = half ? other + part : part + other;   // blocks (i, f) + (g, o), same order on both lanes
  }
  if (valid && dh0 && !half) dh0[(size_t)ped * H + u] = dh;
  if (!decoder) {
    // drel_t = A^T dG_t for every step, from the dG rows this workgroup wrote
    __syncthreads();
    for (int e = q; e < 2 * T; e += TPP) {
      const int t = e >> 1, cc = e & 1;
      if (!valid) continue;
      const float* gr = dG + ((size_t)t * B + ped) * G4;
      float s0 = 0.f, s1 = 0.f;
      for (int r = 0; r < G4; r += 2) {
        s0 = fmaf(A[2 * r + cc], gr[r], s0);
        s1 = fmaf(A[2 * (r + 1) + cc], gr[r + 1], s1);
      }
      drel_in[((size_t)t * B + ped) * 2 + cc] = s0 + s1;
    }
  }
}

template <int H>
int launch_fwd(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0, const float* c0,
               const float* Wp, const float* bp, int T, int B, int decoder, float* h_all, float* c_all, float* act_all,
               float* rel_out, hipStream_t st) {
  const int grid = (B + UnitCfg<H>::PPW - 1) / UnitCfg<H>::PPW;
  hipLaunchKernelGGL(lstm_unit_fwd_kernel<H>, dim3(grid), dim3(UnitCfg<H>::NT), 0, st, rel, A, Whh, bias, h0, c0, Wp,
                     bp, T, B, decoder, h_all, c_all, act_all, rel_out);
  SGG_RETURN_LAUNCH("sgg_lstm_fwd");
}

template <int H>
int launch_bwd(const float* A, const float* Whh, const float* Wp, const float* c_all, const float* act_all,
               const float* dh_last, const float* dout, int T, int B, int decoder, float* dG, float* dh0, float* drel_in,
               float* drel_tot, hipStream_t st) {
  const int grid = (B + UnitCfg<H>::PPW - 1) / UnitCfg<H>::PPW;
  hipLaunchKernelGGL(lstm_unit_bwd_kernel<H>, dim3(grid), dim3(UnitCfg<H>::NT), 0, st, A, Whh, Wp, c_all, act_all,
                     dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot);
  SGG_RETURN_LAUNCH("sgg_lstm_bwd");
}

}  // namespace

// H in {16, 32}: the ped's 2H threads sit in one wavefront (lane-shuffle
// sums).  H = 48 (the discriminator) measured faster on the row-per-thread
// kernels of lstm.hip (this form needs 168+ VGPRs there: 3 waves per SIMD
// with spills, or 2 waves and two rounds of the chip at B = 2560).
bool lstm_unit_ok(int H, int decoder) {
  (void)decoder;
  return H == 16 || H == 32;
}

int lstm_unit_fwd(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0,
                  const float* c0, const float* Wp, const float* bp, int T, int B, int H, int decoder, float* h_all,
                  float* c_all, float* act_all, float* rel_out, hipStream_t st) {
  switch (H) {
    case 16: return launch_fwd<16>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st);
    case 32: return launch_fwd<32>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st);
    case 48: return launch_fwd<48>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st);
    default: return launch_fwd<64>(rel, A, Whh, bias, h0, c0, Wp, bp, T, B, decoder, h_all, c_all, act_all, rel_out, st);
  }
}

int lstm_unit_bwd(const float* A, const float* Whh, const float* Wp, const float* c_all, const float* act_all,
                  const float* dh_last, const float* dout, int T, int B, int H, int decoder, float* dG, float* dh0,
                  float* drel_in, float* drel_tot, hipStream_t st) {
  switch (H) {
    case 16: return launch_bwd<16>(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot, st);
    case 32: return launch_bwd<32>(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot, st);
    case 48: return launch_bwd<48>(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot, st);
    default: return launch_bwd<64>(A, Whh, Wp, c_all, act_all, dh_last, dout, T, B, decoder, dG, dh0, drel_in, drel_tot, st);
  }
}

}  // namespace sgg
