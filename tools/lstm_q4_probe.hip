// Probe: an LSTM encoder recurrence with FOUR peds per workgroup on
// v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4, K = 1) against the 16-ped
// four-wave form.  Block b of wave w holds unit u = 16 w + b: rows = its four
// gates, columns = the four peds, so a lane ends the k loop holding i, f, g, o
// of one (unit, ped).  H / 16 waves per workgroup.  Checks the result against
// a CPU recurrence (double) and times T-step launches for B peds.
//   hipcc -O3 --offload-arch=gfx950 tools/lstm_q4_probe.hip -o tools/bin/lstm_q4_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
constexpr float kNegLog2e = -1.4426950408889634f;
__device__ __forceinline__ float gate_act(float x, float s, float nsl) {
  return fmaf(s, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * nsl)), 1.f - s);
}
__device__ __forceinline__ float tanh_m(float x) {
  return fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * (2.f * kNegLog2e))), -1.f);
}

// NACC independent accumulators over the k loop (summed at the end)
template <int H, int NACC>
__global__ void __launch_bounds__(64 * (H / 16)) q4_fwd(const float* __restrict__ rel, const float* __restrict__ A,
                                                        const float* __restrict__ Whh,
                                                        const float* __restrict__ bias, int T, int B,
                                                        float* __restrict__ h_all) {
  constexpr int NW = H / 16;
  constexpr int HP = H + 4;   // LDS row pitch of h (ped-major)
  __shared__ float hs[2][4][HP];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = lane >> 2, j = lane & 3;   // block (unit), column (ped) / A-row (gate)
  const int u = 16 * w + b;
  const int ped = blockIdx.x * 4 + j, pc = ped < B ? ped : B - 1;
  // A operand: lane (b, i = j) supplies W_hh[gate i of unit u][k] for every k
  float wk[H];
  const int row = j * H + u;
#pragma unroll
  for (int k = 0; k < H; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(Whh + (size_t)row * H + k);
    wk[k] = v.x; wk[k + 1] = v.y; wk[k + 2] = v.z; wk[k + 3] = v.w;
  }
  const float a0 = A[2 * row], a1 = A[2 * row + 1], bb = bias[row];
  float c = 0.f;
  hs[0][j][u] = 0.f;
  if (u < 4) hs[0][j][H + u] = 0.f;
  h_all[(size_t)pc * H + u] = 0.f;
  __syncthreads();
  float2 xn = reinterpret_cast<const float2*>(rel)[pc];
  for (int t = 0; t < T; ++t) {
    const int rb = t & 1;
    const float2 x = xn;   // (loaded a step ahead)
    if (t + 1 < T) xn = reinterpret_cast<const float2*>(rel)[(size_t)(t + 1) * B + pc];
    // input k-steps: the A operand rows (a0, a1, bias) against (r_x, r_y, 1)
    floatx4 acc[NACC];
#pragma unroll
    for (int n = 0; n < NACC; ++n) acc[n] = floatx4{0.f, 0.f, 0.f, 0.f};
    acc[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(a0, x.x, acc[0], 0, 0, 0);
    acc[1 % NACC] = __builtin_amdgcn_mfma_f32_4x4x1f32(a1, x.y, acc[1 % NACC], 0, 0, 0);
    acc[2 % NACC] = __builtin_amdgcn_mfma_f32_4x4x1f32(bb, 1.f, acc[2 % NACC], 0, 0, 0);
    const float* hr = &hs[rb][j][0];
#pragma unroll
    for (int k = 0; k < H; k += 4) {
      const float4 hv = *reinterpret_cast<const float4*>(hr + k);
      acc[(k + 0) % NACC] = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[k], hv.x, acc[(k + 0) % NACC], 0, 0, 0);
      acc[(k + 1) % NACC] = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[k + 1], hv.y, acc[(k + 1) % NACC], 0, 0, 0);
      acc[(k + 2) % NACC] = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[k + 2], hv.z, acc[(k + 2) % NACC], 0, 0, 0);
      acc[(k + 3) % NACC] = __builtin_amdgcn_mfma_f32_4x4x1f32(wk[k + 3], hv.w, acc[(k + 3) % NACC], 0, 0, 0);
    }
    floatx4 g = acc[0];
#pragma unroll
    for (int n = 1; n < NACC; ++n) g += acc[n];
    float a[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = r == 2 ? 2.f : 1.f;
      a[r] = gate_act(g[r], s, s * kNegLog2e);
    }
    c = fmaf(a[1], c, a[0] * a[2]);
    const float h = a[3] * tanh_m(c);
    hs[rb ^ 1][j][u] = h;
    h_all[((size_t)(t + 1) * B + pc) * H + u] = h;
    __syncthreads();
  }
}

static double sig(double x) { return 1.0 / (1.0 + exp(-x)); }

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

template <int H, int NACC>
int run(int B, int T, bool check) {
  const int G4 = 4 * H;
  std::vector<float> W(G4 * H), A(G4 * 2), bias(G4), rel((size_t)T * B * 2);
  srand(7);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& v : W) v = 0.3f * rnd();
  for (auto& v : A) v = 0.5f * rnd();
  for (auto& v : bias) v = 0.2f * rnd();
  for (auto& v : rel) v = rnd();
  float *dW, *dA, *db, *dr, *dh;
  CK(hipMalloc(&dW, W.size() * 4));
  CK(hipMalloc(&dA, A.size() * 4));
  CK(hipMalloc(&db, bias.size() * 4));
  CK(hipMalloc(&dr, rel.size() * 4));
  CK(hipMalloc(&dh, (size_t)(T + 1) * B * H * 4));
  CK(hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, rel.data(), rel.size() * 4, hipMemcpyHostToDevice));
  const dim3 grid((B + 3) / 4), blk(64 * (H / 16));
  hipLaunchKernelGGL((q4_fwd<H, NACC>), grid, blk, 0, 0, dr, dA, dW, db, T, B, dh);
  CK(hipDeviceSynchronize());
  if (check) {
    std::vector<float> out((size_t)(T + 1) * B * H);
    CK(hipMemcpy(out.data(), dh, out.size() * 4, hipMemcpyDeviceToHost));
    double maxerr = 0;
    for (int p = 0; p < B; p += 37) {
      std::vector<double> h(H, 0.0), c(H, 0.0), g(G4);
      for (int t = 0; t < T; ++t) {
        for (int r = 0; r < G4; ++r) {
          double s = bias[r] + A[2 * r] * rel[((size_t)t * B + p) * 2] + A[2 * r + 1] * rel[((size_t)t * B + p) * 2 + 1];
          for (int k = 0; k < H; ++k) s += W[r * H + k] * h[k];
          g[r] = s;
        }
        for (int uu = 0; uu < H; ++uu) {
          const double i = sig(g[uu]), f = sig(g[H + uu]), gg = tanh(g[2 * H + uu]), o = sig(g[3 * H + uu]);
          c[uu] = f * c[uu] + i * gg;
          h[uu] = o * tanh(c[uu]);
        }
        for (int uu = 0; uu < H; ++uu) {
          const double e = fabs(h[uu] - out[((size_t)(t + 1) * B + p) * H + uu]);
          if (e > maxerr) maxerr = e;
        }
      }
    }
    printf("H=%d NACC=%d check: max |h - ref| = %.3g\n", H, NACC, maxerr);
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipGraph_t gph;
  hipGraphExec_t ge;
  const int reps = 20;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((q4_fwd<H, NACC>), grid, blk, 0, st, dr, dA, dW, db, T, B, dh);
  CK(hipStreamEndCapture(st, &gph));
  CK(hipGraphInstantiate(&ge, gph, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("H=%d NACC=%d B=%d T=%d: %.2f us per launch (%d workgroups of %d)\n", H, NACC, B, T, 1000 * ms / reps,
         grid.x, blk.x);
  hipFree(dW); hipFree(dA); hipFree(db); hipFree(dr); hipFree(dh);
  return 0;
}

int main() {
  if (run<48, 1>(1280, 12, true)) return 1;
  if (run<48, 2>(1280, 12, true)) return 1;
  if (run<48, 4>(1280, 12, true)) return 1;
  if (run<48, 2>(2560, 12, false)) return 1;
  if (run<48, 4>(2560, 12, false)) return 1;
  if (run<48, 2>(2560, 20, false)) return 1;
  if (run<32, 2>(1280, 8, true)) return 1;
  if (run<32, 2>(1280, 12, false)) return 1;
  return 0;
}
