// Does VALU work overlap v_mfma_f32_16x16x4_f32 on gfx950?  One wave per
// SIMD (256-thread workgroups, one per CU), a loop of N steps each issuing
// M independent f32 MFMAs (8 accumulators) and V independent VALU
// instructions of one kind (v_exp_f32 or v_fma_f32), all in registers; the
// wave's cycles (s_memtime) per step for each (M, V) pair, and the same with
// bf16 MFMAs (v_mfma_f32_16x16x32_bf16) for comparison.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_valu_probe.hip -o /tmp/mvp && /tmp/mvp
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int M, int V, int KIND, bool BF>
__global__ void __launch_bounds__(256) probe(float* out, long long* cyc, int N, float s) {
  floatx4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  float a = s * threadIdx.x, b = s + threadIdx.x;
  bf16x8 ab, bb;
#pragma unroll
  for (int i = 0; i < 8; ++i) { ab[i] = (__bf16)(a + i); bb[i] = (__bf16)(b - i); }
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = s * (i + 1) + threadIdx.x * 1e-3f;
  const long long t0 = clock64();
  for (int n = 0; n < N; ++n) {
#pragma unroll
    for (int j = 0; j < (M > V ? M : V); ++j) {
      if (j < M) {
        if (BF) acc[j & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, acc[j & 7], 0, 0, 0);
        else acc[j & 7] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j & 7], 0, 0, 0);
      }
      if (j < V) {
        if (KIND == 0) v[j & 15] = __builtin_amdgcn_exp2f(v[j & 15]);
        else v[j & 15] = fmaf(v[j & 15], 0.999f, 0.001f);
      }
    }
    __asm__ volatile("" ::: "memory");
  }
  const long long t1 = clock64();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) r += acc[i][0] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 16; ++i) r += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int M, int V, int KIND, bool BF>
void run(float* out, long long* cyc, long long* h, const char* what) {
  const int N = 2000, G = 256;
  hipLaunchKernelGGL((probe<M, V, KIND, BF>), dim3(G), dim3(256), 0, 0, out, cyc, N, 0.5f);
  hipLaunchKernelGGL((probe<M, V, KIND, BF>), dim3(G), dim3(256), 0, 0, out, cyc, N, 0.5f);
  hipMemcpy(h, cyc, G * sizeof(long long), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < G; ++i) s += h[i];
  printf("%-5s M=%2d V=%2d %-4s  %7.1f cycles per step\n", BF ? "bf16" : "f32", M, V, what, s / G / N);
}

int main() {
  float* out;
  long long* cyc;
  long long h[256];
  hipMalloc(&out, 256 * 256 * sizeof(float));
  hipMalloc(&cyc, 256 * sizeof(long long));
  run<8, 0, 0, false>(out, cyc, h, "-");
  run<0, 8, 0, false>(out, cyc, h, "exp");
  run<0, 8, 1, false>(out, cyc, h, "fma");
  run<0, 16, 1, false>(out, cyc, h, "fma");
  run<8, 8, 0, false>(out, cyc, h, "exp");
  run<8, 8, 1, false>(out, cyc, h, "fma");
  run<8, 16, 1, false>(out, cyc, h, "fma");
  run<8, 24, 1, false>(out, cyc, h, "fma");
  run<8, 16, 0, false>(out, cyc, h, "exp");
  run<8, 0, 0, true>(out, cyc, h, "-");
  run<8, 8, 0, true>(out, cyc, h, "exp");
  run<8, 8, 1, true>(out, cyc, h, "fma");
  run<8, 16, 1, true>(out, cyc, h, "fma");
  return 0;
}
