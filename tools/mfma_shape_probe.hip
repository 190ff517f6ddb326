// Issue rate and dependent latency of the f32 MFMA shapes on gfx950: one
// wave per SIMD, a loop of steps each issuing 8 MFMAs, either on 8
// independent accumulators (rate) or all on one (latency chain).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_shape_probe.hip -o tools/bin/mfma_shape_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// SHAPE 0: 16x16x4 f32, 1: 4x4x1 (16 blocks) f32, 2: 32x32x2 f32
template <int SHAPE, bool DEP>
__global__ void __launch_bounds__(256) probe(float* out, long long* cyc, int N, float s) {
  floatx4 acc[8];
  floatx16 acc16[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    acc16[i] = floatx16{};
  }
  const float a = s * threadIdx.x, b = s + threadIdx.x;
  const long long t0 = clock64();
  for (int n = 0; n < N; ++n) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = DEP ? 0 : j;
      if (SHAPE == 0) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[k], 0, 0, 0);
      if (SHAPE == 1) acc[k] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[k], 0, 0, 0);
      if (SHAPE == 2) acc16[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc16[k], 0, 0, 0);
    }
    __asm__ volatile("" ::: "memory");
  }
  const long long t1 = clock64();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) r += acc[i][0] + acc[i][3] + acc16[i][0] + acc16[i][15];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int SHAPE, bool DEP>
void run(float* out, long long* cyc, long long* h) {
  const int N = 2000, G = 256;
  hipLaunchKernelGGL((probe<SHAPE, DEP>), dim3(G), dim3(256), 0, 0, out, cyc, N, 0.5f);
  hipLaunchKernelGGL((probe<SHAPE, DEP>), dim3(G), dim3(256), 0, 0, out, cyc, N, 0.5f);
  hipMemcpy(h, cyc, G * sizeof(long long), hipMemcpyDeviceToHost);
  double sum = 0;
  for (int i = 0; i < G; ++i) sum += h[i];
  const char* nm[3] = {"16x16x4 f32 (1024 MAC)", "4x4x1 f32 16 blocks (256 MAC)", "32x32x2 f32 (2048 MAC)"};
  printf("%-32s %-11s %7.1f cycles per MFMA\n", nm[SHAPE], DEP ? "dependent" : "independent", sum / G / N / 8);
}

int main() {
  float* out;
  long long* cyc;
  long long h[256];
  hipMalloc(&out, 256 * 256 * sizeof(float));
  hipMalloc(&cyc, 256 * sizeof(long long));
  run<0, false>(out, cyc, h);
  run<0, true>(out, cyc, h);
  run<1, false>(out, cyc, h);
  run<1, true>(out, cyc, h);
  run<2, false>(out, cyc, h);
  run<2, true>(out, cyc, h);
  return 0;
}
