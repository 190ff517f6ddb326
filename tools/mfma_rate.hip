// Issue rate of the f32-input MFMA forms on one SIMD (one wave, 4 independent
// accumulators, s_memtime-free: wall clock over many launches of 1 block).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int KIND>
__global__ void loop(float* out, int iters) {
  const float a = threadIdx.x * 1e-3f, b = 1.0f;
  floatx4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0, e0 = c0, e1 = c0, e2 = c0, e3 = c0;
  floatx16 d0 = {}, d1 = {};
  int x0 = threadIdx.x, x1 = threadIdx.x + 1;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    if (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    } else if (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
    } else if (KIND == 4 || KIND == 5) {
#pragma unroll
      for (int r = 0; r < (KIND == 4 ? 2 : 4); ++r) {
        c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
        e0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, e0, 0, 0, 0);
        e1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, e1, 0, 0, 0);
        e2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, e2, 0, 0, 0);
        e3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, e3, 0, 0, 0);
      }
    } else if (KIND == 7 || KIND == 8) {
      // 8 independent 4x4x1 chains, each MFMA followed by NV independent VALU ops
#define MV(acc) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc, 0, 0, 0); \
      if (KIND == 8) { asm volatile("v_max_i32 %0, 0, %0" : "+v"(x0)); asm volatile("v_max_i32 %0, 0, %0" : "+v"(x1)); } \
      else { asm volatile("v_max_i32 %0, 0, %0" : "+v"(x0)); }
      MV(c0) MV(c1) MV(c2) MV(c3) MV(e0) MV(e1) MV(e2) MV(e3)
#undef MV
    } else if (KIND == 6) {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
    } else if (KIND == 2) {
      d0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, d1, 0, 0, 0);
    } else {
      d0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d1, 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = c0[0] + c1[1] + c2[2] + c3[3] + d0[0] + d1[5] + e0[0] + e1[1] + e2[2] + e3[3] + (float)(x0 + x1);
  if (threadIdx.x == 0) {
    out[0] = (float)(t1 - t0);
    out[1] = s;
  }
}

template <int KIND>
static void run(const char* name, int per_iter, int flop_per_instr, int waves = 1) {
  float* d;
  hipMalloc(&d, 8);
  const int iters = 4096;
  loop<KIND><<<1, 64 * waves>>>(d, 16);
  loop<KIND><<<1, 64 * waves>>>(d, iters);
  float h[2];
  hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  const double cyc = h[0] / (double)(iters * per_iter);
  printf("%-22s %6.2f clock64 ticks / instr  (%d FLOP/instr)\n", name, cyc, flop_per_instr);
  hipFree(d);
}

int main() {
  run<0>("mfma_f32_16x16x4f32", 4, 16 * 16 * 4 * 2);
  run<1>("mfma_f32_4x4x1f32", 4, 16 * 4 * 4 * 2);
  run<4>("4x4x1 x8 indep", 16, 16 * 4 * 4 * 2);
  run<5>("4x4x1 x8 indep (32/it)", 32, 16 * 4 * 4 * 2);
  run<6>("4x4x1 dependent chain", 4, 16 * 4 * 4 * 2);
  run<7>("4x4x1 x8 + 1 VALU each", 8, 16 * 4 * 4 * 2);
  run<8>("4x4x1 x8 + 2 VALU each", 8, 16 * 4 * 4 * 2);
  run<4>("4x4x1 x8, 8 waves/blk", 16, 16 * 4 * 4 * 2, 8);
  run<7>("4x4x1+1VALU, 8 waves", 8, 16 * 4 * 4 * 2, 8);
  run<0>("16x16x4, 8 waves/blk", 4, 16 * 16 * 4 * 2, 8);
  run<2>("mfma_f32_16x16x1f32", 2, 4 * 16 * 16 * 2);
  run<3>("mfma_f32_32x32x2f32", 2, 32 * 32 * 2 * 2);
  return 0;
}
