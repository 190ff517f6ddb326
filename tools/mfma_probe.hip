// Lane-layout probe for v_mfma_f32_4x4x1_16b_f32 on gfx950 (one wave, k = 1):
// run 1: A lane l = l + 1, B = 1 -> D names the A lane feeding each
// (register, lane); run 2: A = 1, B lane l = l + 1 -> the B lane.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out, int which) {
  const int l = threadIdx.x;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const float a = which == 0 ? (float)(l + 1) : 1.f;
  const float b = which == 0 ? 1.f : (float)(l + 1);
  acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[r * 64 + l] = acc[r];
}

int main() {
  float* d;
  hipMalloc(&d, 256 * sizeof(float));
  float ha[256], hb[256];
  probe<<<1, 64>>>(d, 0);
  hipMemcpy(ha, d, sizeof(ha), hipMemcpyDeviceToHost);
  probe<<<1, 64>>>(d, 1);
  hipMemcpy(hb, d, sizeof(hb), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int r = 0; r < 4; ++r) printf("  r%d=A%02d*B%02d", r, (int)ha[r * 64 + l] - 1, (int)hb[r * 64 + l] - 1);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
