// Phase timing of the batch-MFMA decoder rollout (lstm_mfma.hip) at the
// best-of-20 shape (H 32, B peds, T steps, no saved states): wall-clock marks
// per step of workgroups 0 and 300, shader-cycle marks of step 4's phases.
// Diagnostic only: builds its own copy of the kernels with SGG_ROLL_PROF.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -DSGG_ROLL_PROF \
//     -I group-gan-gcn-gat_amd/csrc -I include tools/lstm_roll_probe.hip -o tools/run/lstm_roll_probe
#include "../group-gan-gcn-gat_amd/csrc/lstm_mfma.hip"
#include "../group-gan-gcn-gat_amd/csrc/runtime.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static float* upload(size_t n, float sc) {
  std::vector<float> v(n);
  for (auto& x : v) x = sc * ((float)rand() / RAND_MAX * 2.f - 1.f);
  float* d;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemcpy(d, v.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 26880, T = argc > 2 ? atoi(argv[2]) : 12;
  const int H = 32;
  const int nostate = argc > 3 ? atoi(argv[3]) : 0;   // 1: zero initial state (no h0 / c0 loads)
  srand(1);
  float *rel = upload((size_t)B * 2, 0.3f), *A = upload(4 * H * 2, 0.2f), *Whh = upload(4 * H * H, 0.2f);
  float *bias = upload(4 * H, 0.2f), *h0 = upload((size_t)B * H, 0.5f), *c0 = upload((size_t)B * H, 0.5f);
  float *Wp = upload(2 * H, 0.2f), *bp = upload(2, 0.1f), *rel_out;
  CK(hipMalloc(&rel_out, (size_t)T * B * 2 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto go = [&]() {
    int rc = sgg::lstm_fwd_mfma(rel, A, Whh, bias, nostate ? nullptr : h0, nostate ? nullptr : c0, Wp, bp, T, B, H, 1, nullptr, nullptr, nullptr, rel_out, 0,
                                nullptr);
    if (rc) { printf("launch rc %d\n", rc); exit(1); }
  };
  for (int i = 0; i < 5; ++i) go();
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < 50; ++i) go();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  static long long pr[8192 + 512];
  CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(sgg::g_roll_prof), sizeof pr));
  const int nwg = (B + 63) / 64;
  printf("rollout B=%d T=%d nostate=%d: %.2f us/launch; per workgroup (wave 0, us from workgroup 0's start): start, "
         "loop entry, step 0, step 1, steps 2.. mean, end\n", B, T, nostate, ms * 1e3 / 50);
  const long long z = pr[15];
  for (int wg = 0; wg < nwg && wg < 512; wg += (wg < 8 ? 1 : 23)) {
    const long long* m = pr + 16 * wg;
    double rest = 0;
    for (int t = 3; t <= T && t < 15; ++t) rest += (m[t] - m[t - 1]) * 0.01;
    printf("  wg %3d  %6.2f %6.2f %6.2f %6.2f %6.2f %6.2f\n", wg, (m[15] - z) * 0.01, (m[0] - z) * 0.01,
           (m[1] - m[0]) * 0.01, (m[2] - m[1]) * 0.01, rest / (T - 2), (m[T < 15 ? T : 14] - z) * 0.01);
  }
  printf("  step 4 phases in shader cycles from its start (split done, MFMAs done, cell done, end):\n");
  for (int wg = 0; wg < 2; ++wg)
    for (int w = 0; w < 4; ++w) {
      const long long* m = pr + 8192 + (wg ? 64 : 0) + 8 * w;
      printf("   wg %3d wave %d %6lld %6lld %6lld %6lld\n", wg ? 300 : 0, w, m[1] - m[0], m[2] - m[0], m[3] - m[0],
             m[4] - m[0]);
    }
  return 0;
}
