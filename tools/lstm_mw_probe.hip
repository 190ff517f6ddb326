// Phase timing of the four-wave LSTM encoder forward (workgroup 0, wall
// clock 100 MHz) at the discriminator's shape (H 48, B peds, T steps, saved
// states, U epilogue NU 512).  Diagnostic only: builds its own copy of the
// kernels with SGG_LSTM_PROF.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSGG_LSTM_PROF \
//     -I group-gan-gcn-gat_amd/csrc -I include tools/lstm_mw_probe.hip -o tools/lstm_mw_probe
#include "../group-gan-gcn-gat_amd/csrc/lstm_mw.hip"
#include "../group-gan-gcn-gat_amd/csrc/runtime.hip"
#ifndef SGG_LSTM_PROF
namespace sgg { __device__ long long g_lstm_prof[256]; }   // (the un-instrumented build: launch times only)
#endif

#include <cstdio>
#include <cstdlib>
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
  const int B = argc > 1 ? atoi(argv[1]) : 2560, T = argc > 2 ? atoi(argv[2]) : 20;
  const int withu = argc > 3 ? atoi(argv[3]) : 1, save = argc > 4 ? atoi(argv[4]) : 1;
  const int H = 48, NU = 512;
  srand(1);
  float *rel = upload((size_t)T * B * 2, 0.3f), *A = upload(4 * H * 2, 0.2f), *Whh = upload(4 * H * H, 0.2f);
  float *bias = upload(4 * H, 0.2f), *Wu = upload(NU * H, 0.2f), *cu = upload(NU, 0.2f);
  float *h_all, *c_all, *act, *U;
  CK(hipMalloc(&h_all, (size_t)(T + 1) * B * H * 4));
  CK(hipMalloc(&c_all, (size_t)sgg::lstm_mw_state_floats(T, B, H, 1) * 4));
  CK(hipMalloc(&act, (size_t)sgg::lstm_mw_state_floats(T, B, H, 0) * 4));
  CK(hipMalloc(&U, (size_t)B * NU * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto go = [&]() {
    int rc = sgg::lstm_mw_fwd(rel, A, Whh, bias, nullptr, nullptr, nullptr, nullptr, T, B, H, 0, h_all, c_all,
                              save ? act : nullptr, nullptr, 0, withu ? Wu : nullptr, H, cu, withu ? NU : 0,
                              withu ? U : nullptr);
    if (rc) { printf("launch rc %d\n", rc); exit(1); }
  };
  for (int i = 0; i < 5; ++i) go();
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < 50; ++i) go();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  long long pr[256];
  CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(sgg::g_lstm_prof), sizeof pr));
  printf("B=%d T=%d U=%d save=%d: %.2f us/launch; workgroup 0 (us from entry):\n", B, T, withu, save, ms * 1e3 / 50);
  printf("  staged %.2f\n", (pr[1] - pr[0]) * 0.01);
  for (int t = 0; t < T && t < 60; ++t) printf("  step %2d %.2f (+%.2f)\n", t, (pr[t + 2] - pr[0]) * 0.01,
                                              (pr[t + 2] - (t ? pr[t + 1] : pr[1])) * 0.01);
  printf("  end %.2f (+%.2f)\n", (pr[63] - pr[0]) * 0.01, (pr[63] - pr[T + 1]) * 0.01);
  if (T > 4) {
    printf("  step 4 sub-phases (us after step 3's mark; wave: start, B loaded, MFMAs done, activations, h written, "
           "barrier passed):\n");
    for (int w = 0; w < 4; ++w) {
      printf("   wave %d", w);
      for (int k = 0; k < 6; ++k) printf(" %6.3f", (pr[64 + 8 * w + k] - pr[5]) * 0.01);
      printf("\n");
    }
  }
  return 0;
}
