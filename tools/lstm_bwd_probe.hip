// Phase timing of the four-wave LSTM backward with weight gradients
// (workgroup 0's owner wave 0, wall clock 100 MHz) at the discriminator's
// D-step shape (H 48, B peds, T steps, encoder).  Diagnostic only: builds its
// own copy of the kernels with SGG_LSTM_PROF.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSGG_LSTM_PROF \
//     -I group-gan-gcn-gat_amd/csrc -I include tools/lstm_bwd_probe.hip -o tools/bin/lstm_bwd_probe
#include "../group-gan-gcn-gat_amd/csrc/lstm_mw.hip"
#include "../group-gan-gcn-gat_amd/csrc/runtime.hip"
#ifndef SGG_LSTM_PROF
namespace sgg { __device__ long long g_lstm_prof[256]; }
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
  const int H = 48;
  srand(1);
  float *rel = upload((size_t)T * B * 2, 0.3f), *A = upload(4 * H * 2, 0.2f), *Whh = upload(4 * H * H, 0.2f);
  float* bias = upload(4 * H, 0.2f);
  float *h_all, *c_all, *act, *dh0, *drel, *wpart;
  CK(hipMalloc(&h_all, (size_t)(T + 1) * B * H * 4));
  CK(hipMalloc(&c_all, (size_t)sgg::lstm_mw_state_floats(T, B, H, 1) * 4));
  CK(hipMalloc(&act, (size_t)sgg::lstm_mw_state_floats(T, B, H, 0) * 4));
  float* dh_last = upload((size_t)B * H, 1.f);
  CK(hipMalloc(&dh0, (size_t)B * H * 4));
  CK(hipMalloc(&drel, (size_t)T * B * 2 * 4));
  const size_t P = 4 * H * H + 4 * H + 8 * H + 64;
  CK(hipMalloc(&wpart, (size_t)sgg::lstm_mw_wpart_rows(H, B) * P * 4));
  int rc = sgg::lstm_mw_fwd(rel, A, Whh, bias, nullptr, nullptr, nullptr, nullptr, T, B, H, 0, h_all, c_all, act,
                            nullptr, 0);
  if (rc) { printf("fwd rc %d\n", rc); return 1; }
  CK(hipDeviceSynchronize());
  long long z[64] = {};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(sgg::g_lstm_prof), z, sizeof z));
  auto go = [&]() {
    const int r = sgg::lstm_mw_bwd(A, Whh, nullptr, h_all, c_all, act, rel, nullptr, dh_last, nullptr, T, B, H, 0,
                                   dh0, drel, nullptr, wpart, 0);
    if (r) { printf("bwd rc %d\n", r); exit(1); }
  };
  for (int i = 0; i < 5; ++i) go();
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < 50; ++i) go();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  long long pr[256];
  CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(sgg::g_lstm_prof), sizeof pr));
  printf("bwd B=%d T=%d: %.2f us/launch; workgroup 0 owner wave 0 (us from entry):\n", B, T, ms * 1e3 / 50);
  printf("  prologue %.2f\n", (pr[1] - pr[0]) * 0.01);
  for (int s = 0; s < T && s < 60; ++s) printf("  step %2d %.2f (+%.2f)\n", T - 1 - s, (pr[s + 2] - pr[0]) * 0.01,
                                               (pr[s + 2] - (s ? pr[s + 1] : pr[1])) * 0.01);
  printf("  end %.2f (+%.2f)\n", (pr[62] - pr[0]) * 0.01, (pr[62] - pr[T + 1]) * 0.01);
  printf("  step %d sub-phases (us after its start mark; owners: start, dh read, MFMAs done, part written, barrier; "
         "helpers: barrier, dW MFMAs, sums, staged):\n", T - 5);
  const long long b0 = pr[2 + 4];
  for (int w = 0; w < 8; ++w) {
    printf("   wave %d", w);
    for (int k = 0; k < (w < 4 ? 5 : 4); ++k) printf(" %6.3f", (pr[96 + 8 * w + k] - b0) * 0.01);
    printf("\n");
  }
  return 0;
}
