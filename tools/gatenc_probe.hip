// Phase timing of the fused GAT encoder (workgroup 0's scene, wall clock
// 100 MHz) and whole-launch time, on the bench's shape (64 scenes x 20 peds,
// 5 group labels, 1 head).  Diagnostic only: builds its own copy of the
// kernel with SGG_GATENC_PROF.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSGG_GATENC_PROF \
//     -I group-gan-gcn-gat_amd/csrc -I include tools/gatenc_probe.hip -o gatenc_probe
#include "../group-gan-gcn-gat_amd/csrc/gat_encoder.hip"
#include "../group-gan-gcn-gat_amd/csrc/runtime.hip"
#ifndef SGG_GATENC_PROF
namespace sgg { __device__ long long g_gatenc_prof[2][64]; }   // (the un-instrumented build: launch times only)
#endif

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static float* upload(const std::vector<float>& v) {
  float* d;
  CK(hipMalloc(&d, v.size() * sizeof(float)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
  return d;
}
static std::vector<float> rnd(size_t n, float sc) {
  std::vector<float> v(n);
  for (auto& x : v) x = sc * ((float)rand() / RAND_MAX * 2.f - 1.f);
  return v;
}

int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 64, n = argc > 2 ? atoi(argv[2]) : 20, nh = argc > 3 ? atoi(argv[3]) : 1;
  const int B = S * n;
  srand(1);
  SggGatEncArgs a = {};
  a.X = upload(rnd((size_t)B * 40, 1.f));
  a.ldx = 40;
  std::vector<float> lab(B);
  for (auto& x : lab) x = (float)(rand() % 6);
  a.labels = upload(lab);
  std::vector<int> off(S + 1);
  for (int s = 0; s <= S; ++s) off[s] = s * n;
  int* doff;
  CK(hipMalloc(&doff, off.size() * 4));
  CK(hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  a.scene_off = doff;
  a.S = S;
  a.np = n;
  a.nh = nh;
  a.alpha = 0.2f;
  for (int h = 0; h < nh; ++h) {
    a.w.Wi[h] = upload(rnd(40 * 72, 0.2f));
    a.w.ai[h] = upload(rnd(144, 0.2f));
    a.w.Wg[h] = upload(rnd(16 * 72, 0.2f));
    a.w.ag[h] = upload(rnd(144, 0.2f));
  }
  a.w.Wio = upload(rnd(72 * nh * 16, 0.2f));
  a.w.aio = upload(rnd(32, 0.2f));
  a.w.Wgo = upload(rnd(72 * nh * 16, 0.2f));
  a.w.ago = upload(rnd(32, 0.2f));
  a.w.Woe = upload(rnd(24 * 32, 0.2f));
  a.w.boe = upload(rnd(24, 0.2f));
  float *y, *dx, *slab, *saved;
  CK(hipMalloc(&y, (size_t)B * 24 * 4));
  CK(hipMalloc(&dx, (size_t)B * 40 * 4));
  CK(hipMalloc(&slab, (size_t)S * sgg_gatenc_param_size(nh) * 4));
  CK(hipMalloc(&saved, (size_t)sgg_gatenc_saved_floats(S, n, nh) * 4));
  a.y = y;
  a.ldy = 24;
  a.dy = upload(rnd((size_t)B * 24, 1.f));
  a.lddy = 24;
  a.dX = dx;
  a.lddx = 40;
  a.slab = slab;
  a.saved = argc > 4 && atoi(argv[4]) == 0 ? nullptr : saved;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int bwd = 0; bwd < 2; ++bwd) {
    auto run = [&]() { return bwd ? sgg_gatenc_bwd(&a, nullptr) : sgg_gatenc_fwd(&a, nullptr); };
    for (int i = 0; i < 5; ++i)
      if (run()) { printf("launch failed\n"); return 1; }
    CK(hipDeviceSynchronize());
    const int R = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) run();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long pr[2][64];
    CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(sgg::g_gatenc_prof), sizeof pr));
    printf("%s: %.2f us/launch (back-to-back, %d launches); workgroup 0 phases (us from entry):\n", bwd ? "bwd" : "fwd",
           1e3 * ms / R, R);
    const long long t0 = pr[bwd][40];
    printf("  staged %.2f  scene-start %.2f\n", (pr[bwd][41] - t0) * 0.01, (pr[bwd][0] - t0) * 0.01);
    long long prev = pr[bwd][0];
    if (!bwd && pr[0][53] > pr[0][52])
      printf("  shader clock %.2f GHz (F1..F7)\n", (double)(pr[0][51] - pr[0][50]) / ((pr[0][53] - pr[0][52]) * 10.0));
    for (int i = 1; i < 40; ++i) {
      if (pr[bwd][i] <= 0 || pr[bwd][i] < t0) continue;
      printf("  mark %2d  %7.2f  (+%.2f)\n", i, (pr[bwd][i] - t0) * 0.01, (pr[bwd][i] - prev) * 0.01);
      prev = pr[bwd][i];
    }
    if (bwd && pr[1][42] > 0) {   // per-wave arrival after the backward's preload (marks 42 .. 57)
      printf("  per-wave entry (us from wave 0 entry):");
      for (int w = 0; w < 16; ++w) printf(" %.2f", (pr[1][42 + w] - t0) * 0.01);
      printf("\n");
    }
    CK(hipMemset(pr, 0, 0));
    long long z[2][64] = {};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(sgg::g_gatenc_prof), z, sizeof z));
  }
  return 0;
}
