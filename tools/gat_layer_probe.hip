// Phase timing of the fused batched-GAT layer (sgg_gat_layer_fwd; workgroup
// 0's first (segment, head), wall clock 100 MHz) and whole-launch time, on
// configs[4]'s shapes (64 scenes x 64 peds; layer 1: K 40 -> 4 heads x 16,
// layer 2: K 64 -> 40, bf16 transform, saving).  Diagnostic only:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSGG_GAT_PROF \
//     -I group-gan-gcn-gat_amd/csrc -I include tools/gat_layer_probe.hip -o gat_layer_probe
#include "../group-gan-gcn-gat_amd/csrc/gat.hip"
#include "../group-gan-gcn-gat_amd/csrc/runtime.hip"

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
static float* zeros(size_t n) {
  float* d;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemset(d, 0, n * sizeof(float)));
  return d;
}

int main() {
  const int S = 64, np = 64, B = S * np;
  srand(1);
  std::vector<int> off(S + 1);
  for (int s = 0; s <= S; ++s) off[s] = s * np;
  int* doff;
  CK(hipMalloc(&doff, off.size() * 4));
  CK(hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  struct L { int K, H, F, epi; } layers[2] = {{40, 4, 16, 1}, {64, 1, 40, 0}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const L& l : layers) {
    const int HF = l.H * l.F;
    float* x = upload(rnd((size_t)B * l.K, 1.f));
    float* w = upload(rnd((size_t)l.H * l.K * l.F, 0.2f));
    float* as = upload(rnd((size_t)l.H * l.F, 0.3f));
    float* ad = upload(rnd((size_t)l.H * l.F, 0.3f));
    float* bias = upload(rnd(l.F, 0.1f));
    float *xn = zeros((size_t)B * l.K), *rs = zeros((size_t)S * l.K), *wh = zeros((size_t)B * HF),
          *hp = zeros((size_t)B * HF), *y = zeros((size_t)B * HF);
    auto run = [&]() {
      int rc = sgg_gat_layer_fwd(x, l.K, l.K, nullptr, 0, 0, w, as, ad, bias, doff, S, B, l.H, l.F, 0.2f, 1e-5f, l.epi,
                                 np, 1, xn, rs, wh, hp, y, HF, nullptr);
      if (rc) { printf("rc %d %s\n", rc, sgg_last_error()); exit(1); }
    };
    for (int i = 0; i < 5; ++i) run();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, nullptr));
    for (int i = 0; i < 50; ++i) run();
    CK(hipEventRecord(e1, nullptr));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long prof[64];
    CK(hipMemcpyFromSymbol(prof, HIP_SYMBOL(sgg::g_gat_prof), sizeof(prof)));
    printf("layer K %d heads %d F %d: %.2f us per launch (back-to-back)\n", l.K, l.H, l.F, ms * 1e3 / 50);
    const char* names[] = {"start", "seg loaded", "staged", "normalised", "transformed", "scored", "attended", "end"};
    for (int i = 1; i < 8; ++i) printf("  %-12s +%6.2f us\n", names[i], (prof[i] - prof[i - 1]) * 0.01);
    printf("  total        %6.2f us\n", (prof[7] - prof[0]) * 0.01);
  }
  return 0;
}
