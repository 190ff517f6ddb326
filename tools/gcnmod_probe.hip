// Phase timing of the GCN module backward (sgg_gcnmod_bwd; workgroup 0's
// first scene, wall clock 100 MHz) and whole-launch time on configs[4]'s
// shape (64 scenes x 64 peds, fin 40, fe 24, bf16 transforms).  Diagnostic:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSGG_GCN_PROF \
//     -I group-gan-gcn-gat_amd/csrc -I include tools/gcnmod_probe.hip -o gcnmod_probe
#include "../group-gan-gcn-gat_amd/csrc/gcn_module.hip"
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

int main(int argc, char** argv) {
  const int S = 64, np = argc > 1 ? atoi(argv[1]) : 64, B = S * np, fin = 40, fe = 24;
  srand(1);
  SggGcnModArgs a = {};
  a.X = upload(rnd((size_t)B * fin, 1.f));
  a.ldx = fin;
  std::vector<float> lab(B);
  for (auto& x : lab) x = (float)(rand() % 6);
  a.labels = upload(lab);
  std::vector<int> off(S + 1);
  for (int s = 0; s <= S; ++s) off[s] = s * np;
  int* doff;
  CK(hipMalloc(&doff, off.size() * 4));
  CK(hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  a.scene_off = doff;
  a.S = S;
  a.np = np;
  a.fin = fin;
  a.fe = fe;
  a.bf16 = 1;
  a.W0i = upload(rnd((size_t)fin * 72, 0.2f));
  a.W1i = upload(rnd(72 * 16, 0.2f));
  a.W0g = upload(rnd(16 * 72, 0.2f));
  a.W1g = upload(rnd(72 * 16, 0.2f));
  a.Woe = upload(rnd((size_t)fe * 32, 0.2f));
  a.boe = upload(rnd(fe, 0.1f));
  a.dy = upload(rnd((size_t)B * fe, 1.f));
  a.lddy = fe;
  a.dy_copies = 1;
  a.dy_cstride = 0;
  float* dX;
  CK(hipMalloc(&dX, (size_t)B * fin * 4));
  a.dX = dX;
  a.lddx = fin;
  const size_t slab = (size_t)sgg_gcnmod_slab_rows(S) * sgg_gcnmod_param_size(fin, fe);
  float* sl;
  CK(hipMalloc(&sl, slab * 4));
  a.slab = sl;
  auto run = [&]() {
    int rc = sgg_gcnmod_bwd(&a, nullptr);
    if (rc) { printf("rc %d %s\n", rc, sgg_last_error()); exit(1); }
  };
  for (int i = 0; i < 5; ++i) run();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < 50; ++i) run();
  CK(hipEventRecord(e1, nullptr));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  long long prof[64];
  CK(hipMemcpyFromSymbol(prof, HIP_SYMBOL(g_gcn_prof), sizeof(prof)));
  printf("gcnmod_bwd %d scenes x %d peds: %.2f us per launch (back-to-back)\n", S, np, ms * 1e3 / 50);
  const char* names[] = {"start", "weights", "groups+dY", "group mean", "h1 h2", "inter fwd + dcat", "inter bwd + dWoe",
                         "Sg + dW1g dW0g", "layer 2", "layer 1 + dX"};
  for (int i = 1; i < 10; ++i) printf("  %-18s +%6.2f us\n", names[i], (prof[i] - prof[i - 1]) * 0.01);
  printf("  total              %6.2f us\n", (prof[9] - prof[0]) * 0.01);
  return 0;
}
