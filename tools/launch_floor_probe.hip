// Launch floor of this runtime: per-kernel time of a chain of N dependent
// launches captured in one HIP graph, for an empty kernel and for kernels
// doing one / two dependent rounds of global loads, at 1 and 256 workgroups.
// usage: hipcc --offload-arch=gfx950 -O3 tools/launch_floor_probe.hip -o /tmp/lfp && /tmp/lfp
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__global__ void k_empty(float* p) {
  if (p == nullptr) p[threadIdx.x] = 0.f;   // never taken
}

// ROUNDS dependent load rounds: x = buf[idx(x)], then one store
template <int ROUNDS>
__global__ void k_loads(float* __restrict__ buf, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int j = i % n;
  float x = 0.f;
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    x += buf[j];
    j = (j + 1 + (int)(x * 0.f)) % n;   // the next address depends on the load
  }
  buf[(i + n / 2) % n] = x * 0.5f;
}

template <typename F>
static int time_chain(const char* name, int nk, F launch, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int k = 0; k < nk; ++k) launch();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));   // warm
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-34s %3d launches: %.3f us per launch\n", name, nk, 1000.f * ms / (reps * nk));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int n = 1 << 22;
  float* buf;
  CK(hipMalloc(&buf, sizeof(float) * n));
  CK(hipMemset(buf, 0, sizeof(float) * n));
  const int nk = 50;
  for (int wg : {1, 256, 1024}) {
    char nm[64];
    snprintf(nm, sizeof nm, "empty, %d wg", wg);
    if (time_chain(nm, nk, [&] { hipLaunchKernelGGL(k_empty, dim3(wg), dim3(256), 0, st, buf); }, st)) return 1;
    snprintf(nm, sizeof nm, "1 load round, %d wg", wg);
    if (time_chain(nm, nk, [&] { hipLaunchKernelGGL(k_loads<1>, dim3(wg), dim3(256), 0, st, buf, n); }, st)) return 1;
    snprintf(nm, sizeof nm, "2 load rounds, %d wg", wg);
    if (time_chain(nm, nk, [&] { hipLaunchKernelGGL(k_loads<2>, dim3(wg), dim3(256), 0, st, buf, n); }, st)) return 1;
    snprintf(nm, sizeof nm, "4 load rounds, %d wg", wg);
    if (time_chain(nm, nk, [&] { hipLaunchKernelGGL(k_loads<4>, dim3(wg), dim3(256), 0, st, buf, n); }, st)) return 1;
  }
  CK(hipFree(buf));
  return 0;
}
