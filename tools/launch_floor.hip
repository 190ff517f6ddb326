// Device time per launch of (near) empty kernels replayed from a HIP graph:
// the fixed cost every kernel of the training step pays.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void tiny(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.f;
}

struct Big {
  float* p[100];
  int n;
};
__global__ void tiny_bigarg(Big a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n) a.p[i & 63][i] += 1.f;
}

__global__ void empty_k() {}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  float* d;
  CK(hipMalloc(&d, 1 << 24));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int blocks[] = {1, 64, 256, 1024};
  for (int b : blocks) {
    const int K = 100;
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(tiny, dim3(b), dim3(256), 0, st, d, b * 256);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    const int R = 20;
    for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("graph of %d launches x %4d blocks: %.2f us per launch\n", K, b, ms * 1e3 / (R * K));
    // the same launches issued directly on the stream
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < R; ++r)
      for (int k = 0; k < K; ++k) hipLaunchKernelGGL(tiny, dim3(b), dim3(256), 0, st, d, b * 256);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("stream launches x %4d blocks:        %.2f us per launch\n", b, ms * 1e3 / (R * K));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // variants at 64 blocks: empty kernel, a 808-byte by-value argument, 4 MB written per launch
  for (int v = 0; v < 3; ++v) {
    const int K = 100, b = v == 2 ? 4096 : 64;
    Big big;
    for (int j = 0; j < 100; ++j) big.p[j] = d;
    big.n = 64 * 256;
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int k = 0; k < K; ++k) {
      if (v == 0) hipLaunchKernelGGL(empty_k, dim3(b), dim3(256), 0, st);
      else if (v == 1) hipLaunchKernelGGL(tiny_bigarg, dim3(b), dim3(256), 0, st, big);
      else hipLaunchKernelGGL(tiny, dim3(b), dim3(256), 0, st, d, b * 256);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const char* nm[3] = {"empty kernel, 64 blocks", "808-B argument, 64 blocks", "4 MB written, 4096 blocks"};
    printf("graph of %d launches, %s: %.2f us per launch\n", K, nm[v], ms * 1e3 / (20 * K));
  }
  return 0;
}
