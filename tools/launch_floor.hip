// Device time per launch of (near) empty kernels replayed from a HIP graph:
// the fixed cost every kernel of the training step pays.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o tools/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void tiny(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.f;
}

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
  return 0;
}
