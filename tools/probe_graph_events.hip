// Probe: timing events recorded inside a captured hipGraph (event record
// nodes) — does hipEventElapsedTime on them give the kernel's duration?
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
__global__ void spin(float* p, int n) {
  float v = p[threadIdx.x];
  for (int i = 0; i < n; ++i) v = v * 0.999f + 0.001f;
  p[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
int main() {
  float* d;
  CK(hipMalloc(&d, 1 << 24));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1, a, b;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  // eager reference
  CK(hipEventRecord(a, s));
  hipLaunchKernelGGL(spin, dim3(1024), dim3(256), 0, s, d, 20000);
  CK(hipEventRecord(b, s));
  CK(hipStreamSynchronize(s));
  float ms_eager; CK(hipEventElapsedTime(&ms_eager, a, b));
  hipGraph_t g; hipGraphExec_t ex;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  hipLaunchKernelGGL(spin, dim3(1024), dim3(256), 0, s, d, 1000);
  CK(hipEventRecord(e0, s));
  hipLaunchKernelGGL(spin, dim3(1024), dim3(256), 0, s, d, 20000);
  CK(hipEventRecord(e1, s));
  hipLaunchKernelGGL(spin, dim3(1024), dim3(256), 0, s, d, 1000);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) {
    CK(hipEventRecord(a, s));
    CK(hipGraphLaunch(ex, s));
    CK(hipEventRecord(b, s));
    CK(hipStreamSynchronize(s));
    float ms_in, ms_all;
    CK(hipEventElapsedTime(&ms_in, e0, e1));
    CK(hipEventElapsedTime(&ms_all, a, b));
    printf("eager %.4f ms | in-graph event pair %.4f ms | whole graph %.4f ms\n", ms_eager, ms_in, ms_all);
  }
  return 0;
}
