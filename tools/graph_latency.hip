// Microbenchmark: per-kernel cost of dependent trivial kernels in a hipGraph,
// vs the same kernels split over 2 / 4 parallel graph branches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void tiny(float* p, int n) { int i = blockIdx.x * 256 + threadIdx.x; if (i < n) p[i] = p[i] * 0.5f + 1.0f; }

int run(int branches, int kernels, int blocks, float* buf, float* ms_out) {
  std::vector<hipStream_t> s(branches);
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(branches * 2);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  hipGraph_t g; hipGraphExec_t ex;
  CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeRelaxed));
  CK(hipEventRecord(ev[0], s[0]));
  for (int b = 1; b < branches; ++b) CK(hipStreamWaitEvent(s[b], ev[0], 0));
  for (int k = 0; k < kernels / branches; ++k)
    for (int b = 0; b < branches; ++b)
      hipLaunchKernelGGL(tiny, dim3(blocks), dim3(256), 0, s[b], buf + b * 1024 * 1024, blocks * 256);
  for (int b = 1; b < branches; ++b) { CK(hipEventRecord(ev[branches + b], s[b])); CK(hipStreamWaitEvent(s[0], ev[branches + b], 0)); }
  CK(hipStreamEndCapture(s[0], &g));
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ex, s[0]));
  CK(hipEventRecord(a, s[0]));
  for (int w = 0; w < 10; ++w) CK(hipGraphLaunch(ex, s[0]));
  CK(hipEventRecord(z, s[0]));
  CK(hipEventSynchronize(z));
  float ms; CK(hipEventElapsedTime(&ms, a, z));
  *ms_out = ms / 10;
  return 0;
}

int main() {
  float* buf; CK(hipMalloc(&buf, 64 << 20));
  CK(hipMemset(buf, 0, 64 << 20));
  for (int blocks : {1, 256, 2048}) {
    for (int br : {1, 2, 4}) {
      float ms;
      if (run(br, 400, blocks, buf, &ms)) return 1;
      printf("blocks=%5d branches=%d: %.2f us per kernel (400 kernels, %.3f ms per graph)\n", blocks, br, ms * 1e3 / 400, ms);
    }
  }
  return 0;
}
