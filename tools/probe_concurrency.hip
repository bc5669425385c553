// Probe: do kernels on two HIP streams of ONE process run at the same time?
//
// A spin kernel (one workgroup, busy for ~US microseconds by the constant-rate
// wall clock) is launched K times on stream A and K times on stream B.  If the
// streams' hardware queues run together the whole takes ~K*US; serialised it
// takes ~2*K*US.  Also times the two streams' chains of many short dependent
// kernels (the decoder-step pattern).  Run two copies at once to see the
// cross-process case.  Build: hipcc --offload-arch=gfx950 -O2 -o tools/probe_concurrency tools/probe_concurrency.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                       \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void spin(unsigned long long ticks, float* out) {
  const unsigned long long t0 = wall_clock64();
  float v = threadIdx.x;
  while (wall_clock64() - t0 < ticks) v = v * 0.999f + 0.001f;
  if (v == -1.f) out[threadIdx.x] = v;  // keep the loop
}

static double run(hipStream_t* st, int ns, int K, unsigned long long ticks, float* d, int wgs) {
  for (int i = 0; i < ns; ++i) (void)hipStreamSynchronize(st[i]);
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < K; ++k)
    for (int i = 0; i < ns; ++i) hipLaunchKernelGGL(spin, dim3(wgs), dim3(64), 0, st[i], ticks, d);
  for (int i = 0; i < ns; ++i) (void)hipStreamSynchronize(st[i]);
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  const int us = argc > 1 ? atoi(argv[1]) : 200;
  int dev = 0, khz = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  const unsigned long long ticks = (unsigned long long)us * khz / 1000;
  for (const char* v : {"AMD_SERIALIZE_KERNEL", "AMD_SERIALIZE_COPY", "GPU_MAX_HW_QUEUES", "HIP_LAUNCH_BLOCKING",
                        "DEBUG_CLR_GRAPH_PACKET_CAPTURE", "HSA_ENABLE_SDMA", "HIP_FORCE_DEV_KERNARG",
                        "AMD_LOG_LEVEL", "HSA_CU_MASK", "ROC_ACTIVE_WAIT_TIMEOUT"}) {
    const char* e = getenv(v);
    printf("env %s=%s\n", v, e ? e : "(unset)");
  }
  float* d;
  CK(hipMalloc(&d, 4096));
  hipStream_t st[4];
  for (int i = 0; i < 4; ++i) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  const int K = 20;
  run(st, 2, 2, ticks, d, 1);  // warm
  for (int wgs : {1, 64}) {
    const double one = run(st, 1, K, ticks, d, wgs);
    const double two = run(st, 2, K, ticks, d, wgs);
    const double four = run(st, 4, K, ticks, d, wgs);
    printf("spin %d us x %d, %d WG: 1 stream %.0f us, 2 streams %.0f us (%.2fx of 1), 4 streams %.0f us (%.2fx)\n",
           us, K, wgs, one, two, two / one, four, four / one);
  }
  // short dependent kernels (decoder-step pattern): 2000 x ~5 us per stream
  const unsigned long long t5 = 5ull * khz / 1000;
  const double c1 = run(st, 1, 2000, t5, d, 64);
  const double c2 = run(st, 2, 2000, t5, d, 64);
  printf("chain 2000 x 5 us, 64 WG: 1 stream %.0f us, 2 streams %.0f us (%.2fx)\n", c1, c2, c2 / c1);
  return 0;
}
