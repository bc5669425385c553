// Microbenchmark: cost of a device-wide barrier inside one persistent kernel
// against the boundary between dependent kernels of a hipGraph.
//
// Both run P phases of the same toy work: every workgroup writes its own 4 KB
// block, then (after the barrier / kernel boundary) reads the block of a
// workgroup 37 places further on (another XCD) and folds it into a checksum.
// The persistent form launches exactly one workgroup per CU (co-resident by
// construction: 256 threads, no LDS) and its barrier is a monotonically
// increasing agent-scope counter: release add, acquire poll with s_sleep, and a
// bounded poll (a workgroup that gives up raises an error word and leaves, so
// every wave reaches the end whatever happens).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

#define BLK 1024  // floats per workgroup block
#ifndef RELAXED_POLL
#define RELAXED_POLL 1
#endif

__device__ __forceinline__ bool grid_barrier(unsigned* cnt, unsigned target, int* err) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    unsigned it = 0;
    while (__hip_atomic_load(cnt, RELAXED_POLL ? __ATOMIC_RELAXED : __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      // bounded: ~0.1 s, or at once when another workgroup gave up already
      if (++it > (1u << 18) || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
    }
    if (RELAXED_POLL) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // one L2 invalidate after the poll, not one per poll
  }
  __shared__ int bad;
  if (threadIdx.x == 0) bad = !ok;
  __syncthreads();
  return !bad;
}

__global__ void __launch_bounds__(256) persistent(float* buf, unsigned* cnt, int* err, int phases, float* out) {
  const int b = blockIdx.x, n = gridDim.x, t = threadIdx.x;
  float acc = 0.f;
  for (int p = 0; p < phases; ++p) {
    float4* mine = reinterpret_cast<float4*>(buf + (size_t)b * BLK);
    mine[t] = make_float4(p + b, p, b, 1.f);
    if (!grid_barrier(cnt, (unsigned)(2 * p + 1) * n, err)) break;
    const float4 v = reinterpret_cast<const float4*>(buf + (size_t)((b + 37) % n) * BLK)[t];
    acc += v.x + v.y;
    if (!grid_barrier(cnt, (unsigned)(2 * p + 2) * n, err)) break;  // WAR on buf
  }
  out[b * 256 + t] = acc;
}

__global__ void __launch_bounds__(256) phase_write(float* buf, int p) {
  const int b = blockIdx.x, t = threadIdx.x;
  reinterpret_cast<float4*>(buf + (size_t)b * BLK)[t] = make_float4(p + b, p, b, 1.f);
}
__global__ void __launch_bounds__(256) phase_read(const float* buf, float* out) {
  const int b = blockIdx.x, n = gridDim.x, t = threadIdx.x;
  const float4 v = reinterpret_cast<const float4*>(buf + (size_t)((b + 37) % n) * BLK)[t];
  out[b * 256 + t] += v.x + v.y;
}

int main() {
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int n = cus, phases = 200;
  float *buf, *out;
  unsigned* cnt;
  int* err;
  CK(hipMalloc(&buf, (size_t)n * BLK * 4));
  CK(hipMalloc(&out, (size_t)n * 256 * 4));
  CK(hipMalloc(&cnt, 8));
  CK(hipMalloc(&err, 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&z));

  // graph: 2 kernels per phase
  hipGraph_t g;
  hipGraphExec_t ex;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  for (int p = 0; p < phases; ++p) {
    hipLaunchKernelGGL(phase_write, dim3(n), dim3(256), 0, s, buf, p);
    hipLaunchKernelGGL(phase_read, dim3(n), dim3(256), 0, s, buf, out);
  }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ex, s));
  CK(hipEventRecord(a, s));
  for (int w = 0; w < 10; ++w) CK(hipGraphLaunch(ex, s));
  CK(hipEventRecord(z, s));
  CK(hipEventSynchronize(z));
  float ms;
  CK(hipEventElapsedTime(&ms, a, z));
  printf("graph chain: %.3f us per boundary (%d kernels x 10, %d workgroups)\n", ms * 1e3 / 10 / (2 * phases),
         2 * phases, n);

  // persistent: 2 barriers per phase
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipMemsetAsync(cnt, 0, 8, s));
    CK(hipMemsetAsync(err, 0, 4, s));
    CK(hipEventRecord(a, s));
    hipLaunchKernelGGL(persistent, dim3(n), dim3(256), 0, s, buf, cnt, err, phases, out);
    CK(hipGetLastError());
    CK(hipEventRecord(z, s));
    CK(hipEventSynchronize(z));
    CK(hipEventElapsedTime(&ms, a, z));
    int e = 0;
    CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    printf("persistent: %.3f us per barrier (%d barriers in %.3f ms)%s\n", ms * 1e3 / (2 * phases), 2 * phases, ms,
           e ? "  BARRIER TIMED OUT" : "");
    if (e) return 2;
  }
  return 0;
}
