// LDS canary (diagnostic tool, not part of the engine): workgroups that fill
// their dynamic LDS with a pattern, spin for a while re-checking it, and count
// mismatches into a device word.  Run beside a suspect kernel on another
// stream: a co-resident workgroup of the suspect that writes outside its own
// LDS allocation shows up as mismatches.
// Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o tools/liblds_canary.so tools/lds_canary.hip
#include <hip/hip_runtime.h>

__global__ void lds_canary_kernel(unsigned* err, int words, unsigned long long ticks) {
  extern __shared__ unsigned lds[];
  const unsigned tag = 0x5a000000u ^ (blockIdx.x << 12);
  for (int i = threadIdx.x; i < words; i += blockDim.x) lds[i] = tag ^ (unsigned)i;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  unsigned bad = 0, first = 0xffffffffu;
  do {
    for (int i = threadIdx.x; i < words; i += blockDim.x)
      if (lds[i] != (tag ^ (unsigned)i)) {
        ++bad;
        first = min(first, (unsigned)i);
      }
    __builtin_amdgcn_s_sleep(2);
  } while (wall_clock64() - t0 < ticks);
  if (bad) {
    atomicAdd(err, bad);
    atomicMin(err + 1, first);  // lowest corrupted word index
  }
}

extern "C" int lds_canary(unsigned* err, int wgs, int lds_bytes, int us, void* stream) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev))
    return 1;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)lds_canary_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return 3;
  hipLaunchKernelGGL(lds_canary_kernel, dim3(wgs), dim3(64), lds_bytes, (hipStream_t)stream, err, lds_bytes / 4,
                     (unsigned long long)us * khz / 1000);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
