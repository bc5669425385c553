// Probe: how fast can one workgroup per chunk stream a chunk's 512 KB memory
// bank (512 rows of 1 KB) when it does nothing else?  This is the ceiling of
// the memory-bank attention kernel's load side (mem_attention.hip): same row
// ownership (wave w, tile r: rows 64 r + KW w .. + KW - 1), register tiles
// kept DEPTH deep, one 16 B load per lane per row.  Variants change the waves
// per workgroup, the rows per wave per tile, the depth and the workgroups per
// chunk.  Build: hipcc -O3 --offload-arch=gfx950 tools/probe_stream.hip -o tools/probe_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

// SPLIT workgroups per chunk, each over T / SPLIT consecutive rows
template <int NW, int KW, int DEPTH, int SPLIT>
__global__ void __launch_bounds__(NW * 64) stream(const float* __restrict__ mem, float* out, int T) {
  extern __shared__ float lds_pad[];  // PROBE_LDS: dynamic LDS per workgroup (occupancy as the attention kernels)
  if (T < 0) lds_pad[threadIdx.x] = 0.f;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x / SPLIT, part = blockIdx.x % SPLIT;
  const int rows = T / SPLIT, tile = NW * KW, nt = rows / tile;
  const float* base = mem + ((size_t)c * T + part * rows) * 256 + 4 * lane;
  f4 R[DEPTH][KW];
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
#pragma unroll
    for (int k = 0; k < KW; ++k)
      R[d][k] = *reinterpret_cast<const f4*>(base + (size_t)(d * tile + w * KW + k) * 256);
  for (int r = 0; r < nt; r += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int k = 0; k < KW; ++k) acc += R[d][k];
      const int nr = r + d + DEPTH;
      if (nr < nt) {
#pragma unroll
        for (int k = 0; k < KW; ++k)
          R[d][k] = *reinterpret_cast<const f4*>(base + (size_t)(nr * tile + w * KW + k) * 256);
      }
    }
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[threadIdx.x] = acc.x;
}

__global__ void fill_random(unsigned* p, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u + 12345u;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    p[i] = (x & 0x807FFFFFu) | 0x3F000000u;  // finite floats in [0.5, 1) with random sign
  }
}

template <int NW, int KW, int DEPTH, int SPLIT>
int run(const char* name, const float* mem, float* out, int C, int T) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int lb = getenv("PROBE_LDS") ? atoi(getenv("PROBE_LDS")) : 0;
  CK(hipFuncSetAttribute((const void*)stream<NW, KW, DEPTH, SPLIT>, hipFuncAttributeMaxDynamicSharedMemorySize, lb));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((stream<NW, KW, DEPTH, SPLIT>), dim3(C * SPLIT), dim3(NW * 64), lb, 0, mem, out, T);
  CK(hipDeviceSynchronize());
  const int n = 50;
  CK(hipEventRecord(e0));
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL((stream<NW, KW, DEPTH, SPLIT>), dim3(C * SPLIT), dim3(NW * 64), lb, 0, mem, out, T);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / n;
  printf("%-34s C=%4d: %8.2f us  %7.1f GB/s\n", name, C, us, (double)C * T * 1024 / (us * 1e-6) / 1e9);
  return 0;
}

int main() {
  const int T = 512, Cmax = 512;
  float *mem, *out;
  CK(hipMalloc(&mem, (size_t)Cmax * T * 1024));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(mem, 0, (size_t)Cmax * T * 1024));
  if (getenv("PROBE_RANDOM")) {  // random bits instead of zeros (zero lines may stream faster)
    hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, reinterpret_cast<unsigned*>(mem),
                       (size_t)Cmax * T * 256);
    CK(hipDeviceSynchronize());
  }
  for (int C : {64, 256, 512}) {
    run<8, 8, 2, 1>("nw8 kw8 depth2 (engine-like)", mem, out, C, T);
    run<8, 8, 4, 1>("nw8 kw8 depth4", mem, out, C, T);
    run<16, 4, 4, 1>("nw16 kw4 depth4", mem, out, C, T);
    run<16, 4, 8, 1>("nw16 kw4 depth8", mem, out, C, T);
    run<8, 8, 2, 2>("nw8 kw8 depth2 split2", mem, out, C, T);
    run<8, 8, 4, 2>("nw8 kw8 depth4 split2", mem, out, C, T);
    run<4, 8, 4, 4>("nw4 kw8 depth4 split4", mem, out, C, T);
  }
  return 0;
}
