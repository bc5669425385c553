// Which LDS instruction forms go wrong above 64 KB when another kernel's
// workgroups share the CU?  (Diagnostic tool, not part of the engine;
// DESIGN.md section 5.)
//
// Victim: 512-thread workgroups, one per CU (96 or 128 KB of dynamic LDS).
// Each wave writes a tagged pattern into a private region with ONE
// instruction form (inline asm, so the compiler cannot pick another), then
// re-reads it with the matching form for a while and counts mismatches.
// Scribbler: 256-thread workgroups with 32 KB of LDS that rewrite their own
// LDS for the same while, launched on another stream just before.
//
//   mode 0  ds_write_b32 / ds_read_b32, address VGPR >= 64 KB
//   mode 1  ds_write_b32 / ds_read_b32, VGPR < 64 KB, offset:32768 -> >= 64 KB
//   mode 2  ds_write2_b32 / ds_read2_b32 offset1:1, VGPR >= 64 KB
//   mode 3  ds_write2st64_b32 / ds_read2st64_b32 offset1:192, VGPR < 64 KB,
//           the second address >= 64 KB
//   mode 4  ds_write_b128 / ds_read_b128, VGPR >= 64 KB
//   mode 5  ds_write2_b32 / ds_read2_b32 offset1:1, every address < 64 KB
//   mode 6  ds_write2_b64 / ds_read2_b64 offset1:1, VGPR >= 64 KB
// Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o tools/liblds_forms.so tools/lds_forms_probe.hip
#include <hip/hip_runtime.h>

typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned tagof(unsigned a) { return 0x3c000000u ^ (blockIdx.x << 17) ^ a; }

template <int MODE>
__device__ __forceinline__ unsigned vaddr(int w, int lane, int j) {
  switch (MODE) {
    case 0: return 65536u + w * 2048 + j * 256 + lane * 4;
    case 1: return 32768u + w * 2048 + j * 256 + lane * 4;
    case 2: return 65536u + w * 4096 + j * 512 + lane * 8;
    case 3: return 16384u + w * 2048 + j * 256 + lane * 4;
    case 4: return 65536u + w * 8192 + j * 1024 + lane * 16;
    case 5: return (unsigned)w * 4096 + j * 512 + lane * 8;
    default: return 65536u + w * 8192 + j * 1024 + lane * 16;
  }
}

// write the pattern of access j (the tag of the byte address each dword lands on)
template <int MODE>
__device__ __forceinline__ void put(unsigned a) {
  if constexpr (MODE == 0 || MODE == 1) {
    const unsigned p = a + (MODE == 1 ? 32768u : 0u);
    if constexpr (MODE == 0)
      asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(tagof(p)) : "memory");
    else
      asm volatile("ds_write_b32 %0, %1 offset:32768" ::"v"(a), "v"(tagof(p)) : "memory");
  } else if constexpr (MODE == 2 || MODE == 5) {
    asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(a), "v"(tagof(a)), "v"(tagof(a + 4)) : "memory");
  } else if constexpr (MODE == 3) {
    asm volatile("ds_write2st64_b32 %0, %1, %2 offset1:192" ::"v"(a), "v"(tagof(a)), "v"(tagof(a + 49152))
                 : "memory");
  } else if constexpr (MODE == 4) {
    const u4 v = {tagof(a), tagof(a + 4), tagof(a + 8), tagof(a + 12)};
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
  } else {
    const u2 x = {tagof(a), tagof(a + 4)}, y = {tagof(a + 8), tagof(a + 12)};
    asm volatile("ds_write2_b64 %0, %1, %2 offset1:1" ::"v"(a), "v"(x), "v"(y) : "memory");
  }
}

// mismatching dwords of access j
template <int MODE>
__device__ __forceinline__ unsigned check(unsigned a) {
  if constexpr (MODE == 0 || MODE == 1) {
    unsigned r;
    if constexpr (MODE == 0)
      asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    else
      asm volatile("ds_read_b32 %0, %1 offset:32768\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    return r != tagof(a + (MODE == 1 ? 32768u : 0u));
  } else if constexpr (MODE == 2 || MODE == 5) {
    u2 r;
    asm volatile("ds_read2_b32 %0, %1 offset1:1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    return (r.x != tagof(a)) + (r.y != tagof(a + 4));
  } else if constexpr (MODE == 3) {
    u2 r;
    asm volatile("ds_read2st64_b32 %0, %1 offset1:192\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    return (r.x != tagof(a)) + (r.y != tagof(a + 49152));
  } else if constexpr (MODE == 4) {
    u4 r;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    return (r.x != tagof(a)) + (r.y != tagof(a + 4)) + (r.z != tagof(a + 8)) + (r.w != tagof(a + 12));
  } else {
    u4 r;
    asm volatile("ds_read2_b64 %0, %1 offset1:1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    return (r.x != tagof(a)) + (r.y != tagof(a + 4)) + (r.z != tagof(a + 8)) + (r.w != tagof(a + 12));
  }
}

template <int MODE>
__global__ void __launch_bounds__(512) victim_kernel(unsigned* err, unsigned long long ticks) {
  extern __shared__ unsigned lds[];
  (void)lds;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) put<MODE>(vaddr<MODE>(w, lane, j));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned long long t0 = wall_clock64();
  unsigned bad = 0;
  do {
#pragma unroll
    for (int j = 0; j < 8; ++j) bad += check<MODE>(vaddr<MODE>(w, lane, j));
    __builtin_amdgcn_s_sleep(1);
  } while (wall_clock64() - t0 < ticks);
  if (bad) atomicAdd(err, bad);
}

__global__ void __launch_bounds__(256) scribbler_kernel(unsigned long long ticks, unsigned* sink) {
  extern __shared__ unsigned lds[];
  const unsigned long long t0 = wall_clock64();
  unsigned s = threadIdx.x * 2654435761u + blockIdx.x, acc = 0;
  do {
    for (int i = threadIdx.x; i < 8192; i += 256) lds[i] = s ^ i;
    __syncthreads();
    for (int i = threadIdx.x; i < 8192; i += 256) acc += lds[8191 - i];
    __syncthreads();
    s = s * 1664525u + 1013904223u;
  } while (wall_clock64() - t0 < ticks);
  if (acc == 0x12345678u) sink[0] = acc;  // keep the loop
}

// short-lived workgroups shaped like the decoder's split-K GEMM reduction
// (gemm_p16_kernel<1, 8, 256>: 8 waves, 8 KB of LDS, one b128 write per
// lane, a barrier, wave 0 reads them back): LDS allocated and released on
// every CU all the time
__global__ void __launch_bounds__(512) churn_kernel(unsigned* sink) {
  __shared__ uint4 red[8][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  red[w][lane] = uint4{blockIdx.x, (unsigned)threadIdx.x, 7u, 9u};
  __syncthreads();
  if (w != 0) return;
  unsigned a = 0;
  for (int v = 0; v < 8; ++v) a += red[v][lane].x + red[v][lane].y;
  if (a == 0x12345678u) sink[0] = a;
}

template <int MODE>
static hipError_t launch_victim(unsigned* err, int wgs, unsigned long long ticks, hipStream_t s) {
  const int bytes = (MODE == 4 || MODE == 6) ? 131072 : 98304;
  hipError_t e = hipFuncSetAttribute((const void*)victim_kernel<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     bytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(victim_kernel<MODE>, dim3(wgs), dim3(512), bytes, s, err, ticks);
  return hipGetLastError();
}

// mode 0..6: victims on stream a; scribblers (if > 0) on stream b, launched
// first; scribblers < 0: -scribblers launches of 2048 short churn workgroups instead
extern "C" int lds_forms(int mode, unsigned* err, int victims, int scribblers, int us, void* sa, void* sb) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev))
    return 1;
  const unsigned long long ticks = (unsigned long long)us * khz / 1000;
  for (int i = 0; i < -scribblers; ++i)
    hipLaunchKernelGGL(churn_kernel, dim3(2048), dim3(512), 0, (hipStream_t)sb, err + 1);
  if (scribblers > 0) {
    if (hipFuncSetAttribute((const void*)scribbler_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 32768))
      return 3;
    hipLaunchKernelGGL(scribbler_kernel, dim3(scribblers), dim3(256), 32768, (hipStream_t)sb, 2 * ticks, err + 1);
  }
  hipError_t e;
  switch (mode) {
    case 0: e = launch_victim<0>(err, victims, ticks, (hipStream_t)sa); break;
    case 1: e = launch_victim<1>(err, victims, ticks, (hipStream_t)sa); break;
    case 2: e = launch_victim<2>(err, victims, ticks, (hipStream_t)sa); break;
    case 3: e = launch_victim<3>(err, victims, ticks, (hipStream_t)sa); break;
    case 4: e = launch_victim<4>(err, victims, ticks, (hipStream_t)sa); break;
    case 5: e = launch_victim<5>(err, victims, ticks, (hipStream_t)sa); break;
    case 6: e = launch_victim<6>(err, victims, ticks, (hipStream_t)sa); break;
    default: return 4;
  }
  return e == hipSuccess ? 0 : 2;
}
