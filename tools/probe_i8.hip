// Operand-map probes for the 24-bit fixed-point memory bank (diagnostic
// tool, not part of the engine):
//  tr_b8:  what ds_read_b64_tr_b8 hands each lane.  LDS holds a byte matrix
//          M[r][c] = (r << 5) | c (r < 8, c < 32, 32-byte rows); every lane
//          supplies the address given in addr[lane]; out[lane] = the 8 bytes.
//  mfma:   v_mfma_i32_16x16x64_i8 on random int8 A / B fragments; out = D
//          (16 x 16 int32 as the C/D map: col = lane & 15, row = 4 (lane >> 4) + i).
// Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o tools/libprobe_i8.so tools/probe_i8.hip
#include <hip/hip_runtime.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__global__ void tr_b8_kernel(const unsigned* addr, unsigned long long* out) {
  __shared__ volatile unsigned char m[256];  // volatile: the stores stay (only the asm reads them)
  const int l = threadIdx.x;
  for (int i = l; i < 256; i += 64) m[i] = (unsigned char)(((i >> 5) << 5) | (i & 31));
  __syncthreads();
  u2 r;
  asm volatile("ds_read_b64_tr_b8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr[l]) : "memory");
  out[l] = ((unsigned long long)r.y << 32) | r.x;
}

__global__ void mfma_i8_kernel(const i32x4* a, const i32x4* b, i32x4* d) {
  const int l = threadIdx.x;
  i32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], acc, 0, 0, 0);
  d[l] = acc;
}

extern "C" int probe_tr_b8(const unsigned* addr, unsigned long long* out) {
  hipLaunchKernelGGL(tr_b8_kernel, dim3(1), dim3(64), 0, 0, addr, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

extern "C" int probe_mfma_i8(const void* a, const void* b, void* d) {
  hipLaunchKernelGGL(mfma_i8_kernel, dim3(1), dim3(64), 0, 0, (const i32x4*)a, (const i32x4*)b, (i32x4*)d);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
