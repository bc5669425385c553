// Probe: semantics and issue rate of v_mfma_f32_4x4x1_16b_f32 against
// v_mfma_f32_16x16x4_f32 on gfx950 (f32 in / f32 accumulate), at 1 and 8
// waves per SIMD and 4 / 8 / 16 independent accumulator chains per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void sem(float* out) {
  const int l = threadIdx.x;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32((float)l, (float)(1000 * (l + 1)), c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

template <int KIND, int CH>
__global__ void rate(float* out, int iters) {
  const int l = threadIdx.x;
  float a = l * 1e-3f, b = 1e-3f;
  f4 c[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) c[j] = {0, 0, 0, 0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 32 / CH; ++u)
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        if (KIND == 0) c[j] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[j], 0, 0, 0);
        else c[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[j], 0, 0, 0);
      }
  }
  f4 s = c[0];
#pragma unroll
  for (int j = 1; j < CH; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + l] = s[0] + s[1] + s[2] + s[3];
}

template <int KIND, int CH>
int run(float* d, int blocks, int threads, const char* tag) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 2048;
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((rate<KIND, CH>), dim3(blocks), dim3(threads), 0, 0, d, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double per_simd = (double)blocks * (threads / 64) * iters * 32 / 1024.0;  // MFMAs per SIMD
  printf("%s %-9s chains=%2d waves/SIMD=%d: %.2f ns per MFMA per SIMD\n", tag, KIND == 0 ? "4x4x1_16b" : "16x16x4",
         CH, blocks * threads / 64 / 1024, best * 1e6 / per_simd);
  return 0;
}

int main() {
  float* d;
  CK(hipMalloc(&d, 1 << 24));
  hipLaunchKernelGGL(sem, dim3(1), dim3(64), 0, 0, d);
  float h[256];
  CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  int ok = 1;  // D[lane 4b+j][reg i] = A[lane 4b+i] * B[lane 4b+j]
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int bb = l / 4, j = l % 4;
      const float want = (float)(4 * bb + i) * 1000.f * (4 * bb + j + 1);
      if (h[l * 4 + i] != want) ok = 0;
    }
  printf("4x4x1_16b layout D[4b+j][i] = A[4b+i] B[4b+j]: %s\n", ok ? "confirmed" : "MISMATCH");
  run<0, 4>(d, 256, 256, "1w");
  run<0, 8>(d, 256, 256, "1w");
  run<0, 16>(d, 256, 256, "1w");
  run<1, 4>(d, 256, 256, "1w");
  run<0, 4>(d, 2048, 256, "8w");
  run<0, 8>(d, 2048, 256, "8w");
  run<1, 4>(d, 2048, 256, "8w");
  return 0;
}
