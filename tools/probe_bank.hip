// Probe: the split-fp16 memory-bank attention (dec_bank_h3_kernel) timed with
// plain back-to-back launches on hipMalloc'd buffers, the harness of
// tools/probe_stream.hip (which reads the same 512 KB per chunk and nothing
// else).  Build: hipcc -O3 --offload-arch=gfx950 -Inanodecoder_amd/csrc -Iinclude
//   tools/probe_bank.hip -o tools/probe_bank
#include "../nanodecoder_amd/csrc/mem_attention.hip"

#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void fill(float* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u + seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    p[i] = ((x >> 8) * (1.0f / 16777216.0f) - 0.5f) * 2.f;
  }
}

int main() {
  const int T = 512, Cmax = 512;
  float *x, *qp, *sig, *out;
  uint16_t* bank;
  int *span, *ovf;
  CK(hipMalloc(&x, (size_t)Cmax * T * 1024));
  CK(hipMalloc(&bank, (size_t)Cmax * T * 1024));
  CK(hipMalloc(&qp, (size_t)Cmax * 2048 * 4));
  CK(hipMalloc(&sig, (size_t)Cmax * T * 4));
  CK(hipMalloc(&out, (size_t)Cmax * 2048 * 4));
  CK(hipMalloc(&span, Cmax * 4));
  CK(hipMalloc(&ovf, 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, x, (size_t)Cmax * T * 256, 1u);
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, qp, (size_t)Cmax * 2048, 2u);
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, sig, (size_t)Cmax * T, 3u);
  std::vector<int> sp(Cmax, T);
  CK(hipMemcpy(span, sp.data(), Cmax * 4, hipMemcpyHostToDevice));
  CK(nd::init_mem_attributes());
  CK(nd::launch_bank_pack_h3(x, nullptr, nullptr, bank, Cmax, T, ovf, 0));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int C : {64, 128, 256, 512}) {
    for (int i = 0; i < 3; ++i) CK(nd::launch_dec_bank_h3(qp, bank, sig, span, 1.0f, out, C, T, 0, nullptr, nullptr, 0, ovf));
    CK(hipDeviceSynchronize());
    const int n = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < n; ++i) CK(nd::launch_dec_bank_h3(qp, bank, sig, span, 1.0f, out, C, T, 0, nullptr, nullptr, 0, ovf));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / n;
    printf("bank-h3 plain launches C=%4d: %8.2f us  %7.1f GB/s\n", C, us, (double)C * T * 1024 / (us * 1e-6) / 1e9);
  }
  return 0;
}
