// Signal front end on the device: the per-read
// normalisation and windowing of utils/labelop.py:194-243
// (extract_fast5_raw), so raw reads go to the engine's [chunks, T] signal
// batch without a host pass.
//
// Normalisation (labelop.py:220-223), in fp64 like numpy / statsmodels on
// the float64 raw read, then rounded to float32 (the chunk dtype):
//   median: (x - median(x)) / median(|x - median(x)| / 0.6744897501960817)
//           (statsmodels robust.mad: the scaling happens before the median)
//   mean:   (x - median(x)) / std(x)   (population std; the reference centres
//           on the median here too)
//   none:   x
// Medians are exact order statistics: a radix select over the
// order-preserving 64-bit image of the doubles, 8 passes of 8 bits with a
// 256-bin LDS histogram, one workgroup per read; an even count averages the
// two middle values as numpy does ((a + b) / 2).
#include "common.hpp"
#include "kernels.hpp"

namespace nd {

#define FE_THREADS 256
#define FE_MAD_C 0.6744897501960817

__device__ __forceinline__ unsigned long long fe_key(double v) {
  const unsigned long long b = __double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double fe_val(unsigned long long k) {
  return __longlong_as_double((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k);
}

// value at MODE: 0 x_i, 1 |x_i - c| / MAD_C
template <int MODE>
__device__ __forceinline__ double fe_elem(const double* __restrict__ x, long long i, double c) {
  return MODE == 0 ? x[i] : fabs(x[i] - c) / FE_MAD_C;
}

// k-th smallest (0-based) of the n values fe_elem<MODE>(x, i, c); every thread returns it
template <int MODE>
__device__ double fe_select(const double* __restrict__ x, long long n, double c, long long k, unsigned* hist,
                            unsigned long long* s_prefix, long long* s_k) {
  const int tid = threadIdx.x;
  unsigned long long prefix = 0, mask = 0;
  for (int shift = 56; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    for (long long i = tid; i < n; i += FE_THREADS) {
      const unsigned long long key = fe_key(fe_elem<MODE>(x, i, c));
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      long long cum = 0;
      int b = 0;
      for (; b < 255; ++b) {
        if (cum + hist[b] > k) break;
        cum += hist[b];
      }
      *s_k = k - cum;
      *s_prefix = prefix | ((unsigned long long)b << shift);
    }
    __syncthreads();
    k = *s_k;
    prefix = *s_prefix;
    mask |= 0xFFull << shift;
    __syncthreads();
  }
  return fe_val(prefix);
}

template <int MODE>
__device__ double fe_median(const double* __restrict__ x, long long n, double c, unsigned* hist,
                            unsigned long long* s_prefix, long long* s_k) {
  const double hi = fe_select<MODE>(x, n, c, n / 2, hist, s_prefix, s_k);
  if (n & 1) return hi;
  const double lo = fe_select<MODE>(x, n, c, n / 2 - 1, hist, s_prefix, s_k);
  return (lo + hi) / 2.0;  // numpy: mean of the two middle values
}

__device__ double fe_block_sum(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = FE_THREADS / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(FE_THREADS)
read_normalize_kernel(const double* __restrict__ raw, const long long* __restrict__ off, int method,
                      float* __restrict__ out) {
  __shared__ unsigned hist[256];
  __shared__ double red[FE_THREADS];
  __shared__ unsigned long long s_prefix;
  __shared__ long long s_k;
  const int r = blockIdx.x, tid = threadIdx.x;
  const long long o = off[r], n = off[r + 1] - o;
  if (n <= 0) return;
  const double* x = raw + o;
  float* y = out + o;
  if (method == 0) {
    for (long long i = tid; i < n; i += FE_THREADS) y[i] = (float)x[i];
    return;
  }
  const double med = fe_median<0>(x, n, 0.0, hist, &s_prefix, &s_k);
  double scale;
  if (method == 1) {
    scale = fe_median<1>(x, n, med, hist, &s_prefix, &s_k);
  } else {
    double s = 0.0;
    for (long long i = tid; i < n; i += FE_THREADS) s += x[i];
    const double mean = fe_block_sum(s, red) / (double)n;
    double q = 0.0;
    for (long long i = tid; i < n; i += FE_THREADS) q += (x[i] - mean) * (x[i] - mean);
    scale = sqrt(fe_block_sum(q, red) / (double)n);
  }
  for (long long i = tid; i < n; i += FE_THREADS) y[i] = (float)((x[i] - med) / scale);
}

hipError_t launch_read_normalize(const double* raw, const long long* off, int R, int method, float* out,
                                 hipStream_t s) {
  if (R < 0 || method < 0 || method > 2 || (R > 0 && (!raw || !off || !out))) return hipErrorInvalidValue;
  if (R == 0) return hipSuccess;
  hipLaunchKernelGGL(read_normalize_kernel, dim3(R), dim3(FE_THREADS), 0, s, raw, off, method, out);
  return hipGetLastError();
}

// chunk c = samples [start[c], start[c] + len[c]) of read rd[c] (utils/labelop.py:225-233),
// zero padded to T, into row c of the engine's [C, T] signal batch; one wave per chunk row
__global__ void __launch_bounds__(256)
read_window_kernel(const float* __restrict__ sig, const long long* __restrict__ off, const int* __restrict__ rd,
                   const int* __restrict__ start, const int* __restrict__ len, int C, int T, float* __restrict__ out) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;
  const float* src = sig + off[rd[c]] + start[c];
  const int L = min(len[c], T);
  for (int t = lane; t < T; t += 64) out[(size_t)c * T + t] = t < L ? src[t] : 0.f;
}

hipError_t launch_read_window(const float* sig, const long long* off, const int* rd, const int* start,
                              const int* len, int C, int T, float* out, hipStream_t s) {
  if (C < 0 || T < 1 || (C > 0 && (!sig || !off || !rd || !start || !len || !out))) return hipErrorInvalidValue;
  if (C == 0) return hipSuccess;
  hipLaunchKernelGGL(read_window_kernel, dim3((C + 3) / 4), dim3(256), 0, s, sig, off, rd, start, len, C, T, out);
  return hipGetLastError();
}

}  // namespace nd
