// Average self-attention (AAN) decoder step kernels, gfx950.
//
// Replaces onmt/modules/average_attn.py:55-106 in decoding mode (layer cache
// "prev_g", decoder/transformer.py:82-84,262-263) for
// `self_attn_type = average` checkpoints:
//   xn   = LayerNorm_1(x)
//   avg  = (xn + step * prev_g) / (step + 1);  prev_g <- avg
//   a    = avg + W2 relu(W1 LN(avg) + b1) + b2          (PositionwiseFeedForward(d, d))
//   g    = W_g [xn ; a] + b_g                            (Linear(2d, 2d))
//   q1   = sigmoid(g[:d]) * xn + sigmoid(g[d:]) * a + x  (+ the decoder layer's residual)
// The two Linear stages run on the P16 GEMMs; these kernels do the row-wise
// parts.  prev_g lives in the decoder's per-layer history slab (the K/V cache
// of the scaled-dot form, [slot][t][512], first 256 floats) so beam reordering
// reads the parent's state through the same ancestry table as the self-
// attention cache (anc[r][t] = slot holding step t of row r's history).
#include "common.hpp"
#include "kernels.hpp"

namespace nd {

// one wave per row; lane owns columns 4 lane .. 4 lane + 3
__global__ void __launch_bounds__(256)
aan_prep_kernel(const float* __restrict__ x, const float* __restrict__ g1, const float* __restrict__ b1,
                float* __restrict__ hist, const int* __restrict__ anc, int anc_ld, int step, int S,
                float* __restrict__ xn_out, float* __restrict__ avg_out, float* __restrict__ avg_part, int R) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  const f32x4 v = ld4(x + pk(r, 4 * lane, ND_D));
  // nn.LayerNorm(d, eps=1e-6): biased variance, two passes
  const float mu = wave_sum(v.x + v.y + v.z + v.w) * (1.0f / ND_D);
  const f32x4 d = v - mu;
  const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / ND_D);
  const f32x4 xn = d * ln_rsqrt(var + ND_LN_EPS) * ld4(g1 + 4 * lane) + ld4(b1 + 4 * lane);
  f32x4 prev = {0.f, 0.f, 0.f, 0.f};
  if (step > 0) {
    const int slot = anc ? anc[(size_t)r * anc_ld + step - 1] : r;
    prev = ld4(hist + ((size_t)slot * S + step - 1) * 2 * ND_D + 4 * lane);
  }
  // (inputs + step * prev_g) / (step + 1), as average_attn.py:79-80 evaluates it
  const float fs = (float)step, fs1 = (float)(step + 1);
  const f32x4 avg = (xn + fs * prev) / fs1;
  st4(hist + ((size_t)r * S + step) * 2 * ND_D + 4 * lane, avg);
  st4(xn_out + pk(r, 4 * lane, ND_D), xn);
  st4(avg_out + pk(r, 4 * lane, ND_D), avg);
  // full-row statistics of avg for the average_layer's LayerNorm (one partial)
  const float am = wave_sum(avg.x + avg.y + avg.z + avg.w) * (1.0f / ND_D);
  const f32x4 ad = avg - am;
  const float m2 = wave_sum(ad.x * ad.x + ad.y * ad.y + ad.z * ad.z + ad.w * ad.w);
  if (lane == 0) {
    avg_part[(size_t)r * ND_PART_LD * 2] = am;
    avg_part[(size_t)r * ND_PART_LD * 2 + 1] = m2;
  }
}

__device__ __forceinline__ float sigm(float z) { return 1.0f / (1.0f + __expf(-z)); }

// q1 = sigmoid(g_in) * xn + sigmoid(g_forget) * a + x, with q1's full-row
// statistics (one partial) for LayerNorm_2.  g [R, 512], the rest [R, 256],
// all P16.
__global__ void __launch_bounds__(256)
aan_gate_kernel(const float* __restrict__ g, const float* __restrict__ xn, const float* __restrict__ a,
                const float* __restrict__ x, float* __restrict__ out, float* __restrict__ part, int R) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  const f32x4 gi = ld4(g + pk(r, 4 * lane, 2 * ND_D)), gf = ld4(g + pk(r, ND_D + 4 * lane, 2 * ND_D));
  const f32x4 vx = ld4(xn + pk(r, 4 * lane, ND_D)), va = ld4(a + pk(r, 4 * lane, ND_D));
  const f32x4 si = {sigm(gi.x), sigm(gi.y), sigm(gi.z), sigm(gi.w)};
  const f32x4 sf = {sigm(gf.x), sigm(gf.y), sigm(gf.z), sigm(gf.w)};
  const f32x4 q = (si * vx + sf * va) + ld4(x + pk(r, 4 * lane, ND_D));
  st4(out + pk(r, 4 * lane, ND_D), q);
  const float qm = wave_sum(q.x + q.y + q.z + q.w) * (1.0f / ND_D);
  const f32x4 qd = q - qm;
  const float m2 = wave_sum(qd.x * qd.x + qd.y * qd.y + qd.z * qd.z + qd.w * qd.w);
  if (lane == 0) {
    part[(size_t)r * ND_PART_LD * 2] = qm;
    part[(size_t)r * ND_PART_LD * 2 + 1] = m2;
  }
}

hipError_t launch_aan_prep(const float* x, const float* ln_g, const float* ln_b, float* hist, const int* anc,
                           int anc_ld, int step, int max_steps, float* xn, float* avg, float* avg_part, int R,
                           hipStream_t s) {
  if (step < 0 || step >= max_steps) return hipErrorInvalidValue;
  hipLaunchKernelGGL(aan_prep_kernel, dim3((R + 3) / 4), dim3(256), 0, s, x, ln_g, ln_b, hist, anc, anc_ld, step,
                     max_steps, xn, avg, avg_part, R);
  return hipGetLastError();
}

hipError_t launch_aan_gate(const float* g, const float* xn, const float* a, const float* x, float* out, float* part,
                           int R, hipStream_t s) {
  hipLaunchKernelGGL(aan_gate_kernel, dim3((R + 3) / 4), dim3(256), 0, s, g, xn, a, x, out, part, R);
  return hipGetLastError();
}

}  // namespace nd
