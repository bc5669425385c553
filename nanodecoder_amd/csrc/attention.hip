// Attention and row kernels of the translate path (gfx950).
//
// * enc_attention: the Transformer encoder's self-attention
//   (onmt/modules/multi_headed_attn.py:154-177 with the key mask of
//   encoder/transformer.py:117-121, ``src == 0.0``).  One workgroup owns one
//   (chunk, head): all of that head's K (row-major) and V (transposed) sit in
//   LDS (<= 512 keys, 140 KB), and 16 waves each stream 32 queries through
//   them with fp32 MFMA and an online softmax — the [T, T] score matrix the
//   reference materialises is never written.  Scores are computed transposed
//   (S^T = K Q^T) so a query's 32 keys live in one lane's accumulator
//   registers: the row max/sum is 15 register ops + one cross-half shuffle,
//   and the exponentiated tile is directly the B operand of the P.V MFMA.
// * dec_self_attention / dec_ctx_attention: the decoder's q_len = 1
//   attention (multi_headed_attn.py:124-153 cache modes), bandwidth bound.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "head.hpp"
#include "kernels.hpp"

namespace nd {

// ------------------------------------------------------------------ encoder
// Full-row statistics {mean, M2} of a 256-wide row held as float4 per lane
// (the part_n = 1 form of the GEMM row-statistics hand-off).
__device__ __forceinline__ void row_part(f32x4 v, int lane, float* part) {
  const float mu = wave_sum(v.x + v.y + v.z + v.w) * (1.0f / ND_D);
  const f32x4 d = v - mu;
  const float q = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w);
  if (lane == 0) {
    part[0] = mu;
    part[1] = q;
  }
}

template <bool QKV>
__global__ void __launch_bounds__(256)
enc_embed_kernel(const float* __restrict__ signal, const float* __restrict__ w, const float* __restrict__ b,
                 float* __restrict__ x, float* __restrict__ part, int n_rows, EmbedQkv eq) {
  // encoder/transformer.py:104,113 — Linear(1, d) applied to the scalar sample
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const float s = signal[row];
  const f32x4 wv = ld4(w + lane * 4), bv = ld4(b + lane * 4);
  const f32x4 v = s * wv + bv;
  st4(x + (size_t)row * ND_D + lane * 4, v);
  if (part) row_part(v, lane, part + (size_t)row * ND_PART_LD * 2);
  if constexpr (QKV) {  // layer 0's q | k | v (encoder/transformer.py:44, the rank-2 form of EmbedQkv)
    const float rs = ln_rsqrt(fmaf(s, fmaf(s, eq.mww, 2.0f * eq.mwb), eq.mbb) + ND_LN_EPS);
    float* o = eq.qkv + (size_t)row * 3 * ND_D + lane * 4;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int n = j * ND_D + lane * 4;
      st4(o + j * ND_D, (s * ld4(eq.ac + n) + ld4(eq.ac + 3 * ND_D + n)) * rs + ld4(eq.bias + n));
    }
  }
}

hipError_t launch_enc_embed(const float* signal, const float* w_in, const float* b_in, float* x, float* part, int B,
                            int T, hipStream_t s, const EmbedQkv* eq) {
  const int rows = B * T;
  if (eq) {
    if (!eq->ac || !eq->bias || !eq->qkv) return hipErrorInvalidValue;
    hipLaunchKernelGGL(enc_embed_kernel<true>, dim3((rows + 3) / 4), dim3(256), 0, s, signal, w_in, b_in, x, part,
                       rows, *eq);
  } else {
    hipLaunchKernelGGL(enc_embed_kernel<false>, dim3((rows + 3) / 4), dim3(256), 0, s, signal, w_in, b_in, x, part,
                       rows, EmbedQkv());
  }
  return hipGetLastError();
}

// EmbedQkv's a, c (thread n of 768) and means (block 0), accumulated in double
__global__ void __launch_bounds__(256)
embed_qkv_prep_kernel(const float* __restrict__ w, const float* __restrict__ b, const float* __restrict__ W,
                      float* __restrict__ ac, double* __restrict__ scal) {
  __shared__ double wd[ND_D], bd[ND_D];
  const int tid = threadIdx.x;
  wd[tid] = w[tid];
  bd[tid] = b[tid];
  __syncthreads();
  double wm = 0.0, bm = 0.0;
  for (int d = 0; d < ND_D; ++d) {
    wm += wd[d];
    bm += bd[d];
  }
  wm /= ND_D;
  bm /= ND_D;
  const int n = blockIdx.x * 256 + tid;
  double a = 0.0, c = 0.0;
  for (int d = 0; d < ND_D; ++d) {
    const double wt = W[(size_t)n * ND_D + d];
    a += (wd[d] - wm) * wt;
    c += (bd[d] - bm) * wt;
  }
  ac[n] = (float)a;
  ac[3 * ND_D + n] = (float)c;
  if (blockIdx.x == 0 && tid == 0) {
    double ww = 0.0, wb = 0.0, bb = 0.0;
    for (int d = 0; d < ND_D; ++d) {
      ww += (wd[d] - wm) * (wd[d] - wm);
      wb += (wd[d] - wm) * (bd[d] - bm);
      bb += (bd[d] - bm) * (bd[d] - bm);
    }
    scal[0] = ww / ND_D;
    scal[1] = wb / ND_D;
    scal[2] = bb / ND_D;
  }
}

hipError_t launch_embed_qkv_prep(const float* w_in, const float* b_in, const float* nwqkv, float* ac, double* scal,
                                 hipStream_t s) {
  hipLaunchKernelGGL(embed_qkv_prep_kernel, dim3(3), dim3(256), 0, s, w_in, b_in, nwqkv, ac, scal);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256)
layernorm_kernel(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
                 float* __restrict__ out, int rows) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  f32x4 v = ld4(x + (size_t)row * ND_D + lane * 4);
  const float mu = wave_sum(v.x + v.y + v.z + v.w) * (1.0f / ND_D);
  const f32x4 d = v - mu;
  const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / ND_D);
  const float rs = ln_rsqrt(var + ND_LN_EPS);
  st4(out + (size_t)row * ND_D + lane * 4, d * rs * ld4(g + lane * 4) + ld4(b + lane * 4));
}

hipError_t launch_layernorm(const float* x, const float* g, const float* b, float* out, int rows, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, g, b, out, rows);
  return hipGetLastError();
}

#define ENC_MAXT 512
#define ENC_KLD 36    // K row stride (floats): conflict-free ds_read_b128
#define ENC_VLD 516   // V^T row stride

__global__ void __launch_bounds__(1024)
enc_attention_kernel(const float* __restrict__ qkv, const float* __restrict__ signal, const int* __restrict__ span,
                     float* __restrict__ out, int T) {
#ifdef ND_SKIP_EATTN32  // timing probe only (tools/marginal_exact.sh): the kernel's marginal cost
  if (threadIdx.x < 100000) return;
#endif
  __shared__ __attribute__((aligned(16))) float Ks[ENC_MAXT * ENC_KLD];
  __shared__ __attribute__((aligned(16))) float Vt[ND_DH * ENC_VLD];
  __shared__ int kflag[ENC_MAXT];  // 0 = key, 1 = masked (signal == 0), 2 = absent (t >= span)

  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = min(span[b], T);
  const int nkt = (L + 31) >> 5;
  const size_t base = (size_t)b * T;

  for (int idx = tid; idx < nkt * 32 * 8; idx += 1024) {
    const int t = idx >> 3, c = (idx & 7) * 4;
    f32x4 k = {0.f, 0.f, 0.f, 0.f}, v = {0.f, 0.f, 0.f, 0.f};
    if (t < L) {
      const float* row = qkv + (base + t) * (3 * ND_D) + h * ND_DH + c;
      k = ld4(row + ND_D);
      v = ld4(row + 2 * ND_D);
    }
    st4(&Ks[t * ENC_KLD + c], k);
    Vt[(c + 0) * ENC_VLD + t] = v.x;
    Vt[(c + 1) * ENC_VLD + t] = v.y;
    Vt[(c + 2) * ENC_VLD + t] = v.z;
    Vt[(c + 3) * ENC_VLD + t] = v.w;
  }
  for (int t = tid; t < nkt * 32; t += 1024) kflag[t] = t < L ? (signal[base + t] == 0.0f ? 1 : 0) : 2;
  __syncthreads();

  const int q0 = wave * 32;
  if (q0 >= L) return;
  const int lr = lane & 31, lh = lane >> 5;
  const int q = q0 + lr;
  const int qc = min(q, T - 1);

  // query fragment: step s = 4j+i uses d = 8j + 4*lh + i; pre-scaled like
  // ``query / math.sqrt(dim_per_head)`` (multi_headed_attn.py:167)
  f32x4 qf[4];
  {
    const float* qrow = qkv + (base + qc) * (3 * ND_D) + h * ND_DH + 4 * lh;
#pragma unroll
    for (int j = 0; j < 4; ++j) qf[j] = ld4(qrow + 8 * j) / ND_SQRT_DH;
  }

  f32x16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
  float m = -INFINITY, l = 0.f;

  for (int kt = 0; kt < nkt; ++kt) {
    f32x16 sacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
    const float* krow = &Ks[(kt * 32 + lr) * ENC_KLD + 4 * lh];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 kf = ld4(krow + 8 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) sacc = mfma32(kf[i], qf[j][i], sacc);
    }
    // sacc[r] = score(query q, key kt*32 + mfma32_row(r, lane))
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int f = kflag[kt * 32 + mfma32_row(r, lane)];
      float sv = sacc[r];
      sv = f == 1 ? ND_MASK_FILL : sv;
      sv = f == 2 ? -INFINITY : sv;
      sacc[r] = sv;
      mx = fmaxf(mx, sv);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = __expf(m - mn);
    float rsum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sacc[r] = __expf(sacc[r] - mn);
      rsum += sacc[r];
    }
    rsum += __shfl_xor(rsum, 32, 64);
    l = l * alpha + rsum;
    m = mn;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] *= alpha;
    // O^T[d][q] += V^T[d][key] P^T[key][q]; step s = 4j+i uses key 8j + 4*lh + i
    const float* vrow = &Vt[lr * ENC_VLD + kt * 32 + 4 * lh];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 vf = ld4(vrow + 8 * j);
#pragma unroll
      for (int i = 0; i < 4; ++i) o = mfma32(vf[i], sacc[4 * j + i], o);
    }
  }
  if (q < L) {
    const float inv = 1.0f / l;
    float* orow = out + (base + q) * ND_D + h * ND_DH + 4 * lh;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v = {o[4 * g + 0] * inv, o[4 * g + 1] * inv, o[4 * g + 2] * inv, o[4 * g + 3] * inv};
      st4(orow + 8 * g, v);
    }
  }
}

// Split-fp16 form of enc_attention_kernel (same work split, same accumulator
// layouts): K, V^T are staged into LDS already split into fp16 hi / lo planes
// and Q is split in registers, so every product is hi*hi + hi*lo + lo*hi on
// v_mfma_f32_32x32x16_f16 into the fp32 accumulators (the GEMM's H3 scheme,
// gemm.hip) — 6 MFMAs of 32 cycles per 32 x 32 x 32 product instead of 16 of
// 64 cycles.  Scores S^T = K Q^T: A = K rows (lane: key l&31, dims
// 16 s + 8 (l>>5) + j), B = Q^T.  P.V: O^T += V^T P^T with the 16 keys of
// k-step s taken in the order the score accumulator hands them to a lane
// (registers 8 s .. 8 s + 7 = keys 4 h + {0..3, 8..11} + 16 s), which V^T's
// LDS image stores contiguously (key k of a 16-group at position
// (k & 3) + 4 ((k >> 3) & 1) + 8 ((k >> 2) & 1)).
typedef _Float16 eh8 __attribute__((ext_vector_type(8)));
#define ENC_KH 20      // K plane row stride (dwords): 32 halves + 8 pad, conflict-free ds_read_b128
#define ENC_VH 260     // V^T plane row stride (dwords): 512 halves + 8 pad

__device__ __forceinline__ f32x16 mfma32h(eh8 a, eh8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void esplit8(const float (&x)[8], eh8& hi, eh8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = (_Float16)x[j];
    lo[j] = (_Float16)(x[j] - (float)hi[j]);
  }
}

// Softmax in log2 units (Q pre-scaled by log2(e) / sqrt(dh): p = 2^(s - m)
// on v_exp_f32 with no multiply) with a lazy running maximum: O and l are
// rescaled only when a query's tile maximum exceeds m by more than
// ENC_THR (p <= 2^8, far inside fp16 once split).  Tiles with no masked or
// absent key (the common case) skip the per-element mask selects; the row
// sum stays per lane until the end.  These cut the loop's VALU work, which
// (at head dim 32) is what bounds this kernel, not the MFMAs.
#define ENC_THR 8.0f
typedef float ef2 __attribute__((ext_vector_type(2)));

// Persistent form: one workgroup per CU walks the (chunk, head) items
// blockIdx.x, + gridDim.x, ...; the next item's K / V loads are issued right
// after the current item is staged into LDS and land while its key loop runs
// (one workgroup per CU: 150 KB of LDS).  NQ = query blocks of 32 per wave:
//  - NQ = 1: 16 waves, 128 VGPRs each; only half of the next K / V fits
//    beside the loop (the whole prefetch spills);
//  - NQ = 2: 8 waves of 64 queries, 256 VGPRs each: the whole next item
//    (K, V and the wave's Q rows) is prefetched, and every K / V fragment
//    read from LDS feeds two query blocks.
template <int NQ>
__global__ void __launch_bounds__(1024 / NQ)
enc_attention_h3_kernel(const float* __restrict__ qkv, const float* __restrict__ signal, const int* __restrict__ span,
                        float* __restrict__ out, int T, int B, int* ovf) {
#ifdef ND_SKIP_EATTN  // timing probe only (tools/build_variant.sh): the kernel's marginal cost
  if (threadIdx.x < 100000) return;
#endif
  __shared__ __attribute__((aligned(16))) unsigned Kp[2][ENC_MAXT * ENC_KH];  // [hi|lo][key][32 halves + pad]
  __shared__ __attribute__((aligned(16))) unsigned Vp[2][ND_DH * ENC_VH];     // [hi|lo][dim][512 halves + pad]
  __shared__ int kflag[ENC_MAXT];          // 0 = key, 1 = masked (signal == 0), 2 = absent (t >= span)
  __shared__ int tdirty[ENC_MAXT / 32];    // 32-key tile holds a masked or absent key

  constexpr int NT = 1024 / NQ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int n_items = B * ND_H;

  // staging loads of item it (head it % 8 of chunk it / 8): every K / V load
  // of its 512 keys (IT x 2 per thread, rows clamped into the span),
  // straight-line (a load under `t < L` in each pass of a loop made hipcc
  // drain them pass by pass).  The first PF passes (and with QPF the wave's
  // Q rows) are prefetched under the previous item's loop; the rest go out
  // with the item's own staging.
  static_assert(ENC_MAXT * 8 % NT == 0 && ENC_MAXT <= NT, "staging passes / one key per thread");
  constexpr int IT = ENC_MAXT * 8 / NT;
  constexpr int PF = NQ == 1 ? 2 : IT;
  constexpr bool QPF = false;  // the Q rows too: 5 registers beyond 256 at NQ = 2 (a spill)
  f32x4 kr[IT], vr[IT];
  f32x4 qraw[NQ][4];  // this lane's query rows (see the Q^T operand below)
  auto issue = [&](int it, int i0, int i1) {
    const int h = it % ND_H, b = it / ND_H;
    const int L = min(span[b], T);
    const size_t base = (size_t)b * T;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      if (i < i0 || i >= i1) continue;  // compile-time after unrolling
      const int idx = tid + i * NT, t = min(idx >> 3, L - 1), c = (idx & 7) * 4;
      const float* row = qkv + (base + t) * (3 * ND_D) + h * ND_DH + c;
      kr[i] = ld4(row + ND_D);
      vr[i] = ld4(row + 2 * ND_D);
    }
  };
  auto issue_q = [&](int it) {
    const int h = it % ND_H, b = it / ND_H;
    const size_t base = (size_t)b * T;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const float* qrow = qkv + (base + min((wave * NQ + j) * 32 + lr, T - 1)) * (3 * ND_D) + h * ND_DH + 8 * lh;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        qraw[j][2 * s2] = ld4(qrow + 16 * s2);
        qraw[j][2 * s2 + 1] = ld4(qrow + 16 * s2 + 4);
      }
    }
  };
  int item = blockIdx.x;
  if (item < n_items) {
    issue(item, 0, PF);
    if constexpr (QPF) issue_q(item);
  }
  for (; item < n_items; item += gridDim.x) {
    const int h = item % ND_H, b = item / ND_H;
    const int L = min(span[b], T);
    const int nkt = (L + 31) >> 5;
    const size_t base = (size_t)b * T;
    issue(item, PF, IT);
    if constexpr (!QPF) issue_q(item);
    const float sgv = signal[base + min(tid, L - 1)];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = tid + i * NT, t = idx >> 3, c = (idx & 7) * 4;
      const bool in = t < L;
      const f32x4 k = in ? kr[i] : f32x4{0.f, 0.f, 0.f, 0.f}, v = in ? vr[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      amax = fmaxf(amax, fmaxf(absmax4(k), absmax4(v)));
      _Float16* kh = reinterpret_cast<_Float16*>(&Kp[0][t * ENC_KH]) + c;
      _Float16* kl = reinterpret_cast<_Float16*>(&Kp[1][t * ENC_KH]) + c;
      const int pos = (t & ~15) + (t & 3) + 4 * ((t >> 3) & 1) + 8 * ((t >> 2) & 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const _Float16 a = (_Float16)k[j], vv = (_Float16)v[j];
        kh[j] = a;
        kl[j] = (_Float16)(k[j] - (float)a);
        reinterpret_cast<_Float16*>(&Vp[0][(c + j) * ENC_VH])[pos] = vv;
        reinterpret_cast<_Float16*>(&Vp[1][(c + j) * ENC_VH])[pos] = (_Float16)(v[j] - (float)vv);
      }
    }
    flag_overflow(ovf, amax);
    {
      // one key per thread; wave w covers tiles 2w, 2w + 1
      const bool have = tid < nkt * 32;
      int f = 0;
      if (have) {
        f = tid < L ? (sgv == 0.0f ? 1 : 0) : 2;
        kflag[tid] = f;
      }
      const unsigned long long bal = __ballot(have && f != 0);
      if (lane == 0 && 64 * wave < nkt * 32) {
        tdirty[2 * wave] = (unsigned)bal != 0u;
        tdirty[2 * wave + 1] = (unsigned)(bal >> 32) != 0u;
      }
    }
    // Q^T operand of k-step s: dims 16 s + 8 lh .. + 7 of query q, pre-scaled
    // like ``query / math.sqrt(dim_per_head)`` (multi_headed_attn.py:167)
    // and by log2(e) (scores in log2 units)
    eh8 qh[NQ][2], ql[NQ][2];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const float qs = 1.4426950408889634f / ND_SQRT_DH;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const f32x4 r0 = qraw[j][2 * s2], r1 = qraw[j][2 * s2 + 1];
        const f32x4 x0 = r0 * qs, x1 = r1 * qs;
        flag_overflow(ovf, fmaxf(absmax4(x0), absmax4(x1)));  // the values split, log2(e) included
        const float x[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        esplit8(x, qh[j][s2], ql[j][s2]);
      }
    }
    __syncthreads();
    // the next item's loads go out now and land under this item's key loop
    if (item + (int)gridDim.x < n_items) {
      issue(item + gridDim.x, 0, PF);
      if constexpr (QPF) issue_q(item + gridDim.x);
    }

    const int q0 = wave * NQ * 32;
    if (q0 < L) {
      f32x16 o[NQ];
      float m[NQ], l[NQ];  // l: this lane's 16 keys of each tile
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) o[j][r] = 0.f;
        m[j] = -INFINITY;
        l[j] = 0.f;
      }

      for (int kt = 0; kt < nkt; ++kt) {
        f32x16 sacc[NQ];
#pragma unroll
        for (int j = 0; j < NQ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc[j][r] = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int off = (kt * 32 + lr) * ENC_KH + 8 * s2 + 4 * lh;  // dwords: dims 16 s2 + 8 lh
          const eh8 kh = __builtin_bit_cast(eh8, *reinterpret_cast<const f32x4*>(&Kp[0][off]));
          const eh8 kl = __builtin_bit_cast(eh8, *reinterpret_cast<const f32x4*>(&Kp[1][off]));
#pragma unroll
          for (int j = 0; j < NQ; ++j) {
            sacc[j] = mfma32h(kh, ql[j][s2], sacc[j]);
            sacc[j] = mfma32h(kl, qh[j][s2], sacc[j]);
            sacc[j] = mfma32h(kh, qh[j][s2], sacc[j]);
          }
        }
        // sacc[j][r] = score(query q0 + 32 j + lr, key kt*32 + mfma32_row(r, lane)), log2 units
        if (tdirty[kt]) {  // wave-uniform
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int f = kflag[kt * 32 + mfma32_row(r, lane)];
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
              float sv = sacc[j][r];
              sv = f == 1 ? ND_MASK_FILL : sv;
              sv = f == 2 ? -INFINITY : sv;
              sacc[j][r] = sv;
            }
          }
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
          float mx = sacc[j][0];
#pragma unroll
          for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sacc[j][r]);
          mx = xor32_max(mx);
          if (__any(mx > m[j] + ENC_THR)) {
            const float mn = fmaxf(m[j], mx);
            const float alpha = __builtin_amdgcn_exp2f(m[j] - mn);  // m = -inf: 0
            m[j] = mn;
            l[j] *= alpha;
#pragma unroll
            for (int r = 0; r < 16; ++r) o[j][r] *= alpha;
          }
          ef2 ls = {0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const ef2 d = ef2{sacc[j][r], sacc[j][r + 1]} - m[j];
            const ef2 p = {__builtin_amdgcn_exp2f(d.x), __builtin_amdgcn_exp2f(d.y)};
            sacc[j][r] = p.x;
            sacc[j][r + 1] = p.y;
            ls += p;
          }
          l[j] += ls.x + ls.y;
        }
        // O^T[d][q] += V^T[d][key] P^T[key][q] over the tile's two 16-key k-steps
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int off = lr * ENC_VH + (kt * 32 + 16 * s2 + 8 * lh) / 2;  // dwords
          const eh8 vh = __builtin_bit_cast(eh8, *reinterpret_cast<const f32x4*>(&Vp[0][off]));
          const eh8 vl = __builtin_bit_cast(eh8, *reinterpret_cast<const f32x4*>(&Vp[1][off]));
#pragma unroll
          for (int j = 0; j < NQ; ++j) {
            const float pv[8] = {sacc[j][8 * s2 + 0], sacc[j][8 * s2 + 1], sacc[j][8 * s2 + 2], sacc[j][8 * s2 + 3],
                                 sacc[j][8 * s2 + 4], sacc[j][8 * s2 + 5], sacc[j][8 * s2 + 6], sacc[j][8 * s2 + 7]};
            eh8 ph, pl;
            esplit8(pv, ph, pl);
            o[j] = mfma32h(vh, pl, o[j]);
            o[j] = mfma32h(vl, ph, o[j]);
            o[j] = mfma32h(vh, ph, o[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const float lj = xor32_sum(l[j]);  // both lane halves of query q
        const int q = q0 + 32 * j + lr;
        if (q < L) {
          const float inv = 1.0f / lj;
          float* orow = out + (base + q) * ND_D + h * ND_DH + 4 * lh;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            f32x4 v = {o[j][4 * g + 0] * inv, o[j][4 * g + 1] * inv, o[j][4 * g + 2] * inv, o[j][4 * g + 3] * inv};
            st4(orow + 8 * g, v);
          }
        }
      }
    }
    lds_barrier();  // every wave is done with this item's K / V / flags in LDS
  }
}

// persistent grid of the split-fp16 encoder attention: one workgroup per CU
static int enc_attn_grid() {
  static const int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return cus > 0 ? cus : 256;
  }();
  return n;
}

hipError_t launch_enc_attention(const float* qkv, const float* signal, const int* span, float* out, int B, int T,
                                hipStream_t s, bool exact, int* ovf) {
  if (T > ENC_MAXT || T <= 0) return hipErrorInvalidValue;
  static const bool f32 = [] {
    const char* e = getenv("ND_ENC_ATTN_F32");  // 1: the fp32-MFMA kernel
    return e && atoi(e) != 0;
  }();
  if (f32 || exact)
    hipLaunchKernelGGL(enc_attention_kernel, dim3(ND_H, B), dim3(1024), 0, s, qkv, signal, span, out, T);
  else
    hipLaunchKernelGGL(enc_attention_h3_kernel<2>, dim3(std::min(B * ND_H, enc_attn_grid())), dim3(512), 0, s, qkv,
                       signal, span, out, T, B, ovf);
  return hipGetLastError();
}

// Layer 0's attention in closed form (kernels.hpp launch_enc_attention_rank2;
// multi_headed_attn.py:154-177 with the key mask of encoder/transformer.py:
// 117-121).  One workgroup per chunk, one query per thread: the unmasked keys'
// (y, r) are compacted (a masked key's score is the -1e18 fill, whose weight
// is exactly 0 beside any unmasked key; a chunk with no unmasked key is
// uniform over its keys, which all share s = 0, so one representative key
// gives the same expectations); two passes over them per (query, head): the
// maximum, then exp2 and the three sums.
// No data crosses between waves: every wave compacts all of the chunk's keys
// into its OWN LDS slab (8 keys per lane, ballots and popcounts) and stages
// its own 64 queries' E[y], E[r] for its coalesced row stores, so the kernel
// has no barrier.  (The first form shared one key list and the 8 waves'
// counts through LDS across barriers; its output went wrong by whole chunks
// when another engine's decoder GEMMs ran beside it on the GPU)
// LDS: 8 wave slabs of 8 KB = exactly 64 KB.  Each slab holds the keys (y, r)
// and then its 64 queries' E[y], E[r] as [64][16] floats, column c of row q at
// c ^ (q & 15) (the 64 lanes' row writes hit 64 distinct banks).  The round-3
// layout ([64][17], 67,584 B in all) put wave 7's rows q >= 34 past byte
// 65,536 and went wrong beside other engines' kernels (DESIGN.md section 5;
// the probe layouts of that experiment live in git history, round 4).
#define R2_SLAB (8 * ENC_MAXT + 64 * 16 * 4)  // bytes per wave: keys (y, r), then its queries' E[y], E[r]
__device__ __forceinline__ int r2_col(int q, int c) { return c ^ (q & 15); }
__global__ void __launch_bounds__(512)
enc_attention_rank2_kernel(R2Args A, int T) {
  const float* __restrict__ signal = A.signal;
  const int* __restrict__ span = A.span;
  const EmbedQkv eq = A.eq;
  const float* __restrict__ coef = A.coef;
  float* __restrict__ out = A.out;
  __shared__ __attribute__((aligned(16))) char smem[8 * R2_SLAB];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float2* kyr = reinterpret_cast<float2*>(smem + wave * R2_SLAB);                                   // [ENC_MAXT]
  float(*ex)[16] = reinterpret_cast<float(*)[16]>(smem + wave * R2_SLAB + 8 * ENC_MAXT);  // [64][16]
  const int L = min(span[b], T);
  const float* sig = signal + (size_t)b * T;
  // every key of the chunk in this wave: key u = 64 j + lane
  float ky[ENC_MAXT / 64], kr[ENC_MAXT / 64];
  unsigned long long bal[ENC_MAXT / 64];
#pragma unroll
  for (int j = 0; j < ENC_MAXT / 64; ++j) {
    const int u = 64 * j + lane;
    const float s = sig[max(min(u, L - 1), 0)];
    kr[j] = ln_rsqrt(fmaf(s, fmaf(s, eq.mww, 2.0f * eq.mwb), eq.mbb) + ND_LN_EPS);
    ky[j] = s * kr[j];
    bal[j] = __ballot(u < L && s != 0.0f);
  }
  int n_um = 0;
#pragma unroll
  for (int j = 0; j < ENC_MAXT / 64; ++j) {
    if ((bal[j] >> lane) & 1ull) kyr[n_um + __popcll(bal[j] & ((1ull << lane) - 1ull))] = make_float2(ky[j], kr[j]);
    n_um += __popcll(bal[j]);
  }
  if (n_um == 0 && lane == 0) kyr[0] = make_float2(0.0f, ln_rsqrt(eq.mbb + ND_LN_EPS));  // all masked: s = 0
  const int nk = n_um > 0 ? n_um : 1;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's slab written (its own reads follow in order)
  // this thread's query t: its (y, r) is key t's, held by lane t % 64 as key slot t / 64
  const float y = ky[wave], r = kr[wave];
  if (t < L) {
    // alpha_h, beta_h of this query (log2 units); heads in pairs for packed math
    ef2 al[4], be[4];
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      const float* k = coef + h * 6;
      const float a = fmaf(k[0], y, fmaf(k[1], r, k[2])), bb = fmaf(k[3], y, fmaf(k[4], r, k[5]));
      al[h >> 1][h & 1] = a;
      be[h >> 1][h & 1] = bb;
    }
    ef2 m[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) m[p] = ef2{-INFINITY, -INFINITY};
    for (int u = 0; u < nk; ++u) {
      const float2 k = kyr[u];
      const ef2 kyv = {k.x, k.x}, krv = {k.y, k.y};
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const ef2 l = al[p] * kyv + be[p] * krv;
        m[p] = ef2{fmaxf(m[p].x, l.x), fmaxf(m[p].y, l.y)};
      }
    }
    ef2 sp[4], sy[4], sr[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) sp[p] = sy[p] = sr[p] = ef2{0.f, 0.f};
    for (int u = 0; u < nk; ++u) {
      const float2 k = kyr[u];
      const ef2 kyv = {k.x, k.x}, krv = {k.y, k.y};
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const ef2 d = al[p] * kyv + (be[p] * krv - m[p]);
        const ef2 e = {__builtin_amdgcn_exp2f(d.x), __builtin_amdgcn_exp2f(d.y)};
        sp[p] += e;
        sy[p] += e * kyv;
        sr[p] += e * krv;
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float inv = __builtin_amdgcn_rcpf(sp[p][j]);
        ex[lane][r2_col(lane, 2 * (2 * p + j))] = sy[p][j] * inv;
        ex[lane][r2_col(lane, 2 * (2 * p + j) + 1)] = sr[p][j] * inv;
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's E[y], E[r] staged
  // out[t][32 h + d] = a_v[h][d] E[y] + c_v[h][d] E[r] + b_v[h][d]: the wave's 64 rows, 1 KB each
  const int n = 2 * ND_D + lane * 4, h = lane >> 3;
  const f32x4 av = ld4(eq.ac + n), cv = ld4(eq.ac + 3 * ND_D + n), bv = ld4(eq.bias + n);
  const int q1 = min(64, L - 64 * wave);
  for (int q = 0; q < q1; ++q) {
    const f32x4 o = av * ex[q][r2_col(q, 2 * h)] + cv * ex[q][r2_col(q, 2 * h + 1)] + bv;
    *reinterpret_cast<f32x4*>(out + ((size_t)b * T + 64 * wave + q) * ND_D + lane * 4) = o;
  }
}

hipError_t launch_enc_attention_rank2(const float* signal, const int* span, const EmbedQkv& eq, const float* coef,
                                      float* out, int B, int T, hipStream_t s) {
  if (T > ENC_MAXT || T <= 0 || !eq.ac || !eq.bias || !coef) return hipErrorInvalidValue;
  R2Args a;
  a.signal = signal;
  a.span = span;
  a.eq = eq;
  a.coef = coef;
  a.out = out;
  hipLaunchKernelGGL(enc_attention_rank2_kernel, dim3(B), dim3(512), 0, s, a, T);
  return hipGetLastError();
}


// ------------------------------------------------------------------ decoder
__global__ void __launch_bounds__(256)
dec_embed_kernel(const int* __restrict__ tok, const float* __restrict__ emb, const float* __restrict__ pe, int step,
                 float* __restrict__ x, float* __restrict__ part, int R) {
  // onmt/modules/embeddings.py:189-207 (+ PositionalEncoding.forward :36-43)
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  f32x4 e = ld4(emb + (size_t)tok[row] * ND_D + lane * 4);
  if (pe) e = e * 16.0f + ld4(pe + (size_t)step * ND_D + lane * 4);  // sqrt(256) = 16
  st4(x + pk(row, lane * 4, ND_D), e);  // decoder activations are P16-packed
  if (part) row_part(e, lane, part + (size_t)row * ND_PART_LD * 2);
}

hipError_t launch_dec_embed(const int* tok, const float* emb, const float* pe, int step, float* x, float* part,
                            int R, hipStream_t s) {
  hipLaunchKernelGGL(dec_embed_kernel, dim3((R + 3) / 4), dim3(256), 0, s, tok, emb, pe, step, x, part, R);
  return hipGetLastError();
}

// the layer-0 QKV table's input: row s * V + v = emb[v] (* 16 + pe[s]), the
// same arithmetic as dec_embed_kernel / embed_row (search.hip) for token v
// at step s; rows past S * V are zero (the GEMM's padded row block)
__global__ void __launch_bounds__(256)
dec_embed_table_kernel(const float* __restrict__ emb, const float* __restrict__ pe, int V, int S,
                       float* __restrict__ x, float* __restrict__ part, int rows) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  f32x4 e = {0.f, 0.f, 0.f, 0.f};
  if (row < S * V) {
    const int st = row / V, tk = row - st * V;
    e = ld4(emb + (size_t)tk * ND_D + lane * 4);
    if (pe) e = e * 16.0f + ld4(pe + (size_t)st * ND_D + lane * 4);
  }
  st4(x + pk(row, lane * 4, ND_D), e);
  row_part(e, lane, part + (size_t)row * ND_PART_LD * 2);
}

hipError_t launch_dec_embed_table(const float* emb, const float* pe, int V, int S, float* x, float* part, int rows,
                                  hipStream_t s) {
  if (V < 1 || S < 1 || rows < S * V || rows % 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dec_embed_table_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, emb, pe, V, S, x, part, rows);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Single-pass (flash-decoding) building blocks shared by the decoder's self-
// and context attention.  Lane owns dims 4*lane..4*lane+3 of a 256-wide row
// (head = lane / 8); a wave keeps a running (max m, sum l, acc) per
// (row, head) over the keys it owns, and the waves' partial states merge
// through LDS at the end.  softmax is exp(s - max) / sum as torch computes
// it; masked keys carry the reference's finite -1e18 fill, keys that do not
// exist carry -inf (weight 0).
template <int RPC, int U>
__device__ __forceinline__ void online_update(const float (&s)[RPC][U], const f32x4 (&v)[U], float (&m)[RPC],
                                              float (&l)[RPC], f32x4 (&acc)[RPC]) {
#pragma unroll
  for (int j = 0; j < RPC; ++j) {
    float mx = m[j];
#pragma unroll
    for (int u = 0; u < U; ++u) mx = fmaxf(mx, s[j][u]);  // finite: the block's first key exists
    const float sc = __expf(m[j] - mx);
    acc[j] = acc[j] * sc;
    l[j] *= sc;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float p = __expf(s[j][u] - mx);
      l[j] += p;
      acc[j] += p * v[u];
    }
    m[j] = mx;
  }
}

// The same update with a lazy maximum (flash-attention style): a row's running
// maximum moves only when a score exceeds it by more than tau = 8 (weights up
// to e^8 relative to the kept maximum; (m, l, acc) stay mutually consistent,
// so the merge and the final division are exact).  The rescale (one exp and
// 5 multiplies per row) then runs only on blocks where some row of some lane
// needs it, a wave-uniform branch: after a chunk's first keys, almost never.
template <int RPC, int U>
__device__ __forceinline__ void online_update_lazy(const float (&s)[RPC][U], const f32x4 (&v)[U], float (&m)[RPC],
                                                   float (&l)[RPC], f32x4 (&acc)[RPC]) {
  constexpr float TAU = 8.0f;
  float mxs[RPC];
  bool need = false;
#pragma unroll
  for (int j = 0; j < RPC; ++j) {
    float mx = s[j][0];
#pragma unroll
    for (int u = 1; u < U; ++u) mx = fmaxf(mx, s[j][u]);
    mxs[j] = mx;
    need |= mx > m[j] + TAU;  // m = -inf: any existing key
  }
  if (__builtin_amdgcn_ballot_w64(need)) {
#pragma unroll
    for (int j = 0; j < RPC; ++j) {
      const float mx = fmaxf(m[j], mxs[j]);
      const float sc = __expf(m[j] - mx);  // m = -inf: 0 (acc, l are 0)
      acc[j] = acc[j] * sc;
      l[j] *= sc;
      m[j] = mx;
    }
  }
#pragma unroll
  for (int j = 0; j < RPC; ++j)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float p = __expf(s[j][u] - m[j]);
      l[j] += p;
      acc[j] += p * v[u];
    }
}

// LDS image: accs [NW][RPC][256], ms / ls [NW][RPC][8].  Output rows
// row0 .. row0+RPC-1 of the P16-packed [*, 256] matrix out.
template <int RPC, int NW>
__device__ __forceinline__ void merge_waves(float* accs, float* ms, float* ls, const float (&m)[RPC],
                                            const float (&l)[RPC], const f32x4 (&acc)[RPC], int wave, int lane,
                                            int tid, float* __restrict__ out, int row0) {
#pragma unroll
  for (int j = 0; j < RPC; ++j) {
    st4(accs + ((size_t)wave * RPC + j) * ND_D + lane * 4, acc[j]);
    if ((lane & 7) == 0) {
      ms[(wave * RPC + j) * ND_H + (lane >> 3)] = m[j];
      ls[(wave * RPC + j) * ND_H + (lane >> 3)] = l[j];
    }
  }
  lds_barrier();  // (the self-attention's cache append may still be in flight)
  for (int e = tid; e < RPC * ND_D; e += NW * 64) {
    const int j = e / ND_D, d = e % ND_D, h = d / ND_DH;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, ms[(w * RPC + j) * ND_H + h]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float mw = ms[(w * RPC + j) * ND_H + h];
      const float f = mw == -INFINITY ? 0.f : __expf(mw - M);  // waves that owned no key
      num += f * accs[((size_t)w * RPC + j) * ND_D + d];
      den += f * ls[(w * RPC + j) * ND_H + h];
    }
    out[pk(row0 + j, d & ~3, ND_D) + (d & 3)] = den > 0.f ? num * __builtin_amdgcn_rcpf(den) : 0.f;
  }
}

// merge_waves without the normalisation: per row j the workgroup's partial
// state {num[256], max[8], den[8]} at part + j * CTX_PART (the split
// context attention; ctx_split_merge_kernel combines the splits).
#define CTX_PART (ND_D + 2 * ND_H)
template <int RPC, int NW>
__device__ __forceinline__ void merge_waves_part(float* accs, float* ms, float* ls, const float (&m)[RPC],
                                                 const float (&l)[RPC], const f32x4 (&acc)[RPC], int wave, int lane,
                                                 int tid, float* __restrict__ part) {
#pragma unroll
  for (int j = 0; j < RPC; ++j) {
    st4(accs + ((size_t)wave * RPC + j) * ND_D + lane * 4, acc[j]);
    if ((lane & 7) == 0) {
      ms[(wave * RPC + j) * ND_H + (lane >> 3)] = m[j];
      ls[(wave * RPC + j) * ND_H + (lane >> 3)] = l[j];
    }
  }
  lds_barrier();
  for (int e = tid; e < RPC * ND_D; e += NW * 64) {
    const int j = e / ND_D, d = e % ND_D, h = d / ND_DH;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, ms[(w * RPC + j) * ND_H + h]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float mw = ms[(w * RPC + j) * ND_H + h];
      const float f = mw == -INFINITY ? 0.f : __expf(mw - M);
      num += f * accs[((size_t)w * RPC + j) * ND_D + d];
      den += f * ls[(w * RPC + j) * ND_H + h];
    }
    part[j * CTX_PART + d] = num;
    if ((d & (ND_DH - 1)) == 0) {
      part[j * CTX_PART + ND_D + h] = M;
      part[j * CTX_PART + ND_D + ND_H + h] = den;
    }
  }
}

// Decoder self-attention, one workgroup per row, single pass.
// cache layout: [slot][t][512] = k (256) | v (256), one slot per row; key t
// of row r lives in slot anc[r][t] (beam ancestry; identity when anc is
// null), so beam reordering never moves the cache.  This step's k, v come
// from registers and are appended to the row's own slot
// (multi_headed_attn.py:124-141).  Wave w owns the KW consecutive keys
// w*KW .. w*KW+KW-1 and issues every one of their loads before the first
// score (one memory round trip per step; a loop over key blocks would pay
// one per block), then the NW partial states merge through LDS.
#define SELF_MAXS 512  // max_steps bound (nd_create); the beam rows' kernel holds two lane-indexed slot tables
#define SELF_TABV 8  // vocabulary bound of the head-fused form (its candidate table rows sit in LDS)
// HEAD (greedy, layer 0 in table mode, step > 0): wave 0 first runs the
// previous step's greedy head for the row (head.hpp), whose token picks the
// row's q | k | v in the table; the other waves' cache loads are in flight
// meanwhile.  One launch per step fewer than a standalone head kernel.
// Q24 (round 5; beam rows outside exact fp32, engine.hip enqueue_dec_step; greedy rows keep fp32, which
// measured faster for them; the greedy Q24 form is the op entry's): the cache holds each (slot,
// t) as the 24-bit image of the beam's context K/V (k's 256 integers | v's |
// per head {k scale, v scale}: SELF_Q24_ROW = 1600 B instead of 2 KB,
// common.hpp q24_quant); a lane's key is its 12 bytes of k and of v and its
// head's scales, the step's own key is quantised the same way in registers
// (the one value every later step reads back), and the scores and v are
// dequantised exactly as the context attention does.
#define SELF_Q24_ROW CTXQ_ROW
template <int NW, int KW, bool ANC, bool HEAD, bool Q24>
__global__ void __launch_bounds__(NW * 64)
dec_self_attention_kernel(const float* __restrict__ qkv, float* __restrict__ cache, const int* __restrict__ anc,
                          int anc_ld, int step, int S, float* __restrict__ out, int rpc, const int* __restrict__ skip,
                          int skip_rpc, QkvRows qr, GreedyHead hd, const int* __restrict__ clist) {
#ifdef ND_SKIP_SELF  // timing probe only (tools/build_variant.sh): the kernel's marginal cost
  if (threadIdx.x < 100000) return;
#endif
  __shared__ float accs[NW * ND_D];
  __shared__ float ms[NW * ND_H], ls[NW * ND_H];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // beam rows of a chunk mostly read the same ancestor slots: with rpc > 1
  // (and a chunk count that is a multiple of 8) workgroup b runs chunk
  // 8 (b / 8 / rpc) + b % 8, beam (b / 8) % rpc, so one chunk's rows share an
  // XCD and its L2 serves their common history once
  int r = blockIdx.x;
  if (clist) {  // --fast beam tail: workgroups over the listed chunks only (-1: none)
    const int cc = clist[r / skip_rpc];
    if (cc < 0) return;
    r = cc * skip_rpc + r % skip_rpc;
  } else if (rpc > 1) {
    const int j = r >> 3;
    r = ((j / rpc) * 8 + (r & 7)) * rpc + j % rpc;
  }
  // --fast beam: rows of finished chunks are out of the decode loop
  // (translate/translator.py:793-823 drops their batches)
  if (skip && skip[r / skip_rpc]) return;
  const int n = step + 1;
  // this wave's keys of pass `base`: the cached history (t < step); the
  // step's own key (t == step) and keys past it are patched in below.  The
  // loads are straight-line (t clamped into the history; a branch around
  // each made hipcc wait vmcnt(0) before the next, one round trip per key)
  f32x4 k[KW], v[KW];
  u32v3 kr[KW], vr[KW];  // Q24: the lane's 12 bytes of k and of v
  f32x2 sr[KW];          // Q24: its head's {k scale, v scale}
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  auto load_pass = [&](int base) {
    // Q24: the wave index from an SGPR, so each key's row address is a scalar base plus the lane's constant
    // offsets (its three loads per key otherwise held two 64-bit vector addresses per key in flight and
    // spilled at KW = 16); the fp32 forms keep the vector form, whose schedule has no drain
    const int t0 = base + (Q24 ? wu : wave) * KW, tmax = max(step - 1, 0);
    // slots of this wave's keys (lane u < KW: key t0 + u; beam ancestry)
    int sv = r;
    if constexpr (ANC) sv = anc[(size_t)r * anc_ld + min(t0 + (lane % KW), tmax)];
#pragma unroll
    for (int u = 0; u < KW; ++u) {
      const int t = min(t0 + u, tmax);  // wave-uniform
      const int slot = ANC ? __builtin_amdgcn_readlane(sv, u) : r;
      if constexpr (Q24) {
        // straight into the registers the arithmetic reads (a composed f32x4 made hipcc stage and wait)
        const uint8_t* rb = reinterpret_cast<const uint8_t*>(cache) + ((size_t)slot * S + t) * SELF_Q24_ROW;
        const u32v3* kp = reinterpret_cast<const u32v3*>(rb + 12 * lane);
        const u32v3* vp = reinterpret_cast<const u32v3*>(rb + CTXQ_V + 12 * lane);
        const f32x2* sp = reinterpret_cast<const f32x2*>(rb + CTXQ_S + 8 * (lane >> 3));
        if constexpr (!ANC) {  // non-temporal, as the fp32 form below
          kr[u] = __builtin_nontemporal_load(kp);
          vr[u] = __builtin_nontemporal_load(vp);
          sr[u] = __builtin_nontemporal_load(sp);
        } else {
          kr[u] = *kp;
          vr[u] = *vp;
          sr[u] = *sp;
        }
        continue;
      }
      const float* row = cache + ((size_t)slot * S + t) * 2 * ND_D + lane * 4;
      if constexpr (!ANC) {
        // a greedy row's history is read by that row alone: non-temporal, which leaves the Infinity Cache to
        // the memory bank that every layer re-reads (pooled configs[1] 16.05 / 16.00 -> 15.88 / 15.77 ms per
        // call, same box; beam rows share their ancestors' slots and keep the default policy: non-temporal
        // there cost configs[3] 69.8 -> 71.7 ms)
        k[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row));
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + ND_D));
      } else {
        k[u] = ld4(row);
        v[u] = ld4(row + ND_D);
      }
    }
  };
  // the first pass's cache loads go out before the row's q | k | v, whose
  // address (table mode) waits on the row's token
  // HEAD: wave 0 runs the head before its own cache loads (its registers are
  // then free of the keys: no spill); the other waves first load the step's
  // V candidate table rows (every token the head can pick) for LDS, then
  // their cache loads, so the row's q | k | v is an LDS read once the token
  // is known (not a global round trip after the barrier)
  f32x4 qv, kme, vme;
  if constexpr (HEAD) {
    __shared__ float hlp[ND_MAXV];
    __shared__ int htok;
    __shared__ __attribute__((aligned(16))) float tabs[SELF_TABV * 3 * ND_D];
    if (wu == 0) {
      const int b = greedy_head_row(hd, r, step - 1, lane, hlp);
      if (lane == 0) htok = b;
      load_pass(0);
    } else {
      // V x 192 float4 pieces over (NW - 1) x 64 threads, clamped (straight-line:
      // a load under a branch would make the stores below wait for the cache loads)
      constexpr int TPT = (SELF_TABV * 3 * ND_D / 4 + (NW - 1) * 64 - 1) / ((NW - 1) * 64);
      const int n4 = qr.V * (3 * ND_D / 4), t0 = tid - 64;
      f32x4 tv[TPT];
#pragma unroll
      for (int i = 0; i < TPT; ++i) {
        const int e = min(t0 + i * (NW - 1) * 64, n4 - 1), v = e / (3 * ND_D / 4), c4 = e % (3 * ND_D / 4);
        const int tr = step * qr.V + v;
        tv[i] = ld4(qkv + (qr.rm ? (size_t)tr * 3 * ND_D + 4 * c4 : pk(tr, 4 * c4, 3 * ND_D)));
      }
      load_pass(0);
#pragma unroll
      for (int i = 0; i < TPT; ++i) {
        const int e = min(t0 + i * (NW - 1) * 64, n4 - 1);
        st4(tabs + 4 * e, tv[i]);
      }
    }
    lds_barrier();  // LDS only: the cache loads stay in flight
    const float* trow = tabs + htok * (3 * ND_D);
    qv = ld4(trow + lane * 4) / ND_SQRT_DH;
    kme = ld4(trow + ND_D + lane * 4);
    vme = ld4(trow + 2 * ND_D + lane * 4);
  } else {
    load_pass(0);
    // qkv is P16-packed [R, 768], or the layer-0 table [S * V, 768] (QkvRows)
    const int qrow = qr.tok ? step * qr.V + (step == 0 ? qr.tok0 : qr.tok[r]) : r;
    const float* qr0 = qkv + (qr.rm ? (size_t)qrow * 3 * ND_D + lane * 4 : pk(qrow, lane * 4, 3 * ND_D));
    const size_t qstep = qr.rm ? (size_t)ND_D : pk(0, ND_D, 3 * ND_D);  // q -> k -> v: 256 columns on
    qv = ld4(qr0) / ND_SQRT_DH;
    kme = ld4(qr0 + qstep);
    vme = ld4(qr0 + 2 * qstep);
  }
  if constexpr (Q24) {  // the step's own key as every later step will read it back
    kme = q24_raw(kme);
    vme = q24_raw(vme);
  }
  float m[1] = {-INFINITY}, l[1] = {0.f};
  f32x4 acc[1] = {{0.f, 0.f, 0.f, 0.f}};
  // one pass covers NW * KW keys (every step of max_length <= 128 in one)
  for (int base = 0; base < n; base += NW * KW) {
    if (base > 0) load_pass(base);
    const int t0 = base + wave * KW;
#pragma unroll
    for (int u = 0; u < KW; ++u)
      if (t0 + u >= step) {  // this step's own key (and masked keys past it)
        if constexpr (Q24) {
          kr[u] = u32v3{__float_as_uint(kme.x), __float_as_uint(kme.y), __float_as_uint(kme.z)};
          vr[u] = u32v3{__float_as_uint(vme.x), __float_as_uint(vme.y), __float_as_uint(vme.z)};
          sr[u] = f32x2{kme.w, vme.w};
        } else {
          k[u] = kme;
          v[u] = vme;
        }
      }
    if (t0 < n) {
      float sc[1][KW];
      f32x4 vf[KW];
#pragma unroll
      for (int u = 0; u < KW; ++u) {
        f32x4 kf = k[u];
        float ks = 1.f;
        vf[u] = v[u];
        if constexpr (Q24) {
          kf = q24_unpack(f32x4{__uint_as_float(kr[u].x), __uint_as_float(kr[u].y), __uint_as_float(kr[u].z), 0.f});
          ks = sr[u].x;
          vf[u] = q24_unpack(f32x4{__uint_as_float(vr[u].x), __uint_as_float(vr[u].y), __uint_as_float(vr[u].z), 0.f}) *
                  sr[u].y;
        }
        float d = sum8(qv.x * kf.x + qv.y * kf.y + qv.z * kf.z + qv.w * kf.w);
        if constexpr (Q24) d *= ks;
        sc[0][u] = t0 + u < n ? d : -INFINITY;
      }
      online_update<1, KW>(sc, vf, m, l, acc);
    }
  }
  if (wave == 0) {
    if constexpr (Q24) {
      uint8_t* mine = reinterpret_cast<uint8_t*>(cache) + ((size_t)r * S + step) * SELF_Q24_ROW;
      *reinterpret_cast<u32x3*>(mine + 12 * lane) = u32x3{__float_as_uint(kme.x), __float_as_uint(kme.y),
                                                          __float_as_uint(kme.z)};
      *reinterpret_cast<u32x3*>(mine + CTXQ_V + 12 * lane) = u32x3{__float_as_uint(vme.x), __float_as_uint(vme.y),
                                                                   __float_as_uint(vme.z)};
      if ((lane & 7) == 0) *reinterpret_cast<f32x2*>(mine + CTXQ_S + 8 * (lane >> 3)) = f32x2{kme.w, vme.w};
    } else {
      float* mine = cache + ((size_t)r * S + step) * 2 * ND_D;
      st4(mine + lane * 4, kme);
      st4(mine + ND_D + lane * 4, vme);
    }
  }
  merge_waves<1, NW>(accs, ms, ls, m, l, acc, wave, lane, tid, out, r);
}

// Beam rows (round 5): one workgroup per chunk for its RPC rows.  The rows of
// a chunk are hypotheses that share most of their history (anc[r][t] is the
// same slot for every row until they diverge), so the per-row kernel above
// pulled the same cache lines into up to RPC CUs, once per row.  Here a wave
// walks its keys for all RPC rows at once: the RPC loads of a key that name
// one slot are consecutive instructions of one wave, so the repeats are
// served by the CU's L1.  Per key and row the per-row kernel's scores and
// online softmax, keys one at a time with the next key's loads in flight.
// The rows' own keys (t == step) are appended first (Q24: quantised as the
// per-row kernel does), and after a workgroup barrier every key, the own one
// included, is read from the cache.
// LONG: steps from NW * 64 on (max_length > 256): a second lane-indexed slot table
template <int RPC, int NW, bool Q24, bool LONG>
__global__ void __launch_bounds__(NW * 64)
dec_self_attention_beam_kernel(const float* __restrict__ qkv, float* __restrict__ cache, const int* __restrict__ anc,
                               int anc_ld, int step, int S, float* __restrict__ out, const int* __restrict__ skip,
                               QkvRows qr, const int* __restrict__ clist) {
  __shared__ float accs[NW * RPC * ND_D];
  __shared__ float ms[NW * RPC * ND_H], ls[NW * RPC * ND_H];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = clist ? clist[blockIdx.x] : (int)blockIdx.x;
  if (c < 0 || (skip && skip[c])) return;  // finished chunk (translate/translator.py:793-823)
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  const int n = step + 1;
  // this step's q | k | v of row j: P16 [R, 768] or the layer-0 table (row-major, by the row's token)
  auto qkv_at = [&](int j, int part) -> const float* {
    const int r = c * RPC + j;
    const int qrow = qr.tok ? step * qr.V + (step == 0 ? qr.tok0 : qr.tok[r]) : r;
    return qkv + (qr.rm ? (size_t)qrow * 3 * ND_D + part * ND_D + lane * 4 : pk(qrow, part * ND_D + lane * 4, 3 * ND_D));
  };
  // append every row's k | v at t = step to its own slot
  for (int j = wu; j < RPC; j += NW) {
    const f32x4 kme = ld4(qkv_at(j, 1)), vme = ld4(qkv_at(j, 2));
    const size_t at = (size_t)(c * RPC + j) * S + step;
    if constexpr (Q24) {
      const f32x4 kr = q24_raw(kme), vr = q24_raw(vme);
      uint8_t* mine = reinterpret_cast<uint8_t*>(cache) + at * SELF_Q24_ROW;
      *reinterpret_cast<u32x3*>(mine + 12 * lane) = u32x3{__float_as_uint(kr.x), __float_as_uint(kr.y),
                                                          __float_as_uint(kr.z)};
      *reinterpret_cast<u32x3*>(mine + CTXQ_V + 12 * lane) = u32x3{__float_as_uint(vr.x), __float_as_uint(vr.y),
                                                                   __float_as_uint(vr.z)};
      if ((lane & 7) == 0) *reinterpret_cast<f32x2*>(mine + CTXQ_S + 8 * (lane >> 3)) = f32x2{kr.w, vr.w};
    } else {
      float* mine = cache + at * 2 * ND_D;
      st4(mine + lane * 4, kme);
      st4(mine + ND_D + lane * 4, vme);
    }
  }
  f32x4 qv[RPC], acc[RPC];
  float m[RPC], l[RPC];
#pragma unroll
  for (int j = 0; j < RPC; ++j) {
    qv[j] = ld4(qkv_at(j, 0)) / ND_SQRT_DH;
    acc[j] = {0.f, 0.f, 0.f, 0.f};
    m[j] = -INFINITY;
    l[j] = 0.f;
  }
  // this wave's keys t = wu + NW i: every row's slot for them (t == step: its own slot), key i in lane i & 63
  // of sl (i < 64) or (LONG) sl2 (64 <= i < 128: steps past NW * 64, SELF_MAXS)
  int sl[RPC], sl2[RPC];
  {
    const int t = wu + NW * lane, t2 = t + NW * 64;
#pragma unroll
    for (int j = 0; j < RPC; ++j) {
      const int r = c * RPC + j;
      sl[j] = t < step ? anc[(size_t)r * anc_ld + t] : r;
      if constexpr (LONG) sl2[j] = t2 < step ? anc[(size_t)r * anc_ld + t2] : r;
    }
  }
  static_assert(SELF_MAXS <= NW * 128, "two slot tables of 64 keys per wave");
  // the appends are visible to every wave of the workgroup: each storing wave's stores retired, then a barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // key i of this wave for every row: fp32 k | v, or (Q24) the raw image loaded into the registers the
  // arithmetic reads (12 + 12 bytes and the head's two scales: composing them into one f32x4 per row made
  // hipcc wait for each key's loads right after issuing them)
  struct Key {
    f32x4 k, v;   // fp32 form
    u32v3 kq, vq;  // Q24 form
    f32x2 sq;
  };
  auto load = [&](int i, Key (&kk)[RPC]) {
    const int t = min(wu + NW * i, n - 1);  // wave-uniform; clamped (straight-line loads)
#pragma unroll
    for (int j = 0; j < RPC; ++j) {
      const size_t at = LONG ? (size_t)__builtin_amdgcn_readlane(i < 64 ? sl[j] : sl2[j], i & 63) * S + t
                             : (size_t)__builtin_amdgcn_readlane(sl[j], min(i, 63)) * S + t;
      if constexpr (Q24) {
        const uint8_t* rb = reinterpret_cast<const uint8_t*>(cache) + at * SELF_Q24_ROW;
        kk[j].kq = *reinterpret_cast<const u32v3*>(rb + 12 * lane);
        kk[j].vq = *reinterpret_cast<const u32v3*>(rb + CTXQ_V + 12 * lane);
        kk[j].sq = *reinterpret_cast<const f32x2*>(rb + CTXQ_S + 8 * (lane >> 3));
      } else {
        const float* p = cache + at * 2 * ND_D + lane * 4;
        kk[j].k = ld4(p);
        kk[j].v = ld4(p + ND_D);
      }
    }
  };
  const int nk = wu < n ? (n - 1 - wu) / NW + 1 : 0;  // this wave's keys
  auto update = [&](const Key (&kk)[RPC]) {
#pragma unroll
    for (int j = 0; j < RPC; ++j) {
      f32x4 kf, vf;
      if constexpr (Q24) {
        kf = q24_unpack(f32x4{__uint_as_float(kk[j].kq.x), __uint_as_float(kk[j].kq.y), __uint_as_float(kk[j].kq.z), 0.f});
        vf = q24_unpack(f32x4{__uint_as_float(kk[j].vq.x), __uint_as_float(kk[j].vq.y), __uint_as_float(kk[j].vq.z), 0.f}) *
             kk[j].sq.y;
      } else {
        kf = kk[j].k;
        vf = kk[j].v;
      }
      float d = sum8(qv[j].x * kf.x + qv[j].y * kf.y + qv[j].z * kf.z + qv[j].w * kf.w);
      if constexpr (Q24) d *= kk[j].sq.x;
      const float mx = fmaxf(m[j], d);
      const float sc = __expf(m[j] - mx);  // m = -inf: 0 (acc, l are 0)
      const float p = __expf(d - mx);
      acc[j] = acc[j] * sc + p * vf;
      l[j] = l[j] * sc + p;
      m[j] = mx;
    }
  };
  // two register sets in turn (a copy from one to the other would make hipcc wait for the loads it
  // just issued); the loads past the last key are clamped to it (straight-line) and never used
  Key ka[RPC], kb[RPC];
  if (nk > 0) {
    load(0, ka);
    for (int i = 0; i < nk; i += 2) {
      load(min(i + 1, nk - 1), kb);
      update(ka);
      if (i + 1 >= nk) break;
      load(min(i + 2, nk - 1), ka);
      update(kb);
    }
  }
  merge_waves<RPC, NW>(accs, ms, ls, m, l, acc, wave, lane, tid, out, c * RPC);
}

// the chunk-per-workgroup form for rpc beam rows (ancestry, no fused head)
static bool use_self_beam(const int* anc, int rpc, const GreedyHead* head) { return anc && rpc >= 2 && !head; }

hipError_t launch_dec_self_attention(const float* qkv, float* cache, const int* anc, int anc_ld, int step,
                                     int max_steps, float* out, int R, hipStream_t s, int rpc, const int* skip,
                                     const QkvRows& qr, const GreedyHead* head, const int* clist, int ccap,
                                     bool q24) {
  if (use_self_beam(anc, rpc, head) && R % rpc == 0) {
    if (qr.tok && (qr.V < 1 || qr.tok0 < 0 || qr.tok0 >= qr.V)) return hipErrorInvalidValue;
    if (clist && (ccap < 1 || (long)ccap * rpc > R)) return hipErrorInvalidValue;
    if (step >= max_steps || step >= SELF_MAXS) return hipErrorInvalidValue;
    const int grid = clist ? ccap : R / rpc;
    const bool lng = step >= 4 * 64;  // keys past the first slot table (4 waves x 64 lanes)
    switch (rpc) {
#define ND_SELFB2(RP, Q, L)                                                                                       \
  hipLaunchKernelGGL((dec_self_attention_beam_kernel<RP, 4, Q, L>), dim3(grid), dim3(4 * 64), 0, s, qkv, cache,    \
                     anc, anc_ld, step, max_steps, out, skip, qr, clist)
#define ND_SELFB(RP)                    \
  case RP:                              \
    if (q24 && !lng)                    \
      ND_SELFB2(RP, true, false);       \
    else if (q24)                       \
      ND_SELFB2(RP, true, true);        \
    else if (!lng)                      \
      ND_SELFB2(RP, false, false);      \
    else                                \
      ND_SELFB2(RP, false, true);       \
    break;
      ND_SELFB(2)
      ND_SELFB(3)
      ND_SELFB(4)
      ND_SELFB(5)
      ND_SELFB(6)
      ND_SELFB(7)
      ND_SELFB(8)
#undef ND_SELFB
#undef ND_SELFB2
      default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (qr.tok && (qr.V < 1 || qr.tok0 < 0 || qr.tok0 >= qr.V)) return hipErrorInvalidValue;
  if (head) {
    if (!qr.tok || anc || skip || rpc != 1 || step < 1 || head->V != qr.V || head->V > SELF_TABV ||
        head->S > max_steps)
      return hipErrorInvalidValue;
    const hipError_t e = check_greedy_head(*head);
    if (e != hipSuccess) return e;
  }
  const GreedyHead hd = head ? *head : GreedyHead();
  const int skip_rpc = rpc;
  if (rpc < 2 || R % (8 * rpc)) rpc = 1;
  if (clist && (ccap < 1 || (long)ccap * skip_rpc > R || head)) return hipErrorInvalidValue;
  const int grid = clist ? ccap * skip_rpc : R;
  if (step >= max_steps || step >= SELF_MAXS) return hipErrorInvalidValue;
  const int n = step + 1;
#define ND_SELF3(NW, KW, A, HD, Q)                                                                                \
  hipLaunchKernelGGL((dec_self_attention_kernel<NW, KW, A, HD, Q>), dim3(grid), dim3(NW * 64), 0, s, qkv, cache,   \
                     anc, anc_ld, step, max_steps, out, rpc, skip, skip_rpc, qr, hd, clist)
#define ND_SELF2(NW, KW, A, HD)       \
  do {                                \
    if (q24)                          \
      ND_SELF3(NW, KW, A, HD, true);  \
    else                              \
      ND_SELF3(NW, KW, A, HD, false); \
  } while (0)
#define ND_SELF(NW, KW)                \
  if (anc)                             \
    ND_SELF2(NW, KW, true, false);     \
  else if (head)                       \
    ND_SELF2(NW, KW, false, true);     \
  else                                 \
    ND_SELF2(NW, KW, false, false)
  // 4 waves of up to 16 keys per row up to 64 keys (beam rows: configs[3]
  // pooled 75.62 -> 74.59 ms, one call 94.28 -> 93.60 ms; greedy rows pooled
  // 16.75 / 16.84 -> 16.72 / 16.70 ms), then 8 waves of 16 keys (the 16-wave
  // forms fill a CU's whole register file and shut other pool lanes out:
  // pooled 17.85 -> 17.73 ms per call); round 3-4 same-box A/B pairs
  if (n <= 16) ND_SELF(4, 4);
  else if (n <= 32) ND_SELF(4, 8);
  else if (n <= 64) ND_SELF(4, 16);
  else ND_SELF(8, 16);  // two passes beyond 128 keys
#undef ND_SELF
#undef ND_SELF2
#undef ND_SELF3
  return hipGetLastError();
}

// Context attention, one workgroup (16 waves) per chunk, single pass over
// the chunk's context K/V (flash-decoding): the chunk's K/V stream from HBM
// exactly once for all of its rows (beam rows share the same memory bank,
// translate/translator.py:667-676 tiles it only logically).  Each wave owns
// blocks of U consecutive keys (K and V of a key are one contiguous 2 KB run
// of the ctx K/V row), keeps a running (max, sum, acc) per (row, head) and
// prefetches its next block while computing the current one, so
// 16 waves x 2 blocks x U x 2 KB are in flight per CU.  The 16 partial states
// merge through LDS at the end.  softmax(QK^T/sqrt(d), mask src == pad_idx
// -> -1e18) V as decoder/transformer.py:220-221 + modules/multi_headed_attn.py.
// 8 waves per chunk: the 16-wave form filled a CU's register file (16 x 114
// VGPRs at rpc 5) and shut the other pool lanes out; beam configs[3] pooled
// 83.6 -> 82.1 ms per call, one call 102.2 -> 101.5 ms (two reps, same box,
// tools/_g44.sh); round 2 measured the two forms equal alone.  Round 4: 4
// waves per chunk (more chunks' workgroups per CU beside the other lanes):
// configs[3] pooled 77.3 -> 75.9 ms on one box (profiles/r04_beam_ab.txt)
// Measured and dropped (round 4, profiles/r04_beam_ab.txt): scores in log2
// units, a select-free path for plain key blocks, waves-per-EU hints, 2 / 8 /
// 16 waves per chunk, 4-key blocks above 2 rows per chunk.
#define CTX_NW 4
#define CTX_URPC 2  // rows per chunk up to which a block holds 4 keys (else 2)
#define CTX_UHI 2   // keys per block above CTX_URPC rows
#define CTX_MAXR 8  // beam_size bound (nd_create max_beam; search.hip BEAM_MAX)
template <int RPC>
struct CtxTile {
  static constexpr int U = RPC <= CTX_URPC ? 4 : CTX_UHI;  // keys per block (register budget)
};

// fp32 K/V (exact fp32 calls): K at kv[(c*T + t)*ld + koff], V at + 256.
// The 24-bit image (every other beam call) runs dec_ctx_q24_kernel below.
template <int RPC>
__global__ void __launch_bounds__(CTX_NW * 64)
dec_ctx_attention_kernel(const float* __restrict__ q, const float* __restrict__ kv, int ld, int koff,
                         const float* __restrict__ signal, const int* __restrict__ span, float pad_val,
                         float* __restrict__ out, int T, unsigned long long* stamp, float* __restrict__ dbg,
                         size_t dbg_stride, const int* __restrict__ skip, const int* __restrict__ clist, int nsplit,
                         float* __restrict__ part) {
  // --fast beam tail: workgroups over the listed chunks only (-1: none), nsplit
  // workgroups per chunk (the keys in nsplit ranges; their unnormalised states
  // go to part and ctx_split_merge_kernel combines them)
  const int c = clist ? clist[blockIdx.x / nsplit] : (int)blockIdx.x;
  if (c < 0 || (skip && skip[c])) return;  // finished chunk (--fast beam, translator.py:793-823)
  stamp_begin(stamp);
  constexpr int U = CtxTile<RPC>::U;
  extern __shared__ float sm[];
  float* accs = sm;                              // [NW][RPC][256]
  float* ms = sm + CTX_NW * RPC * ND_D;          // [NW][RPC][8]
  float* ls = ms + CTX_NW * RPC * ND_H;          // [NW][RPC][8]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = min(span[c], T);
  const size_t base = (size_t)c * T;
  const float* sgc = signal + base;
  // lane owns dims 4*lane..4*lane+3 of every row; head = lane / 8
  f32x4 qv[RPC], acc[RPC];
  float m[RPC], l[RPC];
#pragma unroll
  for (int j = 0; j < RPC; ++j) {
    // q, out P16-packed
    qv[j] = ld4(q + pk(c * RPC + j, lane * 4, ND_D)) / ND_SQRT_DH;
    acc[j] = {0.f, 0.f, 0.f, 0.f};
    m[j] = -INFINITY;
    l[j] = 0.f;
  }
  f32x4 kc[U], vc[U];
  float sg[U];
  auto load = [&](int blk, f32x4* kk, f32x4* vv, float* ss) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(blk * U + u, L - 1);
      const float* kvc = kv + (base + t) * ld + koff + lane * 4;
      kk[u] = ld4(kvc);
      vv[u] = ld4(kvc + ND_D);
      ss[u] = sgc[t];
    }
  };
  // this workgroup's key blocks [b0, b1) (all of them unless split)
  const int nblk = (L + U - 1) / U, bps = (nblk + nsplit - 1) / nsplit;
  const int b0 = (blockIdx.x % nsplit) * bps, b1 = min(nblk, b0 + bps);
  int blk = b0 + wave;
  if (blk < b1) load(blk, kc, vc, sg);
  for (; blk < b1; blk += CTX_NW) {
    f32x4 kn[U], vn[U];
    float sn[U];
    const bool more = blk + CTX_NW < b1;
    if (more) load(blk + CTX_NW, kn, vn, sn);
    float sc[RPC][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool valid = blk * U + u < L;
      const bool masked = sg[u] == pad_val;
#pragma unroll
      for (int j = 0; j < RPC; ++j) {
        const float d = sum8(qv[j].x * kc[u].x + qv[j].y * kc[u].y + qv[j].z * kc[u].z + qv[j].w * kc[u].w);
        sc[j][u] = valid ? (masked ? ND_MASK_FILL : d) : -INFINITY;
      }
      // -attn_debug / coverage: head 0 (lanes 0..7 after sum8) of every row of the chunk
      if (dbg && lane == 0 && valid)
#pragma unroll
        for (int j = 0; j < RPC; ++j)  // natural units (the -1e18 fill as it stands)
          dbg[((size_t)c * RPC + j) * dbg_stride + blk * U + u] = sc[j][u];
    }
    online_update_lazy<RPC, U>(sc, vc, m, l, acc);
    if (more) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kc[u] = kn[u];
        vc[u] = vn[u];
        sg[u] = sn[u];
      }
    }
  }
  if (part)
    merge_waves_part<RPC, CTX_NW>(accs, ms, ls, m, l, acc, wave, lane, tid,
                                            part + (size_t)blockIdx.x * RPC * CTX_PART);
  else
    merge_waves<RPC, CTX_NW>(accs, ms, ls, m, l, acc, wave, lane, tid, out, c * RPC);
  stamp_end(stamp);
}

// The 24-bit image (round 4, ctx_pack_q24_kernel below / the K/V GEMM's
// epilogue): per key 1600 B instead of 2 KB; the integers convert exactly to
// fp32 and the per-(key, head) power-of-two scales fold into the score (after
// the head's 8-lane sum) and into v.
//
// Its key rows reach LDS by DMA (round 5).  The round-4 form (the fp32
// kernel above on the image) kept one block of U keys in flight per wave in
// registers (2 x 1600 B at 5 rows: every more key costs 9 VGPRs and the 4th
// wave per SIMD); timed alone at B = 1024 x 5 rows (tools/ctx_time.py) its
// loads by themselves took 158 us (5.3 TB/s), its arithmetic by itself 89
// us, and the kernel 204-211 us: the two barely overlapped.  Here every wave streams its
// blocks through a private ring of CQ_D LDS slots by global_load_lds (no VGPR
// holds a block in flight, no barrier: the wave that copies a block is the
// one that reads it), CQ_P blocks ahead of the one it computes, and waits for
// a block with a counted vmcnt.  The block's rows land in LDS byte for byte
// as in HBM (16-B pieces: row u's bytes at u * 1600), followed by its keys'
// signal samples; the lane reads its 12 bytes of k and of v as three dwords
// each (12-B lane stride: a ds_read_b96 off its 16-B alignment replays) and
// its head's two scales as one b64.  The LDS reads are inline asm: an
// ordinary LDS read after an LDS-DMA makes hipcc wait for every DMA in
// flight (vmcnt(0)), which is the prefetch this kernel exists for.  Same
// arithmetic as the register form, key for key (bitwise equal outputs,
// checked on the GPU before that form was deleted: 493,824 outputs, rpc 1, 2,
// 5, 6, ragged spans).  Alone: 205 -> 195 us; with the layer-major image
// (every chunk's keys of a layer one contiguous run) 172 us (its copies
// alone 150 us); configs[3] pooled 70.0 -> 69.0 ms (profiles/r05_ctx_ab.txt).
#ifndef CQ_P
#define CQ_P 2  // blocks in flight beyond the one computed
#endif
#define CQ_D (CQ_P + 1)  // ring slots per wave
static_assert(CTXQ_ROW % 16 == 0, "16-B pieces");
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) char lds_char_t;
// a block of U keys (the register form's blocking, CtxTile): U rows + their U
// signal samples (16-B aligned); DMA instructions per block
template <int U>
struct CqBlock {
  static constexpr int PIECES = U * CTXQ_ROW / 16;
  static constexpr int SLOT = U * CTXQ_ROW + 16;
  static constexpr int NI = (PIECES + 63) / 64 + 1;
};

template <int OFF>
__device__ __forceinline__ float cq_ld32(uint32_t a) {
  float r;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=&v"(r) : "v"(a), "n"(OFF) : "memory");
  return r;
}
template <int OFF>
__device__ __forceinline__ f32x2 cq_ld64(uint32_t a) {
  f32x2 r;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=&v"(r) : "v"(a), "n"(OFF) : "memory");
  return r;
}
// key u of the slot at sb: the lane's 12 bytes of k and of v (three dwords
// each), its head's two scales, the key's signal sample; every value passes
// through the lgkmcnt wait (the reads land there, not at the asm statements).
// Each call waits for everything the wave has in flight on LDS, so the keys'
// reads go out together only when the caller issues them all first: it
// calls cq_key_issue for every key, then cq_key_land for every key.
struct CqKey {
  float k0, k1, k2, v0, v1, v2, sg;
  f32x2 s;
};
template <int U, int u>
__device__ __forceinline__ void cq_key_issue(CqKey& o, uint32_t a12, uint32_t a8, uint32_t sb) {
  o.k0 = cq_ld32<u * CTXQ_ROW>(a12);
  o.k1 = cq_ld32<u * CTXQ_ROW + 4>(a12);
  o.k2 = cq_ld32<u * CTXQ_ROW + 8>(a12);
  o.v0 = cq_ld32<u * CTXQ_ROW + CTXQ_V>(a12);
  o.v1 = cq_ld32<u * CTXQ_ROW + CTXQ_V + 4>(a12);
  o.v2 = cq_ld32<u * CTXQ_ROW + CTXQ_V + 8>(a12);
  o.s = cq_ld64<u * CTXQ_ROW>(a8);
  o.sg = cq_ld32<U * CTXQ_ROW + 4 * u>(sb);
}
__device__ __forceinline__ void cq_key_land(CqKey& o) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(o.k0), "+v"(o.k1), "+v"(o.k2), "+v"(o.v0), "+v"(o.v1), "+v"(o.v2), "+v"(o.s), "+v"(o.sg)
               :
               : "memory");
}

template <int RPC>
__global__ void __launch_bounds__(CTX_NW * 64)
dec_ctx_q24_kernel(const float* __restrict__ q, const uint8_t* __restrict__ kv, int ld, int koff,
                   const float* __restrict__ signal, const int* __restrict__ span, float pad_val,
                   float* __restrict__ out, int T, unsigned long long* stamp, float* __restrict__ dbg,
                   size_t dbg_stride, const int* __restrict__ skip, const int* __restrict__ clist, int nsplit,
                   float* __restrict__ part) {
  constexpr int U = CtxTile<RPC>::U;
  using BK = CqBlock<U>;
  const int c = clist ? clist[blockIdx.x / nsplit] : (int)blockIdx.x;
  if (c < 0 || (skip && skip[c])) return;  // finished chunk (--fast beam, translator.py:793-823)
  stamp_begin(stamp);
  extern __shared__ __attribute__((aligned(16))) char cq_sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  char* ring = cq_sm + wu * (CQ_D * BK::SLOT);  // this wave's slots
  const int L = min(span[c], T);
  const size_t base = (size_t)c * T;
  const float* sgc = signal + base;
  f32x4 qv[RPC], acc[RPC];
  float m[RPC], l[RPC];
#pragma unroll
  for (int j = 0; j < RPC; ++j) {
    qv[j] = ld4(q + pk(c * RPC + j, lane * 4, ND_D)) / ND_SQRT_DH;
    acc[j] = {0.f, 0.f, 0.f, 0.f};
    m[j] = -INFINITY;
    l[j] = 0.f;
  }
  // q is in registers before the first DMA goes out (its wait stays out of the loop): the values
  // feed an empty statement that no memory operation may cross
#pragma unroll
  for (int j = 0; j < RPC; ++j) asm volatile("" ::"v"(qv[j].x), "v"(qv[j].y), "v"(qv[j].z), "v"(qv[j].w) : "memory");
  // this lane's 16-B piece of each DMA instruction: key pu of the block, byte po of its row
  int pu[BK::NI - 1], po[BK::NI - 1];
#pragma unroll
  for (int j = 0; j < BK::NI - 1; ++j) {
    const int p = min(j * 64 + lane, BK::PIECES - 1);
    pu[j] = p / (CTXQ_ROW / 16);
    po[j] = (p % (CTXQ_ROW / 16)) * 16;
  }
  const uint8_t* kvc = kv + base * ld + koff;
  // block b (keys clamped into the span: the copies stay straight-line) into slot s
  auto issue = [&](int b, int s) {
    char* dst = ring + s * BK::SLOT;
#pragma unroll
    for (int j = 0; j < BK::NI - 1; ++j) {
      const int t = min(b * U + pu[j], L - 1);
      const uint8_t* src = kvc + (size_t)t * ld + po[j];
      if (j < BK::PIECES / 64 || lane < BK::PIECES % 64)
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(dst + j * 1024), 16, 0, 0);
    }
    if (lane < U)
      __builtin_amdgcn_global_load_lds((const void*)(sgc + min(b * U + lane, L - 1)),
                                       (lds_void_t*)(dst + U * CTXQ_ROW), 4, 0, 0);
  };
  const int nblk = (L + U - 1) / U, bps = (nblk + nsplit - 1) / nsplit;
  const int b0 = (blockIdx.x % nsplit) * bps, b1 = min(nblk, b0 + bps);
  int blk = b0 + wu;
  if (blk < b1) {
#pragma unroll
    for (int p = 0; p < CQ_P; ++p) issue(min(blk + p * CTX_NW, b1 - 1), p);
    int slot = 0;
    const uint32_t lbase = (uint32_t)reinterpret_cast<uintptr_t>((lds_char_t*)ring);  // LDS byte address
    for (; blk < b1; blk += CTX_NW) {
      {
        const int s2 = slot + CQ_P;
        issue(min(blk + CQ_P * CTX_NW, b1 - 1), s2 >= CQ_D ? s2 - CQ_D : s2);
      }
      // block blk's copies are the oldest NI of the (CQ_P + 1) NI in flight
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BK::NI * CQ_P) : "memory");
      const uint32_t sb = lbase + (uint32_t)(slot * BK::SLOT);
      const uint32_t a12 = sb + 12 * lane, a8 = sb + CTXQ_S + 8 * (lane >> 3);
      CqKey key[U];
      cq_key_issue<U, 0>(key[0], a12, a8, sb);
      cq_key_issue<U, 1>(key[1], a12, a8, sb);
      if constexpr (U > 2) {
        cq_key_issue<U, 2>(key[2], a12, a8, sb);
        cq_key_issue<U, 3>(key[3], a12, a8, sb);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) cq_key_land(key[u]);
      float sc[RPC][U];
      f32x4 vf[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool valid = blk * U + u < L;
        const bool masked = key[u].sg == pad_val;
        const f32x4 kf = q24_unpack(f32x4{key[u].k0, key[u].k1, key[u].k2, 0.f});
        const float ks = key[u].s.x;
        vf[u] = q24_unpack(f32x4{key[u].v0, key[u].v1, key[u].v2, 0.f}) * key[u].s.y;
#pragma unroll
        for (int j = 0; j < RPC; ++j) {
          const float d = sum8(qv[j].x * kf.x + qv[j].y * kf.y + qv[j].z * kf.z + qv[j].w * kf.w) * ks;
          sc[j][u] = valid ? (masked ? ND_MASK_FILL : d) : -INFINITY;
        }
        if (dbg && lane == 0 && valid)
#pragma unroll
          for (int j = 0; j < RPC; ++j) dbg[((size_t)c * RPC + j) * dbg_stride + blk * U + u] = sc[j][u];
      }
      online_update_lazy<RPC, U>(sc, vf, m, l, acc);
      slot = slot + 1 == CQ_D ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped copies past b1 land before the rings are reused
  }
  __syncthreads();  // every wave is out of its ring: the rings become the merge image
  float* accs = reinterpret_cast<float*>(cq_sm);  // [NW][RPC][256]
  float* ms = accs + CTX_NW * RPC * ND_D;         // [NW][RPC][8]
  float* ls = ms + CTX_NW * RPC * ND_H;           // [NW][RPC][8]
  if (part)
    merge_waves_part<RPC, CTX_NW>(accs, ms, ls, m, l, acc, wave, lane, tid, part + (size_t)blockIdx.x * RPC * CTX_PART);
  else
    merge_waves<RPC, CTX_NW>(accs, ms, ls, m, l, acc, wave, lane, tid, out, c * RPC);
  stamp_end(stamp);
}

static size_t cq_lds_bytes(int rpc) {
  const size_t slot = rpc <= CTX_URPC ? CqBlock<4>::SLOT : CqBlock<CTX_UHI>::SLOT;
  return std::max((size_t)CTX_NW * CQ_D * slot, (size_t)CTX_NW * rpc * (ND_D + 2 * ND_H) * sizeof(float));
}

// The split form's combine: row j of listed chunk b from its nsplit partial
// states {num[256], max[8], den[8]} (one workgroup of 256 threads per row).
__global__ void __launch_bounds__(256)
ctx_split_merge_kernel(const float* __restrict__ part, const int* __restrict__ clist, const int* __restrict__ skip,
                       int nsplit, int rpc, float* __restrict__ out) {
  const int b = blockIdx.x / rpc, j = blockIdx.x % rpc, d = threadIdx.x, h = d / ND_DH;
  const int c = clist[b];
  if (c < 0 || (skip && skip[c])) return;
  const float* p = part + ((size_t)b * nsplit * rpc + j) * CTX_PART;
  const size_t ps = (size_t)rpc * CTX_PART;  // one split's states
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, p[s * ps + ND_D + h]);
  float num = 0.f, den = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float ms = p[s * ps + ND_D + h];
    const float f = ms == -INFINITY ? 0.f : __expf(ms - M);  // a split with no key
    num += f * p[s * ps + d];
    den += f * p[s * ps + ND_D + ND_H + h];
  }
  out[pk(c * rpc + j, d & ~3, ND_D) + (d & 3)] = den > 0.f ? num * __builtin_amdgcn_rcpf(den) : 0.f;
}

// fp32 K/V [M][ld] (layer l's k | v at column l * 512) -> the 24-bit image
// [Ld][M][CTXQ_ROW] bytes: per (layer, key) k's and v's 256 integers
// (3 bytes each, little-endian two's complement, lane-major: lane i's 12
// bytes hold dims 4i..4i+3), then per head {2^(e_k - 23), 2^(e_v - 23)} as
// floats.  e = the head's exponent: max|x| < 2^e, so |x| 2^(23-e) < 2^23 and
// rounding to the nearest integer (clamped to 2^23 - 1) leaves an error of at
// most 2^(e-24) <= 2^-23 max|x| per element (an fp32 value's own rounding is
// 2^-24 |x|; the split-fp16 GEMM that produced K / V carries 2^-22 operands).
// Rows t >= span of their chunk are never read and not written.
// One wave per (key row, layer).
__global__ void __launch_bounds__(256)
ctx_pack_q24_kernel(const float* __restrict__ kv, int ld, int Ld, uint8_t* __restrict__ out,
                    const int* __restrict__ span, int T, int n) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= n) return;
  const int row = w / Ld, layer = w % Ld;
  if (row % T >= min(span[row / T], T)) return;
  const float* src = kv + (size_t)row * ld + (size_t)layer * 2 * ND_D + lane * 4;
  uint8_t* dst = out + ((size_t)layer * (n / Ld) + row) * CTXQ_ROW;  // layer-major planes of n / Ld rows
  float scl[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) scl[h] = q24_quant_store(ld4(src + h * ND_D), dst + h * CTXQ_V + 12 * lane);
  if ((lane & 7) == 0) *reinterpret_cast<f32x2*>(dst + CTXQ_S + 8 * (lane >> 3)) = f32x2{scl[0], scl[1]};
}

hipError_t launch_ctx_pack_q24(const float* kv, int ld, int Ld, uint8_t* out, const int* span, int B, int T,
                               hipStream_t s) {
  if (Ld < 1 || ld < Ld * 2 * ND_D || B < 1 || T < 1) return hipErrorInvalidValue;
  const int n = B * T * Ld;
  hipLaunchKernelGGL(ctx_pack_q24_kernel, dim3((n + 3) / 4), dim3(256), 0, s, kv, ld, Ld, out, span, T, n);
  return hipGetLastError();
}

static size_t ctx_lds_bytes(int rpc) { return (size_t)CTX_NW * rpc * (ND_D + 2 * ND_H) * sizeof(float); }

hipError_t launch_dec_ctx_attention(const float* q, const void* kv, int ld, int koff, const float* signal,
                                    const int* span, float pad_val, float* out, int C, int rpc, int T,
                                    hipStream_t s, unsigned long long* stamp, float* attn_dbg, size_t dbg_stride,
                                    const int* skip, bool q24, const int* clist, int ccap, int nsplit, float* part) {
  if (rpc < 1 || rpc > CTX_MAXR || T > 512) return hipErrorInvalidValue;
  if (clist && (ccap < 1 || ccap > C)) return hipErrorInvalidValue;
  if (!clist || !part || attn_dbg) nsplit = 1;  // the split form runs over a chunk list (the -attn_debug form whole)
  if (nsplit < 1 || nsplit > 64) return hipErrorInvalidValue;
  float* const pout = nsplit > 1 ? part : nullptr;
  const int grid = clist ? ccap * nsplit : C;
  const size_t lds = q24 ? cq_lds_bytes(rpc) : ctx_lds_bytes(rpc);
  switch (rpc) {
#define ND_CTX_CASE(R)                                                                                            \
  case R:                                                                                                         \
    if (q24)                                                                                                      \
      hipLaunchKernelGGL((dec_ctx_q24_kernel<R>), dim3(grid), dim3(CTX_NW * 64), lds, s, q,                       \
                         static_cast<const uint8_t*>(kv), ld, koff, signal, span, pad_val, out, T, stamp,         \
                         attn_dbg, dbg_stride, skip, clist, nsplit, pout);                                        \
    else                                                                                                          \
      hipLaunchKernelGGL((dec_ctx_attention_kernel<R>), dim3(grid), dim3(CTX_NW * 64), lds, s, q,                 \
                         static_cast<const float*>(kv), ld, koff, signal, span, pad_val, out, T, stamp, attn_dbg, \
                         dbg_stride, skip, clist, nsplit, pout);                                                  \
    break;
    ND_CTX_CASE(1)
    ND_CTX_CASE(2)
    ND_CTX_CASE(3)
    ND_CTX_CASE(4)
    ND_CTX_CASE(5)
    ND_CTX_CASE(6)
    ND_CTX_CASE(7)
    ND_CTX_CASE(8)
#undef ND_CTX_CASE
  }
  if (nsplit > 1) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ctx_split_merge_kernel, dim3(ccap * rpc), dim3(ND_D), 0, s, part, clist, skip, nsplit, rpc, out);
  }
  return hipGetLastError();
}

}  // namespace nd

namespace nd {

__global__ void fill_i32_kernel(int* p, int v, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = v;
}

hipError_t launch_fill_i32(int* p, int v, int n, hipStream_t s) {
  hipLaunchKernelGGL(fill_i32_kernel, dim3((n + 255) / 256), dim3(256), 0, s, p, v, n);
  return hipGetLastError();
}

// --fast beam tail: the chunks not yet done, in ascending order, into
// list[0 .. cap) (the rest -1).  One workgroup; a wave ballot per 64 chunks.
// The engine builds it at the start of a tail segment, when at most cap
// chunks are alive (chunks finishing inside the segment are skipped by their
// done flag); more than cap alive sets *ovf (the caller's guard is violated).
__global__ void __launch_bounds__(64)
alive_list_kernel(const int* __restrict__ done, int C, int* __restrict__ list, int cap, int* __restrict__ ovf) {
  const int lane = threadIdx.x;
  int n = 0;
  for (int c0 = 0; c0 < C; c0 += 64) {
    const int c = c0 + lane;
    const bool alive = c < C && done[c] == 0;
    const unsigned long long m = __ballot(alive);
    const int k = n + __popcll(m & ((1ull << lane) - 1ull));
    if (alive && k < cap) list[k] = c;
    n += __popcll(m);
  }
  for (int k = n + lane; k < cap; k += 64) list[k] = -1;
  if (n > cap && lane == 0 && ovf) *ovf = 1;
}

hipError_t launch_alive_list(const int* done, int C, int* list, int cap, int* ovf, hipStream_t s) {
  if (C < 1 || cap < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(alive_list_kernel, dim3(1), dim3(64), 0, s, done, C, list, cap, ovf);
  return hipGetLastError();
}

hipError_t init_kernel_attributes() {
  const void* fns[] = {
      (const void*)dec_ctx_attention_kernel<1>, (const void*)dec_ctx_attention_kernel<2>,
      (const void*)dec_ctx_attention_kernel<3>, (const void*)dec_ctx_attention_kernel<4>,
      (const void*)dec_ctx_attention_kernel<5>, (const void*)dec_ctx_attention_kernel<6>,
      (const void*)dec_ctx_attention_kernel<7>, (const void*)dec_ctx_attention_kernel<8>,
      (const void*)dec_ctx_q24_kernel<1>,              (const void*)dec_ctx_q24_kernel<2>,
      (const void*)dec_ctx_q24_kernel<3>,              (const void*)dec_ctx_q24_kernel<4>,
      (const void*)dec_ctx_q24_kernel<5>,              (const void*)dec_ctx_q24_kernel<6>,
      (const void*)dec_ctx_q24_kernel<7>,              (const void*)dec_ctx_q24_kernel<8>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  {
    hipError_t e = init_mem_attributes();
    if (e != hipSuccess) return e;
  }
  {
    hipError_t e = init_bank8_attributes();
    if (e != hipSuccess) return e;
  }
  return init_gemm_attributes();
}

}  // namespace nd
