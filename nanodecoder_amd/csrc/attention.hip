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
#include "common.hpp"
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

__global__ void __launch_bounds__(256)
enc_embed_kernel(const float* __restrict__ signal, const float* __restrict__ w, const float* __restrict__ b,
                 float* __restrict__ x, float* __restrict__ part, int n_rows) {
  // encoder/transformer.py:104,113 — Linear(1, d) applied to the scalar sample
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const float s = signal[row];
  const f32x4 wv = ld4(w + lane * 4), bv = ld4(b + lane * 4);
  const f32x4 v = s * wv + bv;
  st4(x + (size_t)row * ND_D + lane * 4, v);
  if (part) row_part(v, lane, part + (size_t)row * ND_PART_LD * 2);
}

hipError_t launch_enc_embed(const float* signal, const float* w_in, const float* b_in, float* x, float* part, int B,
                            int T, hipStream_t s) {
  const int rows = B * T;
  hipLaunchKernelGGL(enc_embed_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, signal, w_in, b_in, x, part, rows);
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
  const float rs = 1.0f / sqrtf(var + ND_LN_EPS);
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

hipError_t launch_enc_attention(const float* qkv, const float* signal, const int* span, float* out, int B, int T,
                                hipStream_t s) {
  if (T > ENC_MAXT || T <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(enc_attention_kernel, dim3(ND_H, B), dim3(1024), 0, s, qkv, signal, span, out, T);
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
  st4(x + (size_t)row * ND_D + lane * 4, e);
  if (part) row_part(e, lane, part + (size_t)row * ND_PART_LD * 2);
}

hipError_t launch_dec_embed(const int* tok, const float* emb, const float* pe, int step, float* x, float* part,
                            int R, hipStream_t s) {
  hipLaunchKernelGGL(dec_embed_kernel, dim3((R + 3) / 4), dim3(256), 0, s, tok, emb, pe, step, x, part, R);
  return hipGetLastError();
}

// Decoder self-attention, one workgroup (256 threads = 4 waves) per row.
// cache layout: [slot][t][512] = k (256) | v (256).  Lane owns dims
// 4*lane..4*lane+3 (head = lane/8); waves split the keys, 4 per iteration, so
// every K/V row is one coalesced 1 KB wave load.
#define SELF_MAXS 256
#define SELF_NW 8
__global__ void __launch_bounds__(SELF_NW * 64)
dec_self_attention_kernel(const float* __restrict__ qkv, float* __restrict__ cache, const int* __restrict__ anc,
                          int anc_ld, int step, int S, float* __restrict__ out) {
  __shared__ float p[ND_H][SELF_MAXS];
  __shared__ float part[SELF_NW][ND_D];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* qrow = qkv + (size_t)r * 3 * ND_D;
  const f32x4 q = ld4(qrow + lane * 4) / ND_SQRT_DH;
  const f32x4 kme = ld4(qrow + ND_D + lane * 4), vme = ld4(qrow + 2 * ND_D + lane * 4);
  // append this step's k, v to the row's own slot (multi_headed_attn.py:124-141)
  if (wave == 0) {
    float* mine = cache + ((size_t)r * S + step) * 2 * ND_D;
    st4(mine + lane * 4, kme);
    st4(mine + ND_D + lane * 4, vme);
  }
  const int n = step + 1;
  const int hh = lane >> 3;
  auto krow = [&](int t) -> const float* {
    const int slot = (anc && t < step) ? anc[(size_t)r * anc_ld + t] : r;
    return cache + ((size_t)slot * S + t) * 2 * ND_D;
  };
  // scores: keys t < step come from the cache, key `step` from registers
  for (int t0 = wave; t0 < n; t0 += 4 * SELF_NW) {
    f32x4 k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + SELF_NW * u;
      k[u] = (t < step) ? ld4(krow(t) + lane * 4) : kme;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + SELF_NW * u;
      float d = q.x * k[u].x + q.y * k[u].y + q.z * k[u].z + q.w * k[u].w;
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 4, 64);
      if ((lane & 7) == 0 && t < n) p[hh][t] = d;
    }
  }
  __syncthreads();
  // softmax per head (no mask while stepping): wave w handles heads w, w+4
  for (int h2 = wave; h2 < ND_H; h2 += SELF_NW) {
    float mx = -INFINITY;
    for (int t = lane; t < n; t += 64) mx = fmaxf(mx, p[h2][t]);
    mx = wave_max(mx);
    float sm = 0.f;
    for (int t = lane; t < n; t += 64) {
      const float e = __expf(p[h2][t] - mx);
      p[h2][t] = e;
      sm += e;
    }
    sm = wave_sum(sm);
    const float inv = 1.0f / sm;
    for (int t = lane; t < n; t += 64) p[h2][t] *= inv;
  }
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int t0 = wave; t0 < n; t0 += 4 * SELF_NW) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + SELF_NW * u;
      v[u] = (t < step) ? ld4(krow(t) + ND_D + lane * 4) : vme;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + SELF_NW * u;
      if (t < n) acc += p[hh][t] * v[u];
    }
  }
  st4(&part[wave][lane * 4], acc);
  __syncthreads();
  if (tid < ND_D) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < SELF_NW; ++w) v += part[w][tid];
    out[(size_t)r * ND_D + tid] = v;
  }
}

hipError_t launch_dec_self_attention(const float* qkv, float* cache, const int* anc, int anc_ld, int step,
                                     int max_steps, float* out, int R, hipStream_t s) {
  if (step >= max_steps || step >= SELF_MAXS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dec_self_attention_kernel, dim3(R), dim3(SELF_NW * 64), 0, s, qkv, cache, anc, anc_ld, step, max_steps,
                     out);
  return hipGetLastError();
}

// Context attention, one workgroup (512 threads) per chunk: the chunk's
// context K/V stream from HBM once for all of its rows (beam rows share the
// same memory bank, translate/translator.py:667-676 tiles it only logically).
#define CTX_THREADS 512
#define CTX_MAXR 6
template <int RPC>
__global__ void __launch_bounds__(CTX_THREADS)
dec_ctx_attention_kernel(const float* __restrict__ q, const float* __restrict__ kv, int ld, int koff,
                         const float* __restrict__ signal, const int* __restrict__ span, float pad_val,
                         float* __restrict__ out, int T) {
  constexpr int rpc = RPC;
  extern __shared__ float sm[];
  float* sc = sm;                                   // [rpc][8][T]
  float* part = sm + rpc * ND_H * T;                // [8 waves][rpc][256]
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = min(span[c], T);
  const size_t base = (size_t)c * T;
  // lane owns dims 4*lane..4*lane+3 of every row; head = lane / 8
  f32x4 qv[RPC];
#pragma unroll
  for (int j = 0; j < RPC; ++j) qv[j] = ld4(q + ((size_t)c * rpc + j) * ND_D + lane * 4) / ND_SQRT_DH;
  // pass 1: scores (mask src == pad_idx, decoder/transformer.py:220-221);
  // wave w takes keys w, w+8, ... four at a time so 4 KB are in flight per wave
  constexpr int NW = CTX_THREADS / 64;
  for (int t0 = wave; t0 < L; t0 += 4 * NW) {
    f32x4 k[4];
    bool masked[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = min(t0 + u * NW, L - 1);
      k[u] = ld4(kv + (base + t) * ld + koff + lane * 4);
      masked[u] = signal[base + t] == pad_val;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + u * NW;
#pragma unroll
      for (int j = 0; j < RPC; ++j) {
        float d = qv[j].x * k[u].x + qv[j].y * k[u].y + qv[j].z * k[u].z + qv[j].w * k[u].w;
        d += __shfl_xor(d, 1, 64);
        d += __shfl_xor(d, 2, 64);
        d += __shfl_xor(d, 4, 64);
        if ((lane & 7) == 0 && t < L) sc[(j * ND_H + (lane >> 3)) * T + t] = masked[u] ? ND_MASK_FILL : d;
      }
    }
  }
  __syncthreads();
  // softmax over keys for each (row, head)
  for (int rh = wave; rh < rpc * ND_H; rh += CTX_THREADS / 64) {
    float* s = sc + rh * T;
    float mx = -INFINITY;
    for (int t = lane; t < L; t += 64) mx = fmaxf(mx, s[t]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int t = lane; t < L; t += 64) {
      const float e = __expf(s[t] - mx);
      s[t] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float inv = 1.0f / sum;
    for (int t = lane; t < L; t += 64) s[t] *= inv;
  }
  __syncthreads();
  // pass 2: out[j] = sum_t p[j][head][t] * V[t]
  f32x4 acc[RPC];
#pragma unroll
  for (int j = 0; j < RPC; ++j) acc[j] = {0.f, 0.f, 0.f, 0.f};
  const int hh = lane >> 3;
  for (int t0 = wave; t0 < L; t0 += 4 * NW) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld4(kv + (base + min(t0 + u * NW, L - 1)) * ld + koff + ND_D + lane * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + u * NW;
      if (t < L) {
#pragma unroll
        for (int j = 0; j < RPC; ++j) acc[j] += sc[(j * ND_H + hh) * T + t] * v[u];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RPC; ++j) st4(part + ((size_t)wave * rpc + j) * ND_D + lane * 4, acc[j]);
  __syncthreads();
  for (int e = tid; e < rpc * ND_D; e += CTX_THREADS) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < CTX_THREADS / 64; ++w) v += part[(size_t)w * rpc * ND_D + e];
    out[(size_t)c * rpc * ND_D + e] = v;
  }
}

hipError_t launch_dec_ctx_attention(const float* q, const float* kv, int ld, int koff, const float* signal,
                                    const int* span, float pad_val, float* out, int C, int rpc, int T,
                                    hipStream_t s) {
  if (rpc < 1 || rpc > CTX_MAXR || T > 512) return hipErrorInvalidValue;
  const size_t lds = ((size_t)rpc * ND_H * T + (size_t)(CTX_THREADS / 64) * rpc * ND_D) * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  switch (rpc) {
#define ND_CTX_CASE(R)                                                                                            \
  case R:                                                                                                         \
    hipLaunchKernelGGL(dec_ctx_attention_kernel<R>, dim3(C), dim3(CTX_THREADS), lds, s, q, kv, ld, koff, signal, \
                       span, pad_val, out, T);                                                                    \
    break;
    ND_CTX_CASE(1)
    ND_CTX_CASE(2)
    ND_CTX_CASE(3)
    ND_CTX_CASE(4)
    ND_CTX_CASE(5)
    ND_CTX_CASE(6)
#undef ND_CTX_CASE
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

hipError_t init_kernel_attributes() {
  const void* fns[] = {(const void*)dec_ctx_attention_kernel<1>, (const void*)dec_ctx_attention_kernel<2>,
                       (const void*)dec_ctx_attention_kernel<3>, (const void*)dec_ctx_attention_kernel<4>,
                       (const void*)dec_ctx_attention_kernel<5>, (const void*)dec_ctx_attention_kernel<6>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace nd
