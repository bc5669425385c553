// 24-bit fixed-point memory bank: the greedy decoder's context attention in
// memory-bank form (kernels.hpp launch_dec_bank_d8) on 3 bytes per bank
// element instead of the split-fp16 bank's 4 (mem_attention.hip,
// dec_bank_h3_kernel).  Reference: onmt/modules/multi_headed_attn.py:142-177
// (scores, mask, softmax, context) with the context K/V projections folded
// into the query side (W_qk) and the output side (W_vo) as in the h3 form.
//
// Bank (bank_pack_d8_kernel, once per call): every key row t of the LN'd
// encoder output is m_t = s_t A_t with s_t = max|m_t| / (126 * 2^16) and A_t
// integer, |A_t| <= 126 * 2^16 < 2^23, held as three signed 8-bit digits
// A = a2 2^16 + a1 2^8 + a0 (balanced: a0 = sext8(A), ...; |a2| <= 126).
// Error per element <= 0.75 s_t ~ 2^-23.3 max|m_t|.  Layout: 1 KB fragments
// (chunk, key block kb of 16 keys, dim block db of 64, digit plane), lane l
// holding key 16 kb + (l & 15), dims 64 db + 16 (l >> 4) .. +15; per key s_t,
// per chunk max_t s_t.
//
// S = M q'^T on v_mfma_i32_16x16x64_i8: q' of head h is quantised the same
// way per (chunk, head) in the prologue (sigma_h, digits q2 q1 q0); B1 =
// [q2 | q1] and B2 = [0 | q0] over the 16 columns (8 heads each); five
// products per 64 dims, a2 B1, a2 B2, a1 B1, a0 B1 + a1 B2 (one accumulator:
// a0 q1 and a1 q0 share the weight 2^8), hold every digit product of weight
// >= 2^8 (only a0 q0 dropped), summed exactly in int32 and combined in fp32
// with their power-of-two weights.  Score error on LN-like rows: below a
// plain fp32 dot product's rounding (tests/test_bank_d8_scheme.py).
//
// U = P^T M on f16 MFMAs as in the h3 form, the digits turned into exact f16
// integers (magic-number conversion) from a per-wave transposed LDS image
// read by ds_read_b64_tr_b8: one 16x16x32 product per dim block takes
// [P, P] against [a2 * 2^8 (4 keys), a1 (4 keys)], one 16x16x16 product P
// against a0 * 2^-8.  P is p s_t 2^7 / s_max (s_max: the chunk's largest s_t,
// so <= 2^7 e^6 < 65504) split hi | lo as in the h3 form.
//
// 3 bytes per element: 103.9 MB per launch at 256 chunks against 138.9 MB.
#include "common.hpp"
#include "kernels.hpp"

namespace nd {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 d8h2 __attribute__((ext_vector_type(2)));
typedef _Float16 d8h4 __attribute__((ext_vector_type(4)));
typedef _Float16 d8h8 __attribute__((ext_vector_type(8)));
typedef unsigned d8u2 __attribute__((ext_vector_type(2)));

#define B8_NW 8                          // waves per chunk, 64 keys each
#define B8_KB 32                         // key blocks of 16 per chunk
#define B8_KPW (B8_KB / B8_NW)           // key blocks per wave
#define B8_THR 6.0f                      // lazy-rescale threshold (natural log units), as the h3 form
#define B8_ROW 272                       // bytes per key row of one digit plane in the image (256 + 16)
#define B8_PLANE (16 * B8_ROW)           // one plane of a key block
#define B8_IMG 16384                     // bytes per wave: the 3-plane image (13 KB), then its U partial (16 KB)
#define B8_QD (B8_NW * B8_IMG)           // q' digits [3 planes][8 heads][256 dims]
#define B8_ZERO (B8_QD + 3 * ND_H * ND_D)  // 16 zero bytes (B2 of columns 8..15)
#define B8_SIG (B8_ZERO + 16)            // [8 heads] sigma_h * 2^16
#define B8_ML (B8_SIG + ND_H * 4)        // merge (m, l) [wave][8 heads][2]
#define B8_FW (B8_ML + B8_NW * 16 * 4)   // merge weights [wave][8 heads], then [8 heads] output scales
#define B8_LDS (B8_FW + (B8_NW + 1) * ND_H * 4)
#define B8_AMAX (126.0f * 65536.0f)       // |A| <= 126 * 2^16: |a2| <= 126 after the balanced carries
static_assert(3 * B8_PLANE <= B8_IMG && ND_H * ND_D * 2 * 4 <= B8_IMG, "wave image");
static_assert(B8_LDS <= 160 * 1024, "LDS");

__device__ __forceinline__ int sext8(int x) { return (x << 24) >> 24; }

// the three balanced digits of an integer |A| <= 126 * 2^16 + 1 (|a2| <= 126)
__device__ __forceinline__ void digits(int A, int& d2, int& d1, int& d0) {
  d0 = sext8(A);
  const int A1 = (A - d0) >> 8;
  d1 = sext8(A1);
  d2 = (A1 - d1) >> 8;
}

// x / s for the scale s = max|x| / (126 * 2^16) of its row (or head), rounded to an integer: |result| <=
// 126 * 2^16 + 1 (IEEE division: the quotient's rounding is below the rint's)
__device__ __forceinline__ int fix_q(float x, float s) { return s > 0.f ? (int)rintf(x / s) : 0; }

__device__ __forceinline__ i32x4 mfma_i8(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_d8h32(d8h8 a, d8h8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_d8h16(d8h4 a, d8h4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}

// 4 signed bytes -> 4 exact f16: f16 bits 0x64uu = 1024 + u with u = b + 128
// (b ^ 0x80), minus 1152 (exact); then the plane weight (exact power of two)
__device__ __forceinline__ d8h4 d8_cvt(unsigned x, int plane) {
  const unsigned t = x ^ 0x80808080u;
  const d8h2 lo = __builtin_bit_cast(d8h2, __builtin_amdgcn_perm(0x64646464u, t, 0x04010400u));
  const d8h2 hi = __builtin_bit_cast(d8h2, __builtin_amdgcn_perm(0x64646464u, t, 0x04030402u));
  d8h2 a, b;
  if (plane == 2) {  // a2 * 2^8
    const d8h2 k = {(_Float16)1152.0f, (_Float16)1152.0f}, s = {(_Float16)256.0f, (_Float16)256.0f};
    a = (lo - k) * s;
    b = (hi - k) * s;
  } else if (plane == 1) {  // a1
    const d8h2 k = {(_Float16)1152.0f, (_Float16)1152.0f};
    a = lo - k;
    b = hi - k;
  } else {  // a0 * 2^-8: u / 256 - 4.5 (exact)
    const d8h2 s = {(_Float16)0.00390625f, (_Float16)0.00390625f}, k = {(_Float16)4.5f, (_Float16)4.5f};
    a = lo * s - k;
    b = hi * s - k;
  }
  return d8h4{a.x, a.y, b.x, b.y};
}

// ds_read_b64_tr_b8 (tools/probe_i8.py): per 16-lane group, lane 2q + p
// supplies the address of row q (0..7), bytes 8p .. 8p + 7 of a 16-byte
// column run; lane i receives byte i of the 8 rows
__device__ __forceinline__ d8u2 tr_b8(const char* p) {
  typedef int v2i __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  return __builtin_bit_cast(d8u2, __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)p));
}

template <bool NT>
__device__ __forceinline__ void bank_d8_chunk(int c, const float* __restrict__ qp, const i32x4* __restrict__ bank,
                                              const float* __restrict__ kscale, const int* __restrict__ kemax,
                                              const float* __restrict__ signal, const int* __restrict__ span,
                                              float pad_val, float* __restrict__ out, int T,
                                              unsigned long long* stamp, float* __restrict__ dbg, size_t dbg_stride,
                                              int* ovf, unsigned long long t_entry) {
  extern __shared__ float lds[];
  char* lb = reinterpret_cast<char*>(lds);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  char* img = lb + w * B8_IMG;
  // half block h: key block w + 8 (h >> 1), dim blocks 2 (h & 1) + j (j = 0, 1), planes 2, 1, 0: f[3 j + 2 - pl]
  auto hload = [&](int h, i32x4(&f)[6]) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int db = 2 * (h & 1) + i / 3, pl = 2 - i % 3;
      const i32x4* p = bank + ((((size_t)c * B8_KB + w + B8_NW * (h >> 1)) * 4 + db) * 3 + pl) * 64 + lane;
      if constexpr (NT)
        f[i] = __builtin_nontemporal_load(p);
      else
        f[i] = *p;
    }
  };
  // q' of head w (4 dims per lane), this lane's key scales (keys 16 (w + 8 kb) + 4 g + i), the signal,
  // e_max: then the first half blocks
  const f32x4 qv = ld4(qp + (size_t)c * (ND_H * ND_D) + w * ND_D + 4 * lane);
  f32x4 ksc[B8_KPW];
#pragma unroll
  for (int kb = 0; kb < B8_KPW; ++kb) ksc[kb] = ld4(kscale + (size_t)c * 512 + 16 * (w + B8_NW * kb) + 4 * g);
  float sg;
  {
    const int bkey = 16 * (w + B8_NW * (lane >> 4)) + (lane & 15);  // lane l: row l & 15 of key block w + 8 (l >> 4)
    sg = signal[(size_t)c * T + min(bkey, T - 1)];
  }
  const float smax = __builtin_bit_cast(float, kemax[c]);  // the chunk's largest row scale
  i32x4 F[3][6];
  // issue order = retire order: q' and the scales first, then half block 0, then 1 (a wait for an
  // earlier load leaves the later ones in flight)
  __builtin_amdgcn_sched_barrier(0);
  hload(0, F[0]);
  __builtin_amdgcn_sched_barrier(0);
  hload(1, F[1]);
  __builtin_amdgcn_sched_barrier(0);
  stamp_begin_at(stamp, t_entry);
  const int L = min(span[c], T);
  // q' of head w in digits (every wave one head)
  {
    const float qm = wave_max(absmax4(qv));
    if (!(qm <= 3.0e38f) && ovf != nullptr) ovf[0] = 1;  // non-finite q'
    const float qs = qm * (1.0f / B8_AMAX);
    unsigned pw[3] = {0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int d2, d1, d0;
      digits(fix_q(qv[j], qs), d2, d1, d0);
      pw[2] |= (unsigned)(d2 & 255) << (8 * j);
      pw[1] |= (unsigned)(d1 & 255) << (8 * j);
      pw[0] |= (unsigned)(d0 & 255) << (8 * j);
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<unsigned*>(lb + B8_QD + pl * ND_H * ND_D + w * ND_D + 4 * lane) = pw[pl];
    if (lane == 0) reinterpret_cast<float*>(lb + B8_SIG)[w] = qs * 65536.0f;  // sigma_h * 2^16 (exact)
    if (w == 0 && lane < 4) reinterpret_cast<unsigned*>(lb + B8_ZERO)[lane] = 0u;
  }
  lds_barrier();  // LDS only: the bank loads stay in flight
  // B operands: column col = head col & 7; B1 = q2 (col < 8) | q1, B2 = 0 (col < 8) | q0; dims 64 db + 16 g ..
  i32x4 qb1[4], qb2[4];
  {
    const char* q1p = lb + B8_QD + (col < 8 ? 2 : 1) * ND_H * ND_D + (col & 7) * ND_D + 16 * g;
    const char* q2p = col < 8 ? lb + B8_ZERO : lb + B8_QD + (col & 7) * ND_D + 16 * g;
    const int q2s = col < 8 ? 0 : 64;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      qb1[db] = *reinterpret_cast<const i32x4*>(q1p + 64 * db);
      qb2[db] = *reinterpret_cast<const i32x4*>(q2p + q2s * db);
    }
  }
  const float sgm = reinterpret_cast<const float*>(lb + B8_SIG)[col & 7];
  // digit-product weights (x 2^-16, folded into sgm): X1 = a2 [q2 | q1], X2 = a2 [0 | q0], X3 = a1 [q2 | q1],
  // X4 = a0 [q2 | q1] + a1 [0 | q0]
  const float w1 = col < 8 ? 65536.0f : 256.0f, w2 = col < 8 ? 0.0f : 1.0f, w3 = col < 8 ? 256.0f : 1.0f,
              w4 = col < 8 ? 1.0f : 0.00390625f;
  const float kp = smax > 0.f ? 128.0f / smax : 0.f;  // P scale: p s_t 2^7 / s_max
  const unsigned long long padm = __ballot(sg == pad_val);
  // transposed reads: lane 2q + p of its group supplies row q (keys 4 g + (q & 3)); planes (a2 | a1) at
  // dim block k, or a0 at dim blocks (k | k + 1)
  const int q8 = (lane & 15) >> 1, p8 = lane & 1;
  const char* rb1 = img + (q8 < 4 ? 2 : 1) * B8_PLANE + (4 * g + (q8 & 3)) * B8_ROW + 8 * p8;
  const char* rb3 = img + (4 * g + (q8 & 3)) * B8_ROW + 8 * p8 + (q8 < 4 ? 0 : 16);
  char* wimg = img + col * B8_ROW + 16 * g;  // this lane's fragment row in the image

  f32x4 ua[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) ua[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

#pragma unroll
  for (int kb = 0; kb < B8_KPW; ++kb) {
    i32x4 X1 = {0, 0, 0, 0}, X2 = X1, X3 = X1, X4 = X1;
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const int h = 2 * kb + part;
      i32x4(&f)[6] = F[h % 3];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int db = 2 * part + j;
        X1 = mfma_i8(f[3 * j], qb1[db], X1);
        X2 = mfma_i8(f[3 * j], qb2[db], X2);
        X3 = mfma_i8(f[3 * j + 1], qb1[db], X3);
        X4 = mfma_i8(f[3 * j + 2], qb1[db], X4);
        X4 = mfma_i8(f[3 * j + 1], qb2[db], X4);
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int db = 2 * part + i / 3, pl = 2 - i % 3;
        *reinterpret_cast<i32x4*>(wimg + pl * B8_PLANE + 64 * db) = f[i];
      }
      __builtin_amdgcn_sched_barrier(0);  // the next loads reuse f's registers
      if (h + 2 < 2 * B8_KPW) hload(h + 2, F[(h + 2) % 3]);
    }
    // ---- scores: columns h and h + 8 hold the high and low digit products of head h
    f32x4 s;
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = (float)X1[i] * w1 + (float)X2[i] * w2 + (float)X3[i] * w3 + (float)X4[i] * w4;
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = (s[i] + dpp_mov<0x128>(s[i])) * (ksc[kb][i] * sgm);
    const int kbase = 16 * (w + B8_NW * kb) + 4 * g;  // key of row i
    const unsigned pb = (unsigned)(padm >> (16 * kb + 4 * g)) & 0xFu;
    float gm = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s[i] = kbase + i < L ? (((pb >> i) & 1u) ? ND_MASK_FILL : s[i]) : -INFINITY;
      gm = fmaxf(gm, s[i]);
    }
    if (dbg && col == 0) {  // -attn_debug: head 0's scores
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (kbase + i < L) dbg[(size_t)c * dbg_stride + kbase + i] = s[i];
    }
    gm = xor32_max(xor16_max(gm));
    if (__any(gm > m + B8_THR)) {
      const float nm = fmaxf(m, gm);
      const float sc = nm == m ? 1.f : __expf(m - nm);
      m = nm;
      l *= sc;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float si = __shfl(sc, (lane & 48) | (4 * (g & 1) + i));
#pragma unroll
        for (int k = 0; k < 16; ++k) ua[k][i] *= si;
      }
    }
    f32x4 p;
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = s[i] == -INFINITY ? 0.f : __expf(s[i] - m);
    l += (p[0] + p[1]) + (p[2] + p[3]);
    // ---- A operand of U: row col = (P plane col >> 3, head col & 7), keys 4 g .. 4 g + 3
    d8h4 pa;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = p[i] * (ksc[kb][i] * kp);
      const _Float16 hi = (_Float16)x;
      pa[i] = col < 8 ? hi : (_Float16)(x - (float)hi);
    }
    const d8h8 pa8 = {pa[0], pa[1], pa[2], pa[3], pa[0], pa[1], pa[2], pa[3]};
    // ---- U += P^T M': dim blocks (2 kp, 2 kp + 1) of 16 dims, dims 16 k + col
#pragma unroll
    for (int kp2 = 0; kp2 < 8; ++kp2) {
      const d8u2 r1 = tr_b8(rb1 + 32 * kp2), r2 = tr_b8(rb1 + 32 * kp2 + 16), r3 = tr_b8(rb3 + 32 * kp2);
      const d8h4 b1a = d8_cvt(r1.x, 2), b1b = d8_cvt(r1.y, 1), b2a = d8_cvt(r2.x, 2), b2b = d8_cvt(r2.y, 1);
      const d8h8 b1 = {b1a[0], b1a[1], b1a[2], b1a[3], b1b[0], b1b[1], b1b[2], b1b[3]};
      const d8h8 b2 = {b2a[0], b2a[1], b2a[2], b2a[3], b2b[0], b2b[1], b2b[2], b2b[3]};
      ua[2 * kp2] = mfma_d8h32(pa8, b1, ua[2 * kp2]);
      ua[2 * kp2] = mfma_d8h16(pa, d8_cvt(r3.x, 0), ua[2 * kp2]);
      ua[2 * kp2 + 1] = mfma_d8h32(pa8, b2, ua[2 * kp2 + 1]);
      ua[2 * kp2 + 1] = mfma_d8h16(pa, d8_cvt(r3.y, 0), ua[2 * kp2 + 1]);
    }
  }

  // ---- merge the 8 waves (as dec_bank_h3_kernel): unmerged U^T fragments to the wave's own image, (m, l)
  //      beside, wave 0 turns them into merge weights and the output scale 2 s_max / den
  l = xor32_sum(xor16_sum(l));
  float* ml = reinterpret_cast<float*>(lb + B8_ML);  // [wave][8 heads][2]
  {
    f32x4* red = reinterpret_cast<f32x4*>(img);
#pragma unroll
    for (int k = 0; k < 16; ++k) red[k * 64 + lane] = ua[k];
  }
  if (lane < 8) {
    ml[(w * ND_H + lane) * 2] = m;
    ml[(w * ND_H + lane) * 2 + 1] = l;
  }
  __syncthreads();
  float* fw = reinterpret_cast<float*>(lb + B8_FW);  // [wave][8 heads] weights, then [8 heads] output scales
  if (w == 0) {
    const int v = lane >> 3, hh = lane & 7;
    const float mv = ml[(v * ND_H + hh) * 2], lv = ml[(v * ND_H + hh) * 2 + 1];
    float M = fmaxf(mv, __shfl_xor(mv, 8, 64));
    M = fmaxf(M, __shfl_xor(M, 16, 64));
    M = fmaxf(M, __shfl_xor(M, 32, 64));
    const float f = mv == -INFINITY ? 0.f : __expf(mv - M);  // waves that owned no key
    float den = f * lv;
    den += __shfl_xor(den, 8, 64);
    den += __shfl_xor(den, 16, 64);
    den += __shfl_xor(den, 32, 64);
    fw[v * ND_H + hh] = f;
    if (v == 0) fw[B8_NW * ND_H + hh] = den > 0.f ? __builtin_amdgcn_rcpf(den) * (2.0f * smax) : 0.f;
  }
  lds_barrier();
#pragma unroll
  for (int e = threadIdx.x; e < 512; e += B8_NW * 64) {
    const int hs = e >> 8, d = e & 255, k = d >> 4, cl = d & 15;
    const int lh = k * 64 + cl + 16 * hs, ll = k * 64 + cl + 16 * (2 + hs);  // P hi rows g = hs, lo rows g = 2 + hs
    f32x4 num = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < B8_NW; ++v) {
      const f32x4* red = reinterpret_cast<const f32x4*>(lb + v * B8_IMG);
      num += ld4(fw + v * ND_H + 4 * hs) * (red[lh] + red[ll]);
    }
    num *= ld4(fw + B8_NW * ND_H + 4 * hs);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = (4 * hs + i) * ND_D + d;
      out[pk(c, n & ~3, ND_H * ND_D) + (n & 3)] = num[i];
    }
  }
}

template <bool NT, bool WALK>
__global__ void __launch_bounds__(B8_NW * 64)
dec_bank_d8_kernel(const float* __restrict__ qp, const i32x4* __restrict__ bank, const float* __restrict__ kscale,
                   const int* __restrict__ kemax, const float* __restrict__ signal, const int* __restrict__ span,
                   float pad_val, float* __restrict__ out, int T, int C, unsigned long long* stamp,
                   float* __restrict__ dbg, size_t dbg_stride, int* ovf) {
#ifdef ND_SKIP_BANK  // timing probe only (tools/build_variant.sh, tools/marginal.sh): the kernel's marginal cost
  if (threadIdx.x < 100000) return;
#endif
  const unsigned long long t_entry = wall_clock64();
  if constexpr (WALK) {
    for (int c = blockIdx.x; c < C; c += gridDim.x) {
      if (c != (int)blockIdx.x) lds_barrier();  // the previous chunk's merge reads of LDS are done
      bank_d8_chunk<NT>(c, qp, bank, kscale, kemax, signal, span, pad_val, out, T, stamp, dbg, dbg_stride, ovf,
                        t_entry);
    }
  } else {
    bank_d8_chunk<NT>(blockIdx.x, qp, bank, kscale, kemax, signal, span, pad_val, out, T, stamp, dbg, dbg_stride, ovf,
                      t_entry);
  }
  stamp_end(stamp);
}

// Encoder output -> the 24-bit digit bank: one workgroup per (chunk, key
// block of 16 rows): LayerNorm (as bank_pack_h3_kernel), per row the scale
// s_t and the digits into LDS, then the 12 fragments as coalesced 1 KB
// stores; the row scales and the chunk's largest (atomicMax on the float's
// bits, non-negative; kemax zeroed by the caller).  Rows t >= T, and rows at
// or past the chunk's span (never attended; the encoder leaves them
// unspecified), are zero with scale 0, so s_max is a function of the
// attended rows alone.
__global__ void __launch_bounds__(256)
bank_pack_d8_kernel(const float* __restrict__ x, const float* __restrict__ gm, const float* __restrict__ bt,
                    i32x4* __restrict__ bank, float* __restrict__ kscale, int* __restrict__ kemax,
                    const int* __restrict__ span, int T, int* ovf) {
  __shared__ __attribute__((aligned(16))) unsigned char dg[3][16][ND_D];
  const int c = blockIdx.x / B8_KB, kb = blockIdx.x % B8_KB, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int L = span ? min(span[c], T) : T;
  float smx = 0.f;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = wv + 4 * rr, t = 16 * kb + r;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (t < L) {
      v = ld4(x + ((size_t)c * T + t) * ND_D + lane * 4);
      if (gm) {
        const float mu = wave_sum(v.x + v.y + v.z + v.w) * (1.0f / ND_D);
        const f32x4 d = v - mu;
        const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / ND_D);
        v = d * ln_rsqrt(var + ND_LN_EPS) * ld4(gm + lane * 4) + ld4(bt + lane * 4);
      }
    }
    const float mx = wave_max(absmax4(v));
    if (!(mx <= 3.0e38f) && ovf != nullptr) ovf[0] = 1;  // non-finite encoder output
    const float st = mx * (1.0f / B8_AMAX);
    unsigned pw[3] = {0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int d2, d1, d0;
      digits(fix_q(v[j], st), d2, d1, d0);
      pw[2] |= (unsigned)(d2 & 255) << (8 * j);
      pw[1] |= (unsigned)(d1 & 255) << (8 * j);
      pw[0] |= (unsigned)(d0 & 255) << (8 * j);
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<unsigned*>(&dg[pl][r][4 * lane]) = pw[pl];
    if (lane == 0) kscale[(size_t)c * 512 + t] = st;
    smx = fmaxf(smx, st);
  }
  if (lane == 0) atomicMax(kemax + c, __builtin_bit_cast(int, smx));  // non-negative floats order as ints
  __syncthreads();
  // fragment (db, pl): lane ln holds key ln & 15, dims 64 db + 16 (ln >> 4) .. +15
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int item = threadIdx.x + 256 * j, fr = item >> 6, ln = item & 63, db = fr / 3, pl = fr % 3;
    bank[((((size_t)c * B8_KB + kb) * 4 + db) * 3 + pl) * 64 + ln] =
        *reinterpret_cast<const i32x4*>(&dg[pl][ln & 15][64 * db + 16 * (ln >> 4)]);
  }
}

hipError_t launch_bank_pack_d8(const float* x, const float* ln_g, const float* ln_b, void* bank, float* kscale,
                               int* kemax, const int* span, int B, int T, int* ovf, hipStream_t s) {
  if (T < 1 || T > 512 || B < 1 || !bank || !kscale || !kemax) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(kemax, 0, (size_t)B * sizeof(int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(bank_pack_d8_kernel, dim3(B * B8_KB), dim3(256), 0, s, x, ln_g, ln_b,
                     reinterpret_cast<i32x4*>(bank), kscale, kemax, span, T, ovf);
  return hipGetLastError();
}

hipError_t launch_dec_bank_d8(const float* qp, const void* bank, const float* kscale, const int* kemax,
                              const float* signal, const int* span, float pad_val, float* out, int C, int T,
                              hipStream_t s, unsigned long long* stamp, float* attn_dbg, size_t dbg_stride, int* ovf,
                              bool nt, int grid) {
  if (T < 1 || T > 512 || C < 1 || grid < 0 || !bank || !kscale || !kemax) return hipErrorInvalidValue;
  const int G = grid > 0 ? std::min(C, grid) : C;
#define ND_BANK8_GO(N, W)                                                                                         \
  hipLaunchKernelGGL((dec_bank_d8_kernel<N, W>), dim3(G), dim3(B8_NW * 64), B8_LDS, s, qp,                       \
                     reinterpret_cast<const i32x4*>(bank), kscale, kemax, signal, span, pad_val, out, T, C, stamp,  \
                     attn_dbg, dbg_stride, ovf)
  if (G < C) {
    if (nt)
      ND_BANK8_GO(true, true);
    else
      ND_BANK8_GO(false, true);
  } else if (nt) {
    ND_BANK8_GO(true, false);
  } else {
    ND_BANK8_GO(false, false);
  }
#undef ND_BANK8_GO
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// --fast beam rows in memory-bank form (translate/translator.py:700-823 runs
// the decoder on beam x batch rows; decoder/transformer.py:178-189 their
// context attention): the RPC (2..6) rows of a chunk share ONE pass over the
// chunk's digit bank, against the K/V form's 1 MB per chunk.
//  - The chunk's key blocks (12 KB each: 4 dim blocks x 3 planes of 1 KB
//    fragments) stream through a 3-slot LDS ring by buffer_load ... lds
//    (waves 0..5 copy two fragments each), two blocks ahead; slots are 1152 B
//    apart so the a2 and a1 planes of a dim block sit on opposite bank halves
//    for the transposed reads.
//  - Scores: wave p < ceil(RPC / 2) owns the row pair (2p, 2p + 1): its 16
//    MFMA columns are (row 2p + (col >> 3), head col & 7), so every column
//    carries a score (the one-row form duplicates each head over a column
//    pair).  Eight i8 products per 64 dims on the block from LDS, grouped by
//    digit weight into four exact int32 sums: a2 q2 (2^16); a2 q1 + a1 q2
//    (2^8); a2 q0 + a1 q1 + a0 q2 (1); a1 q0 + a0 q1 (2^-8) -- the digit
//    products the greedy form keeps (only a0 q0 dropped).  Then the lazy
//    online softmax per column and P (hi | lo f16, the U A-operand layout) and
//    the rescale factors to LDS.
//  - Context: every wave owns two 16-dim blocks of U for ALL rows (row pair
//    b = MFMA rows 0..15 of accumulator block b), converts only those digits
//    (tr_b8 + the exact f16 conversion) and runs two 16x16x32 products
//    ([hi | lo] against [a2 | a2] and [a1 | a1]) and one 16x16x16 (hi against
//    a0) per pair: no U merge across waves, the digits of a block converted
//    once per workgroup.
// Output U [C * RPC, 2048] P16 (row c * RPC + j), as dec_bank_d8_kernel's.
#define BB_NW 8
#define BB_MAXR 6
#define BB_MAXP 3                          // row pairs
#ifndef BB_EXPT
#define BB_EXPT 0  // timing probes only (tools/bb_time.py with a variant library): 1 no score MFMAs,
                   // 2 no context MFMAs, 4 no key-block copies (stale LDS), 8 no softmax / P VALU
#endif
#ifndef BB_WPE
#define BB_WPE 4                           // waves per SIMD: two workgroups per CU (128 VGPRs)
#endif
#define BB_FR 1152                         // LDS bytes per 1 KB fragment slot
#define BB_BLK (12 * BB_FR)                // one key block
#define BB_NBUF 3                          // ring slots
#define BB_KS (BB_NBUF * BB_BLK)           // [512] row scales s_t
#define BB_PM (BB_KS + 512 * 4)            // [512] pad flags (bytes)
#define BB_P (BB_PM + 512)                 // [pair][4 key groups][16 columns] P hi x 4 | lo x 4 (16 B)
#define BB_SC (BB_P + BB_MAXP * 1024)      // [pair][16 columns] rescale factors of the current block
#define BB_FIN (BB_SC + BB_MAXP * 16 * 4)  // [pair][16 columns] output scales 2 s_max / l
#define BB_LDS (BB_FIN + BB_MAXP * 16 * 4)
static_assert(BB_LDS <= 65536, "beam bank LDS within 64 KB (DESIGN.md section 5, co-residency rule)");

template <int RPC>
__device__ __forceinline__ void bank_d8_beam_chunk(char* lb, int c, const float* __restrict__ qp, const char* bank,
                                                   const float* __restrict__ kscale, const int* __restrict__ kemax,
                                                   const float* __restrict__ signal, const int* __restrict__ span,
                                                   float pad_val, float* __restrict__ out, int T, int* ovf) {
  constexpr int NP = (RPC + 1) / 2;  // row pairs = score waves = U accumulator blocks
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int L = min(span[c], T);
  const int nkb = (L + 15) >> 4;  // key blocks holding a key < L
  const float smax = __builtin_bit_cast(float, kemax[c]);
  const __amdgpu_buffer_rsrc_t src = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(bank) + (size_t)c * (B8_KB * 12 * 1024), 0, B8_KB * 12 * 1024, 0x00020000);
  // key block kb -> ring slot kb % 3: waves 0..5 copy fragments 2w, 2w + 1 (db * 3 + plane)
  auto issue = [&](int kb) {
    if ((BB_EXPT & 4) == 0 && w < 6) {
      char* dst = lb + (kb % BB_NBUF) * BB_BLK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int f = 2 * w + i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (__attribute__((address_space(3))) void*)(dst + f * BB_FR), 16,
                                                 lane * 16, kb * 12288 + f * 1024, 0, 0);
      }
    }
  };
  // ---- prologue: the first two key blocks, then every prologue load at once (one memory round trip):
  //      this lane's q' (row 2 w + (col >> 3), head col & 7, dims 64 db + 16 g + 4 i ..; P16 [R][2048]),
  //      the chunk's row scales and pad flags (one key per thread)
  const int jq = 2 * w + (col >> 3);  // this lane's row (score waves)
  const bool rowq = w < NP && jq < RPC;
  if (nkb > 0) issue(0);
  if (nkb > 1) issue(1);
  const float* qrow = qp + pk(c * RPC + (rowq ? jq : 0), (col & 7) * ND_D + 16 * g, ND_H * ND_D);
  f32x4 qv[16];
  if (w < NP) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      qv[k] = rowq ? ld4(qrow + pk(0, 64 * (k >> 2) + 4 * (k & 3), ND_H * ND_D)) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int tk = threadIdx.x;  // 512 threads, 512 keys
  const float ksv = kscale[(size_t)c * 512 + tk];
  const float sgv = signal[(size_t)c * T + min(tk, T - 1)];
  reinterpret_cast<float*>(lb + BB_KS)[tk] = ksv;
  reinterpret_cast<unsigned char*>(lb + BB_PM)[tk] = (tk < T && sgv == pad_val) ? 1 : 0;
  // B operands of the scores: the three digit planes of this lane's column
  i32x4 qd[3][4];
  float sgm = 0.f;
  if (w < NP) {
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) mx = fmaxf(mx, absmax4(qv[k]));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (!(mx <= 3.0e38f) && ovf != nullptr) ovf[0] = 1;  // non-finite q'
    const float qs = mx * (1.0f / B8_AMAX);
    const float qdiv = qs > 0.f ? qs : 1.0f;  // a zero head is all zeros: x / 1 = 0 (fix_q without its branch)
    sgm = qs * 65536.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      unsigned u2 = 0u, u1 = 0u, u0 = 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int d2, d1, d0;
        digits((int)rintf(qv[k][e] / qdiv), d2, d1, d0);
        u2 |= (unsigned)(d2 & 255) << (8 * e);
        u1 |= (unsigned)(d1 & 255) << (8 * e);
        u0 |= (unsigned)(d0 & 255) << (8 * e);
      }
      qd[2][k >> 2][k & 3] = (int)u2;
      qd[1][k >> 2][k & 3] = (int)u1;
      qd[0][k >> 2][k & 3] = (int)u0;
      __builtin_amdgcn_sched_barrier(0);  // four values at a time (the divisions' temporaries)
    }
  }
  const float kp = smax > 0.f ? 128.0f / smax : 0.f;  // P scale: p s_t 2^7 / s_max
  // ---- this wave's U dim blocks 2w, 2w + 1 (dim block db_u, 16-dim groups G0, G0 + 1) in the transposed
  //      reads: lane 2q + p of its group supplies row q (keys 4 g + (q & 3); planes a2 | a1, or a0 of G0 | G0 + 1)
  const int db_u = w >> 1, G0 = 2 * (w & 1);
  const int q8 = (lane & 15) >> 1, p8 = lane & 1;
  const int o1 = (db_u * 3 + (q8 < 4 ? 2 : 1)) * BB_FR + (4 * g + (q8 & 3) + 16 * G0) * 16 + 8 * p8;
  const int o3 = db_u * 3 * BB_FR + (4 * g + (q8 & 3) + 16 * (G0 + (q8 < 4 ? 0 : 1))) * 16 + 8 * p8;
  // U accumulators: block b = row pair b (MFMA rows = columns of the pair's scores); P's hi and lo parts
  // ride in the K dimension against the same digits twice
  f32x4 ua[NP][2];
#pragma unroll
  for (int b = 0; b < NP; ++b) ua[b][0] = ua[b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  for (int kb = 0; kb < nkb; ++kb) {
    // block kb landed (this wave's copies; the barrier: everyone's), and every wave is done with
    // block kb - 1 (its ring slot takes block kb + 2)
    if (kb + 1 < nkb)
      asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kb + 2 < nkb) issue(kb + 2);
    const char* buf = lb + (kb % BB_NBUF) * BB_BLK;
    if (w < NP) {
      // ---- scores of row pair w, grouped by digit weight (x 2^-16): X1 2^16, X2 2^8, X3 1, X4 2^-8
      i32x4 X1 = {0, 0, 0, 0}, X2 = X1, X3 = X1, X4 = X1;
      const char* fb = buf + lane * 16;
      // the next dim block's fragments load under this one's products; the products alternate between
      // the four accumulators (a dependent MFMA waits for its predecessor's result)
      i32x4 fr[2][3];
      auto fload = [&](int db, i32x4(&f)[3]) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) f[pl] = *reinterpret_cast<const i32x4*>(fb + (db * 3 + pl) * BB_FR);
      };
      fload(0, fr[0]);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        if (db < 3) fload(db + 1, fr[(db + 1) & 1]);
        const i32x4(&f)[3] = fr[db & 1];
        if (BB_EXPT & 1) {
          X1 += f[2];
          X2 += f[1];
          X3 += f[0];
          continue;
        }
        X1 = mfma_i8(f[2], qd[2][db], X1);
        X2 = mfma_i8(f[2], qd[1][db], X2);
        X3 = mfma_i8(f[2], qd[0][db], X3);
        X4 = mfma_i8(f[1], qd[0][db], X4);
        X2 = mfma_i8(f[1], qd[2][db], X2);
        X3 = mfma_i8(f[1], qd[1][db], X3);
        X4 = mfma_i8(f[0], qd[1][db], X4);
        X3 = mfma_i8(f[0], qd[2][db], X3);
        __builtin_amdgcn_sched_barrier(0);  // two dim blocks' fragments live at most (registers)
      }
      const f32x4 ks4 = *reinterpret_cast<const f32x4*>(lb + BB_KS + (16 * kb + 4 * g) * 4);
      const unsigned pf = *reinterpret_cast<const unsigned*>(lb + BB_PM + 16 * kb + 4 * g);
      const int kbase = 16 * kb + 4 * g;  // key of row i
      f32x4 s;
      float gm = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = fmaf((float)X1[i], 65536.0f, fmaf((float)X2[i], 256.0f, fmaf((float)X4[i], 0.00390625f,
                                                                                   (float)X3[i])));
        s[i] = v * (ks4[i] * sgm);
        s[i] = kbase + i < L ? (((pf >> (8 * i)) & 1u) ? ND_MASK_FILL : s[i]) : -INFINITY;
        gm = fmaxf(gm, s[i]);
      }
      gm = xor32_max(xor16_max(gm));
      const bool resc = __any(gm > m + B8_THR);  // wave-uniform
      float sc = 1.f;
      if (resc) {
        const float nm = fmaxf(m, gm);
        sc = nm == m ? 1.f : __expf(m - nm);
        m = nm;
        l *= sc;
      }
      // every block (1 when this column did not rescale): the accumulators rescale unconditionally
      if (g == 0) reinterpret_cast<float*>(lb + BB_SC)[w * 16 + col] = sc;
      f32x4 p;
#pragma unroll
      for (int i = 0; i < 4; ++i) p[i] = s[i] == -INFINITY ? 0.f : __expf(s[i] - m);
      l += (p[0] + p[1]) + (p[2] + p[3]);
      // the U A operand of column col, keys 4 g .. 4 g + 3: hi x 4 | lo x 4 at P[pair][g][col]
      d8h8 pa;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = p[i] * (ks4[i] * kp);
        const _Float16 hi = (_Float16)x;
        pa[i] = hi;
        pa[4 + i] = (_Float16)(x - (float)hi);
      }
      *reinterpret_cast<d8h8*>(lb + BB_P + w * 1024 + (g * 16 + col) * 16) = pa;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // P, rescale factors visible
    // ---- U += P^T M' for every row pair on this wave's two dim blocks
    const d8u2 r1 = tr_b8(buf + o1), r2 = tr_b8(buf + o1 + 256), r3 = tr_b8(buf + o3);
    const d8h4 c2a = d8_cvt(r1.x, 2), c1a = d8_cvt(r1.y, 1), c2b = d8_cvt(r2.x, 2), c1b = d8_cvt(r2.y, 1);
    const d8h8 b2a = {c2a[0], c2a[1], c2a[2], c2a[3], c2a[0], c2a[1], c2a[2], c2a[3]};  // [a2 | a2] 2^8
    const d8h8 b1a = {c1a[0], c1a[1], c1a[2], c1a[3], c1a[0], c1a[1], c1a[2], c1a[3]};  // [a1 | a1]
    const d8h8 b2b = {c2b[0], c2b[1], c2b[2], c2b[3], c2b[0], c2b[1], c2b[2], c2b[3]};
    const d8h8 b1b = {c1b[0], c1b[1], c1b[2], c1b[3], c1b[0], c1b[1], c1b[2], c1b[3]};
    const d8h4 b0a = d8_cvt(r3.x, 0), b0b = d8_cvt(r3.y, 0);  // a0 2^-8 (the hi parts only)
#pragma unroll
    for (int b = 0; b < NP; ++b) {
      // the running-maximum rescale, every block (factor 1 when the column did not rescale).  Branch-free
      // on purpose: a branch around these multiplies gave wrong components 0, 1 of the second dim
      // block's accumulator on gfx950 (tools/bb_debug.py; cause not isolated, this form is exact).
      // Accumulator rows 4 g + i = columns 4 g + i of the pair's scores
      const f32x4 sc4 = *reinterpret_cast<const f32x4*>(lb + BB_SC + b * 64 + 16 * g);
      ua[b][0] *= sc4;
      ua[b][1] *= sc4;
      const d8h8 pa = *reinterpret_cast<const d8h8*>(lb + BB_P + b * 1024 + (g * 16 + col) * 16);
      const d8h4 ph = {pa[0], pa[1], pa[2], pa[3]};
      if (BB_EXPT & 2) {
        ua[b][0] += f32x4{(float)pa[0], (float)b2a[1], (float)b1a[2], (float)b0a[3]};
        ua[b][1] += f32x4{(float)pa[1], (float)b2b[1], (float)b1b[2], (float)b0b[3]};
        continue;
      }
      ua[b][0] = mfma_d8h32(pa, b2a, ua[b][0]);
      ua[b][1] = mfma_d8h32(pa, b2b, ua[b][1]);
      ua[b][0] = mfma_d8h32(pa, b1a, ua[b][0]);
      ua[b][1] = mfma_d8h32(pa, b1b, ua[b][1]);
      ua[b][0] = mfma_d8h16(ph, b0a, ua[b][0]);
      ua[b][1] = mfma_d8h16(ph, b0b, ua[b][1]);
    }
  }
  // ---- output scales 2 s_max / l per column; U [row][h * 256 + d] P16
  if (w < NP) {
    l = xor32_sum(xor16_sum(l));
    if (g == 0)
      reinterpret_cast<float*>(lb + BB_FIN)[w * 16 + col] = l > 0.f ? __builtin_amdgcn_rcpf(l) * (2.0f * smax) : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < NP; ++b) {
    const int j = 2 * b + (g >> 1);  // accumulator rows 4 g + i: row 2 b + (g >> 1), head 4 (g & 1) + i
    if (j < RPC) {
      const f32x4 fs = *reinterpret_cast<const f32x4*>(lb + BB_FIN + b * 64 + 16 * g);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int d = 16 * (2 * w + kk) + col;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = (4 * (g & 1) + i) * ND_D + d;
          out[pk(c * RPC + j, n & ~3, ND_H * ND_D) + (n & 3)] = ua[b][kk][i] * fs[i];
        }
      }
    }
  }
}

// one workgroup per chunk (two per CU: 8 waves of <= 128 VGPRs each, 47.5 KB of LDS)
template <int RPC>
__global__ void __launch_bounds__(BB_NW * 64) __attribute__((amdgpu_waves_per_eu(BB_WPE)))
dec_bank_d8_beam_kernel(const float* __restrict__ qp, const char* __restrict__ bank,
                        const float* __restrict__ kscale, const int* __restrict__ kemax,
                        const float* __restrict__ signal, const int* __restrict__ span, float pad_val,
                        float* __restrict__ out, int T, const int* __restrict__ done, unsigned long long* stamp,
                        int* ovf) {
  // ONE shared array (a second __shared__ object beside LDS-DMA staging can make hipcc drain vmcnt
  // before every ds_read)
  __shared__ __attribute__((aligned(16))) char lb[BB_LDS];
  const unsigned long long t_entry = wall_clock64();
  stamp_begin_at(stamp, t_entry);
  const int c = blockIdx.x;
  if (!(done && done[c])) bank_d8_beam_chunk<RPC>(lb, c, qp, bank, kscale, kemax, signal, span, pad_val, out, T, ovf);
  stamp_end(stamp);
}

// Pipelined form (default; ND_BB_PIPE=0 keeps the two-phase kernel above): the score waves (0 .. NP-1, one
// row pair each) work on key block t while the four context waves (4..7, one 64-dim block each) work on
// block t - 1, one barrier per block.  P and the rescale factors are double-buffered by block parity, the
// key-block ring has 4 slots (block t + 2 in flight; a slot is free once block t - 2's context products
// are done).  The context waves issue the key-block copies (3 fragments each).
#define B3_NBUF 4
#define B3_KS (B3_NBUF * BB_BLK)                // [512] row scales
#define B3_PM (B3_KS + 512 * 4)                 // [512] pad flags
#define B3_P (B3_PM + 512)                      // [parity][pair][g][16 columns] hi x 4 | lo x 4
#define B3_SC (B3_P + 2 * BB_MAXP * 1024)       // [parity][pair][16 columns] rescale factors
#define B3_FIN (B3_SC + 2 * BB_MAXP * 64)       // [pair][16 columns] output scales
#define B3_LDS (B3_FIN + BB_MAXP * 64)
static_assert(B3_LDS <= 65536, "pipelined beam bank LDS within 64 KB (DESIGN.md section 5, co-residency rule)");

// block-loop barrier: block t + 1 landed (the copying waves wait for their own copies first), block t's P
// and factors visible, block t - 1's context products done
__device__ __forceinline__ void b3_barrier(bool more) {
  if (more)
    asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int RPC>
__device__ __forceinline__ void bank_d8_beam3_chunk(char* lb, int c, const float* __restrict__ qp, const char* bank,
                                                    const float* __restrict__ kscale, const int* __restrict__ kemax,
                                                    const float* __restrict__ signal, const int* __restrict__ span,
                                                    float pad_val, float* __restrict__ out, int T, int* ovf) {
  constexpr int NP = (RPC + 1) / 2;
  static_assert(NP <= 4, "score waves 0..3");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int L = min(span[c], T);
  const int nkb = (L + 15) >> 4;
  const float smax = __builtin_bit_cast(float, kemax[c]);
  // the chunk's row scales and pad flags (one key per thread), before the roles split
  {
    const int tk = threadIdx.x;
    const float ksv = kscale[(size_t)c * 512 + tk];
    const float sgv = signal[(size_t)c * T + min(tk, T - 1)];
    reinterpret_cast<float*>(lb + B3_KS)[tk] = ksv;
    reinterpret_cast<unsigned char*>(lb + B3_PM)[tk] = (tk < T && sgv == pad_val) ? 1 : 0;
  }
  if (w < NP) {
    // ======== score wave: row pair w (rows 2w, 2w + 1), columns (row 2w + (col >> 3), head col & 7)
    const int jq = 2 * w + (col >> 3);
    const bool rowq = jq < RPC;
    const float* qrow = qp + pk(c * RPC + (rowq ? jq : 0), (col & 7) * ND_D + 16 * g, ND_H * ND_D);
    f32x4 qv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      qv[k] = rowq ? ld4(qrow + pk(0, 64 * (k >> 2) + 4 * (k & 3), ND_H * ND_D)) : f32x4{0.f, 0.f, 0.f, 0.f};
    i32x4 qd[3][4];
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) mx = fmaxf(mx, absmax4(qv[k]));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (!(mx <= 3.0e38f) && ovf != nullptr) ovf[0] = 1;
    const float qs = mx * (1.0f / B8_AMAX);
    const float qdiv = qs > 0.f ? qs : 1.0f;
    const float sgm = qs * 65536.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      unsigned u2 = 0u, u1 = 0u, u0 = 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int d2, d1, d0;
        digits((int)rintf(qv[k][e] / qdiv), d2, d1, d0);
        u2 |= (unsigned)(d2 & 255) << (8 * e);
        u1 |= (unsigned)(d1 & 255) << (8 * e);
        u0 |= (unsigned)(d0 & 255) << (8 * e);
      }
      qd[2][k >> 2][k & 3] = (int)u2;
      qd[1][k >> 2][k & 3] = (int)u1;
      qd[0][k >> 2][k & 3] = (int)u0;
      __builtin_amdgcn_sched_barrier(0);
    }
    const float kp = smax > 0.f ? 128.0f / smax : 0.f;
    float m = -INFINITY, l = 0.f;
    b3_barrier(nkb > 1);  // block 0 landed, tables visible
    for (int t = 0; t <= nkb && nkb > 0; ++t) {
      if (t < nkb) {
        const char* fb = lb + (t % B3_NBUF) * BB_BLK + lane * 16;
        const int par = t & 1;
        i32x4 X1 = {0, 0, 0, 0}, X2 = X1, X3 = X1, X4 = X1;
        i32x4 fr[2][3];
        auto fload = [&](int db, i32x4(&f)[3]) {
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) f[pl] = *reinterpret_cast<const i32x4*>(fb + (db * 3 + pl) * BB_FR);
        };
        fload(0, fr[0]);
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          if (db < 3) fload(db + 1, fr[(db + 1) & 1]);
          const i32x4(&f)[3] = fr[db & 1];
          if (BB_EXPT & 1) {
            X1 += f[2];
            X2 += f[1];
            X3 += f[0];
            continue;
          }
          X1 = mfma_i8(f[2], qd[2][db], X1);
          X2 = mfma_i8(f[2], qd[1][db], X2);
          X3 = mfma_i8(f[2], qd[0][db], X3);
          X4 = mfma_i8(f[1], qd[0][db], X4);
          X2 = mfma_i8(f[1], qd[2][db], X2);
          X3 = mfma_i8(f[1], qd[1][db], X3);
          X4 = mfma_i8(f[0], qd[1][db], X4);
          X3 = mfma_i8(f[0], qd[2][db], X3);
          __builtin_amdgcn_sched_barrier(0);
        }
        const f32x4 ks4 = *reinterpret_cast<const f32x4*>(lb + B3_KS + (16 * t + 4 * g) * 4);
        const unsigned pf = *reinterpret_cast<const unsigned*>(lb + B3_PM + 16 * t + 4 * g);
        const int kbase = 16 * t + 4 * g;
        f32x4 sv;
        float gm = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = fmaf((float)X1[i], 65536.0f,
                               fmaf((float)X2[i], 256.0f, fmaf((float)X4[i], 0.00390625f, (float)X3[i])));
          sv[i] = v * (ks4[i] * sgm);
          sv[i] = kbase + i < L ? (((pf >> (8 * i)) & 1u) ? ND_MASK_FILL : sv[i]) : -INFINITY;
          gm = fmaxf(gm, sv[i]);
        }
        gm = xor32_max(xor16_max(gm));
        const bool resc = __any(gm > m + B8_THR);
        float sc = 1.f;
        if (resc) {
          const float nm = fmaxf(m, gm);
          sc = nm == m ? 1.f : __expf(m - nm);
          m = nm;
          l *= sc;
        }
        if (g == 0) reinterpret_cast<float*>(lb + B3_SC + (par * BB_MAXP + w) * 64)[col] = sc;
        f32x4 p;
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = sv[i] == -INFINITY ? 0.f : __expf(sv[i] - m);
        l += (p[0] + p[1]) + (p[2] + p[3]);
        d8h8 pa;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float x = p[i] * (ks4[i] * kp);
          const _Float16 hi = (_Float16)x;
          pa[i] = hi;
          pa[4 + i] = (_Float16)(x - (float)hi);
        }
        *reinterpret_cast<d8h8*>(lb + B3_P + (par * BB_MAXP + w) * 1024 + (g * 16 + col) * 16) = pa;
      }
      b3_barrier(t + 2 < nkb);
    }
    l = xor32_sum(xor16_sum(l));
    if (g == 0)
      reinterpret_cast<float*>(lb + B3_FIN)[w * 16 + col] = l > 0.f ? __builtin_amdgcn_rcpf(l) * (2.0f * smax) : 0.f;
    __syncthreads();
  } else if (w >= 4) {
    // ======== context wave u = w - 4: 64-dim block u (16-dim groups 0..3 as the pairs 0|1, 2|3), every
    //          row pair; issues the key-block copies (fragments 3u .. 3u + 2; block kb -> slot kb % 4)
    const int u = w - 4;
    const __amdgpu_buffer_rsrc_t src = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(bank) + (size_t)c * (B8_KB * 12 * 1024), 0, B8_KB * 12 * 1024, 0x00020000);
    auto issue = [&](int kb) {
      if ((BB_EXPT & 4) == 0) {
        char* dst = lb + (kb % B3_NBUF) * BB_BLK;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int f = 3 * u + i;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (__attribute__((address_space(3))) void*)(dst + f * BB_FR),
                                                   16, lane * 16, kb * 12288 + f * 1024, 0, 0);
        }
      }
    };
    if (nkb > 0) issue(0);
    if (nkb > 1) issue(1);
    const int q8 = (lane & 15) >> 1, p8 = lane & 1;
    const int o1 = (u * 3 + (q8 < 4 ? 2 : 1)) * BB_FR + (4 * g + (q8 & 3)) * 16 + 8 * p8;
    const int o3 = u * 3 * BB_FR + (4 * g + (q8 & 3) + 16 * (q8 < 4 ? 0 : 1)) * 16 + 8 * p8;
    f32x4 ua[NP][4];
#pragma unroll
    for (int b = 0; b < NP; ++b)
#pragma unroll
      for (int k = 0; k < 4; ++k) ua[b][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    b3_barrier(nkb > 1);
    for (int t = 0; t <= nkb && nkb > 0; ++t) {
      if (t + 2 < nkb) issue(t + 2);
      if (t >= 1) {
        const char* buf = lb + ((t - 1) % B3_NBUF) * BB_BLK;
        const int par = (t - 1) & 1;
        d8h8 pa[NP];
#pragma unroll
        for (int b = 0; b < NP; ++b) {
          // branch-free running-maximum rescale (bank_d8_beam_chunk); rows 4 g + i = columns 4 g + i
          const f32x4 sc4 = *reinterpret_cast<const f32x4*>(lb + B3_SC + (par * BB_MAXP + b) * 64 + 16 * g);
#pragma unroll
          for (int k = 0; k < 4; ++k) ua[b][k] *= sc4;
          pa[b] = *reinterpret_cast<const d8h8*>(lb + B3_P + (par * BB_MAXP + b) * 1024 + (g * 16 + col) * 16);
        }
#pragma unroll
        for (int gp = 0; gp < 2; ++gp) {
          const d8u2 r1 = tr_b8(buf + o1 + 512 * gp), r2 = tr_b8(buf + o1 + 512 * gp + 256),
                     r3 = tr_b8(buf + o3 + 512 * gp);
          const d8h4 c2a = d8_cvt(r1.x, 2), c1a = d8_cvt(r1.y, 1), c2b = d8_cvt(r2.x, 2), c1b = d8_cvt(r2.y, 1);
          const d8h8 b2a = {c2a[0], c2a[1], c2a[2], c2a[3], c2a[0], c2a[1], c2a[2], c2a[3]};
          const d8h8 b1a = {c1a[0], c1a[1], c1a[2], c1a[3], c1a[0], c1a[1], c1a[2], c1a[3]};
          const d8h8 b2b = {c2b[0], c2b[1], c2b[2], c2b[3], c2b[0], c2b[1], c2b[2], c2b[3]};
          const d8h8 b1b = {c1b[0], c1b[1], c1b[2], c1b[3], c1b[0], c1b[1], c1b[2], c1b[3]};
          const d8h4 b0a = d8_cvt(r3.x, 0), b0b = d8_cvt(r3.y, 0);
#pragma unroll
          for (int b = 0; b < NP; ++b) {
            const d8h4 ph = {pa[b][0], pa[b][1], pa[b][2], pa[b][3]};
            f32x4& u0 = ua[b][2 * gp];
            f32x4& u1 = ua[b][2 * gp + 1];
            if (BB_EXPT & 2) {
              u0 += f32x4{(float)ph[0], (float)b2a[1], (float)b1a[2], (float)b0a[3]};
              u1 += f32x4{(float)ph[1], (float)b2b[1], (float)b1b[2], (float)b0b[3]};
              continue;
            }
            u0 = mfma_d8h32(pa[b], b2a, u0);
            u1 = mfma_d8h32(pa[b], b2b, u1);
            u0 = mfma_d8h32(pa[b], b1a, u0);
            u1 = mfma_d8h32(pa[b], b1b, u1);
            u0 = mfma_d8h16(ph, b0a, u0);
            u1 = mfma_d8h16(ph, b0b, u1);
          }
        }
      }
      b3_barrier(t + 2 < nkb);
    }
    __syncthreads();  // FIN written by the score waves
#pragma unroll
    for (int b = 0; b < NP; ++b) {
      const int j = 2 * b + (g >> 1);  // accumulator rows 4 g + i: row 2 b + (g >> 1), head 4 (g & 1) + i
      if (j < RPC) {
        const f32x4 fs = *reinterpret_cast<const f32x4*>(lb + B3_FIN + b * 64 + 16 * g);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int d = 64 * u + 16 * kk + col;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = (4 * (g & 1) + i) * ND_D + d;
            out[pk(c * RPC + j, n & ~3, ND_H * ND_D) + (n & 3)] = ua[b][kk][i] * fs[i];
          }
        }
      }
    }
  } else {
    // ======== idle waves (NP .. 3): the block loop's barriers only
    b3_barrier(nkb > 1);
    for (int t = 0; t <= nkb && nkb > 0; ++t) b3_barrier(t + 2 < nkb);
    __syncthreads();
  }
}

template <int RPC>
__global__ void __launch_bounds__(BB_NW * 64) __attribute__((amdgpu_waves_per_eu(BB_WPE)))
dec_bank_d8_beam3_kernel(const float* __restrict__ qp, const char* __restrict__ bank,
                         const float* __restrict__ kscale, const int* __restrict__ kemax,
                         const float* __restrict__ signal, const int* __restrict__ span, float pad_val,
                         float* __restrict__ out, int T, const int* __restrict__ done, unsigned long long* stamp,
                         int* ovf) {
  __shared__ __attribute__((aligned(16))) char lb[B3_LDS];  // one shared array (see dec_bank_d8_beam_kernel)
  const unsigned long long t_entry = wall_clock64();
  stamp_begin_at(stamp, t_entry);
  const int c = blockIdx.x;
  if (!(done && done[c])) bank_d8_beam3_chunk<RPC>(lb, c, qp, bank, kscale, kemax, signal, span, pad_val, out, T, ovf);
  stamp_end(stamp);
}

hipError_t launch_dec_bank_d8_beam(const float* qp, const void* bank, const float* kscale, const int* kemax,
                                   const float* signal, const int* span, float pad_val, float* out, int C, int rpc,
                                   int T, const int* done, hipStream_t s, unsigned long long* stamp, int* ovf) {
  if (T < 1 || T > 512 || C < 1 || rpc < 2 || rpc > BB_MAXR || !qp || !bank || !kscale || !kemax || !signal ||
      !span || !out)
    return hipErrorInvalidValue;
  static const bool pipe = [] {
    const char* e = getenv("ND_BB_PIPE");  // 0: the two-phase kernel (A/B timing)
    return !(e && atoi(e) == 0);
  }();
#define ND_BANK8B_GO(R)                                                                                          \
  if (pipe)                                                                                                      \
    hipLaunchKernelGGL((dec_bank_d8_beam3_kernel<R>), dim3(C), dim3(BB_NW * 64), 0, s, qp,                      \
                       reinterpret_cast<const char*>(bank), kscale, kemax, signal, span, pad_val, out, T, done, stamp, \
                       ovf);                                                                                     \
  else                                                                                                           \
    hipLaunchKernelGGL((dec_bank_d8_beam_kernel<R>), dim3(C), dim3(BB_NW * 64), 0, s, qp,                       \
                       reinterpret_cast<const char*>(bank), kscale, kemax, signal, span, pad_val, out, T, done, stamp, \
                       ovf)
  switch (rpc) {
    case 2: ND_BANK8B_GO(2); break;
    case 3: ND_BANK8B_GO(3); break;
    case 4: ND_BANK8B_GO(4); break;
    case 5: ND_BANK8B_GO(5); break;
    default: ND_BANK8B_GO(6); break;
  }
#undef ND_BANK8B_GO
  return hipGetLastError();
}

hipError_t init_bank8_attributes() {
  const void* fns[] = {(const void*)dec_bank_d8_kernel<false, false>, (const void*)dec_bank_d8_kernel<true, false>,
                       (const void*)dec_bank_d8_kernel<false, true>, (const void*)dec_bank_d8_kernel<true, true>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, B8_LDS);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace nd
