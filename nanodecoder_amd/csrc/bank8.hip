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
// U = P^T M on f16 MFMAs, the digits turned into exact f16 integers
// (magic-number conversion) from a per-wave transposed LDS image read by
// ds_read_b64_tr_b8: one 16x16x32 product per dim block takes [P, P] against
// [a2 * 2^8 (4 keys), a1 (4 keys)], a second [P, 0] against a0 * 2^-8 (one
// MFMA shape per accumulator: mfma_d8h16as32).  P is p s_t 2^7 / s_max
// (s_max: the chunk's largest s_t, so <= 2^7 e^6 < 65504) split hi | lo (the
// rows of head h carry hi, the rows of h + 8 lo).
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
// The a0 plane's product on the same 16x16x32 form as the a2 / a1 products ([P | 0] against [a0 | a0]: the
// same lane pairs, zeros in the second k half): every MFMA of an accumulator then has ONE shape.  A
// 16x16x16_f16 that accumulates onto a 16x16x32_f16's destination reads components 0-1 of srcC stale
// unless >= 4 VALU / 5 other instructions separate them (tools/probe_mfma_hazard.py, profiles/
// r05_mfma_hazard_probe.json); hipcc 7.2 pads such a pair with nothing.
__device__ __forceinline__ f32x4 mfma_d8h16as32(d8h4 a, d8h4 b, f32x4 c) {
  const d8h8 a8 = {a[0], a[1], a[2], a[3], (_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
  const d8h8 b8 = {b[0], b[1], b[2], b[3], b[0], b[1], b[2], b[3]};
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c, 0, 0, 0);
}

// 4 signed bytes -> 4 exact f16: f16 bits 0x64uu = 1024 + u with u = b + 128
// (b ^ 0x80), minus 1152 (exact); then the plane weight (exact power of two)
__device__ __forceinline__ d8h4 d8_cvt(unsigned x, int plane) {
#ifdef B8_PROBE_NOCVT  // timing probe only: the bytes reinterpreted, no conversion
  return __builtin_bit_cast(d8h4, d8u2{x, x ^ (unsigned)plane});
#endif
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

// timing probe only (tools/bank_phases.py, B8_PROBE_PHASES): wave w of chunk c writes the wall clock at
// phase i to the u64 slot [c][w][i] past the C16 x 2048 output (the probe allocates it)
#ifdef B8_PROBE_PHASES
#define B8_PHASE(i)                                                                                                  \
  if (lane == 0)                                                                                                     \
    reinterpret_cast<unsigned long long*>(out + (size_t)((C_ + 15) / 16 * 16) * (ND_H * ND_D))[(c * B8_NW + w) * 8 + \
                                                                                          (i)] = wall_clock64()
#else
#define B8_PHASE(i)
#endif

// What a chunk's prologue loads: q' of the wave's head (4 dims per lane), this lane's key scales (keys
// 16 (w + 8 kb) + 4 g + i), the signal, the chunk's largest row scale, then the first two half blocks.
// WALK: the next chunk's head is loaded before this chunk's merge (its latency hides behind the merge).
struct B8Head {
  f32x4 qv;
  f32x4 ksc[B8_KPW];  // the first KPW used
  float sg, smax;
  i32x4 F[3][6];
};

// half block h of chunk c: key block w + 8 (h >> 1), dim blocks 2 (h & 1) + j (j = 0, 1), planes 2, 1, 0:
// f[3 j + 2 - pl]
template <bool NT>  // non-temporal loads (a runtime condition around loads makes hipcc drain every load in flight)
__device__ __forceinline__ void b8_hload(const i32x4* __restrict__ bank, int c, int h, int w, int lane,
                                         i32x4 (&f)[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int db = 2 * (h & 1) + i / 3, pl = 2 - i % 3;
#ifdef B8_PROBE_NOLOAD  // timing probe only (tools/bank_probe.sh): every chunk reads chunk 0's bank (L2-resident)
    const i32x4* p = bank + (((((size_t)0) * B8_KB + w + B8_NW * (h >> 1)) * 4 + db) * 3 + pl) * 64 + lane;
#else
    const i32x4* p = bank + ((((size_t)c * B8_KB + w + B8_NW * (h >> 1)) * 4 + db) * 3 + pl) * 64 + lane;
#endif
    if constexpr (NT)
      f[i] = __builtin_nontemporal_load(p);
    else
      f[i] = *p;
  }
}

// KPW: the key blocks per wave this launch processes (T <= 128 KPW; bank8_kpw)
template <bool NT, bool BOTH, int KPW>  // BOTH: the first two half blocks (else the first only: the WALK prefetch)
__device__ __forceinline__ void b8_head(int c, const float* __restrict__ qp, const i32x4* __restrict__ bank,
                                        const float* __restrict__ kscale, const int* __restrict__ kemax,
                                        const float* __restrict__ signal, int T, B8Head& hd) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  hd.qv = ld4(qp + (size_t)c * (ND_H * ND_D) + w * ND_D + 4 * lane);
#pragma unroll
  for (int kb = 0; kb < KPW; ++kb) hd.ksc[kb] = ld4(kscale + (size_t)c * 512 + 16 * (w + B8_NW * kb) + 4 * g);
  {
    const int bkey = 16 * (w + B8_NW * (lane >> 4)) + (lane & 15);  // lane l: row l & 15 of key block w + 8 (l >> 4)
    hd.sg = signal[(size_t)c * T + min(bkey, T - 1)];
  }
  hd.smax = __builtin_bit_cast(float, kemax[c]);  // the chunk's largest row scale
  // issue order = retire order: q' and the scales first, then half block 0, then 1 (a wait for an
  // earlier load leaves the later ones in flight)
  __builtin_amdgcn_sched_barrier(0);
  b8_hload<NT>(bank, c, 0, w, lane, hd.F[0]);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (BOTH) {
    b8_hload<NT>(bank, c, 1, w, lane, hd.F[1]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// chunk c from its loaded head (need1: its second half block still to load); nx >= 0: the next chunk this
// workgroup walks to, whose head (first half block) goes into hd before the merge
template <bool NT, bool NXNT, int KPW>  // this chunk's and the next chunk's load policy; key blocks per wave
__device__ __forceinline__ void bank_d8_chunk(int c, B8Head& hd, bool need1, int nx,
                                              const float* __restrict__ qp, const i32x4* __restrict__ bank,
                                              const float* __restrict__ kscale, const int* __restrict__ kemax,
                                              const float* __restrict__ signal, const int* __restrict__ span,
                                              float pad_val, float* __restrict__ out, int T,
                                              unsigned long long* stamp, float* __restrict__ dbg, size_t dbg_stride,
                                              int* ovf, unsigned long long t_entry, int C_) {
  extern __shared__ float lds[];
  char* lb = reinterpret_cast<char*>(lds);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  char* img = lb + w * B8_IMG;
  (void)C_;
  B8_PHASE(0);
  i32x4(&F)[3][6] = hd.F;
  if (need1) {
    b8_hload<NT>(bank, c, 1, w, lane, F[1]);
    __builtin_amdgcn_sched_barrier(0);
  }
  const f32x4 qv = hd.qv;
  const float sg = hd.sg, smax = hd.smax;
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
  B8_PHASE(1);
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
  for (int kb = 0; kb < KPW; ++kb) {
    i32x4 X1 = {0, 0, 0, 0}, X2 = X1, X3 = X1, X4 = X1;
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const int h = 2 * kb + part;
      i32x4(&f)[6] = F[h % 3];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int db = 2 * part + j;
#ifdef B8_PROBE_NOSCORE  // timing probe only: no score products (X stays 0 + the fragments' first word)
        X1[0] += f[3 * j][0] ^ f[3 * j + 1][1] ^ f[3 * j + 2][2];
        continue;
#endif
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
      if (h + 2 < 2 * KPW) b8_hload<NT>(bank, c, h + 2, w, lane, F[(h + 2) % 3]);
    }
    // ---- scores: columns h and h + 8 hold the high and low digit products of head h
    f32x4 s;
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = (float)X1[i] * w1 + (float)X2[i] * w2 + (float)X3[i] * w3 + (float)X4[i] * w4;
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = (s[i] + dpp_mov<0x128>(s[i])) * (hd.ksc[kb][i] * sgm);
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
      const float x = p[i] * (hd.ksc[kb][i] * kp);
      const _Float16 hi = (_Float16)x;
      pa[i] = col < 8 ? hi : (_Float16)(x - (float)hi);
    }
    const d8h8 pa8 = {pa[0], pa[1], pa[2], pa[3], pa[0], pa[1], pa[2], pa[3]};
    // ---- U += P^T M': dim blocks (2 kp, 2 kp + 1) of 16 dims, dims 16 k + col
#ifdef B8_PROBE_NOU  // timing probe only: no context product (U stays the P sums)
    ua[kb][0] += pa[0] + pa[1];
    continue;
#endif
#pragma unroll
    for (int kp2 = 0; kp2 < 8; ++kp2) {
      const d8u2 r1 = tr_b8(rb1 + 32 * kp2), r2 = tr_b8(rb1 + 32 * kp2 + 16), r3 = tr_b8(rb3 + 32 * kp2);
      const d8h4 b1a = d8_cvt(r1.x, 2), b1b = d8_cvt(r1.y, 1), b2a = d8_cvt(r2.x, 2), b2b = d8_cvt(r2.y, 1);
      const d8h8 b1 = {b1a[0], b1a[1], b1a[2], b1a[3], b1b[0], b1b[1], b1b[2], b1b[3]};
      const d8h8 b2 = {b2a[0], b2a[1], b2a[2], b2a[3], b2b[0], b2b[1], b2b[2], b2b[3]};
      ua[2 * kp2] = mfma_d8h32(pa8, b1, ua[2 * kp2]);
      ua[2 * kp2] = mfma_d8h16as32(pa, d8_cvt(r3.x, 0), ua[2 * kp2]);
      ua[2 * kp2 + 1] = mfma_d8h32(pa8, b2, ua[2 * kp2 + 1]);
      ua[2 * kp2 + 1] = mfma_d8h16as32(pa, d8_cvt(r3.y, 0), ua[2 * kp2 + 1]);
    }
#ifdef B8_PROBE_PHASES
    if (kb == 0) { B8_PHASE(2); }
    if (kb == 1) { B8_PHASE(3); }
    if (kb == 2) { B8_PHASE(4); }
#endif
  }
  B8_PHASE(5);

  // ---- merge the 8 waves (as dec_bank_h3_kernel): unmerged U^T fragments to the wave's own image, (m, l)
  //      beside, wave 0 turns them into merge weights and the output scale 2 s_max / den
  l = xor32_sum(xor16_sum(l));
  float* ml = reinterpret_cast<float*>(lb + B8_ML);  // [wave][8 heads][2]
  {
    f32x4* red = reinterpret_cast<f32x4*>(img);
#pragma unroll
    for (int k = 0; k < 16; ++k) red[k * 64 + lane] = ua[k];
  }
  // WALK: the next chunk's head (q', scales, its first half blocks) goes out now, into registers that are
  // all dead here (U sits in LDS); its latency hides behind the rest of this chunk's merge
  if (nx >= 0) b8_head<NXNT, false, KPW>(nx, qp, bank, kscale, kemax, signal, T, hd);
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
  B8_PHASE(6);
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
  B8_PHASE(7);
}

// KPW < 4 (T <= 384): the key blocks past 128 KPW keys (zero rows of the pack, keys >= T) are not streamed
template <bool NT, bool WALK, int KPW>
__global__ void __launch_bounds__(B8_NW * 64)
dec_bank_d8_kernel(const float* __restrict__ qp, const i32x4* __restrict__ bank, const float* __restrict__ kscale,
                   const int* __restrict__ kemax, const float* __restrict__ signal, const int* __restrict__ span,
                   float pad_val, float* __restrict__ out, int T, int C, unsigned long long* stamp,
                   float* __restrict__ dbg, size_t dbg_stride, int* ovf, int cached) {
#ifdef ND_SKIP_BANK  // timing probe only (tools/build_variant.sh, tools/marginal.sh): the kernel's marginal cost
  if (threadIdx.x < 100000) return;
#endif
  const unsigned long long t_entry = wall_clock64();
  // NT: chunks c >= cached stream non-temporally; the first `cached` chunks' banks keep the default policy
  // (they stay in the Infinity Cache between the call's 300 launches, bank_cached below)
  auto ntc = [&](int c) { return NT && c >= cached; };
  // every load policy is a template argument (a branch around loads drains them), so each policy pair is its
  // own copy of the chunk body
#define B8_CHUNK(A, B, c_, need1_, nx_)                                                                            \
  bank_d8_chunk<A, B, KPW>(c_, hd, need1_, nx_, qp, bank, kscale, kemax, signal, span, pad_val, out, T, stamp, dbg,      \
                      dbg_stride, ovf, t_entry, C)
  B8Head hd;
  if constexpr (WALK) {
    int c = blockIdx.x;
    const int G = gridDim.x;
    if (C <= 2 * G) {
      // at most two chunks per workgroup (the pool's grid: half the CUs): straight-line, the second chunk's head
      // loaded during the first one's merge (a runtime loop would carry the head's registers across its
      // back-edge and spill)
      // (each policy case one straight-line path: the head's registers never meet at a join).  The second
      // chunk c + G >= G > C / 4 = cached is always past the cached quarter: non-temporal when NT is
      const int nx = c + G < C ? c + G : -1;
      if (!NT || !ntc(c)) {
        b8_head<false, true, KPW>(c, qp, bank, kscale, kemax, signal, T, hd);
        B8_CHUNK(false, NT, c, false, nx);
      } else {
        b8_head<NT, true, KPW>(c, qp, bank, kscale, kemax, signal, T, hd);
        B8_CHUNK(NT, NT, c, false, nx);
      }
      if (nx >= 0) {
        lds_barrier();  // the first chunk's merge reads of LDS are done
        B8_CHUNK(NT, false, nx, true, -1);
      }
    } else {
      for (; c < C; c += G) {
        if (c != (int)blockIdx.x) lds_barrier();  // the previous chunk's merge reads of LDS are done
        if (ntc(c)) {
          b8_head<NT, true, KPW>(c, qp, bank, kscale, kemax, signal, T, hd);
          B8_CHUNK(NT, false, c, false, -1);
        } else {
          b8_head<false, true, KPW>(c, qp, bank, kscale, kemax, signal, T, hd);
          B8_CHUNK(false, false, c, false, -1);
        }
      }
    }
  } else {
    const int c = blockIdx.x;
    if (ntc(c)) {
      b8_head<NT, true, KPW>(c, qp, bank, kscale, kemax, signal, T, hd);
      B8_CHUNK(NT, false, c, false, -1);
    } else {
      b8_head<false, true, KPW>(c, qp, bank, kscale, kemax, signal, T, hd);
      B8_CHUNK(false, false, c, false, -1);
    }
  }
#undef B8_CHUNK
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

// When the bank streams non-temporally (the pool's lanes, EnginePool.bank_nt_lanes), the first quarter of
// a call's chunks keep the default policy: with three lanes that is 75 MB of bank held in the 256 MB
// Infinity Cache across the call's 300 launches.  Pooled configs[1], same box, two reps each (ND_BANK_CACHED
// A/B, round 5): none 16.10 / 16.07 ms per call; 32 of 256 chunks 15.92 / 15.91; 64: 15.91 / 15.90; 96: 15.98
// / 15.95; 128: 15.87 / 15.89; 192: 16.09 / 16.03; all 256: 16.38 / 16.39 (the banks then evict the rest)
// (with the lanes' weights shared, nd_share_weights: a third or half of the chunks 15.50 / 15.58 and 15.54 /
// 15.55 ms against a quarter's 15.48 / 15.53, same box)
static int bank_cached(int C) { return C / 4; }

// key blocks per wave a launch processes: 8 waves x 16 keys per block, so T <= 128 KPW (the pack leaves the
// rows past T zero with scale 0, and they are masked: the blocks past them need not be streamed)
static int bank8_kpw(int T) { return std::min(B8_KPW, (T + 127) / 128); }

hipError_t launch_dec_bank_d8(const float* qp, const void* bank, const float* kscale, const int* kemax,
                              const float* signal, const int* span, float pad_val, float* out, int C, int T,
                              hipStream_t s, unsigned long long* stamp, float* attn_dbg, size_t dbg_stride, int* ovf,
                              bool nt, int grid) {
  if (T < 1 || T > 512 || C < 1 || grid < 0 || !bank || !kscale || !kemax) return hipErrorInvalidValue;
  const int G = grid > 0 ? std::min(C, grid) : C;
  const int kpw = bank8_kpw(T);
#define ND_BANK8_GO(N, W, K)                                                                                      \
  hipLaunchKernelGGL((dec_bank_d8_kernel<N, W, K>), dim3(G), dim3(B8_NW * 64), B8_LDS, s, qp,                    \
                     reinterpret_cast<const i32x4*>(bank), kscale, kemax, signal, span, pad_val, out, T, C, stamp,  \
                     attn_dbg, dbg_stride, ovf, bank_cached(C))
#define ND_BANK8_K(N, W)         \
  do {                           \
    if (kpw == 4)                \
      ND_BANK8_GO(N, W, 4);      \
    else if (kpw == 3)           \
      ND_BANK8_GO(N, W, 3);      \
    else if (kpw == 2)           \
      ND_BANK8_GO(N, W, 2);      \
    else                         \
      ND_BANK8_GO(N, W, 1);      \
  } while (0)
  if (G < C) {
    if (nt)
      ND_BANK8_K(true, true);
    else
      ND_BANK8_K(false, true);
  } else if (nt) {
    ND_BANK8_K(true, false);
  } else {
    ND_BANK8_K(false, false);
  }
#undef ND_BANK8_K
#undef ND_BANK8_GO
  return hipGetLastError();
}

hipError_t init_bank8_attributes() {
#define ND_BANK8_FNS(K)                                                                                           \
  (const void*)dec_bank_d8_kernel<false, false, K>, (const void*)dec_bank_d8_kernel<true, false, K>,              \
      (const void*)dec_bank_d8_kernel<false, true, K>, (const void*)dec_bank_d8_kernel<true, true, K>
  const void* fns[] = {ND_BANK8_FNS(4), ND_BANK8_FNS(3), ND_BANK8_FNS(2), ND_BANK8_FNS(1)};
#undef ND_BANK8_FNS
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, B8_LDS);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace nd
