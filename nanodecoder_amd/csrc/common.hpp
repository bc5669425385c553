// Shared device helpers for the gfx950 kernels of libnanodec_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ND_D 256         // d_model (compiled constant)
#define ND_DH 32         // head dim
#define ND_H 8           // heads
#define ND_MAXV 32       // max vocab
#define ND_MASK_FILL (-1e18f)  // onmt/modules/multi_headed_attn.py:172
#define ND_LN_EPS 1e-6f        // nn.LayerNorm(d, eps=1e-6)
#define ND_SQRT_DH 5.65685424949238f  // math.sqrt(dim_per_head) as torch casts it to f32

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// 12 bytes as one dwordx3 access where only 4-byte alignment holds (a lane's 3 words of the 24-bit images)
typedef unsigned u32v3 __attribute__((ext_vector_type(3), aligned(4)));
struct u32x3 {  // 12 bytes, 4-byte aligned (one dwordx3 access)
  uint32_t x, y, z;
};

// The 24-bit context K/V quantiser (attention.hip ctx_pack_q24_kernel and the
// GEMM epilogue that writes the image directly): x = this lane's 4 values of
// a 32-wide head held by 8 consecutive lanes (lane & 7 = the dims' quad).
// Stores the lane's 12 bytes at dst (little-endian 3-byte integers) and
// returns the head's scale 2^(e-23) (NaN for a head holding a NaN / inf).
__device__ __forceinline__ float q24_quant(f32x4 x, u32x3& b) {
  float mx = fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
  if (!(fabsf(x.x) <= 3.4028235e38f && fabsf(x.y) <= 3.4028235e38f && fabsf(x.z) <= 3.4028235e38f &&
        fabsf(x.w) <= 3.4028235e38f))
    mx = INFINITY;  // NaN / inf anywhere in the head (fmaxf would drop a NaN)
  mx = fmaxf(mx, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, mx), 0xB1, 0xF, 0xF, false)));
  mx = fmaxf(mx, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, mx), 0x4E, 0xF, 0xF, false)));
  mx = fmaxf(mx, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, mx), 0x141, 0xF, 0xF, false)));
  int e = 0;
  frexpf(mx, &e);  // mx = f 2^e, f in [0.5, 1): mx < 2^e (mx == 0: e = 0, the integers are 0)
  e = max(e, -100);  // a head below 2^-100 (2^(23 - e) must stay finite): its integers round to 0
  const float up = ldexpf(1.f, 23 - e);
  int v[4];
  const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (int)fminf(fmaxf(rintf(xs[i] * up), -8388607.f), 8388607.f);
  b.x = (uint32_t)(v[0] & 0xffffff) | ((uint32_t)v[1] << 24);
  b.y = (((uint32_t)v[1] >> 8) & 0xffff) | ((uint32_t)v[2] << 16);
  b.z = (((uint32_t)v[2] >> 16) & 0xff) | ((uint32_t)v[3] << 8);
  // a non-finite head keeps a NaN scale, so its scores / values stay non-finite as in fp32
  return mx <= 3.4028235e38f ? ldexpf(1.f, e - 23) : __builtin_nanf("");
}
__device__ __forceinline__ float q24_quant_store(f32x4 x, uint8_t* dst) {
  u32x3 b;
  const float sc = q24_quant(x, b);
  *reinterpret_cast<u32x3*>(dst) = b;
  return sc;
}
// the same 12 bytes in a register image: .xyz the three words, .w the head's scale (q24_unpack(r) * r.w = x)
__device__ __forceinline__ f32x4 q24_raw(f32x4 x) {
  u32x3 b;
  const float sc = q24_quant(x, b);
  return f32x4{__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), sc};
}

// Four 24-bit two's-complement integers packed little-endian in the bits of
// raw.x, raw.y, raw.z (ctx_pack_q24_kernel) -> exact fp32 values.
__device__ __forceinline__ f32x4 q24_unpack(f32x4 raw) {
  const uint32_t w0 = __float_as_uint(raw.x), w1 = __float_as_uint(raw.y), w2 = __float_as_uint(raw.z);
  const int i0 = (int)(w0 << 8) >> 8;
  const int i1 = (int)(__builtin_amdgcn_alignbit(w1, w0, 24) << 8) >> 8;
  const int i2 = (int)(__builtin_amdgcn_alignbit(w2, w1, 16) << 8) >> 8;
  const int i3 = (int)w2 >> 8;
  return f32x4{(float)i0, (float)i1, (float)i2, (float)i3};
}

// v_mfma_f32_32x32x2_f32: lane l supplies A[l&31][l>>5] and B[l>>5][l&31];
// D lane l, reg r holds D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31].
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int mfma32_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Butterfly reductions inside 4 / 8 / 16-lane groups on DPP lane moves
// (one VALU op per stage, no LDS round trip): quad_perm [1,0,3,2] = xor 1,
// quad_perm [2,3,0,1] = xor 2, row_half_mirror joins the two quads of 8
// lanes, row_mirror the two halves of 16.  Every lane of the group ends with
// the same (commutatively identical) total.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
#define ND_DPP_XOR1 0xB1
#define ND_DPP_XOR2 0x4E
#define ND_DPP_HALF_MIRROR 0x141
#define ND_DPP_MIRROR 0x140
__device__ __forceinline__ float sum4(float v) {
  v += dpp_mov<ND_DPP_XOR1>(v);
  return v + dpp_mov<ND_DPP_XOR2>(v);
}
__device__ __forceinline__ float sum8(float v) {
  v = sum4(v);
  return v + dpp_mov<ND_DPP_HALF_MIRROR>(v);
}
__device__ __forceinline__ float sum16(float v) {
  v = sum8(v);
  return v + dpp_mov<ND_DPP_MIRROR>(v);
}
__device__ __forceinline__ float max16(float v) {
  v = fmaxf(v, dpp_mov<ND_DPP_XOR1>(v));
  v = fmaxf(v, dpp_mov<ND_DPP_XOR2>(v));
  v = fmaxf(v, dpp_mov<ND_DPP_HALF_MIRROR>(v));
  return fmaxf(v, dpp_mov<ND_DPP_MIRROR>(v));
}

// gfx950 cross-row lane swaps (VALU, no LDS): v_permlane16_swap exchanges
// the odd 16-lane rows of one operand with the even rows of the other,
// v_permlane32_swap the upper half with the lower half.  Fed the same value
// twice, the two results hold the partner lanes' values (probe:
// tools/probe_permlane.hip).  Inline asm: hipcc 7.2's builtin reads both
// results from the first operand's register (r[0] + r[1] becomes 2 * r[0]).
// The s_nop covers the VALU-write -> permlane-read hazard.
template <bool ROW32>
__device__ __forceinline__ void lane_swap(float v, float& a, float& b) {
  a = v;
  b = v;
  if constexpr (ROW32)
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  else
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float xor16_sum(float v) {
  float a, b;
  lane_swap<false>(v, a, b);
  return a + b;
}
__device__ __forceinline__ float xor32_sum(float v) {
  float a, b;
  lane_swap<true>(v, a, b);
  return a + b;
}
__device__ __forceinline__ float xor16_max(float v) {
  float a, b;
  lane_swap<false>(v, a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float xor32_max(float v) {
  float a, b;
  lane_swap<true>(v, a, b);
  return fmaxf(a, b);
}

__device__ __forceinline__ float wave_sum(float v) { return xor32_sum(xor16_sum(sum16(v))); }

__device__ __forceinline__ float wave_max(float v) { return xor32_max(xor16_max(max16(v))); }

// Fragment-packed ("P16") layout of an [M, N] fp32 matrix (M, N multiples of
// 16): 16x16 blocks in row-major block order; inside a block, 64 float4
// entries, entry e = (m & 15) + 16 * ((n & 15) >> 2) holding columns
// n & ~3 .. +3 of row m.  Entry e is exactly what lane e supplies to (and
// receives from) v_mfma_f32_16x16x4_f32 under the 4-k permutation, so a
// wave moves a whole block with one coalesced 1 KB access.  Float offset of
// element (m, n) with n % 4 == 0:
__device__ __forceinline__ size_t pk(int m, int n, int N) {
  return (((size_t)(m >> 4) * (N >> 4) + (n >> 4)) * 64 + (m & 15) + 16 * ((n >> 2) & 3)) * 4;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// LayerNorm 1 / sqrt(var + eps): v_rsq_f32 (1 ulp; the argument is >= eps,
// never denormal).  1.0f / sqrtf() lowers to an IEEE sqrt plus an IEEE
// division, ~20 dependent instructions on the path of every LN consumer.
__device__ __forceinline__ float ln_rsqrt(float x) { return __builtin_amdgcn_rsqf(x); }

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its outstanding global loads and stores
// (__syncthreads() also waits vmcnt(0), which drains every prefetch in
// flight and every store just issued).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// --fast beam: every row of [r0, r0 + n) (rows < M) belongs to a finished
// chunk (skip[row / rpc] != 0).  Wave-uniform; each wave of a workgroup
// computes the same answer, so a dead tile returns before any barrier.
__device__ __forceinline__ bool rows_dead(const int* __restrict__ skip, int rpc, int r0, int n, int M) {
  if (skip == nullptr) return false;
  const int c0 = r0 / rpc, c1 = (min(r0 + n, M) - 1) / rpc;
  bool alive = false;
  for (int c = c0 + (int)(threadIdx.x & 63); c <= c1; c += 64) alive |= skip[c] == 0;
  return __ballot(alive) == 0;
}

// Split-fp16 range guard.  An activation split as hi = fp16(x), lo =
// fp16(x - hi) leaves the fp16 range from |x| = 65504 on (hi becomes inf
// where the fp32 reference is finite).  Every kernel that splits an
// activation it did not normalise itself records the largest |x| it split
// and raises the ctx's overflow word (plain vector store of 1 from the lanes
// that saw one; all writers store the same value); the host reads the word
// per call (nd_take_overflow) and reruns that call on the exact fp32 path.
#define ND_F16_LIMIT 65504.0f
__device__ __forceinline__ float absmax4(f32x4 v) {
  return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}
__device__ __forceinline__ void flag_overflow(int* ovf, float amax) {
  if (amax >= ND_F16_LIMIT && ovf != nullptr) ovf[0] = 1;
}

// Launch-duration stamps (bench roofline, measured inside the timed graph):
// stamp[0] = earliest workgroup start, stamp[1] = latest workgroup end, in
// wall_clock64() ticks (s_memrealtime, constant rate).  stamp == nullptr: off.
__device__ __forceinline__ void stamp_begin(unsigned long long* stamp) {
  if (stamp && threadIdx.x == 0) atomicMin(stamp, (unsigned long long)wall_clock64());
}
// the same with the clock read at kernel entry (t0 = wall_clock64() as the
// first statement) and published later, so the stamp's branch and atomic do
// not sit ahead of the kernel's first loads
__device__ __forceinline__ void stamp_begin_at(unsigned long long* stamp, unsigned long long t0) {
  if (stamp && threadIdx.x == 0) atomicMin(stamp, t0);
}
__device__ __forceinline__ void stamp_end(unsigned long long* stamp) {
  if (stamp) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(stamp + 1, (unsigned long long)wall_clock64());
  }
}
