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

__device__ __forceinline__ float wave_sum(float v) {
  v = sum16(v);
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

__device__ __forceinline__ float wave_max(float v) {
  v = max16(v);
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
