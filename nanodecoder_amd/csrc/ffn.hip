// Fused position-wise feed-forward block of the transformer encoder, gfx950
// (onmt/modules/position_ffn.py:27-40 inside encoder/transformer.py:36-54):
//
//   x = y + W2 relu(W1 LN(y) + b1) + b2        (LN affine folded into W1, b1)
//
// The unfused form writes the [M, d_ff] hidden to HBM and reads it back:
// 2 x 1.07 GB per layer at B = 256 x 512, which bounded the two GEMMs
// (FFN1 0.71 ms, FFN2 0.50 ms per layer; FFN1 alone ~3x its MFMA time, most
// of it the 256 KB output write of each 256 x 256 tile with nothing left to
// overlap it).  Here the hidden never leaves the CU: a workgroup owns 128
// rows and walks d_ff in chunks of 64 hidden columns,
//
//   phase 1  H_j = relu(W1_j LN(y)^T + b1_j)    [64 x 128] on the MFMA
//   phase 2  out^T += W2_j H_j                  [256 x 128]
//
// both on v_mfma_f32_16x16x32_f16 in the split-fp16 form (hi*hi + hi*lo +
// lo*hi into fp32 accumulators, as gemm.hip H3).  The products run
// transposed so that everything the second product needs is already in a
// lane's registers: phase 1's D fragment of tile t (lane l: rows 4(l>>4)..+3
// of H^T, column l & 15) is, for the tile pair (2p, 2p+1), exactly the
// B operand of phase 2's k-block p in the P16 k-permutation (slot s < 4:
// hidden 32p + 4(l>>4) + s; s >= 4: 32p + 16 + 4(l>>4) + s - 4), which is
// the order the P16H weight images (launch_pack_p16h) and the activation
// fragments below use.  So H is split and consumed in registers, and the
// LN'd activation block (16 rows per wave) is loaded, normalised and split
// ONCE and stays resident in registers for all d_ff / 64 chunks.
//
// Per chunk the two weight slices (W1_j: 4 column tiles x 8 k-blocks,
// W2_j: 16 output tiles x 2 k-blocks, each a hi and a lo 1 KB lane-linear
// block of the P16H image, 64 KB per slice) are copied into LDS by
// global_load_lds_dwordx4 (no VGPR staging) and read by the 8 waves as
// conflict-free ds_read_b128 A operands.  Two LDS slices alternate: W1_{j+1}
// lands while phase 2 of chunk j runs, W2_{j+1} while phase 1 of j+1 runs.
// Raw s_barrier + explicit vmcnt waits (a __syncthreads would drain the
// in-flight copies).  Row statistics of x (for the next LayerNorm) come out
// of the epilogue exactly, from whole rows (one partial).
#include "common.hpp"
#include "kernels.hpp"

namespace nd {

typedef _Float16 fh8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

#define FF_BM 128                   // rows per workgroup (8 waves x 16 rows)
#define FF_HC 64                    // hidden columns per chunk
#define FF_SLICE 65536              // bytes of one weight slice in LDS
#define FF_MAXF 2048                // d_ff bound (b1 staged whole in LDS)

__device__ __forceinline__ f32x4 ffma16(fh8 a, fh8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void ff_split(f32x4 x0, f32x4 x1, fh8& hi, fh8& lo) {
  hi = {(_Float16)x0.x, (_Float16)x0.y, (_Float16)x0.z, (_Float16)x0.w,
        (_Float16)x1.x, (_Float16)x1.y, (_Float16)x1.z, (_Float16)x1.w};
  lo = {(_Float16)(x0.x - (float)hi[0]), (_Float16)(x0.y - (float)hi[1]), (_Float16)(x0.z - (float)hi[2]),
        (_Float16)(x0.w - (float)hi[3]), (_Float16)(x1.x - (float)hi[4]), (_Float16)(x1.y - (float)hi[5]),
        (_Float16)(x1.z - (float)hi[6]), (_Float16)(x1.w - (float)hi[7])};
}

// one wave copies 8 of a slice's 64 lane-linear 1 KB blocks into LDS
__device__ __forceinline__ void ff_copy_w1(const char* w1h, int j, char* dst, int wave, int lane) {
  const char* src = w1h + (size_t)j * FF_SLICE + lane * 16;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int blk = wave * 8 + i;
    __builtin_amdgcn_global_load_lds((const void*)(src + blk * 1024), (lds_void*)(dst + blk * 1024), 16, 0, 0);
  }
}
// W2 slice j: output tile nt, k-block 2j + kb2, plane -> LDS block (nt * 2 + kb2) * 2 + plane
__device__ __forceinline__ void ff_copy_w2(const char* w2h, int kp, int j, char* dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int blk = wave * 8 + i, nt = blk >> 2, kb2 = (blk >> 1) & 1, pl = blk & 1;
    const char* src = w2h + ((size_t)(nt * kp + 2 * j + kb2) * 2 + pl) * 1024 + lane * 16;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + blk * 1024), 16, 0, 0);
  }
}

__global__ void __launch_bounds__(512)
enc_ffn_kernel(const float* __restrict__ y, const uint16_t* __restrict__ w1h, float w1s, const float* __restrict__ b1,
               const uint16_t* __restrict__ w2h, float w2s, const float* __restrict__ b2, float* __restrict__ x,
               float* __restrict__ xpart, int M, int F, int* ovf) {
  // ONE shared array (a second __shared__ object beside LDS-DMA staging can
  // make hipcc drain vmcnt before every ds_read)
  __shared__ __attribute__((aligned(16))) char smem[2 * FF_SLICE + (FF_MAXF + ND_D) * 4];
  char* bufA = smem;                       // W1 slices
  char* bufB = smem + FF_SLICE;            // W2 slices
  float* sb1 = reinterpret_cast<float*>(smem + 2 * FF_SLICE);
  float* sb2 = sb1 + FF_MAXF;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, q = lane >> 4;
  const int nch = F / FF_HC, kp = F / 32;
  const char* W1 = reinterpret_cast<const char*>(w1h);
  const char* W2 = reinterpret_cast<const char*>(w2h);

  // biases (ordinary loads: done before the first copy is issued, so no wait
  // on them later drains an in-flight copy)
  for (int i = tid; i < F; i += 512) sb1[i] = b1[i];
  if (tid < ND_D) sb2[tid] = b2[tid];

  // this lane's activation fragment: row r0 + li, for every k-block kb the
  // 8 columns 32 kb + {4q..4q+3, 16+4q..16+4q+3} (the P16 k-permutation)
  const int row = blockIdx.x * FF_BM + wave * 16 + li;
  const float* yr = y + (size_t)min(row, M - 1) * ND_D + 4 * q;
  f32x4 ya[8], yb[8];
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) {
    ya[kb] = ld4(yr + 32 * kb);
    yb[kb] = ld4(yr + 32 * kb + 16);
  }
  // LayerNorm statistics of the row (the 4 lanes q = 0..3 hold it), two-pass as torch
  float s = 0.f;
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) s += (ya[kb].x + ya[kb].y + ya[kb].z + ya[kb].w) + (yb[kb].x + yb[kb].y + yb[kb].z + yb[kb].w);
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float mu = s * (1.0f / ND_D);
  float v2 = 0.f;
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) {
    const f32x4 da = ya[kb] - mu, db = yb[kb] - mu;
    v2 += (da.x * da.x + da.y * da.y + da.z * da.z + da.w * da.w) + (db.x * db.x + db.y * db.y + db.z * db.z + db.w * db.w);
  }
  v2 += __shfl_xor(v2, 16, 64);
  v2 += __shfl_xor(v2, 32, 64);
  const float rs = 1.0f / sqrtf(v2 * (1.0f / ND_D) + ND_LN_EPS);
  fh8 yh[8], yl[8];  // B operand of phase 1, resident for the whole d_ff walk
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) ff_split((ya[kb] - mu) * rs, (yb[kb] - mu) * rs, yh[kb], yl[kb]);
  __syncthreads();  // biases in LDS (and every ordinary load retired)

  ff_copy_w1(W1, 0, bufA, wave, lane);
  ff_copy_w2(W2, kp, 0, bufB, wave, lane);

  f32x4 acc[16];  // out^T tiles: lane holds out[row][16 nt + 4q + i]
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) acc[nt] = {0.f, 0.f, 0.f, 0.f};
  float hmax = 0.f;  // split-fp16 range guard over the hidden

  const f32x4* A1 = reinterpret_cast<const f32x4*>(bufA) + lane;
  const f32x4* A2 = reinterpret_cast<const f32x4*>(bufB) + lane;
  for (int j = 0; j < nch; ++j) {
    // W1_j landed (this wave's 8 copies; W2_j's 8 are younger), and every wave's
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    // ---- phase 1: H^T tiles t = 0..3 (hidden 64 j + 16 t ..), K = 256
    f32x4 h[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) h[t] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const fh8 wh = __builtin_bit_cast(fh8, A1[((t * 8 + kb) * 2) * 64]);
        const fh8 wl = __builtin_bit_cast(fh8, A1[((t * 8 + kb) * 2 + 1) * 64]);
        h[t] = ffma16(wh, yl[kb], h[t]);
        h[t] = ffma16(wl, yh[kb], h[t]);
        h[t] = ffma16(wh, yh[kb], h[t]);
      }
    fh8 hh[2], hl[2];  // B operand of phase 2 (k-blocks 0, 1 of the chunk)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x4 bv = ld4(sb1 + j * FF_HC + 16 * t + 4 * q);
      f32x4 v = h[t] * w1s + bv;
      v = {fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
      hmax = fmaxf(hmax, absmax4(v));
      h[t] = v;
    }
    ff_split(h[0], h[1], hh[0], hl[0]);
    ff_split(h[2], h[3], hh[1], hl[1]);
    // W2_j landed; every wave is done reading W1_j
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (j + 1 < nch) ff_copy_w1(W1, j + 1, bufA, wave, lane);
    // ---- phase 2: out^T tiles nt = 0..15 += W2_j H_j, K = 64
#pragma unroll
    for (int nt = 0; nt < 16; ++nt)
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2) {
        const fh8 wh = __builtin_bit_cast(fh8, A2[((nt * 2 + kb2) * 2) * 64]);
        const fh8 wl = __builtin_bit_cast(fh8, A2[((nt * 2 + kb2) * 2 + 1) * 64]);
        acc[nt] = ffma16(wh, hl[kb2], acc[nt]);
        acc[nt] = ffma16(wl, hh[kb2], acc[nt]);
        acc[nt] = ffma16(wh, hh[kb2], acc[nt]);
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave is done reading W2_j
    if (j + 1 < nch) ff_copy_w2(W2, kp, j + 1, bufB, wave, lane);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  flag_overflow(ovf, hmax);

  // ---- epilogue: x = out * w2s + b2 + y, and the row's exact statistics
  f32x4 o[16];
  float s2 = 0.f;
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) {
    const int col = 16 * nt + 4 * q;  // nt = 2 kb (+1): the lane's y columns 32 kb (+16) + 4q
    o[nt] = acc[nt] * w2s + ld4(sb2 + col) + ld4(yr + 16 * nt);
    s2 += o[nt].x + o[nt].y + o[nt].z + o[nt].w;
  }
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  const float m2 = s2 * (1.0f / ND_D);
  float q2 = 0.f;
#pragma unroll
  for (int nt = 0; nt < 16; ++nt) {
    const f32x4 d = o[nt] - m2;
    q2 += d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
  }
  q2 += __shfl_xor(q2, 16, 64);
  q2 += __shfl_xor(q2, 32, 64);
  if (row < M) {
    float* xr = x + (size_t)row * ND_D + 4 * q;
#pragma unroll
    for (int nt = 0; nt < 16; ++nt) st4(xr + 16 * nt, o[nt]);
    if (q == 0 && xpart) {
      float* p = xpart + (size_t)row * ND_PART_LD * 2;
      p[0] = m2;
      p[1] = q2;
    }
  }
}

hipError_t launch_enc_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h,
                          float w2s, const float* b2, float* x, float* xpart, int M, int F, int* ovf, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if (F % FF_HC != 0 || F > FF_MAXF || F < FF_HC || !y || !w1h || !b1 || !w2h || !b2 || !x || x == y)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(enc_ffn_kernel, dim3((M + FF_BM - 1) / FF_BM), dim3(512), 0, s, y, w1h, w1s, b1, w2h, w2s, b2,
                     x, xpart, M, F, ovf);
  return hipGetLastError();
}

}  // namespace nd
