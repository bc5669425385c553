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
// rows and walks d_ff in chunks of 32 hidden columns,
//
//   phase 1  H_j = relu(W1_j LN(y)^T + b1_j)    [32 x 128] on the MFMA
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
// ONCE and stays resident in registers for all d_ff / 32 chunks.
//
// Per chunk the two weight slices (W1_j: 2 column tiles x 8 k-blocks,
// W2_j: 16 output tiles x 1 k-block, each a hi and a lo 1 KB lane-linear
// block of the P16H image, 32 KB per slice) are copied into LDS by
// global_load_lds_dwordx4 (no VGPR staging) and read by the 8 waves as
// conflict-free ds_read_b128 A operands.  The loop is software-pipelined
// over the chunks: step k runs phase 2 of chunk k beside
// phase 1 of chunk k + 1 (independent MFMA streams, interleaved), with
// W2_k and W1_{k+1} in two of four 32 KB slots while the copies of W2_{k+1}
// and W1_{k+2} land in the other two: one barrier per step, every copy
// issued a whole step before it is read.  Raw s_barrier + explicit vmcnt
// waits (a __syncthreads would drain the in-flight copies).  Row statistics
// of x (for the next LayerNorm) come out of the epilogue exactly, from whole
// rows (one partial).  The residual and b2 are the accumulators' initial
// value ((y + b2) * 2^s): the epilogue reads nothing.
//
// WO (the attention block's output projection folded in front,
// encoder/transformer.py:45-47): the workgroup first computes its rows of
//
//   y = x + att Wo^T + bo                       (the accumulators start at (x + bo) * 2^s_o)
//
// with Wo's P16H image streamed through the W1 slots in 8 slices of 32
// output columns (each a phase-1 product against the split attention rows),
// whose out^T tiles are exactly y in the P16 k-permutation: its LayerNorm and
// split run in registers, and y never goes to HBM (the unfused form wrote it
// from a GEMM and read it back twice).
//
// QK (the next layer's QKV projection folded behind,
// encoder/transformer.py:44 of layer l + 1): the epilogue's x rows are
// LayerNorm'd from their exact statistics and split into the registers phase
// 1 used, and the 24 slices of 32 columns of W'_qkv stream through the W1
// slots (the first two issued during the last step) as 24 phase-1 products;
// q | k | v leave from the accumulators (x is not re-read by a GEMM).
#include <utility>

#include "common.hpp"
#include "kernels.hpp"

namespace nd {

typedef _Float16 fh8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

#define FF_BM 128                   // rows per workgroup (8 waves x 16 rows)
#define FF_HC 32                    // hidden columns per chunk (one k-block of phase 2)
#define FF_SLICE 32768              // bytes of one weight slice in LDS
#define FF_MAXF 2048                // d_ff bound (b1 staged whole in LDS)
#ifndef FF_SPREAD
#define FF_SPREAD 1  // the main loop's copies issued between its MFMA units (0: all at the step's start)
#endif
#ifndef FF_SPREAD_STRIDE
#define FF_SPREAD_STRIDE 2  // one piece every this many units, from unit 1
#endif
#ifndef FF_AHEAD
#define FF_AHEAD 2                  // units whose LDS reads are in flight beyond the one computed
#endif

__device__ __forceinline__ f32x4 ffma16(fh8 a, fh8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// f(std::integral_constant<int, i>) for i = 0 .. N-1: a loop whose index is a
// constant expression (inline-asm immediates)
template <typename F, int... I>
__device__ __forceinline__ void ff_static_for(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}

// the inline-asm LDS read ring of the main loop (FF_AHEAD + 1 slots): unit
// U's weight pair (hi, lo: two 1 KB lane-linear blocks 1 KB apart) at the
// constant offset (U / 2) 2048 from its slot's base (a1: W1, odd U; a2: W2)
template <int U, int RING>
__device__ __forceinline__ void ff_fetch(f32x4 (&rh)[RING], f32x4 (&rl)[RING], uint32_t a1, uint32_t a2) {
  constexpr int off = (U >> 1) * 2048;
  asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4"
               : "=&v"(rh[U % RING]), "=&v"(rl[U % RING])
               : "v"((U & 1) ? a1 : a2), "n"(off), "n"(off + 1024)
               : "memory");
}
// retire unit U's pair; the younger pairs (up to RING - 1, fewer at the end) stay in flight
template <int U, int RING, int NU>
__device__ __forceinline__ void ff_wait(f32x4 (&rh)[RING], f32x4 (&rl)[RING]) {
  constexpr int left = NU - 1 - U < RING - 1 ? NU - 1 - U : RING - 1;
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(rh[U % RING]), "+v"(rl[U % RING]) : "n"(2 * left));
}

// write-through (sc1) slab store / load of the split form (as gemm.hip's split-K)
typedef unsigned ffu4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ff_store_sc1(__amdgpu_buffer_rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ffu4, v), r, off, 0, 16);  // aux 16 = sc1
}
__device__ __forceinline__ f32x4 ff_load_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

__device__ __forceinline__ void ff_split(f32x4 x0, f32x4 x1, fh8& hi, fh8& lo) {
  hi = {(_Float16)x0.x, (_Float16)x0.y, (_Float16)x0.z, (_Float16)x0.w,
        (_Float16)x1.x, (_Float16)x1.y, (_Float16)x1.z, (_Float16)x1.w};
  lo = {(_Float16)(x0.x - (float)hi[0]), (_Float16)(x0.y - (float)hi[1]), (_Float16)(x0.z - (float)hi[2]),
        (_Float16)(x0.w - (float)hi[3]), (_Float16)(x1.x - (float)hi[4]), (_Float16)(x1.y - (float)hi[5]),
        (_Float16)(x1.z - (float)hi[6]), (_Float16)(x1.w - (float)hi[7])};
}

// NW waves copy a slice's 32 lane-linear 1 KB blocks into LDS, 32 / NW each,
// as buffer_load ... lds: one buffer descriptor per weight image (SGPRs),
// the block's byte offset in an SGPR (soffset) and lane * 16 as the only
// vector operand (the global_load_lds form kept a 64-bit address register
// pair per block live across the loop: spills once the QKV fold was added;
// FF_BUFLDS=0 keeps it)
#ifndef FF_BUFLDS
#define FF_BUFLDS 1
#endif
#if FF_BUFLDS
typedef __amdgpu_buffer_rsrc_t ff_src;
__device__ __forceinline__ ff_src ff_source(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void ff_piece(ff_src s, int off, char* dst, int lane) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s, (lds_void*)dst, 16, lane * 16, off, 0, 0);
}
#else
typedef const char* ff_src;
__device__ __forceinline__ ff_src ff_source(const void* p) { return reinterpret_cast<const char*>(p); }
__device__ __forceinline__ void ff_piece(ff_src s, int off, char* dst, int lane) {
  __builtin_amdgcn_global_load_lds((const void*)(s + off + lane * 16), (lds_void*)dst, 16, 0, 0);
}
#endif
// W1 slice j: column tiles 2j, 2j + 1 (contiguous in the P16H image)
template <int NW>
__device__ __forceinline__ void ff_copy_w1(ff_src w1h, int j, char* dst, int wave, int lane) {
  const int wu = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
  for (int i = 0; i < 32 / NW; ++i) {
    const int blk = wu * (32 / NW) + i;
    ff_piece(w1h, j * FF_SLICE + blk * 1024, dst + blk * 1024, lane);
  }
}
// piece i of this wave's share of the W1 / W2 slice copies (the main loop
// issues them one at a time between its MFMA units)
template <int NW>
__device__ __forceinline__ void ff_piece_w1(ff_src w1h, int j, char* dst, int wave, int lane, int i) {
  const int blk = __builtin_amdgcn_readfirstlane(wave) * (32 / NW) + i;
  ff_piece(w1h, j * FF_SLICE + blk * 1024, dst + blk * 1024, lane);
}
template <int NW>
__device__ __forceinline__ void ff_piece_w2(ff_src w2h, int kp, int j, char* dst, int wave, int lane, int i) {
  const int blk = __builtin_amdgcn_readfirstlane(wave) * (32 / NW) + i, nt = blk >> 1, pl = blk & 1;
  ff_piece(w2h, ((nt * kp + j) * 2 + pl) * 1024, dst + blk * 1024, lane);
}
// W2 slice j: output tile nt, k-block j, plane -> LDS block nt * 2 + plane
template <int NW>
__device__ __forceinline__ void ff_copy_w2(ff_src w2h, int kp, int j, char* dst, int wave, int lane) {
  const int wu = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
  for (int i = 0; i < 32 / NW; ++i) {
    const int blk = wu * (32 / NW) + i, nt = blk >> 1, pl = blk & 1;
    ff_piece(w2h, ((nt * kp + j) * 2 + pl) * 1024, dst + blk * 1024, lane);
  }
}

// RG row groups of 16 rows per wave, FF_BM / (16 RG) waves.  The launch uses
// RG = 1 (8 waves, two per SIMD).  RG = 2 (one wave per SIMD, each weight
// operand read from LDS feeding 6 MFMAs) measured 1.8x slower at M = 131072:
// its 512 registers spill and no second wave covers the LDS latency.
// WO: y is the block's residual input (the layer input x; x may alias it:
// a workgroup reads its rows before it writes them), att the attention
// output.  !WO: y is the FFN's input.
// DEC (launch_dec_ffn, kernels.hpp DecFfn): y and x P16-packed, the d_ff
// chunks of split blockIdx.y only, the splits' partial accumulators summed by
// the row block's last workgroup (no WO / QK fold).
template <int RG, bool WO, bool QK, bool DEC>
__global__ void __launch_bounds__(FF_BM / (16 * RG) * 64)
enc_ffn_kernel(const float* y, const uint16_t* __restrict__ w1h, float w1s, const float* __restrict__ b1,
               const uint16_t* __restrict__ w2h, float w2s, const float* __restrict__ b2, float* x,
               float* __restrict__ xpart, int M, int F, int* ovf, EncWo wo, EncQkv qk, DecFfn df) {
#ifdef ND_SKIP_FFN  // timing probe only (tools/build_variant.sh): the kernel's marginal cost
  if (threadIdx.x < 100000) return;
#endif
  static_assert(!DEC || (!WO && !QK && RG == 1), "the decoder form folds nothing");
  constexpr int NW = FF_BM / (16 * RG), NT = NW * 64;
  // the main loop's copies between its MFMA units (not in the decoder form: 6 VGPRs spilled there)
  constexpr bool SPREAD = FF_SPREAD && !DEC;
  static_assert(!SPREAD || 2 * (32 / NW) == 8, "the spread copies are 8 pieces per wave");
  // every split of a dead row block exits alike (its ticket stays 0)
  if constexpr (DEC)
    if (rows_dead(df.skip, df.skip_rpc, blockIdx.x * FF_BM, FF_BM, M)) return;
  // ONE shared array (a second __shared__ object beside LDS-DMA staging can
  // make hipcc drain vmcnt before every ds_read)
  __shared__ __attribute__((aligned(16))) char smem[4 * FF_SLICE + (FF_MAXF + ND_D + (QK ? 3 * ND_D : 0)) * 4];
  // four 32 KB slots: W1 slices of even / odd chunks, then W2 slices
  auto w1slot = [&](int i) { return smem + (i & 1) * FF_SLICE; };
  auto w2slot = [&](int i) { return smem + (2 + (i & 1)) * FF_SLICE; };
  float* sb1 = reinterpret_cast<float*>(smem + 4 * FF_SLICE);
  float* sb2 = sb1 + FF_MAXF;
  float* sqb = sb2 + ND_D;  // (QK) the next layer's q | k | v bias
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, q = lane >> 4;
  // this workgroup's d_ff chunks c0 .. c0 + nch - 1 (DEC: split sp of nsplit;
  // a chunk's W1 slice and W2 k-block sit at fixed strides in the images, so
  // the split offsets the bases; kp stays the whole W2 image's k-pair count)
  const int nall = F / FF_HC, kp = F / 32;
  const int sp = DEC ? (int)blockIdx.y : 0;
  const int c0 = DEC ? sp * nall / df.nsplit : 0;
  const int nch = DEC ? (sp + 1) * nall / df.nsplit - c0 : nall;
  const ff_src W1 = ff_source(w1h + (size_t)c0 * (FF_SLICE / 2)), W2 = ff_source(w2h + (size_t)c0 * 1024);

  // biases (ordinary loads: done before the first copy is issued, so no wait
  // on them later drains an in-flight copy)
  for (int i = tid; i < nch * FF_HC; i += NT) sb1[i] = b1[c0 * FF_HC + i];
  for (int i = tid; i < ND_D; i += NT) sb2[i] = b2[i];
  if constexpr (QK)
    for (int i = tid; i < 3 * ND_D; i += NT) sqb[i] = qk.bias[i];

  // row group g's activation fragment: row r0 + 16 g + li, for every
  // k-block kb the 8 columns 32 kb + {4q..4q+3, 16+4q..16+4q+3} (the P16
  // k-permutation), LayerNorm'd (two-pass statistics over the 4 lanes
  // q = 0..3 that hold the row, as torch) and split: phase 1's B operand,
  // resident for the whole d_ff walk.  The lane's out^T accumulator tiles
  // nt = 2 kb, 2 kb + 1 hold the same columns (out[row][16 nt + 4q + i])
  fh8 yh[RG][8], yl[RG][8];
  f32x4 acc[RG][16];  // out^T tiles: lane holds out[row g][16 nt + 4q + i]
  int row[RG];
  const float rw2 = 1.0f / w2s;  // 2^s: exact
  // y (pre-LN, fp32, in the accumulator layout) -> the split LN(y) and the
  // accumulators' initial value (y + b2) 2^s (b2 from bsrc: global, or LDS
  // once the copies are in flight: a global load then would wait for them)
  auto ln_split = [&](int g, f32x4 (&ya)[8], f32x4 (&yb)[8], const float* bsrc) {
    float s = 0.f;
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
      s += (ya[kb].x + ya[kb].y + ya[kb].z + ya[kb].w) + (yb[kb].x + yb[kb].y + yb[kb].z + yb[kb].w);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s * (1.0f / ND_D);
    float v2 = 0.f;
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      const f32x4 da = ya[kb] - mu, db = yb[kb] - mu;
      v2 += (da.x * da.x + da.y * da.y + da.z * da.z + da.w * da.w) +
            (db.x * db.x + db.y * db.y + db.z * db.z + db.w * db.w);
    }
    v2 += __shfl_xor(v2, 16, 64);
    v2 += __shfl_xor(v2, 32, 64);
    const float rs = ln_rsqrt(v2 * (1.0f / ND_D) + ND_LN_EPS);
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      ff_split((ya[kb] - mu) * rs, (yb[kb] - mu) * rs, yh[g][kb], yl[g][kb]);
      acc[g][2 * kb] = (ya[kb] + ld4(bsrc + 32 * kb + 4 * q)) * rw2;
      acc[g][2 * kb + 1] = (yb[kb] + ld4(bsrc + 32 * kb + 16 + 4 * q)) * rw2;
    }
  };
  auto p1_mfma = [&](fh8 wh, fh8 wl, int t, int kb, f32x4 (&h)[RG][2]) {
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      h[g][t] = ffma16(wh, yl[g][kb], h[g][t]);
      h[g][t] = ffma16(wl, yh[g][kb], h[g][t]);
      h[g][t] = ffma16(wh, yh[g][kb], h[g][t]);
    }
  };
#pragma unroll
  for (int g = 0; g < RG; ++g) row[g] = blockIdx.x * FF_BM + (wave * RG + g) * 16 + li;

  if constexpr (WO) {
    // the attention rows, split (no LayerNorm: the range guard), and the
    // accumulators' initial value (x + bo) 2^s_o
    const float rwo = 1.0f / wo.wos;
    float amax = 0.f;
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      const float* ar = wo.att + (size_t)min(row[g], M - 1) * ND_D + 4 * q;
      const float* xr = y + (size_t)min(row[g], M - 1) * ND_D + 4 * q;
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        const f32x4 a0 = ld4(ar + 32 * kb), a1 = ld4(ar + 32 * kb + 16);
        amax = fmaxf(amax, fmaxf(absmax4(a0), absmax4(a1)));
        ff_split(a0, a1, yh[g][kb], yl[g][kb]);
        acc[g][2 * kb] = (ld4(xr + 32 * kb) + ld4(wo.bo + 32 * kb + 4 * q)) * rwo;
        acc[g][2 * kb + 1] = (ld4(xr + 32 * kb + 16) + ld4(wo.bo + 32 * kb + 16 + 4 * q)) * rwo;
      }
    }
    flag_overflow(ovf, amax);
    __syncthreads();  // the biases in LDS (and every ordinary load retired)
    // y = the accumulators + att Wo^T: slice j (output columns 32 j .. +31,
    // tiles 2 j, 2 j + 1) from w1slot(j); W1_0 and W2_0 go out with the last
    const ff_src WoH = ff_source(wo.woh);
    ff_copy_w1<NW>(WoH, 0, w1slot(0), wave, lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      if (j + 1 < 8) {
        ff_copy_w1<NW>(WoH, j + 1, w1slot(j + 1), wave, lane);
      } else {
        ff_copy_w1<NW>(W1, 0, w1slot(0), wave, lane);
        ff_copy_w2<NW>(W2, kp, 0, w2slot(0), wave, lane);
      }
      const f32x4* A = reinterpret_cast<const f32x4*>(w1slot(j)) + lane;
      f32x4 h[RG][2];
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        h[g][0] = acc[g][2 * j];
        h[g][1] = acc[g][2 * j + 1];
      }
#pragma unroll
      for (int kb = 0; kb < 8; ++kb)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          p1_mfma(__builtin_bit_cast(fh8, A[((t * 8 + kb) * 2) * 64]),
                  __builtin_bit_cast(fh8, A[((t * 8 + kb) * 2 + 1) * 64]), t, kb, h);
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        acc[g][2 * j] = h[g][0];
        acc[g][2 * j + 1] = h[g][1];
      }
    }
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      f32x4 ya[8], yb[8];
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        ya[kb] = acc[g][2 * kb] * wo.wos;
        yb[kb] = acc[g][2 * kb + 1] * wo.wos;
      }
      ln_split(g, ya, yb, sb2);
    }
    asm volatile("s_barrier" ::: "memory");  // every wave is done with Wo's last slice (slot 1)
    if (nch > 1) ff_copy_w1<NW>(W1, 1, w1slot(1), wave, lane);
  } else {
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      const int rc = min(row[g], M - 1);
      const float* yr = y + (size_t)rc * ND_D + 4 * q;
      f32x4 ya[8], yb[8];
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        if constexpr (DEC) {
          ya[kb] = ld4(y + pk(rc, 32 * kb + 4 * q, ND_D));
          yb[kb] = ld4(y + pk(rc, 32 * kb + 16 + 4 * q, ND_D));
        } else {
          ya[kb] = ld4(yr + 32 * kb);
          yb[kb] = ld4(yr + 32 * kb + 16);
        }
      }
      ln_split(g, ya, yb, b2);
      if constexpr (DEC)
        if (sp > 0)  // b2 and the residual enter once, through split 0
#pragma unroll
          for (int nt = 0; nt < 16; ++nt) acc[g][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();  // the biases in LDS (and every ordinary load retired)
    ff_copy_w1<NW>(W1, 0, w1slot(0), wave, lane);
    ff_copy_w2<NW>(W2, kp, 0, w2slot(0), wave, lane);
    if (nch > 1) ff_copy_w1<NW>(W1, 1, w1slot(1), wave, lane);
  }
  float hmax = 0.f;  // split-fp16 range guard over the hidden
  fh8 hh[RG], hl[RG];  // H of the chunk phase 2 works on, split: its B operand

  // H of chunk j: bias, ReLU, range guard, split into phase 2's B operand
  auto finish_h = [&](int j, f32x4 (&h)[RG][2]) {
#pragma unroll
    for (int g = 0; g < RG; ++g) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 v = h[g][t] * w1s + ld4(sb1 + j * FF_HC + 16 * t + 4 * q);
        v = {fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
        hmax = fmaxf(hmax, absmax4(v));
        h[g][t] = v;
      }
      ff_split(h[g][0], h[g][1], hh[g], hl[g]);
    }
  };
  auto p2_mfma = [&](fh8 wh, fh8 wl, int nt) {
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      acc[g][nt] = ffma16(wh, hl[g], acc[g][nt]);
      acc[g][nt] = ffma16(wl, hh[g], acc[g][nt]);
      acc[g][nt] = ffma16(wh, hh[g], acc[g][nt]);
    }
  };

  // prologue: phase 1 of chunk 0 (W1_0 and W2_0 landed; W1_1 may be in flight)
  {
    if (nch > 1)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(32 / NW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    const f32x4* A1 = reinterpret_cast<const f32x4*>(w1slot(0)) + lane;
    f32x4 h[RG][2];
#pragma unroll
    for (int g = 0; g < RG; ++g) h[g][0] = h[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        p1_mfma(__builtin_bit_cast(fh8, A1[((t * 8 + kb) * 2) * 64]),
                __builtin_bit_cast(fh8, A1[((t * 8 + kb) * 2 + 1) * 64]), t, kb, h);
    finish_h(0, h);
  }
  // step k: phase 2 of chunk k (W2_k, slot k & 1) beside phase 1 of chunk
  // k + 1 (W1_{k+1}, slot (k + 1) & 1); copies of W2_{k+1} and W1_{k+2} land
  // meanwhile in the slots step k - 1 used
  for (int k = 0; k < nch; ++k) {
    // W2_k, W1_{k+1} landed (issued a step ago, the only copies in flight),
    // every wave's too; every wave is done with step k - 1's slots
#ifdef FF_PROBE_NOBAR  // timing probe only: no step barrier (wrong results)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#else
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
#ifndef FF_PROBE_NOCOPY  // timing probe only: no weight copies in the main loop (wrong results)
    if constexpr (!SPREAD) {
      if (k + 1 < nch) ff_copy_w2<NW>(W2, kp, k + 1, w2slot(k + 1), wave, lane);
      if (k + 2 < nch) ff_copy_w1<NW>(W1, k + 2, w1slot(k), wave, lane);
    }
#endif
    const f32x4* A2 = reinterpret_cast<const f32x4*>(w2slot(k)) + lane;
    const f32x4* A1 = reinterpret_cast<const f32x4*>(w1slot(k + 1)) + lane;
    if (k + 1 == nch) {  // the last step: phase 2 alone (QK: the W1 slots take W'_qkv's first slices)
      if constexpr (QK) {
        ff_copy_w1<NW>(ff_source(qk.wh), 0, w1slot(0), wave, lane);
        ff_copy_w1<NW>(ff_source(qk.wh), 1, w1slot(1), wave, lane);
      }
#pragma unroll
      for (int nt = 0; nt < 16; ++nt)
        p2_mfma(__builtin_bit_cast(fh8, A2[(nt * 2) * 64]), __builtin_bit_cast(fh8, A2[(nt * 2 + 1) * 64]), nt);
      continue;
    }
    // 32 units, even: phase 2 of chunk k on output tile u / 2, odd: phase 1
    // of chunk k + 1 on (tile, k-block) = ((u / 2) / 8, (u / 2) % 8); each is
    // a hi and a lo ds_read_b128 operand and 3 RG MFMAs.  The reads go out
    // FF_AHEAD units ahead into a (FF_AHEAD + 1)-deep register ring from
    // inline asm (left to itself hipcc sinks every LDS read to its use and
    // waits on it: 12 % slower), and each unit waits only for its own pair
    // (lgkmcnt(2 FF_AHEAD): the younger pairs stay in flight under this unit's
    // MFMAs).  Addresses are one base register per slot plus the unit's
    // constant offset (immediates: no per-unit address registers).  The "+v"
    // ties make the data defined at the wait; tools/lds_ring_check.py
    // verifies on the compiled code that nothing touches a ring register in
    // between (tests/test_abi.py)
    constexpr int RING = FF_AHEAD + 1;
    const uint32_t a2 = (uint32_t)(uintptr_t)A2, a1 = (uint32_t)(uintptr_t)A1;
    f32x4 rh[RING], rl[RING];
    f32x4 h[RG][2];
#pragma unroll
    for (int g = 0; g < RG; ++g) h[g][0] = h[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    ff_static_for([&](auto uc) { ff_fetch<decltype(uc)::value, RING>(rh, rl, a1, a2); },
                  std::make_integer_sequence<int, FF_AHEAD>{});
    // SPREAD: this step's copies (W2_{k+1}, then W1_{k+2}: its chunk index clamped, so the
    // step before the last re-copies a slice into the free slot instead of branching
    // inside the read ring), one piece every second unit of the first half: each
    // piece's issue sits between MFMAs the SIMD's other wave keeps running, and
    // 16 units remain for the last to land before the next step's vmcnt(0)
    const int j1 = min(k + 2, nch - 1);
    ff_static_for(
        [&](auto uc) {
          constexpr int u = decltype(uc)::value;
          if constexpr (SPREAD && u % FF_SPREAD_STRIDE == 1 && u < 1 + 8 * FF_SPREAD_STRIDE) {
            constexpr int p = u / FF_SPREAD_STRIDE;
            if constexpr (p < 32 / NW)
              ff_piece_w2<NW>(W2, kp, k + 1, w2slot(k + 1), wave, lane, p);
            else
              ff_piece_w1<NW>(W1, j1, w1slot(k), wave, lane, p - 32 / NW);
          }
          if constexpr (u + FF_AHEAD < 32) ff_fetch<u + FF_AHEAD, RING>(rh, rl, a1, a2);
          ff_wait<u, RING, 32>(rh, rl);
          const fh8 wh = __builtin_bit_cast(fh8, rh[u % RING]), wl = __builtin_bit_cast(fh8, rl[u % RING]);
          if constexpr (u & 1)
            p1_mfma(wh, wl, (u >> 1) >> 3, (u >> 1) & 7, h);
          else
            p2_mfma(wh, wl, u >> 1);
        },
        std::make_integer_sequence<int, 32>{});
    finish_h(k + 1, h);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  flag_overflow(ovf, hmax);
  if constexpr (DEC) {
    if (df.nsplit > 1) {
      // the row block's slab [split][16 tiles][NT threads] f32x4: write-through
      // (sc1) stores, every wave's vmcnt(0), one agent-scope ticket; the last
      // arriver reads the other splits back with sc1 loads and sums all of
      // them in split order (its own from registers: the same bits it stored)
      const int S = df.nsplit;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          df.slab + (size_t)blockIdx.x * S * 16 * NT * 4, 0, S * 16 * NT * 16, 0x00020000);
#pragma unroll
      for (int nt = 0; nt < 16; ++nt) ff_store_sc1(rs, ((sp * 16 + nt) * NT + tid) * 16, acc[0][nt]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* tword = reinterpret_cast<int*>(sb2);  // (b2 came from global memory: the slot is free)
      if (tid == 0) tword[0] = __hip_atomic_fetch_add(df.tickets + blockIdx.x, 1, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if (tword[0] != S - 1) return;  // not the row block's last split
      f32x4 sum[16];
#pragma unroll
      for (int nt = 0; nt < 16; ++nt) sum[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s2 = 0; s2 < S; ++s2) {
        if (s2 == sp) {
#pragma unroll
          for (int nt = 0; nt < 16; ++nt) sum[nt] += acc[0][nt];
        } else {
          f32x4 pp[16];
#pragma unroll
          for (int nt = 0; nt < 16; ++nt) pp[nt] = ff_load_sc1(rs, ((s2 * 16 + nt) * NT + tid) * 16);
#pragma unroll
          for (int nt = 0; nt < 16; ++nt) sum[nt] += pp[nt];
        }
      }
#pragma unroll
      for (int nt = 0; nt < 16; ++nt) acc[0][nt] = sum[nt];
      if (tid == 0) __hip_atomic_store(df.tickets + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  // ---- epilogue: x = out * w2s (b2 and the residual were the accumulators'
  //      initial value), and the row's exact statistics
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    f32x4 o[16];
    float s2 = 0.f;
#pragma unroll
    for (int nt = 0; nt < 16; ++nt) {
      o[nt] = acc[g][nt] * w2s;
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
    if (row[g] < M) {
      float* xr = x + (size_t)row[g] * ND_D + 4 * q;
#pragma unroll
      for (int nt = 0; nt < 16; ++nt) {
        if constexpr (DEC)
          st4(x + pk(row[g], 16 * nt + 4 * q, ND_D), o[nt]);
        else
          st4(xr + 16 * nt, o[nt]);
      }
      if (q == 0 && xpart) {
        float* p = xpart + (size_t)row[g] * ND_PART_LD * 2;
        p[0] = m2;
        p[1] = q2;
      }
    }
    if constexpr (QK) {  // LN(x) (the next layer's LayerNorm, affine folded into W'), split
      const float rs = ln_rsqrt(q2 * (1.0f / ND_D) + ND_LN_EPS);
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) ff_split((o[2 * kb] - m2) * rs, (o[2 * kb + 1] - m2) * rs, yh[g][kb], yl[g][kb]);
    }
  }
  if constexpr (QK) {
    // 24 slices of 32 output columns; slice j in W1 slot j & 1, the copy of
    // slice j + 1 issued at the top of step j (slices 0 and 1: during the
    // last main step).  Rows past M store the values of row M - 1 (their
    // inputs were clamped to it): identical bytes, straight-line stores, so
    // vmcnt(2 RG) at the top of a step (the previous step's stores) counts
    // the copy exactly
    const ff_src QH = ff_source(qk.wh);
    for (int j = 0; j < 3 * ND_D / FF_HC; ++j) {
      if (j == 0)
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * RG) : "memory");
      if (j >= 1 && j + 1 < 3 * ND_D / FF_HC) ff_copy_w1<NW>(QH, j + 1, w1slot(j + 1), wave, lane);
      const f32x4* A = reinterpret_cast<const f32x4*>(w1slot(j)) + lane;
      f32x4 h[RG][2];
#pragma unroll
      for (int g = 0; g < RG; ++g) h[g][0] = h[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 8; ++kb)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          p1_mfma(__builtin_bit_cast(fh8, A[((t * 8 + kb) * 2) * 64]),
                  __builtin_bit_cast(fh8, A[((t * 8 + kb) * 2 + 1) * 64]), t, kb, h);
#pragma unroll
      for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int n = FF_HC * j + 16 * t + 4 * q;
          st4(qk.out + (size_t)min(row[g], M - 1) * 3 * ND_D + n, h[g][t] * qk.ws + ld4(sqb + n));
        }
    }
  }
}

hipError_t launch_enc_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h,
                          float w2s, const float* b2, float* x, float* xpart, int M, int F, int* ovf, hipStream_t s,
                          const EncWo* wo, const EncQkv* qk) {
  if (M <= 0) return hipSuccess;
  if (F % FF_HC != 0 || F > FF_MAXF || F < FF_HC || !y || !w1h || !b1 || !w2h || !b2 || !x)
    return hipErrorInvalidValue;
  if (wo && (!wo->att || !wo->woh || !wo->bo || wo->att == x || wo->att == y)) return hipErrorInvalidValue;
  if (!wo && x == y) return hipErrorInvalidValue;  // with wo, x may alias y (the residual): each
                                                    // workgroup reads its rows before it writes them
  if (qk && (!qk->wh || !qk->bias || !qk->out || qk->out == x || qk->out == y || (wo && qk->out == wo->att)))
    return hipErrorInvalidValue;
  const dim3 grid((M + FF_BM - 1) / FF_BM), block(FF_BM / 16 * 64);
  const EncWo w = wo ? *wo : EncWo();
  const EncQkv k = qk ? *qk : EncQkv();
#define ND_FFN_GO(WO, QK)                                                                                          \
  hipLaunchKernelGGL((enc_ffn_kernel<1, WO, QK, false>), grid, block, 0, s, y, w1h, w1s, b1, w2h, w2s, b2, x, xpart, \
                     M, F, ovf, w, k, DecFfn())
  if (wo && qk)
    ND_FFN_GO(true, true);
  else if (wo)
    ND_FFN_GO(true, false);
  else if (qk)
    ND_FFN_GO(false, true);
  else
    ND_FFN_GO(false, false);
#undef ND_FFN_GO
  return hipGetLastError();
}

size_t dec_ffn_slab_floats(int M, int nsplit) {
  return (size_t)((M + FF_BM - 1) / FF_BM) * nsplit * 16 * (FF_BM / 16 * 64) * 4;
}

hipError_t launch_dec_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h,
                          float w2s, const float* b2, float* x, float* xpart, int M, int F, int* ovf,
                          const DecFfn& df, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if (F % FF_HC != 0 || F > FF_MAXF || F < FF_HC || M % 16 || !y || !w1h || !b1 || !w2h || !b2 || !x || x == y)
    return hipErrorInvalidValue;
  if (df.nsplit < 1 || df.nsplit > F / FF_HC || (df.nsplit > 1 && (!df.slab || !df.tickets)) ||
      (df.skip && df.skip_rpc < 1))
    return hipErrorInvalidValue;
  const dim3 grid((M + FF_BM - 1) / FF_BM, df.nsplit), block(FF_BM / 16 * 64);
  hipLaunchKernelGGL((enc_ffn_kernel<1, false, false, true>), grid, block, 0, s, y, w1h, w1s, b1, w2h, w2s, b2, x,
                     xpart, M, F, ovf, EncWo(), EncQkv(), df);
  return hipGetLastError();
}

}  // namespace nd
