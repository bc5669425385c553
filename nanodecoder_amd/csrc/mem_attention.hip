// Memory-bank form of the decoder's context attention (greedy decoding), gfx950.
//
// With the decoder's ctx K/V projections folded into the query and output
// sides (engine finalize: W_qk[h] = W_k,h^T W_q,h / sqrt(d_h),
// W_vo[:, h] = W_o,h W_v,h), head h of a decoder row needs only the encoder
// memory bank m_t (256 floats per source position, shared by all three
// decoder layers) instead of a per-layer K and V
// (onmt/modules/multi_headed_attn.py:142-179, decoder/transformer.py:88-92):
//   s_h(t) = q'_h . m_t        (q'_h = W_qk[h] LN(x) + b_qk[h]; the dropped
//                               q_h . b_k,h is constant in t: softmax-exact)
//   U_h    = sum_t softmax_t(s_h)(t) m_t,   out = W_vo U + b_vo
// Mask: src == pad -> -1e18 (multi_headed_attn.py:172); t >= span: absent.
//
// Per chunk the work is two skinny products over the chunk's [T, 256] bank,
// S = M Q'^T (8 heads) and U = P^T M.  With only 8 query rows a 16-wide MFMA
// tile would be half padding, so both run on v_mfma_f32_4x4x1_16b_f32
// (16 independent 4x4 outer products per instruction, f32 in / f32 acc,
// probe: tools/probe_mfma4x4.hip), whose 4-wide blocks tile 8 heads exactly.
//
// One workgroup (8 waves) per chunk.  Keys are split over the waves, 8 per
// wave per 64-key tile, so every wave works on its own keys only and runs its
// own online softmax; the waves meet once, at the end, to merge (m, l, U).
//  - Staging: each of the wave's 8 key rows (1 KB, contiguous in HBM) is one
//    global_load_lds_dwordx4 into the wave's private LDS slab, double
//    buffered, the next tile in flight while this one computes.  Row k is
//    stored rotated by 4k floats (rotation applied on the per-lane source
//    address, the LDS side stays lane-linear), which makes both read
//    patterns below bank-conflict-free.
//  - S: block b of the 4x4x1 instruction = (dim class dp, key quad kg,
//    head quad hg); dp is the ds_read_b128 lane group the block sits in, so
//    the 16 lanes of a group read 8 distinct rows at distinct bank quads.
//    Lane (b, x) supplies A = m[key 4kg+x][d] and B = q'[head 4hg+x][d] for
//    the 64 dims d of class dp (its q' slice lives in 64 VGPRs for the whole
//    launch).  The 4 class partials meet through a 1 KB LDS slab.
//  - U: block b = (dim octet dg, head quad hg), one key per instruction:
//    A = p[key][4hg+i], B = m[key][dims of the lane] (two 16 B reads of the
//    key's row), 8 accumulators of 4 = the wave's U for all 8 x 256 outputs.
#include <algorithm>

#include "common.hpp"
#include "kernels.hpp"

#include <cstdlib>

namespace nd {

#define MB_NW 8                      // waves per chunk (2 per SIMD)
#define MB_KW 8                      // keys per wave per tile
#define MB_TILE (MB_NW * MB_KW)      // keys per tile
#define MB_WAVE (2 * MB_KW * ND_D + 2 * 256 + 64)  // floats of LDS per wave: 2 tile slabs, 2 S-partial slabs, P
#define MB_U (MB_NW * MB_WAVE)       // q' image [8 heads][256], row h rotated by 4h floats
#define MB_ML (MB_U + ND_H * ND_D)   // merge: per wave and head (m, l)
#define MB_LDS_FLOATS (MB_ML + MB_NW * 16)

__device__ __forceinline__ f32x4 mfma4x4(float a, float b, f32x4 c) {
  // lane 4b+i supplies A_b[i], lane 4b+j supplies B_b[j]; lane 4b+j, reg i
  // accumulates A_b[i] * B_b[j]
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

#define ND_DPP_ROR8 0x128  // row_ror:8 inside a 16-lane row == lane ^ 8

// over the 8 lanes sharing lane & 7
__device__ __forceinline__ float max_by8(float v) {
  v = fmaxf(v, dpp_mov<ND_DPP_ROR8>(v));
  return xor32_max(xor16_max(v));
}
__device__ __forceinline__ float sum_by8(float v) {
  v += dpp_mov<ND_DPP_ROR8>(v);
  return xor32_sum(xor16_sum(v));
}

// NT > 0: the tile count is the compile-time NT (T in (64 (NT-1), 64 NT]);
// every tile is processed (keys >= span masked), so the tile loop unrolls to
// straight-line code and the compiler's wait counts on the in-flight tile
// loads stay exact (a runtime loop makes it drain them every iteration).
template <int NT>
__global__ void __launch_bounds__(MB_NW * 64)
dec_mem_attention_kernel(const float* __restrict__ qp, const float* __restrict__ mem,
                         const float* __restrict__ signal, const int* __restrict__ span, float pad_val,
                         float* __restrict__ out, int T, int ldT, unsigned long long* stamp,
                         float* __restrict__ dbg, size_t dbg_stride) {
  stamp_begin(stamp);
  extern __shared__ float lds[];
  const int c = blockIdx.x, lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar addressing)
  float* slab = lds + w * MB_WAVE;            // [2][8 keys][256], row k rotated by 4k floats
  float* spart = slab + 2 * MB_KW * ND_D;     // [2][4 dp][8 heads][8 keys]
  float* pbuf = spart + 2 * 256;              // [8 heads][8 keys]
  const float* ub = lds + MB_U;
  const int L = min(span[c], T);
  const int ntile = NT > 0 ? NT : (L + MB_TILE - 1) / MB_TILE;
  const float* mc = mem + (size_t)c * ldT * ND_D;

  // ---- lane roles
  // S: block b = lane >> 2, x = lane & 3
  const int b = lane >> 2, x = lane & 3;
  const int dp = 2 * (b >> 3) + (__builtin_popcount(b & 7) & 1);  // ds_read_b128 lane group of block b
  const int kg = (b >> 2) & 1, hg = (b >> 1) & 1;                   // rank within the group
  const int skey = 4 * kg + x, shead = 4 * hg + x;
  // softmax: lane -> (key sk, head sh)
  const int sk = lane >> 3, sh = lane & 7;
  // U: lane's dims 4zm..4zm+3 and 128+4zm..+3; A operand head = sh
  const int zm = 4 * (lane >> 3) + (lane & 3);

  // Staging through registers, four tiles in flight (two in registers, two
  // in LDS): lane l loads 16 B of each of the wave's 8 rows (one coalesced
  // 1 KB row per instruction) and writes them to a slab at the row's rotation.
  auto fetch = [&](int r, f32x4(&dst)[MB_KW]) {
#pragma unroll
    for (int k = 0; k < MB_KW; ++k) {
      const int t = min(r * MB_TILE + w * MB_KW + k, T - 1);
      dst[k] = ld4(mc + (size_t)t * ND_D + 4 * lane);
    }
  };
  auto put = [&](int r, const f32x4(&src)[MB_KW]) {
    float* dst = slab + (r & 1) * (MB_KW * ND_D);
#pragma unroll
    for (int k = 0; k < MB_KW; ++k) st4(dst + k * ND_D + ((4 * lane + 4 * k) & (ND_D - 1)), src[k]);
  };
  // S partial of tile r over dim class dp: lane 4b+j, reg i = s[key 4kg+i][head 4hg+j]
  auto scores = [&](int r) {
    const float* arow = slab + (r & 1) * (MB_KW * ND_D) + skey * ND_D;
    const float* urow = ub + shead * ND_D;
    f32x4 s4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) s4[e] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const f32x4 a = ld4(arow + ((64 * dp + 4 * kk + 4 * skey) & (ND_D - 1)));
      const f32x4 u = ld4(urow + ((64 * dp + 4 * kk + 4 * shead) & (ND_D - 1)));
#pragma unroll
      for (int e = 0; e < 4; ++e) s4[e] = mfma4x4(a[e], u[e], s4[e]);
    }
    return (s4[0] + s4[1]) + (s4[2] + s4[3]);
  };
  auto put_scores = [&](int r, f32x4 v) { st4(spart + (r & 1) * 256 + (dp * 8 + shead) * 8 + 4 * kg, v); };

  // The source samples of this wave's keys (lane l -> tile l >> 3, key l & 7)
  // load FIRST: the waits that retire the tile loads below then retire it
  // too, so no wait for it is left inside the loop (where it would drain
  // the prefetched tiles every iteration).
  const float sgv = signal[(size_t)c * T + min((lane >> 3) * MB_TILE + w * MB_KW + (lane & 7), T - 1)];
  f32x4 R0[MB_KW], R1[MB_KW];
  if (ntile > 0) fetch(0, R0);
  if (ntile > 1) fetch(1, R1);
  // q' image (all heads; 512 threads x 16 B)
  {
    const int h = threadIdx.x >> 6, q = threadIdx.x & 63;
    st4(lds + MB_U + h * ND_D + ((4 * q + 4 * h) & (ND_D - 1)), ld4(qp + pk(c, h * ND_D + 4 * q, ND_H * ND_D)));
  }
  if (ntile > 0) put(0, R0);
  if (ntile > 1) put(1, R1);
  if (ntile > 2) fetch(2, R0);
  if (ntile > 3) fetch(3, R1);
  lds_barrier();  // q' image (tiles 2 and 3 stay in flight)
  if (ntile > 0) put_scores(0, scores(0));

  f32x4 acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = {0.f, 0.f, 0.f, 0.f};
  float mrun = -INFINITY, lrun = 0.f;  // online-softmax state of head sh over this wave's keys

  // Iteration r: the scores of tile r + 1 (MFMA) overlap the softmax of tile r
  // (LDS/VALU latency), then U += P^T M for tile r; then tile r + 2 (in R,
  // fetched two iterations earlier) goes to the freed slab and R refills with
  // tile r + 4.
  auto body = [&](int r, f32x4(&R)[MB_KW]) {
    const f32x4 snext = scores(r + 1);  // tile r + 1's slab (garbage past the last tile, unused)

    // ---- online softmax of head sh over the tile's 8 keys of this wave
    const float* sp = spart + (r & 1) * 256 + sh * 8 + sk;
    float s = (sp[0] + sp[64]) + (sp[128] + sp[192]);
    const int t = r * MB_TILE + w * MB_KW + sk;
    const float sg = __shfl(sgv, r * 8 + sk);
    s = t < L ? (sg == pad_val ? ND_MASK_FILL : s) : -INFINITY;
    if (dbg && sh == 0 && t < L) dbg[(size_t)c * dbg_stride + t] = s;  // -attn_debug: head 0's scores
    const float mnew = fmaxf(mrun, max_by8(s));
    const float scale = mnew == -INFINITY ? 1.f : __expf(mrun - mnew);
    const float p = s == -INFINITY ? 0.f : __expf(s - mnew);
    lrun = lrun * scale + sum_by8(p);
    mrun = mnew;
    pbuf[sh * 8 + sk] = p;
    {
      // acc reg i belongs to head 4((lane>>2)&1) + i = the softmax head of quad lane i
      const float sc0 = dpp_mov<0x00>(scale), sc1 = dpp_mov<0x55>(scale);
      const float sc2 = dpp_mov<0xAA>(scale), sc3 = dpp_mov<0xFF>(scale);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[e][0] *= sc0;
        acc[e][1] *= sc1;
        acc[e][2] *= sc2;
        acc[e][3] *= sc3;
      }
    }

    // ---- U += P^T M over the tile's 8 keys of this wave
    const f32x4 p0 = ld4(pbuf + sh * 8), p1 = ld4(pbuf + sh * 8 + 4);
    const float* tile = slab + (r & 1) * (MB_KW * ND_D);
#pragma unroll
    for (int k = 0; k < MB_KW; ++k) {
      const float* row = tile + k * ND_D;
      const f32x4 b0 = ld4(row + ((4 * zm + 4 * k) & (ND_D - 1)));
      const f32x4 b1 = ld4(row + ((128 + 4 * zm + 4 * k) & (ND_D - 1)));
      const float pk_ = k < 4 ? p0[k] : p1[k - 4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[e] = mfma4x4(pk_, b0[e], acc[e]);
        acc[4 + e] = mfma4x4(pk_, b1[e], acc[4 + e]);
      }
    }
    put_scores(r + 1, snext);
    // the wave's LDS accesses retire in order: tile r + 2 lands after tile r's reads
    if (r + 2 < ntile) put(r + 2, R);
    if (r + 4 < ntile) fetch(r + 4, R);
  };
  if constexpr (NT > 0) {
#pragma unroll
    for (int r = 0; r < NT; r += 2) {
      body(r, R0);
      if (r + 1 < NT) body(r + 1, R1);
    }
  } else {
    for (int r = 0; r < ntile; r += 2) {
      body(r, R0);
      if (r + 1 < ntile) body(r + 1, R1);
    }
  }

  // ---- merge the waves: head h's slots are combined by wave h
  __syncthreads();  // every wave is done with its slabs
  float* red = lds;               // [NW][512 slots][4]; slot = head * 64 + dim quad
  float* ml = lds + MB_ML;        // [NW][8 heads][2]
  if (lane < 8) {
    ml[(w * 8 + lane) * 2] = mrun;  // lane < 8: sh == lane
    ml[(w * 8 + lane) * 2 + 1] = lrun;
  }
  {
    const int hb = 4 * ((lane >> 2) & 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 lo = {acc[0][i], acc[1][i], acc[2][i], acc[3][i]};
      const f32x4 hi = {acc[4][i], acc[5][i], acc[6][i], acc[7][i]};
      st4(red + ((size_t)w * 512 + (hb + i) * 64 + zm) * 4, lo);
      st4(red + ((size_t)w * 512 + (hb + i) * 64 + 32 + zm) * 4, hi);
    }
  }
  __syncthreads();
  const int h = w;  // this wave finishes head h: dims 4 lane .. 4 lane + 3
  float M = -INFINITY;
#pragma unroll
  for (int v = 0; v < MB_NW; ++v) M = fmaxf(M, ml[(v * 8 + h) * 2]);
  f32x4 num = {0.f, 0.f, 0.f, 0.f};
  float den = 0.f;
#pragma unroll
  for (int v = 0; v < MB_NW; ++v) {
    const float mv = ml[(v * 8 + h) * 2];
    const float f = mv == -INFINITY ? 0.f : __expf(mv - M);  // waves that owned no key
    den += f * ml[(v * 8 + h) * 2 + 1];
    num += f * ld4(red + ((size_t)v * 512 + h * 64 + lane) * 4);
  }
  st4(out + pk(c, h * ND_D + 4 * lane, ND_H * ND_D), num * (den > 0.f ? __builtin_amdgcn_rcpf(den) : 0.f));
  stamp_end(stamp);
}

// ---------------------------------------------------------------------------
// Split-fp16 form (T in (448, 512] with 512-row bank buffers: every bench and
// translate batch of 512-sample chunks).  The kernel above runs both
// products on fp32 4x4x1 MFMAs (8192 per chunk, ~9 us of matrix-core time per
// CU) and stages every bank tile through LDS three times; its compute side
// alone takes ~22 us against a ~17-20 us bank stream.  Here:
//  - the bank is packed ONCE per call (bank_pack_h3_kernel) as fp16 hi / lo
//    planes in the A-operand fragment order of v_mfma_f32_16x16x32_f16:
//    fragment (chunk, key block kb of 16 keys, dim block db of 32, plane) is
//    1 KB, lane l holding key 16 kb + (l & 15), dims 32 db + 8 (l >> 4) .. +7.
//    Same 4 bytes per element as fp32; every wave load is one coalesced 1 KB.
//  - S = M Q'^T straight from the load registers: B = q' with its 16 columns
//    [q'_hi of heads 0-7 | q'_lo of heads 0-7], so A_hi B + A_lo B holds all
//    four split products of a head in columns h and h + 8 (one DPP add):
//    16 MFMAs per 16 keys.
//  - U = P^T M on v_mfma_f32_16x16x16_f16 with A = [P_hi | P_lo] (rows =
//    heads, k = keys): the S accumulator hands every lane exactly its A
//    operand (4 keys of its column's head), so P never moves.  B = the key
//    block transposed: the fragments are written once to a per-wave 16 KB
//    LDS image [plane][dim block k of 16][16 keys][16 dims] and read back by
//    ds_read_b64_tr_b16.  A key's 32-byte row holds two 16-byte halves,
//    swapped on rows with bit 2 set: the transposed reads of a 32-lane half
//    cover 256 contiguous bytes (conflict-free), the b128 stores of 8 rows
//    hit 8 distinct bank groups, and every address is a per-lane base plus a
//    compile-time offset (no per-block address registers).  32 MFMAs per 16
//    keys; 64 fp32 accumulators (rows 0-7 P_hi, 8-15 P_lo, summed at the
//    end).  The fragments are plain global loads at constant offsets from
//    one per-wave base (BH_GLOBAL; the buffer-descriptor form, once needed
//    to avoid a spill, is 0.5 us slower now): a register spill here would
//    be a vmcnt(0) drain of every prefetch in flight, so check the .s.
//  - Online softmax with a lazy maximum: p = exp(s - m) <= e^6 and P is
//    split at 2^7 (< 65504; its lo plane out of the fp16 subnormals down to
//    p ~ 5e-7); U and l are rescaled (4 shuffles + 64 multiplies, a
//    wave-uniform branch) only when a head's block maximum exceeds m by
//    more than 6.
//  - One workgroup of 8 waves (two per SIMD) per chunk, wave w owning keys
//    [64 w, 64 w + 64) = 4 key blocks; loads run in half blocks (8 fragments,
//    4 dim blocks x 2 planes), two half blocks ahead of the one computed;
//    the 8 waves' (m, l, U) merge through LDS at the end.
// Matrix-core time per CU: 64 x 16 + 128 x 8 cycles per wave, ~1.8 us.
#ifndef BH_NW
#define BH_NW 8                          // waves per chunk (64 keys each; 4: 128 keys each, half the LDS)
#endif
#define BH_KB 32                         // key blocks per chunk (512 keys)
#define BH_KPW (BH_KB / BH_NW)           // key blocks per wave
static_assert(BH_NW == 4 || BH_NW == 8, "waves per chunk");
#define BH_THR 6.0f                      // lazy-rescale threshold (natural log units)
#define BH_PSCALE 128.0f                 // P split at 2^7
#ifndef BH_AHEAD
#define BH_AHEAD 1                       // half blocks in flight beyond the one computed (2: slower)
#endif
#ifndef BH_INTERLEAVE
#define BH_INTERLEAVE 1                  // key blocks w + 8 kb (1) or 4 w + kb (0)
#endif
#ifndef BH_GLOBAL
#define BH_GLOBAL 1  // global loads (0: buffer loads through one descriptor; 0.5 us slower since the
                     // prologue and merge changes, same box, tools/microbench.py bank; neither spills)
#endif
#ifndef BH_EXPT
#define BH_EXPT 0                        // timing probes only (bit 0 no U, 1 no S, 2 no image writes, 3 no softmax, 4 no merge)
#endif
#define BH_IMG 16384                     // bytes: one wave's transposed image (2 planes x 16 keys x 512 B)
#define BH_ML (BH_NW * BH_IMG)           // merge (m, l) [wave][8 heads][2] floats, behind the images
#define BH_Q (BH_ML + BH_NW * 16 * 4)    // q' image [8 heads][260] floats
#define BH_LDS (BH_Q + ND_H * 260 * 4)
static_assert(ND_H * ND_D * 4 <= BH_IMG, "a wave's partial U fits its own image");

typedef _Float16 bh4 __attribute__((ext_vector_type(4)));
typedef _Float16 bh8 __attribute__((ext_vector_type(8)));
typedef short bs4 __attribute__((vector_size(8)));
typedef __attribute__((address_space(3))) bs4 lds_bs4;

__device__ __forceinline__ f32x4 mfma_h32(bh8 a, bh8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_h16(bh4 a, bh4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}
// byte offset of the 16-byte half hf (dims 8 hf .. +7 of a 16-dim block) of
// key row r in a dim block of one plane of the transposed image
__device__ __forceinline__ int bh_row(int r, int hf) { return 32 * r + 16 * (hf ^ ((r >> 2) & 1)); }

// NT: the bank streamed with non-temporal loads (not kept in the Infinity
// Cache), for an EnginePool lane whose bank should leave the cache to another
// one chunk c (dec_bank_h3_kernel below)
template <bool NT>
__device__ __forceinline__ void bank_h3_chunk(int c, const float* __restrict__ qp, const f32x4* __restrict__ bank,
                                              const float* __restrict__ signal, const int* __restrict__ span,
                                              float pad_val, float* __restrict__ out, int T,
                                              unsigned long long* stamp, float* __restrict__ dbg, size_t dbg_stride,
                                              int* ovf, unsigned long long t_entry) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  char* img = reinterpret_cast<char*>(lds) + w * BH_IMG;  // [plane][dim block][16 keys][32 B]
  // this wave's fragments: key blocks 4w .. 4w + 3 (64 KB from the descriptor base)
#if BH_INTERLEAVE
  // key block kb of this wave = w + 8 kb: the 8 waves stream one contiguous 128 KB window per step
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<f32x4*>(bank + (size_t)c * BH_KB * 8 * 2 * 64), 0,
                                                      BH_KB * 16384, 0x00020000);
  const int kb0 = w, kbs = BH_NW;
#else
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<f32x4*>(bank + ((size_t)c * BH_KB + BH_KPW * w) * 8 * 2 * 64), 0, BH_KPW * 16384, 0x00020000);
  const int kb0 = 0, kbs = 1;
#endif
  const int voff = lane * 16;

  // half block h (0..7): key block 4w + (h >> 1), dim blocks 4 (h & 1) .. +3, both planes
  auto hload = [&](int h, f32x4(&f)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#if BH_GLOBAL
      const f32x4* p = bank + ((size_t)c * BH_KB * 16 + (kb0 + kbs * (h >> 1)) * 16 + 8 * (h & 1) + i) * 64 + lane;
      if constexpr (NT)
        f[i] = __builtin_nontemporal_load(p);
      else
        f[i] = *p;
#else
      f[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rsrc, voff, ((kb0 + kbs * (h >> 1)) * 16 + 8 * (h & 1) + i) * 1024, 0));
#endif
    }
  };
  // this lane's image addresses: write (row col, dim block 2 db + (g >> 1), half g & 1);
  // transposed read (row 4g + q, dims 4p .. 4p + 3 of a dim block)
  char* wimg = img + 512 * (g >> 1) + bh_row(col, g & 1);
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  const char* rimg = img + bh_row(4 * g + q4, p4 >> 1) + 8 * (p4 & 1);
  // q' (one 16 B load per thread, staged in LDS) and the signal FIRST, then
  // the first half blocks: the wait that retires q' leaves them in flight
  float* qimg = lds + BH_Q / 4;  // [8 heads][260] (rows padded: the b128 reads of 8 heads hit 8 bank groups)
  constexpr int QH = ND_H / BH_NW, SGN = BH_KPW / 4;  // q' heads per thread, signal words per lane
  f32x4 qld[QH];
#pragma unroll
  for (int i = 0; i < QH; ++i) qld[i] = ld4(qp + (size_t)c * (ND_H * ND_D) + (w + BH_NW * i) * ND_D + 4 * lane);
  // lane l: row l & 15 of the wave's key block 4 j + (l >> 4)
  float sg[SGN];
#pragma unroll
  for (int j = 0; j < SGN; ++j) {
    const int kl = 4 * j + (lane >> 4);
    const int bkey = 16 * (BH_INTERLEAVE ? w + BH_NW * kl : BH_KPW * w + kl) + (lane & 15);
    sg[j] = signal[(size_t)c * T + min(bkey, T - 1)];
  }
  f32x4 F[3][8];
  hload(0, F[0]);
  hload(1, F[1]);
  if (BH_AHEAD == 2) hload(2, F[2]);
  __builtin_amdgcn_sched_barrier(0);
  // the timing stamp (clock read at entry) and the span after every first
  // load is out (a branch or a scalar load ahead of them split the
  // kernel-argument loads: one more scalar round trip before the stream)
  stamp_begin_at(stamp, t_entry);
  const int L = min(span[c], T);
#pragma unroll
  for (int i = 0; i < QH; ++i) st4(qimg + (w + BH_NW * i) * 260 + 4 * lane, qld[i]);
  lds_barrier();  // LDS only: the bank loads stay in flight
  f32x4 qv[8][2];
  const int hd = col & 7;
#pragma unroll
  for (int db = 0; db < 8; ++db) {
    qv[db][0] = ld4(qimg + hd * 260 + 32 * db + 8 * g);
    qv[db][1] = ld4(qimg + hd * 260 + 32 * db + 8 * g + 4);
  }
  // q' as the B operand: column col = (plane col >> 3, head col & 7), dims 32 db + 8 g .. +7
  bh8 qb[8];
  {
    float amax = 0.f;
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      amax = fmaxf(amax, fmaxf(absmax4(qv[db][0]), absmax4(qv[db][1])));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = qv[db][j >> 2][j & 3];
        const _Float16 hi = (_Float16)x;
        qb[db][j] = col < 8 ? hi : (_Float16)(x - (float)hi);
      }
    }
    flag_overflow(ovf, amax);
  }
  unsigned long long padm[SGN];
#pragma unroll
  for (int j = 0; j < SGN; ++j) padm[j] = __ballot(sg[j] == pad_val);

  f32x4 ua[16];  // U^T... rows 4g + i = (P plane, head), column col of dim block: lane holds rows 4g .. 4g + 3
#pragma unroll
  for (int k = 0; k < 16; ++k) ua[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;  // head col & 7 (l: this lane's keys)

#pragma unroll
  for (int kb = 0; kb < BH_KPW; ++kb) {
    f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0;
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const int h = 2 * kb + part;
      f32x4(&f)[8] = F[h % 3];
      // ---- S partial over dim blocks 4 part .. +3: D[key 4g + i][col]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#if BH_EXPT & 2
        d0 += f[2 * i] + f[2 * i + 1];
#else
        d0 = mfma_h32(__builtin_bit_cast(bh8, f[2 * i]), qb[4 * part + i], d0);
        d1 = mfma_h32(__builtin_bit_cast(bh8, f[2 * i + 1]), qb[4 * part + i], d1);
#endif
      }
      // ---- the fragments into the transposed image: dims 32 db + 8 g .. +7 of key col
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int db = 4 * part + (i >> 1), pl = i & 1;
#if !(BH_EXPT & 4)
        *reinterpret_cast<f32x4*>(wimg + pl * 8192 + 1024 * db) = f[i];
#endif
      }
      __builtin_amdgcn_sched_barrier(0);  // the next loads reuse f's registers
      if (h + BH_AHEAD + 1 < 2 * BH_KPW) hload(h + BH_AHEAD + 1, F[(h + BH_AHEAD + 1) % 3]);
    }
    // ---- scores: columns h and h + 8 hold the hi and lo halves of q'_h
    f32x4 s = d0 + d1;
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] += dpp_mov<ND_DPP_ROR8>(s[i]);
    const int kbase = 16 * (BH_INTERLEAVE ? w + BH_NW * kb : BH_KPW * w + kb) + 4 * g;  // key of row i
    const unsigned pb = (unsigned)(padm[kb >> 2] >> (16 * (kb & 3) + 4 * g)) & 0xFu;
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
#if BH_EXPT & 8
    m = 0.f;
    if (false) {
#else
    gm = xor32_max(xor16_max(gm));
    if (__any(gm > m + BH_THR)) {
#endif
      const float nm = fmaxf(m, gm);
      const float sc = nm == m ? 1.f : __expf(m - nm);
      m = nm;
      l *= sc;
      // U row 4g + i belongs to head 4 (g & 1) + i: that column's scale
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
    // ---- A operand of U: row col = (plane col >> 3, head col & 7), keys 4g .. 4g + 3
    bh4 pa;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = p[i] * BH_PSCALE;
      const _Float16 hi = (_Float16)x;
      pa[i] = col < 8 ? hi : (_Float16)(x - (float)hi);
    }
    // ---- U += P^T M: B = key rows 4g + q, dims 16 k + col (transposed reads)
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {
#if BH_EXPT & 1
        ua[k][pl] += (float)pa[pl];
#else
        const bs4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bs4*)(rimg + pl * 8192 + 512 * k));
        ua[k] = mfma_h16(pa, __builtin_bit_cast(bh4, b), ua[k]);
#endif
      }
  }

  // ---- merge the 8 waves without cross-lane work in the waves: wave w's
  //      unmerged U^T fragments ua[k] (rows 4g .. 4g + 3: plane g >> 1, heads
  //      4 (g & 1) .. + 3; column col: dim 16 k + col) go to its OWN image as 16
  //      b128 writes (its image reads are done: a wave's LDS operations retire
  //      in order), (m, l) beside; wave 0 then turns the 64 (m, l) into the
  //      merge weights exp(m - M) and 1 / den once; every thread combines 4
  //      heads x 1 dim from b128 reads of the hi and lo rows
  l = xor32_sum(xor16_sum(l));  // over the 4 key rows of the column's head
#if BH_EXPT & 16  // timing probe only: no merge
  if (l == 12345.f) out[threadIdx.x] = ua[0][0] + ua[15][3] + m;
  return;
#endif
  float* ml = lds + BH_ML / 4;  // [wave][8 heads][2]
  {
    f32x4* red = reinterpret_cast<f32x4*>(lds + w * (BH_IMG / 4));
#pragma unroll
    for (int k = 0; k < 16; ++k) red[k * 64 + lane] = ua[k];
  }
  if (lane < 8) {
    ml[(w * ND_H + lane) * 2] = m;
    ml[(w * ND_H + lane) * 2 + 1] = l;
  }
  __syncthreads();
  float* fw = lds + BH_Q / 4;  // [wave][8 heads] weights, then [8 heads] 1 / den (the q' image is dead)
  if (w == 0) {
    const int v = lane >> 3, h = lane & 7;
    const float mv = v < BH_NW ? ml[(v * ND_H + h) * 2] : -INFINITY, lv = v < BH_NW ? ml[(v * ND_H + h) * 2 + 1] : 0.f;
    float M = fmaxf(mv, __shfl_xor(mv, 8, 64));
    M = fmaxf(M, __shfl_xor(M, 16, 64));
    M = fmaxf(M, __shfl_xor(M, 32, 64));
    const float f = mv == -INFINITY ? 0.f : __expf(mv - M);  // waves that owned no key
    float den = f * lv;
    den += __shfl_xor(den, 8, 64);
    den += __shfl_xor(den, 16, 64);
    den += __shfl_xor(den, 32, 64);
    if (v < BH_NW) fw[v * ND_H + h] = f;
    if (v == 0) fw[64 + h] = den > 0.f ? __builtin_amdgcn_rcpf(den) * (1.0f / BH_PSCALE) : 0.f;
  }
  lds_barrier();
#pragma unroll
  for (int e = threadIdx.x; e < 512; e += BH_NW * 64) {
    const int hs = e >> 8, d = e & 255, k = d >> 4, cl = d & 15;
    const int lh = k * 64 + cl + 16 * hs, ll = k * 64 + cl + 16 * (2 + hs);  // hi rows g = hs, lo rows g = 2 + hs
    f32x4 num = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < BH_NW; ++v) {
      const f32x4* red = reinterpret_cast<const f32x4*>(lds + v * (BH_IMG / 4));
      num += ld4(fw + v * ND_H + 4 * hs) * (red[lh] + red[ll]);
    }
    num *= ld4(fw + 64 + 4 * hs);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = (4 * hs + i) * ND_D + d;
      out[pk(c, n & ~3, ND_H * ND_D) + (n & 3)] = num[i];
    }
  }
}

// grid = C (one chunk per workgroup, every CU), or (WALK) fewer workgroups
// walking the chunks (nd_set_bank_grid: an EnginePool lane leaves half the
// CUs to the other lanes' kernels, whose LDS does not fit beside this
// kernel's 137 KB).  Two forms: the loop changes the one-chunk code's load
// schedule (a drain of the first half blocks, tests/test_abi.py)
template <bool NT, bool WALK>
__global__ void __launch_bounds__(BH_NW * 64)
dec_bank_h3_kernel(const float* __restrict__ qp, const f32x4* __restrict__ bank, const float* __restrict__ signal,
                   const int* __restrict__ span, float pad_val, float* __restrict__ out, int T, int C,
                   unsigned long long* stamp, float* __restrict__ dbg, size_t dbg_stride, int* ovf) {
#ifdef ND_SKIP_BANK  // timing probe only (tools/build_variant.sh): the kernel's marginal cost
  if (threadIdx.x < 100000) return;
#endif
  const unsigned long long t_entry = wall_clock64();  // the timing stamp's start (published below)
  if constexpr (WALK) {
    for (int c = blockIdx.x; c < C; c += gridDim.x) {
      if (c != (int)blockIdx.x) lds_barrier();  // the previous chunk's merge reads of LDS are done
      bank_h3_chunk<NT>(c, qp, bank, signal, span, pad_val, out, T, stamp, dbg, dbg_stride, ovf, t_entry);
    }
  } else {
    bank_h3_chunk<NT>(blockIdx.x, qp, bank, signal, span, pad_val, out, T, stamp, dbg, dbg_stride, ovf, t_entry);
  }
  stamp_end(stamp);
}

// Encoder output -> the split-fp16 fragment bank of dec_bank_h3_kernel: one
// workgroup per (chunk, key block of 16 rows): LayerNorm (as
// memory_pack_kernel) into LDS, then the 16 fragments (8 dim blocks x hi /
// lo) written as coalesced 1 KB blocks.  Rows t >= T are zero.
__global__ void __launch_bounds__(256)
bank_pack_h3_kernel(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
                    uint16_t* __restrict__ out, int T, int* ovf) {
  __shared__ float rows[16 * ND_D];
  const int c = blockIdx.x / BH_KB, kb = blockIdx.x % BH_KB, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = wv + 4 * rr, t = 16 * kb + r;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (t < T) {
      v = ld4(x + ((size_t)c * T + t) * ND_D + lane * 4);
      if (g) {
        const float mu = wave_sum(v.x + v.y + v.z + v.w) * (1.0f / ND_D);
        const f32x4 d = v - mu;
        const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / ND_D);
        v = d * ln_rsqrt(var + ND_LN_EPS) * ld4(g + lane * 4) + ld4(b + lane * 4);
      }
    }
    st4(rows + r * ND_D + lane * 4, v);
  }
  __syncthreads();
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int item = threadIdx.x + 256 * j, fr = item >> 6, ln = item & 63, db = fr >> 1, pl = fr & 1;
    const float* src = rows + (ln & 15) * ND_D + 32 * db + 8 * (ln >> 4);
    const f32x4 v0 = ld4(src), v1 = ld4(src + 4);
    amax = fmaxf(amax, fmaxf(absmax4(v0), absmax4(v1)));
    bh8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float v = k < 4 ? v0[k] : v1[k - 4];
      const _Float16 hi = (_Float16)v;
      o[k] = pl == 0 ? hi : (_Float16)(v - (float)hi);
    }
    *reinterpret_cast<bh8*>(out + ((((size_t)c * BH_KB + kb) * 8 + db) * 2 + pl) * 512 + ln * 8) = o;
  }
  flag_overflow(ovf, amax);
}

bool bank_h3_eligible(int T, int ldT) {
#ifdef ND_NO_BANK_H3  // A/B builds only (tools/ab_lib.sh): the fp32 LDS-slab kernel everywhere
  return false;
#endif
  return T > 448 && T <= 512 && ldT >= 512;
}

hipError_t launch_bank_pack_h3(const float* x, const float* ln_g, const float* ln_b, uint16_t* out, int B, int T,
                               int* ovf, hipStream_t s) {
  if (T < 1 || T > 512 || B < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bank_pack_h3_kernel, dim3(B * BH_KB), dim3(256), 0, s, x, ln_g, ln_b, out, T, ovf);
  return hipGetLastError();
}

hipError_t launch_dec_bank_h3(const float* qp, const uint16_t* bank, const float* signal, const int* span,
                              float pad_val, float* out, int C, int T, hipStream_t s, unsigned long long* stamp,
                              float* attn_dbg, size_t dbg_stride, int* ovf, bool nt, int grid) {
  if (T < 1 || T > 512 || C < 1 || grid < 0) return hipErrorInvalidValue;
  const int G = grid > 0 ? std::min(C, grid) : C;
#define ND_BANK_GO(N, W)                                                                                          \
  hipLaunchKernelGGL((dec_bank_h3_kernel<N, W>), dim3(G), dim3(BH_NW * 64), BH_LDS, s, qp,                       \
                     reinterpret_cast<const f32x4*>(bank), signal, span, pad_val, out, T, C, stamp, attn_dbg,     \
                     dbg_stride, ovf)
  if (G < C) {
    if (nt)
      ND_BANK_GO(true, true);
    else
      ND_BANK_GO(false, true);
  } else if (nt) {
    ND_BANK_GO(true, false);
  } else {
    ND_BANK_GO(false, false);
  }
#undef ND_BANK_GO
  return hipGetLastError();
}

static constexpr size_t mem_lds_bytes() { return (size_t)MB_LDS_FLOATS * sizeof(float); }
static_assert(MB_LDS_FLOATS * 4 <= 160 * 1024, "LDS");
static_assert(MB_NW * 512 * 4 <= MB_U, "merge slots overlap the q' image");

hipError_t launch_dec_mem_attention(const float* qp, const float* mem, const float* signal, const int* span,
                                    float pad_val, float* out, int C, int rpc, int T, int ldT, hipStream_t s,
                                    unsigned long long* stamp, float* attn_dbg, size_t dbg_stride) {
  if (rpc != 1 || T < 1 || T > 512 || ldT < T || C < 1) return hipErrorInvalidValue;
  const bool full = (T + MB_TILE - 1) / MB_TILE == 8;  // the 512-sample chunks of every bench / translate batch
  if (full)
    hipLaunchKernelGGL((dec_mem_attention_kernel<8>), dim3(C), dim3(MB_NW * 64), mem_lds_bytes(), s, qp, mem, signal,
                       span, pad_val, out, T, ldT, stamp, attn_dbg, dbg_stride);
  else
    hipLaunchKernelGGL((dec_mem_attention_kernel<0>), dim3(C), dim3(MB_NW * 64), mem_lds_bytes(), s, qp, mem, signal,
                       span, pad_val, out, T, ldT, stamp, attn_dbg, dbg_stride);
  return hipGetLastError();
}

// Encoder output -> the decoder's memory bank, row-major with ldT rows per
// chunk: row b*ldT + t = LN(x[b*T + t]) (transformer: encoder.layer_norm,
// encoder/transformer.py:125) or x itself; rows t >= T zero.
__global__ void __launch_bounds__(256)
memory_pack_kernel(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
                   float* __restrict__ out, int B, int T, int ldT) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B * ldT) return;
  const int bb = row / ldT, t = row - bb * ldT;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (t < T) {
    v = ld4(x + ((size_t)bb * T + t) * ND_D + lane * 4);
    if (g) {
      const float mu = wave_sum(v.x + v.y + v.z + v.w) * (1.0f / ND_D);
      const f32x4 d = v - mu;
      const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / ND_D);
      v = d * ln_rsqrt(var + ND_LN_EPS) * ld4(g + lane * 4) + ld4(b + lane * 4);
    }
  }
  st4(out + (size_t)row * ND_D + lane * 4, v);
}

hipError_t launch_memory_pack(const float* x, const float* ln_g, const float* ln_b, float* out, int B, int T, int ldT,
                              hipStream_t s) {
  if (T > ldT || T < 1) return hipErrorInvalidValue;
  const int rows = B * ldT;
  hipLaunchKernelGGL(memory_pack_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, ln_g, ln_b, out, B, T, ldT);
  return hipGetLastError();
}

// -attn_debug: rows of raw head-0 scores (keys t < span) -> softmax in place
// (the reference's attn["std"]: the last layer's context attention, head 0,
// onmt/modules/multi_headed_attn.py:175,187-192).  One wave per row.
__global__ void __launch_bounds__(256)
attn_rows_softmax_kernel(float* __restrict__ a, const int* __restrict__ span, int B, int S, int T) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B * S) return;
  const int c = row / S, L = min(span[c], T);
  float* r = a + (size_t)row * T;
  float mx = -INFINITY;
  for (int t = lane; t < L; t += 64) mx = fmaxf(mx, r[t]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int t = lane; t < L; t += 64) sum += __expf(r[t] - mx);
  sum = wave_sum(sum);
  for (int t = lane; t < T; t += 64) r[t] = t < L ? __expf(r[t] - mx) / sum : 0.f;
}

hipError_t launch_attn_rows_softmax(float* a, const int* span, int B, int S, int T, hipStream_t s) {
  hipLaunchKernelGGL(attn_rows_softmax_kernel, dim3((B * S + 3) / 4), dim3(256), 0, s, a, span, B, S, T);
  return hipGetLastError();
}

__global__ void stamp_reset_kernel(unsigned long long* p, int pairs) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < pairs) {
    p[2 * i] = ~0ull;
    p[2 * i + 1] = 0ull;
  }
}

hipError_t launch_stamp_reset(unsigned long long* stamps, int pairs, hipStream_t s) {
  hipLaunchKernelGGL(stamp_reset_kernel, dim3((pairs + 255) / 256), dim3(256), 0, s, stamps, pairs);
  return hipGetLastError();
}

hipError_t init_mem_attributes() {
  const void* fns[] = {(const void*)dec_mem_attention_kernel<0>, (const void*)dec_mem_attention_kernel<8>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mem_lds_bytes());
    if (e != hipSuccess) return e;
  }
  const void* bh[] = {(const void*)dec_bank_h3_kernel<false, false>, (const void*)dec_bank_h3_kernel<true, false>,
                      (const void*)dec_bank_h3_kernel<false, true>, (const void*)dec_bank_h3_kernel<true, true>};
  for (const void* f : bh) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, BH_LDS);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace nd
