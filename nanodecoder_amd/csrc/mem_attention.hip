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

// What a chunk's prologue loads before its first LDS store: the source samples of the wave's keys, its
// first two tiles, this thread's 16 B of q'.  The walking form (two chunks per workgroup) loads the second
// chunk's head before the first chunk's merge, so its latency hides behind the merge (as bank8.hip's).
struct MbHead {
  float sgv;
  f32x4 qv;
  f32x4 R0[MB_KW], R1[MB_KW];
};

// rows r * 64 + w * 8 + k (k < 8) of a chunk's bank (clamped to T - 1): lane l's 16 B of each
__device__ __forceinline__ void mb_fetch(const float* __restrict__ mc, int r, int w, int lane, int T,
                                         f32x4 (&dst)[MB_KW]) {
#pragma unroll
  for (int k = 0; k < MB_KW; ++k) {
    const int t = min(r * MB_TILE + w * MB_KW + k, T - 1);
    dst[k] = ld4(mc + (size_t)t * ND_D + 4 * lane);
  }
}

__device__ __forceinline__ const float* mb_chunk_base(const float* mem, int c, int ldT) {
#ifdef MB_PROBE_NOLOAD  // timing probe only (tools/mem_probe.sh): every chunk reads chunk 0's bank (L2-resident)
  (void)c;
  (void)ldT;
  return mem;
#else
  return mem + (size_t)c * ldT * ND_D;
#endif
}

// the head of chunk c: the source samples first (the waits that retire the tile loads then retire them
// too, so no wait for them is left inside the loop, where it would drain the prefetched tiles), then the
// first two tiles, then q'
__device__ __forceinline__ void mb_head(int c, const float* __restrict__ qp, const float* __restrict__ mem,
                                        const float* __restrict__ signal, int T, int ldT, int ntile, MbHead& hd) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float* mc = mb_chunk_base(mem, c, ldT);
  hd.sgv = signal[(size_t)c * T + min((lane >> 3) * MB_TILE + w * MB_KW + (lane & 7), T - 1)];
  if (ntile > 0) mb_fetch(mc, 0, w, lane, T, hd.R0);
  if (ntile > 1) mb_fetch(mc, 1, w, lane, T, hd.R1);
  hd.qv = ld4(qp + pk(c, (threadIdx.x >> 6) * ND_D + 4 * (threadIdx.x & 63), ND_H * ND_D));
}

// NT > 0: the tile count is the compile-time NT (T in (64 (NT-1), 64 NT]);
// every tile is processed (keys >= span masked), so the tile loop unrolls to
// straight-line code and the compiler's wait counts on the in-flight tile
// loads stay exact (a runtime loop makes it drain them every iteration).
// hd: chunk c's head (mb_head, loaded by the caller); nx >= 0 (NEXT): the next chunk this workgroup walks to,
// whose head goes into hd before this chunk's merge.
template <int NT, bool NEXT>
__device__ __forceinline__ void mem_chunk(int c, MbHead& hd, int nx, const float* __restrict__ qp,
                                          const float* __restrict__ mem, const float* __restrict__ signal,
                                          const int* __restrict__ span, float pad_val, float* __restrict__ out,
                                          int T, int ldT, float* __restrict__ dbg, size_t dbg_stride) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar addressing)
  float* slab = lds + w * MB_WAVE;            // [2][8 keys][256], row k rotated by 4k floats
  float* spart = slab + 2 * MB_KW * ND_D;     // [2][4 dp][8 heads][8 keys]
  float* pbuf = spart + 2 * 256;              // [8 heads][8 keys]
  const float* ub = lds + MB_U;
  const int L = min(span[c], T);
  const int ntile = NT > 0 ? NT : (L + MB_TILE - 1) / MB_TILE;
  const float* mc = mb_chunk_base(mem, c, ldT);

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
  auto fetch = [&](int r, f32x4(&dst)[MB_KW]) { mb_fetch(mc, r, w, lane, T, dst); };
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
#ifdef MB_PROBE_NOSCORE  // timing probe only: no score reads / MFMAs (scores 0)
    (void)arow;
    (void)urow;
    return s4[0];
#endif
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

  // the source samples of this wave's keys (lane l -> tile l >> 3, key l & 7), tiles 0 and 1, q': hd
  const float sgv = hd.sgv;
  f32x4(&R0)[MB_KW] = hd.R0;
  f32x4(&R1)[MB_KW] = hd.R1;
  // q' image (all heads; 512 threads x 16 B)
  {
    const int h = threadIdx.x >> 6, q = threadIdx.x & 63;
    st4(lds + MB_U + h * ND_D + ((4 * q + 4 * h) & (ND_D - 1)), hd.qv);
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
#ifdef MB_PROBE_NOU  // timing probe only: no context product (U stays the P sums)
    acc[0] += p0 + p1;
    (void)tile;
#else
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
#endif
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

  // NEXT: the next chunk's head goes out now, into registers dead here (R0 / R1's last tiles are in LDS)
  // (fenced: hoisted into the tile loop they would raise its register peak past 256 and spill)
  if constexpr (NEXT) {
    __builtin_amdgcn_sched_barrier(0);
    mb_head(nx, qp, mem, signal, T, ldT, NT, hd);
    __builtin_amdgcn_sched_barrier(0);
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
}

// one workgroup per chunk, or (gridDim.x < C: EnginePool lanes, nd_set_bank_grid) fewer workgroups walking
// the chunks, so the other lanes' kernels fit beside this one's 150 KB of LDS (the digit bank's walking form,
// bank8.hip)
template <int NT>
__global__ void __launch_bounds__(MB_NW * 64)
dec_mem_attention_kernel(const float* __restrict__ qp, const float* __restrict__ mem,
                         const float* __restrict__ signal, const int* __restrict__ span, float pad_val,
                         float* __restrict__ out, int T, int ldT, unsigned long long* stamp,
                         float* __restrict__ dbg, size_t dbg_stride, int C) {
#ifdef ND_SKIP_MEMATT  // timing probe only (tools/marginal_exact.sh): the kernel's marginal cost
  if (threadIdx.x < 100000) return;
#endif
  stamp_begin(stamp);
  MbHead hd;
  auto ntile = [&](int c) { return NT > 0 ? NT : (min(span[c], T) + MB_TILE - 1) / MB_TILE; };
#ifndef MB_NO_PREFETCH  // timing variant only (tools/build_variant.sh): the walking form without the prefetch
  if (NT > 0 && C <= 2 * (int)gridDim.x) {
    // at most two chunks per workgroup (the pool's grid): straight-line, the second chunk's head loaded
    // during the first one's merge (a runtime loop would carry it across the back-edge)
    // (each case loads its own head: a head loaded before the branch is live into both and spills)
    const int c = blockIdx.x, nx = c + (int)gridDim.x;
    if (nx < C) {
      mb_head(c, qp, mem, signal, T, ldT, ntile(c), hd);
      mem_chunk<NT, true>(c, hd, nx, qp, mem, signal, span, pad_val, out, T, ldT, dbg, dbg_stride);
      __syncthreads();  // the first chunk's merge reads of LDS are done
      mem_chunk<NT, false>(nx, hd, -1, qp, mem, signal, span, pad_val, out, T, ldT, dbg, dbg_stride);
    } else {
      mb_head(c, qp, mem, signal, T, ldT, ntile(c), hd);
      mem_chunk<NT, false>(c, hd, -1, qp, mem, signal, span, pad_val, out, T, ldT, dbg, dbg_stride);
    }
    stamp_end(stamp);
    return;
  }
#endif
  for (int c = blockIdx.x; c < C; c += gridDim.x) {
    if (c != (int)blockIdx.x) __syncthreads();  // the previous chunk's merge reads of LDS are done
    mb_head(c, qp, mem, signal, T, ldT, ntile(c), hd);
    mem_chunk<NT, false>(c, hd, -1, qp, mem, signal, span, pad_val, out, T, ldT, dbg, dbg_stride);
  }
  stamp_end(stamp);
}

// The 24-bit digit bank (bank8.hip) serves every chunk length up to 512 (its
// buffer holds 512 rows per chunk whatever max_src_len is, alloc_workspaces;
// below 385 samples it streams ceil(T / 128) key blocks per wave): faster than
// this fp32 kernel at every T (profiles/r06_bank_T_probe.txt: 19.1 vs 26.5 us
// at T = 300, the reference authors' production chunks).  The fp32 kernel
// above serves exact fp32.
bool bank_eligible(int T, int ldT) {
  (void)ldT;
  return T >= 1 && T <= 512;
}

static constexpr size_t mem_lds_bytes() { return (size_t)MB_LDS_FLOATS * sizeof(float); }
static_assert(MB_LDS_FLOATS * 4 <= 160 * 1024, "LDS");
static_assert(MB_NW * 512 * 4 <= MB_U, "merge slots overlap the q' image");

hipError_t launch_dec_mem_attention(const float* qp, const float* mem, const float* signal, const int* span,
                                    float pad_val, float* out, int C, int rpc, int T, int ldT, hipStream_t s,
                                    unsigned long long* stamp, float* attn_dbg, size_t dbg_stride, int grid) {
  if (rpc != 1 || T < 1 || T > 512 || ldT < T || C < 1 || grid < 0) return hipErrorInvalidValue;
#ifdef MB_NO_WALK  // timing variant only (tools/build_variant.sh): one workgroup per chunk always
  grid = 0;
#endif
  const int G = grid > 0 ? std::min(C, grid) : C;
  // the tile count as a compile-time constant for chunks of 257..512 samples (the 512-sample chunks of every bench
  // batch; the reference authors' production runs use 300); shorter ones take the runtime count
#define ND_MEM_GO(N)                                                                                              \
  hipLaunchKernelGGL((dec_mem_attention_kernel<N>), dim3(G), dim3(MB_NW * 64), mem_lds_bytes(), s, qp, mem, signal, \
                     span, pad_val, out, T, ldT, stamp, attn_dbg, dbg_stride, C)
  switch ((T + MB_TILE - 1) / MB_TILE) {
    case 8: ND_MEM_GO(8); break;
    case 7: ND_MEM_GO(7); break;
    case 6: ND_MEM_GO(6); break;
    case 5: ND_MEM_GO(5); break;
    default: ND_MEM_GO(0); break;
  }
#undef ND_MEM_GO
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
  const void* fns[] = {(const void*)dec_mem_attention_kernel<0>, (const void*)dec_mem_attention_kernel<5>,
                       (const void*)dec_mem_attention_kernel<6>, (const void*)dec_mem_attention_kernel<7>,
                       (const void*)dec_mem_attention_kernel<8>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mem_lds_bytes());
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace nd
