// fp32 MFMA GEMMs for gfx950 with fused LayerNorm prologue and
// bias / ReLU / residual / row-statistics epilogue.
//
// Replaces the reference's nn.Linear addmm calls and the LayerNorm that
// precedes them (onmt/modules/multi_headed_attn.py:59-67,155-157,179;
// onmt/modules/position_ffn.py:20-22,38-40; encoder/transformer.py:50,125;
// decoder/transformer.py:75,88).  The reference computes in fp32 and gfx950
// has no xf32 MFMA, so products run on v_mfma_f32_32x32x2_f32 /
// v_mfma_f32_16x16x4_f32 (exact fp32 FMA chains at the fp32 peak).
//
//   C[M,N] = epi( pro(A)[M,K] . W[N,K]^T + bias[N] )
//   pro(A) = (A - mean) * rstd over K                            (LN)
//   (the LayerNorm's gamma/beta are folded into W and bias at load time,
//    fold_layernorm_kernel below)
//   epi(v) = relu(v) (RELU); v + R[M,N] (RESID)
//
// LayerNorm fusion across kernels: every producer of a LayerNorm input (the
// residual GEMMs and the embed kernels) writes per-row partial statistics
// {mean_j, M2_j} of its column tile; the consuming GEMM merges them (Chan's
// parallel-variance formula, exact and stable) instead of re-reading whole
// rows in every column workgroup.
#include "../../include/nanodec.h"
#include "common.hpp"
#include "kernels.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace nd {

// Merge P equal-width partials {mean_j, M2_j} of a 256-wide row.  All
// ND_PART_LD slots are loaded unconditionally (the buffer always holds them)
// so the loads issue together; slots j >= P are discarded by selects.
typedef f32x4 PartRow[ND_PART_LD / 2];  // {mean_2i, M2_2i, mean_2i+1, M2_2i+1}
__device__ __forceinline__ void load_stats(const float* __restrict__ p, PartRow& v) {
#pragma unroll
  for (int i = 0; i < ND_PART_LD / 2; ++i) v[i] = ld4(p + 4 * i);
}
__device__ __forceinline__ void merge_loaded(const PartRow& v, int P, float& mu, float& rs) {
  // P is a power of two (the producer's column tiles, or 1): v_rcp_f32 is
  // exact there, and no IEEE division sits on the LN consumer's path
  const float invP = __builtin_amdgcn_rcpf((float)P), w = 256.0f * invP;
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < ND_PART_LD / 2; ++i) {
    m += 2 * i < P ? v[i].x : 0.f;
    m += 2 * i + 1 < P ? v[i].z : 0.f;
  }
  m *= invP;
  float m2 = 0.f;
#pragma unroll
  for (int i = 0; i < ND_PART_LD / 2; ++i) {
    const float d0 = v[i].x - m, d1 = v[i].z - m;
    m2 += 2 * i < P ? v[i].y + w * d0 * d0 : 0.f;
    m2 += 2 * i + 1 < P ? v[i].w + w * d1 * d1 : 0.f;
  }
  mu = m;
  rs = ln_rsqrt(m2 * (1.0f / 256.0f) + ND_LN_EPS);
}
// The same merge spread over the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 that share
// a row (lane >> 4 = q holds partials 4q .. 4q + 3: two loads per lane
// instead of eight); every lane of the four ends with the row's statistics.
typedef f32x4 PartQuad[2];  // {mean_4q, M2_4q, mean_4q+1, M2_4q+1}, {.. 4q+2, .. 4q+3}
__device__ __forceinline__ void load_stats_quad(const float* __restrict__ prow, int q, PartQuad& v) {
  v[0] = ld4(prow + 8 * q);
  v[1] = ld4(prow + 8 * q + 4);
}
__device__ __forceinline__ void merge_quad(const PartQuad& v, int P, int q, float& mu, float& rs) {
  const float invP = __builtin_amdgcn_rcpf((float)P), w = 256.0f * invP;
  const int j = 4 * q;
  float m = (j < P ? v[0].x : 0.f) + (j + 1 < P ? v[0].z : 0.f) + (j + 2 < P ? v[1].x : 0.f) +
            (j + 3 < P ? v[1].z : 0.f);
  m += __shfl_xor(m, 16, 64);
  m += __shfl_xor(m, 32, 64);
  m *= invP;
  const float d0 = v[0].x - m, d1 = v[0].z - m, d2 = v[1].x - m, d3 = v[1].z - m;
  float m2 = (j < P ? v[0].y + w * d0 * d0 : 0.f) + (j + 1 < P ? v[0].w + w * d1 * d1 : 0.f) +
             (j + 2 < P ? v[1].y + w * d2 * d2 : 0.f) + (j + 3 < P ? v[1].w + w * d3 * d3 : 0.f);
  m2 += __shfl_xor(m2, 16, 64);
  m2 += __shfl_xor(m2, 32, 64);
  mu = m;
  rs = ln_rsqrt(m2 * (1.0f / 256.0f) + ND_LN_EPS);
}
__device__ __forceinline__ void merge_stats(const float* __restrict__ p, int P, float& mu, float& rs) {
  PartRow v;
  load_stats(p, v);
  merge_loaded(v, P, mu, rs);
}


// Sum over aligned groups of TPR lanes (16, 32 or the whole wave).
template <int TPR>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(TPR == 16 || TPR == 32 || TPR == 64, "group of 16, 32 or 64 lanes");
  if constexpr (TPR == 64) return wave_sum(v);
  v = sum16(v);
  if constexpr (TPR == 32) v += __shfl_xor(v, 16, 64);
  return v;
}

// ---------------------------------------------------------------------------
// LDS-tiled kernel (encoder, large M): BM x BN x 32 tiles, WM x WN waves each
// owning (BM/WM) x (BN/WN) as 32x32 MFMA blocks.  A and W tiles are staged
// global -> registers -> LDS (double-buffered, one barrier per K step); row
// stride 36 floats makes the per-lane ds_read_b128 fragment loads
// bank-conflict free.  Inside an 8-wide k block, lane half h reads
// k = 4h..4h+3 with one ds_read_b128 and feeds 4 consecutive MFMAs (MFMA i
// sums k = {i, 4+i}: a permutation of K that A and W share).  The epilogue
// stages the C tile through LDS so output / residual traffic is coalesced
// float4 rows, and row statistics fall out of the same pass.
// Split-fp16 operands (H3): a fp32 value x is carried as hi = fp16(x) and
// lo = fp16(x - hi), 22 significant bits, and a product as
// hi*hi + hi*lo + lo*hi (the dropped lo*lo is below 2^-22 relative) on
// v_mfma_f32_32x32x16_f16, which multiplies exactly into an fp32
// accumulator: fp32-class accuracy at 16/3 of the fp32 MFMA rate.  W is
// split once at load time (scaled by 2^s so its lo plane stays out of the
// fp16 subnormals); A is split while it is staged into LDS (after the
// LayerNorm), so every element is converted once per workgroup.  The LDS
// row image is [k/8][hi 8 | lo 8] halves: the same 144-byte rows as the
// fp32 tile, and each lane's MFMA operand (8 consecutive k of one row) is a
// single ds_read_b128 per plane.
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma32h(h8 a, h8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void split4(f32x4 v, h4& hi, h4& lo) {
  hi = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
  lo = {(_Float16)(v.x - (float)hi.x), (_Float16)(v.y - (float)hi.y), (_Float16)(v.z - (float)hi.z),
        (_Float16)(v.w - (float)hi.w)};
}

// BK: k depth of a main-loop step (32; 64 for the small-tile, long-K shapes,
// whose steps are otherwise too short to cover the next step's load latency)
//
// Exact fp32 products (!H3) at BK = 32 run on v_mfma_f32_16x16x4_f32 (M16)
// rather than 32x32x2: the same cycles per FLOP, but the chip holds a higher
// clock on the 16x16 shape under this load (MI355X_MICROARCH.md 'DVFS
// give-back' item 7; the library's fp32 GEMM at these shapes is a 16x16 one,
// profiles/r06h_mfma_sgemm.json).  Lane (row r = l & 15, k quad q = l >> 4)
// reads 16 B (4 consecutive k) of its row per 16-k block and feeds 4 MFMAs
// (MFMA e sums k = {e, 4 + e, 8 + e, 12 + e}: a permutation of K that A and W
// share).  The LDS rows are unpadded (32 floats) with their 16-B chunks
// XOR-swizzled by (row >> 1) & 7, which makes those reads conflict-free and
// keeps a staging row's 8 chunks one contiguous 128-B store.
#ifndef ND_F32_M16
#define ND_F32_M16 1
#endif
// Epilogue of the row-major LDS-tiled kernels, second half: RP rows of the C tile staged in LDS (Cs, stride
// BN + 4) leave as coalesced float4 rows (+ residual), or as the 24-bit context image; row statistics
template <int BN, int NT, int RP, bool RELU, bool RESID>
__device__ __forceinline__ void f32_tile_rows(const GemmArgs& g, const float* Cs, int row0, int n0, int nbt) {
  constexpr int LDC = BN + 4, TPR = BN / 4, RPP = NT / TPR;
  const int tid = threadIdx.x, c4 = (tid % TPR) * 4, M = g.M;
  for (int r0 = 0; r0 < RP; r0 += RPP) {
    const int rl = r0 + tid / TPR, row = row0 + rl;
    f32x4 v = ld4(&Cs[rl * LDC + c4]);
    if (row < M) {
      const size_t ro = g.p16io ? pk(row, n0 + c4, g.N) : (size_t)row * g.ldr + n0 + c4;
      const size_t co = g.p16io ? pk(row, n0 + c4, g.N) : (size_t)row * g.ldc + n0 + c4;
      if constexpr (RESID) v += ld4(g.R + ro);
      if (!g.q24) st4(g.C + co, v);
    }
    if constexpr (BN % ND_D == 0 && !RESID && !RELU) {
      // the 24-bit context K/V image (q24_quant_store: the head's 8 lanes are
      // this row's threads c4 / 4 .. + 7, every lane of them active here)
      // (BN >= 256: one wave = 64 threads of one row, so `row < M` is wave-uniform)
      if (g.q24 && row < M) {
        const int col = n0 + c4, layer = col / (2 * ND_D), half = (col / ND_D) & 1, d = col % ND_D;
        uint8_t* dst = g.q24 + (size_t)layer * g.q24_plane + (size_t)row * CTXQ_ROW;
        const float sc = q24_quant_store(v, dst + half * CTXQ_V + 3 * d);
        if ((d & (ND_DH - 1)) == 0) reinterpret_cast<float*>(dst + CTXQ_S)[2 * (d / ND_DH) + half] = sc;
      }
    }
    if (g.part_out) {
      const float mu = group_sum<TPR>(v.x + v.y + v.z + v.w) * (1.0f / BN);
      const f32x4 d = v - mu;
      const float q = group_sum<TPR>(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w);
      if ((tid % TPR) == 0 && row < M) {
        float* p = g.part_out + ((size_t)row * ND_PART_LD + nbt) * 2;
        p[0] = mu;
        p[1] = q;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int BK, bool H3, bool LN, bool RELU, bool RESID>
__global__ void __launch_bounds__(WM* WN * 64) gemm_f32_kernel(const GemmArgs g) {
#ifdef ND_SKIP_F32GEMM  // timing probe only (tools/marginal_exact.sh): the fp32 products' marginal cost
  if (!H3 && threadIdx.x < 100000) return;
#endif
  constexpr int NT = WM * WN * 64;
  constexpr bool M16 = ND_F32_M16 && !H3 && BK == 32;
  constexpr int LDK = M16 ? BK : BK + 4, LDC = BN + 4;
  constexpr int FM16 = BM / WM / 16, FN16 = BN / WN / 16;  // M16: 16x16 blocks per wave
  constexpr int TPK = BK / 4;  // threads per row of a row-major BK-wide slice
  constexpr int FM = BM / WM / 32, FN = BN / WN / 32;
  constexpr int A4 = BM * BK / 4 / NT;
  constexpr int W4 = BN * BK / 4 / NT;
  // the epilogue stages the C tile through LDS in EP passes of BM / EP rows
  // (one wave row group per pass when the whole tile would not fit)
  constexpr int EP = (BM * LDC > 2 * (BM + BN) * LDK) ? WM : 1, RP = BM / EP;
  constexpr int SMEM = (2 * (BM + BN) * LDK > RP * LDC) ? 2 * (BM + BN) * LDK : RP * LDC;
  static_assert(A4 >= 1 && W4 >= 1, "tile too small for the thread count");
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  __shared__ float s_mu[LN ? BM : 1], s_rs[LN ? BM : 1];
  float* As = smem;                  // [2][BM*LDK]
  float* Ws = smem + 2 * BM * LDK;   // [2][BN*LDK]
  float* Cs = smem;                  // [BM][LDC] after the main loop

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware tile order: consecutive workgroups land on the 8 XCDs in turn,
  // so workgroup b runs on XCD b % 8; giving XCD x the row blocks x, x+8, ...
  // with all their column tiles keeps each A row block in ONE XCD's L2 (read
  // from HBM once instead of once per column tile), while the whole weight
  // (<= 2 MB) is cached by every XCD.  g.xcd_map == 0: column tile fastest.
  const int ntn = g.N / BN, nmb = (g.M + BM - 1) / BM;
  int nbt, mbk;
  if (g.xcd_map) {
    const int b = blockIdx.x, j = b >> 3;
    nbt = j % ntn;
    mbk = (j / ntn) * 8 + (b & 7);
  } else {
    nbt = blockIdx.x % ntn;
    mbk = blockIdx.x / ntn;
  }
  const int n0 = nbt * BN, m0 = mbk * BM;
  const int M = g.M, K = g.K;
  const float* __restrict__ A = g.A;

  f32x4 ra[A4], rw[W4];
  // A staging piece i of this thread: (row, c) of the BM x BK tile.  Row-major
  // A: 8 threads per 128-B row segment.  P16 A (g.p16io, the decoder's packed
  // activations): one whole 1 KB P16 block per wave instruction, lane e =
  // row e & 15, columns 4 (e >> 4) .. + 3 of the block.
  auto amap = [&](int i, int& row, int& c) {
    if (g.p16io) {
      const int j = wave + (NT / 64) * i;
      row = (j / (BK / 16)) * 16 + (lane & 15);
      c = (j % (BK / 16)) * 16 + 4 * (lane >> 4);
    } else {
      const int f = tid + i * NT;
      row = f / TPK;
      c = (f % TPK) * 4;
    }
  };
  // straight-line loads: the row is clamped into the matrix and rows >= M
  // are zeroed at the LDS store (a guarded load per element made hipcc
  // branch around each one and wait for the previous before issuing it)
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      int row, c;
      amap(i, row, c);
      const int gr = min(m0 + row, M - 1);
      const size_t off = g.p16io ? pk(gr, k0 + c, K) : (size_t)gr * g.lda + k0 + c;
      ra[i] = ld4(A + off);  // raw: the LayerNorm is applied at the LDS store, once the row statistics are in
    }
#pragma unroll
    for (int i = 0; i < W4; ++i) {
      const int f = tid + i * NT, row = f / TPK, c = (f % TPK) * 4;
      if constexpr (H3)  // 16-byte chunk c/4 of the row's [k0, k0+32) image: 8-k group c/8, plane (c/4)&1
        rw[i] = *reinterpret_cast<const f32x4*>(g.Wh + (size_t)(n0 + row) * 2 * K + 2 * k0 + 2 * c);
      else
        rw[i] = ld4(g.W + (size_t)(n0 + row) * g.ldw + k0 + c);
    }
  };
  float amax = 0.f;  // split-fp16 range guard (H3, no LN prologue)
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      int row, c;
      amap(i, row, c);
      if constexpr (LN) ra[i] = (ra[i] - s_mu[row]) * s_rs[row];
      if (m0 + row >= M) ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (H3) {
        if constexpr (!LN) amax = fmaxf(amax, absmax4(ra[i]));
        h4 hi, lo;
        split4(ra[i], hi, lo);
        float* p = &As[buf * BM * LDK + row * LDK + (c >> 3) * 8 + ((c >> 2) & 1) * 2];
        *reinterpret_cast<h4*>(p) = hi;
        *reinterpret_cast<h4*>(p + 4) = lo;
      } else if constexpr (M16) {
        st4(&As[buf * BM * LDK + row * LDK + (((c >> 2) ^ ((row >> 1) & 7)) << 2)], ra[i]);
      } else {
        st4(&As[buf * BM * LDK + row * LDK + c], ra[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < W4; ++i) {
      const int f = tid + i * NT, row = f / TPK, c = (f % TPK) * 4;
      if constexpr (M16)
        st4(&Ws[buf * BN * LDK + row * LDK + (((c >> 2) ^ ((row >> 1) & 7)) << 2)], rw[i]);
      else
        st4(&Ws[buf * BN * LDK + row * LDK + c], rw[i]);
    }
  };

  f32x16 acc[M16 ? 1 : FM][M16 ? 1 : FN];
  f32x4 acc16[M16 ? FM16 : 1][M16 ? FN16 : 1];
  if constexpr (M16) {
#pragma unroll
    for (int a = 0; a < FM16; ++a)
#pragma unroll
      for (int b = 0; b < FN16; ++b) acc16[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int b = 0; b < FN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  }

  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int KT = K / BK;

  // the first step's operands are in flight while the row statistics load
  // (QKV at M = 131072: 271.6 -> 266 us)
  load_tile(0);
  if (rows_dead(g.skip, g.skip_rpc, m0, BM, M)) return;
  if constexpr (LN) {
    if (g.part_in) {
      for (int r = tid; r < BM; r += NT) {
        float mu, rs;
        merge_stats(g.part_in + (size_t)min(m0 + r, M - 1) * ND_PART_LD * 2, g.part_n_in, mu, rs);
        s_mu[r] = mu;
        s_rs[r] = rs;
      }
    } else {
      // two-pass row statistics, one wave per row (K == 256, host-checked);
      // 8 rows' loads are issued together so their latencies overlap
      constexpr int NW = NT / 64, RPW = BM / NW, G = RPW < 8 ? RPW : 8;
      for (int r0 = 0; r0 < RPW; r0 += G) {
        f32x4 v[G];
#pragma unroll
        for (int i = 0; i < G; ++i) v[i] = ld4(A + (size_t)min(m0 + wave + (r0 + i) * NW, M - 1) * g.lda + lane * 4);
#pragma unroll
        for (int i = 0; i < G; ++i) {
          const int r = wave + (r0 + i) * NW;
          const float mu = wave_sum(v[i].x + v[i].y + v[i].z + v[i].w) * (1.0f / 256.0f);
          const f32x4 d = v[i] - mu;
          const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / 256.0f);
          if (lane == 0) {
            s_mu[r] = mu;
            s_rs[r] = ln_rsqrt(var + ND_LN_EPS);
          }
        }
      }
    }
    __syncthreads();
  }
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) load_tile((kt + 1) * BK);
    if constexpr (H3) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        h8 ah[FM], al[FM], bh[FN], bl[FN];
        const int o = (2 * ks + lh) * 8;  // this lane's 8-k group: hi at o, lo at o + 4 (words)
#pragma unroll
        for (int a = 0; a < FM; ++a) {
          const float* p = &As[buf * BM * LDK + (wm * FM * 32 + a * 32 + lr) * LDK + o];
          ah[a] = *reinterpret_cast<const h8*>(p);
          al[a] = *reinterpret_cast<const h8*>(p + 4);
        }
#pragma unroll
        for (int b = 0; b < FN; ++b) {
          const float* p = &Ws[buf * BN * LDK + (wn * FN * 32 + b * 32 + lr) * LDK + o];
          bh[b] = *reinterpret_cast<const h8*>(p);
          bl[b] = *reinterpret_cast<const h8*>(p + 4);
        }
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b) {
            acc[a][b] = mfma32h(ah[a], bl[b], acc[a][b]);
            acc[a][b] = mfma32h(al[a], bh[b], acc[a][b]);
            acc[a][b] = mfma32h(ah[a], bh[b], acc[a][b]);
          }
      }
    } else if constexpr (M16) {
      const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
      for (int kb = 0; kb < BK / 16; ++kb) {
        // a row block at a time: the W operands of the 16-k block stay, one A operand is live (the register
        // peak of holding all eight spilled)
        f32x4 bf[FN16];
#pragma unroll
        for (int b = 0; b < FN16; ++b) {
          const int row = wn * FN16 * 16 + b * 16 + r16;
          bf[b] = ld4(&Ws[buf * BN * LDK + row * LDK + (((kb * 4 + kq) ^ ((row >> 1) & 7)) << 2)]);
        }
#pragma unroll
        for (int a = 0; a < FM16; ++a) {
          const int row = wm * FM16 * 16 + a * 16 + r16;
          const f32x4 af = ld4(&As[buf * BM * LDK + row * LDK + (((kb * 4 + kq) ^ ((row >> 1) & 7)) << 2)]);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int b = 0; b < FN16; ++b) acc16[a][b] = mfma16(af[e], bf[b][e], acc16[a][b]);
        }
      }
    } else
#pragma unroll
    for (int kb = 0; kb < BK / 8; ++kb) {
      f32x4 af[FM], bf[FN];
#pragma unroll
      for (int a = 0; a < FM; ++a)
        af[a] = ld4(&As[buf * BM * LDK + (wm * FM * 32 + a * 32 + lr) * LDK + kb * 8 + lh * 4]);
#pragma unroll
      for (int b = 0; b < FN; ++b)
        bf[b] = ld4(&Ws[buf * BN * LDK + (wn * FN * 32 + b * 32 + lr) * LDK + kb * 8 + lh * 4]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b) acc[a][b] = mfma32(af[a][i], bf[b][i], acc[a][b]);
    }
    if (kt + 1 < KT) store_tile(buf ^ 1);
    __syncthreads();
  }
  if constexpr (H3 && !LN) flag_overflow(g.ovf, amax);

#pragma unroll
  for (int ep = 0; ep < EP; ++ep) {
    // epilogue 1: bias (+relu) into the LDS C tile (rows ep*RP .. +RP)
    if constexpr (M16) {
      // lane l, reg r of block (a, b): row 16 a + 4 (l >> 4) + r, column 16 b + (l & 15)
      if (EP == 1 || wm == ep) {
#pragma unroll
        for (int b = 0; b < FN16; ++b) {
          const int cl = wn * FN16 * 16 + b * 16 + (lane & 15);
          const float bv = g.bias ? g.bias[n0 + cl] : 0.f;
#pragma unroll
          for (int a = 0; a < FM16; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc16[a][b][r] + bv;
              if constexpr (RELU) v = fmaxf(v, 0.f);
              Cs[(wm * FM16 * 16 + a * 16 + 4 * (lane >> 4) + r - ep * RP) * LDC + cl] = v;
            }
        }
      }
    } else if (EP == 1 || wm == ep) {
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) {
          const int cl = wn * FN * 32 + b * 32 + lr;
          const float bv = g.bias ? g.bias[n0 + cl] : 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float v = (H3 ? acc[a][b][r] * g.wscale : acc[a][b][r]) + bv;
            if constexpr (RELU) v = fmaxf(v, 0.f);
            Cs[(wm * FM * 32 + a * 32 + mfma32_row(r, lane) - ep * RP) * LDC + cl] = v;
          }
        }
    }
    __syncthreads();
    f32_tile_rows<BN, NT, RP, RELU, RESID>(g, Cs, m0 + ep * RP, n0, nbt);
    if (EP > 1) __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Exact fp32 at large M (the encoder's GEMMs under exact fp32) with the
// operands brought to LDS by DMA (ND_F32D): the 256x256 tile, 8 waves of
// 128x64 and 16x16x4 MFMAs of gemm_f32_kernel's M16 form, in its k order (so
// bitwise its C), on a ring instead of register staging.
//  - k steps of 16 (A 16 KB + W 16 KB) in a ring of 4 LDS slots, every wave
//    copying 4 KB of each by buffer_load ... lds (lane-linear 1 KB per
//    instruction; the lane's row offset its only vector operand, the k step
//    in the scalar offset); FD_SLOTS - 1 steps in flight beyond the one
//    computed, one barrier per step;
//  - a row's four 16-B k chunks stored XOR-swizzled by (row >> 1) & 3, so a
//    lane's (row, 4-k) operand read is a conflict-free ds_read_b128;
//  - the LDS reads are inline asm with a counted lgkmcnt wait (an ordinary
//    LDS read after an LDS-DMA makes hipcc wait for every copy in flight),
//    the barrier a raw s_barrier behind a counted vmcnt;
//  - the LayerNorm applied to the operand registers, (a - mean) * rstd, as
//    the register-staged kernel applies it at its LDS store.
// (The 32x32x2 form of this ring, ca5ef35, was busier but held a 9% lower
// clock: DESIGN.md §3 "Exact fp32 encoder GEMMs".)
#ifndef ND_F32D
#define ND_F32D 1
#endif
#define FD_BK 16                       // k per step
// Ring slots and epilogue passes: the smaller LDS footprint wins under the pool's three calls in flight
// (exact leg, same box: register-staged 27.21 ms per call, 4 slots / 2 passes (135 KB) 27.10, 4 / 4 (133 KB)
// 27.06, 3 / 4 (100 KB) 27.00; profiles/r06_ab_f32d_ring.txt), although alone the ring kernel runs FFN1 and FFN2
// 5-8% slower than the register-staged one (lower clock, profiles/r06_f32d_s3e4_check.txt)
#ifndef FD_SLOTS
#define FD_SLOTS 3                     // ring slots (two steps in flight beyond the one computed)
#endif
#ifndef FD_EP
#define FD_EP 4                        // epilogue passes (row groups of 256 / FD_EP rows staged in LDS)
#endif
#define FD_SLOT (2 * 256 * FD_BK * 4)  // bytes per slot: A tile, then W tile
typedef __attribute__((address_space(3))) void fd_lds_void;

template <int OFF>
__device__ __forceinline__ f32x4 fd_ld(uint32_t a) {
  f32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(r) : "v"(a), "n"(OFF) : "memory");
  return r;
}
// a step's operands of one lane: its 8 A row blocks and 4 W row blocks (16 rows = 1 KB apart)
struct FdOps {
  f32x4 a[8], b[4];
};
__device__ __forceinline__ void fd_issue(FdOps& o, uint32_t aa, uint32_t ab) {
  o.a[0] = fd_ld<0>(aa);
  o.a[1] = fd_ld<1024>(aa);
  o.a[2] = fd_ld<2048>(aa);
  o.a[3] = fd_ld<3072>(aa);
  o.a[4] = fd_ld<4096>(aa);
  o.a[5] = fd_ld<5120>(aa);
  o.a[6] = fd_ld<6144>(aa);
  o.a[7] = fd_ld<7168>(aa);
  o.b[0] = fd_ld<0>(ab);
  o.b[1] = fd_ld<1024>(ab);
  o.b[2] = fd_ld<2048>(ab);
  o.b[3] = fd_ld<3072>(ab);
}
__device__ __forceinline__ void fd_land(FdOps& o) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(o.a[0]), "+v"(o.a[1]), "+v"(o.a[2]), "+v"(o.a[3]), "+v"(o.a[4]), "+v"(o.a[5]), "+v"(o.a[6]),
                 "+v"(o.a[7]), "+v"(o.b[0]), "+v"(o.b[1]), "+v"(o.b[2]), "+v"(o.b[3])
               :
               : "memory");
}

template <bool LN, bool RELU, bool RESID>
__global__ void __launch_bounds__(512) gemm_f32d_kernel(const GemmArgs g) {
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4, NT = 512, EP = FD_EP, RP = BM / EP, LDC = BN + 4;
  static_assert(EP == 2 || EP == 4, "a pass is one wave row group or half of one");
  constexpr int FM16 = 8, FN16 = 4;
  constexpr int RING = FD_SLOTS * FD_SLOT, CBYTES = RP * LDC * 4;
  __shared__ __attribute__((aligned(16))) char fd_sm[RING > CBYTES ? RING : CBYTES];
  __shared__ float s_mu[LN ? BM : 1], s_rs[LN ? BM : 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  const int ntn = g.N / BN;
  int nbt, mbk;
  if (g.xcd_map) {  // as gemm_f32_kernel
    const int b = blockIdx.x, j = b >> 3;
    nbt = j % ntn;
    mbk = (j / ntn) * 8 + (b & 7);
  } else {
    nbt = blockIdx.x % ntn;
    mbk = blockIdx.x / ntn;
  }
  const int n0 = nbt * BN, m0 = mbk * BM;
  const int M = g.M, KT = g.K / FD_BK;

  // copies: wave w moves pieces 2w, 2w + 1 of each tile (1 KB each: 16 rows x 4 chunks); the lane's piece is
  // row 16 j + lane / 4, k chunk (lane & 3) ^ ((lane >> 3) & 3) (rows past M clamped: never stored)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.A + (size_t)m0 * g.lda), 0,
                                                                      0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.W + (size_t)n0 * g.ldw), 0,
                                                                      0x7fffffff, 0x00020000);
  const int kc = (lane & 3) ^ ((lane >> 3) & 3);
  int voa[2], vow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (2 * wu + i) * 16 + (lane >> 2);
    voa[i] = min(row, M - 1 - m0) * g.lda * 4 + kc * 16;
    vow[i] = row * g.ldw * 4 + kc * 16;
  }
  auto issue = [&](int st) {  // k step st into slot st % FD_SLOTS
    char* sl = fd_sm + (st % FD_SLOTS) * FD_SLOT;
    const int so = st * FD_BK * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (fd_lds_void*)(sl + (2 * wu + i) * 1024), 16, voa[i], so, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (fd_lds_void*)(sl + FD_SLOT / 2 + (2 * wu + i) * 1024), 16,
                                               vow[i], so, 0, 0);
  };

  if (rows_dead(g.skip, g.skip_rpc, m0, BM, M)) return;
#pragma unroll
  for (int p = 0; p < FD_SLOTS - 1; ++p) issue(p);  // KT >= FD_SLOTS (host-checked)

  const int wm = wave / WN, wn = wave % WN;
  const int r16 = lane & 15, kq = lane >> 4;
  float mu[FM16], rs[FM16];
  if constexpr (LN) {
    // the row statistics' loads go out beside the first copies (the LDS stores below wait for both)
    if (g.part_in) {
      for (int r = tid; r < BM; r += NT) {
        float m_, r_;
        merge_stats(g.part_in + (size_t)min(m0 + r, M - 1) * ND_PART_LD * 2, g.part_n_in, m_, r_);
        s_mu[r] = m_;
        s_rs[r] = r_;
      }
    } else {
      // two-pass row statistics, one wave per row (K == 256, host-checked)
      constexpr int NW = NT / 64, RPW = BM / NW, G = 8;
      for (int r0 = 0; r0 < RPW; r0 += G) {
        f32x4 v[G];
#pragma unroll
        for (int i = 0; i < G; ++i) v[i] = ld4(g.A + (size_t)min(m0 + wave + (r0 + i) * NW, M - 1) * g.lda + lane * 4);
#pragma unroll
        for (int i = 0; i < G; ++i) {
          const int r = wave + (r0 + i) * NW;
          const float m_ = wave_sum(v[i].x + v[i].y + v[i].z + v[i].w) * (1.0f / 256.0f);
          const f32x4 d = v[i] - m_;
          const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / 256.0f);
          if (lane == 0) {
            s_mu[r] = m_;
            s_rs[r] = ln_rsqrt(var + ND_LN_EPS);
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < FM16; ++a) {
      mu[a] = s_mu[wm * FM16 * 16 + a * 16 + r16];
      rs[a] = s_rs[wm * FM16 * 16 + a * 16 + r16];
    }
  }

  f32x4 acc16[FM16][FN16];
#pragma unroll
  for (int a = 0; a < FM16; ++a)
#pragma unroll
    for (int b = 0; b < FN16; ++b) acc16[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the lane's operand addresses in a slot: its A / W row in block 0 and its swizzled 16-B chunk
  const uint32_t lbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)fd_sm);
  const uint32_t x = (uint32_t)((kq ^ ((r16 >> 1) & 3)) * 16);
  const uint32_t oa = (uint32_t)((wm * FM16 * 16 + r16) * 64) + x;
  const uint32_t ob = (uint32_t)(FD_SLOT / 2 + (wn * FN16 * 16 + r16) * 64) + x;
  FdOps o;
  for (int kt = 0; kt < KT; ++kt) {
    // step kt landed for every wave (younger steps in flight: kt + 1, kt + 2 when they exist), and every wave is
    // done reading slot kt - 1: it takes step kt + 3
    const int younger = KT - 1 - kt;
    if (FD_SLOTS >= 4 && younger >= 2)
      asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else if (younger >= 1)
      asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + FD_SLOTS - 1 < KT) issue(kt + FD_SLOTS - 1);
    const uint32_t sb = lbase + (uint32_t)((kt % FD_SLOTS) * FD_SLOT);
    fd_issue(o, sb + oa, sb + ob);
    fd_land(o);
    if constexpr (LN) {
#pragma unroll
      for (int a = 0; a < FM16; ++a) o.a[a] = (o.a[a] - mu[a]) * rs[a];
    }
#pragma unroll
    for (int a = 0; a < FM16; ++a)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int b = 0; b < FN16; ++b) acc16[a][b] = mfma16(o.a[a][e], o.b[b][e], acc16[a][b]);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is done with the ring: it becomes the C tile
  float* Cs = reinterpret_cast<float*>(fd_sm);
#pragma unroll
  for (int ep = 0; ep < EP; ++ep) {
    constexpr int AP = FM16 * WM / EP;  // row blocks of a wave per pass
    if (wm == ep * WM / EP) {
      // lane l, reg r of block (a, b): row 16 a + 4 (l >> 4) + r, column 16 b + (l & 15)
      const int a0 = (ep % (EP / WM)) * AP;
#pragma unroll
      for (int b = 0; b < FN16; ++b) {
        const int cl = wn * FN16 * 16 + b * 16 + r16;
        const float bv = g.bias ? g.bias[n0 + cl] : 0.f;
#pragma unroll
        for (int a = 0; a < FM16; ++a) {
          if (a < a0 || a >= a0 + AP) continue;  // compile-time per pass after unrolling
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc16[a][b][r] + bv;
            if constexpr (RELU) v = fmaxf(v, 0.f);
            Cs[((a - a0) * 16 + 4 * kq + r) * LDC + cl] = v;
          }
        }
      }
    }
    __syncthreads();
    f32_tile_rows<BN, NT, RP, RELU, RESID>(g, Cs, m0 + ep * RP, n0, nbt);
    if (EP > 1) __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Decoder-step kernel (small M: the batch's rows) on the fragment-packed
// layout (common.hpp, pk()).  A [M,K], W [N,K], R and C [M,N] are all P16
// packed, so every operand fragment, the residual and the output tile move
// as ONE coalesced 1 KB wave access (row-major fragments touch 16 rows per
// instruction and keep the address path ~3x busier).  The product runs
// transposed, C^T = W A^T, because the 16x16x4 MFMA's D fragment of W A^T is
// exactly a P16 entry of C (lane l: row l&15, columns 4(l>>4)..+3).
//
// Workgroup = 16 rows x (NT*16) columns; wave (t, s) owns column block t and
// K slice s (K = KS*KW).  Each wave issues all of its loads up front (fragments,
// bias, residual, the LayerNorm row statistics) before the first MFMA; two
// interleaved accumulator chains; K slices are summed through LDS.
// LN: rows are normalised with statistics merged from the producer's
// partials (part_in); gamma/beta are folded into W / bias.
// the bias operand of a GEMM without one: its load stays unconditional (a
// branch around it made hipcc wait vmcnt(0) there, draining every A / W
// load in flight before the epilogue operands were even requested)
__device__ __attribute__((aligned(16))) float nd_zero16[16];


// Split-fp16 form on the P16 layout (H3, see the row-major kernel): the
// 16x16x32 f16 MFMA takes 8 k per lane; lane l supplies the 4 k of its P16
// entry in k-block 2p followed by the 4 of k-block 2p+1, for the weight and
// the activation alike (one shared permutation of the pair's 32 k), and its D
// fragment is the P16 entry of C as with 16x16x4.  The weight image (P16H,
// launch_pack_p16h) holds per column block and k pair a hi plane and a lo
// plane, each one 1 KB wave access: [nb][K/32][hi | lo][64 lanes][8 halves].
__device__ __forceinline__ f32x4 mfma16h(h8 a, h8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void split8(f32x4 x0, f32x4 x1, h8& hi, h8& lo) {
  h4 h0, l0, h1, l1;
  split4(x0, h0, l0);
  split4(x1, h1, l1);
  hi = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
  lo = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
}

template <int NT, int KS, int KW, bool H3, bool LN, bool RELU, bool RESID>
__global__ void __launch_bounds__(NT* KS * 64) gemm_p16_kernel(const GemmArgs g) {
#ifdef ND_SKIP_P16  // timing probe only (tools/build_variant.sh): the kernel's marginal cost
  if (g.M >= 0) return;
#endif
  constexpr int WAVES = NT * KS;
  constexpr int NF = KW / 16;  // 16-k blocks per wave
  __shared__ f32x4 red[KS > 1 ? WAVES : 1][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wt = wave % NT, ws = wave / NT;
  // XCD-aware block order: consecutive workgroups go to the 8 XCDs in turn
  // (b % 8 share one), so XCD x is given a rectangle of (GY / a) row blocks x
  // (GX / (8 / a)) column groups; each XCD's L2 then fetches 1 / a of A and
  // a / 8 of W instead of all of A (grid order: x fastest, every XCD saw
  // every row block; measured 4.2x the algorithmic fabric bytes at K = 2048)
  int bx = blockIdx.x, by = blockIdx.y;
  if (g.xcd_a) {
    const int GX = gridDim.x, GY = gridDim.y, a = g.xcd_a, lc = GX / (8 / a);
    const int lin = by * GX + bx, x = lin & 7, j = lin >> 3;
    by = (x / (8 / a)) * (GY / a) + j / lc;
    bx = (x % (8 / a)) * lc + j % lc;
  }
  const int nb = bx * NT + wt, mb = by;
  const int KB = g.K >> 4, NB = g.N >> 4;
  if (rows_dead(g.skip, g.skip_rpc, mb * 16, 16, g.M)) return;
  const f32x4* __restrict__ ap = reinterpret_cast<const f32x4*>(g.A) + ((size_t)mb * KB + ws * NF) * 64 + lane;
  // fp32 P16 blocks, or (H3) the P16H image: per 32-k pair a hi and a lo 1 KB plane
  const f32x4* __restrict__ wp = H3 ? reinterpret_cast<const f32x4*>(g.Wh) + ((size_t)nb * KB + ws * NF) * 64 + lane
                                    : reinterpret_cast<const f32x4*>(g.W) + ((size_t)nb * KB + ws * NF) * 64 + lane;
  // every load straight-line, in the order of use: LN partials, A / W, then
  // the epilogue's bias and residual (the waits below count down in order)
  PartRow pr;
  if constexpr (LN) load_stats(g.part_in + (size_t)(mb * 16 + (lane & 15)) * ND_PART_LD * 2, pr);
  f32x4 a[NF], w[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    a[f] = ap[f * 64];
    w[f] = wp[f * 64];
  }
  const size_t ct = ((size_t)mb * NB + nb) * 64 + lane;  // this lane's output entry
  const f32x4 bv = ld4((g.bias ? g.bias + nb * 16 : nd_zero16) + 4 * (lane >> 4));
  f32x4 rv = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RESID) rv = reinterpret_cast<const f32x4*>(g.R)[ct];
  float mu = 0.f, rs = 1.f;
  if constexpr (LN) merge_loaded(pr, g.part_n_in, mu, rs);
  // keep every load in flight before the first MFMA waits
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (LN) {
#pragma unroll
    for (int f = 0; f < NF; ++f) a[f] = (a[f] - mu) * rs;
  }
  if constexpr (H3 && !LN) {
    float amax = 0.f;
#pragma unroll
    for (int f = 0; f < NF; ++f) amax = fmaxf(amax, absmax4(a[f]));
    flag_overflow(g.ovf, amax);
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (H3) {
#pragma unroll
    for (int p = 0; p < NF / 2; ++p) {
      h8 ah, al;
      split8(a[2 * p], a[2 * p + 1], ah, al);
      const h8 wh = __builtin_bit_cast(h8, w[2 * p]), wl = __builtin_bit_cast(h8, w[2 * p + 1]);
      acc0 = mfma16h(wh, ah, acc0);
      acc1 = mfma16h(wh, al, acc1);
      acc1 = mfma16h(wl, ah, acc1);
    }
  } else {
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      acc0 = mfma16(w[f][0], a[f][0], acc0);
      acc1 = mfma16(w[f][1], a[f][1], acc1);
      acc0 = mfma16(w[f][2], a[f][2], acc0);
      acc1 = mfma16(w[f][3], a[f][3], acc1);
    }
  }
  f32x4 v = acc0 + acc1;
  if constexpr (H3) v *= g.wscale;
  if constexpr (KS > 1) {
    red[wave][lane] = v;
    __syncthreads();
    if (ws != 0) return;
    v = red[wt][lane];
#pragma unroll
    for (int s2 = 1; s2 < KS; ++s2) v += red[s2 * NT + wt][lane];
  }
  v += bv;
  if constexpr (RELU) v = {fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
  if constexpr (RESID) v += rv;
  if (g.c_rm)
    st4(g.C + (size_t)(mb * 16 + (lane & 15)) * g.N + nb * 16 + 4 * (lane >> 4), v);
  else
    reinterpret_cast<f32x4*>(g.C)[ct] = v;
  if (g.part_out) {
    // row statistics over this block's 16 columns: lanes l, l^16, l^32, l^48
    const float m_ = xor32_sum(xor16_sum(v.x + v.y + v.z + v.w)) * (1.0f / 16.0f);
    const f32x4 d = v - m_;
    const float q = xor32_sum(xor16_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w));
    if (lane < 16) {
      float* p = g.part_out + ((size_t)(mb * 16 + lane) * ND_PART_LD + nb) * 2;
      p[0] = m_;
      p[1] = q;
    }
  }
}

// K = 256 variant with both operands staged through LDS: workgroup tile =
// BMB row blocks x BNB column blocks (one 16x16 output block per wave).
// The A row blocks and W column blocks are each loaded ONCE per workgroup
// (coalesced 1 KB P16 blocks, the LayerNorm applied on the way in) instead
// of once per wave, which cuts the L2 -> CU traffic that bounds these
// small-M GEMMs (FFN1 / query projections: 256 -> 96 KB per workgroup).
template <int BMB, int BNB, bool H3, bool LN, bool RELU, bool RESID>
__global__ void __launch_bounds__(BMB* BNB * 64) gemm_p16s_kernel(const GemmArgs g) {
#ifdef ND_SKIP_P16  // timing probe only
  if (g.M >= 0) return;
#endif
  constexpr int NW = BMB * BNB, KB = ND_D / 16;
  extern __shared__ f32x4 sh[];
  f32x4* As = sh;                  // [BMB][KB][64]  (H3: [BMB][KB/2][hi | lo][64])
  f32x4* Ws = sh + BMB * KB * 64;  // [BNB][KB][64]  (H3: the P16H image)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb0 = blockIdx.x * BNB, mb0 = blockIdx.y * BMB, NB = g.N >> 4;
  const int MB = (g.M + 15) >> 4;  // row blocks that exist (buffers are padded to 16 rows, not 16*BMB)
  if (rows_dead(g.skip, g.skip_rpc, mb0 * 16, BMB * 16, g.M)) return;
  const f32x4* __restrict__ A4 = reinterpret_cast<const f32x4*>(g.A);
  const f32x4* __restrict__ W4 = reinterpret_cast<const f32x4*>(H3 ? (const void*)g.Wh : (const void*)g.W);
  // stage: block j of A = (row block mb0 + j / KB, k block j % KB), likewise W.
  // H3 stages A in k-block pairs (i even / odd = blocks 2 jp, 2 jp + 1) so a
  // thread holds both halves of each 32-k operand it splits.
  constexpr int AJ = BMB * KB / NW, WJ = BNB * KB / NW;
  static_assert(AJ * NW == BMB * KB && WJ * NW == BNB * KB, "blocks per wave");
  static_assert(!H3 || AJ % 2 == 0, "H3 stages A block pairs");
  auto aj = [&](int i) { return H3 ? 2 * (wave + (i >> 1) * NW) + (i & 1) : wave + i * NW; };
  // LN partials first (every lane: the rows lane & 15 of the BMB row blocks,
  // the rows its staged A blocks and its output block belong to), then A /
  // W, then bias and residual: straight-line, waits in order.  The row
  // statistics stay in registers: no LDS hand-off, no barrier for them (a
  // wave-0 LDS hand-off measured a corrupted tile when another kernel's
  // workgroups shared the CU, EnginePool)
  PartQuad pr[LN ? BMB : 1];
  if constexpr (LN)
#pragma unroll
    for (int b = 0; b < BMB; ++b)
      load_stats_quad(g.part_in + (size_t)min(mb0 * 16 + b * 16 + (lane & 15), MB * 16 - 1) * ND_PART_LD * 2,
                      lane >> 4, pr[b]);
  f32x4 av[AJ], wv[WJ];
#pragma unroll
  for (int i = 0; i < AJ; ++i) {
    const int j = aj(i);
    av[i] = A4[((size_t)min(mb0 + j / KB, MB - 1) * KB + j % KB) * 64 + lane];
  }
#pragma unroll
  for (int i = 0; i < WJ; ++i) {
    const int j = wave + i * NW;
    wv[i] = W4[((size_t)(nb0 + j / KB) * KB + j % KB) * 64 + lane];
  }
  // this wave's output block (rb, cb) and its epilogue operands
  const int rb = wave / BNB, cb = wave % BNB, nb = nb0 + cb, mb = mb0 + rb;
  const bool live = mb < MB;
  const size_t ct = ((size_t)min(mb, MB - 1) * NB + nb) * 64 + lane;
  const f32x4 bv = ld4((g.bias ? g.bias + nb * 16 : nd_zero16) + 4 * (lane >> 4));
  f32x4 rv = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RESID) rv = reinterpret_cast<const f32x4*>(g.R)[ct];
  // LayerNorm row statistics of rows b * 16 + (lane & 15)
  float smu[BMB], srs[BMB];
  if constexpr (LN)
#pragma unroll
    for (int b = 0; b < BMB; ++b) merge_quad(pr[b], g.part_n_in, lane >> 4, smu[b], srs[b]);
  if constexpr (H3) {
    // normalise and split while staging: every A element converted once per workgroup
    if constexpr (!LN) {
      float amax = 0.f;
#pragma unroll
      for (int i = 0; i < AJ; ++i) amax = fmaxf(amax, absmax4(av[i]));
      flag_overflow(g.ovf, amax);
    }
#pragma unroll
    for (int i = 0; i < AJ; i += 2) {
      const int j = aj(i);
      f32x4 x0 = av[i], x1 = av[i + 1];
      if constexpr (LN) {
        const int b = j / KB;  // the block's row block (its row: b * 16 + (lane & 15))
        const float m_ = smu[b], r_ = srs[b];
        x0 = (x0 - m_) * r_;
        x1 = (x1 - m_) * r_;
      }
      h8 hi, lo;
      split8(x0, x1, hi, lo);
      As[j * 64 + lane] = __builtin_bit_cast(f32x4, hi);
      As[(j + 1) * 64 + lane] = __builtin_bit_cast(f32x4, lo);
    }
  } else {
#pragma unroll
    for (int i = 0; i < AJ; ++i) As[(wave + i * NW) * 64 + lane] = av[i];
  }
#pragma unroll
  for (int i = 0; i < WJ; ++i) Ws[(wave + i * NW) * 64 + lane] = wv[i];
  __syncthreads();
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const f32x4* ar = As + rb * KB * 64 + lane;
  const f32x4* wr = Ws + cb * KB * 64 + lane;
  if constexpr (H3) {
#pragma unroll
    for (int p = 0; p < KB / 2; ++p) {
      const h8 ah = __builtin_bit_cast(h8, ar[2 * p * 64]), al = __builtin_bit_cast(h8, ar[(2 * p + 1) * 64]);
      const h8 wh = __builtin_bit_cast(h8, wr[2 * p * 64]), wl = __builtin_bit_cast(h8, wr[(2 * p + 1) * 64]);
      acc0 = mfma16h(wh, ah, acc0);
      acc1 = mfma16h(wh, al, acc1);
      acc1 = mfma16h(wl, ah, acc1);
    }
  } else {
    float mu = 0.f, rs = 1.f;
    if constexpr (LN) {
      mu = smu[rb];
      rs = srs[rb];
    }
#pragma unroll
    for (int f = 0; f < KB; ++f) {
      f32x4 a = ar[f * 64];
      const f32x4 w = wr[f * 64];
      if constexpr (LN) a = (a - mu) * rs;
      acc0 = mfma16(w[0], a[0], acc0);
      acc1 = mfma16(w[1], a[1], acc1);
      acc0 = mfma16(w[2], a[2], acc0);
      acc1 = mfma16(w[3], a[3], acc1);
    }
  }
  f32x4 v = acc0 + acc1;
  if constexpr (H3) v *= g.wscale;
  v += bv;
  if constexpr (RELU) v = {fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
  if constexpr (RESID) v += rv;
  if (!live) return;
  if (g.c_rm)
    st4(g.C + (size_t)(mb * 16 + (lane & 15)) * g.N + nb * 16 + 4 * (lane >> 4), v);
  else
    reinterpret_cast<f32x4*>(g.C)[ct] = v;
  if (g.part_out) {
    const float m_ = xor32_sum(xor16_sum(v.x + v.y + v.z + v.w)) * (1.0f / 16.0f);
    const f32x4 d = v - m_;
    const float q = xor32_sum(xor16_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w));
    if (lane < 16) {
      float* p = g.part_out + ((size_t)(mb * 16 + lane) * ND_PART_LD + nb) * 2;
      p[0] = m_;
      p[1] = q;
    }
  }
}

// Long-K decoder products (the memory bank's output projection W_vo and
// FFN2, K = 2048, at 128 < M <= 1024 rows) split over workgroups.  The
// one-block-per-workgroup kernel above (16 x 16 outputs, the whole K on 8
// waves) pulls 256 KB of A and W into every CU for 16 x 16 outputs; here a
// workgroup owns a 32 x 32 tile (2 x 2 blocks) over one K-slice of 512 (4
// waves of 128 k), so a CU takes in 128 KB for 4 blocks and the launch moves
// half the L2 -> CU bytes (MI355X_MICROARCH.md: per-CU ingest bounds these
// latency-bound shapes).  The 4 waves' partials are summed through LDS in wave
// order; the K / 512 slices of a tile meet in an fp32 slab: write-through
// (sc1) stores, every wave's vmcnt(0), one agent-scope ticket per workgroup;
// the workgroup that draws the last ticket reads the slabs back with sc1 loads
// and sums them in slice order (deterministic: the result does not depend on
// which slice arrives last), adds bias / residual, writes C and the row
// statistics, and resets the tile's ticket for the next launch
// (cdna_hip_programming.md §5 "Projection GEMM at M = 256", §6 Guideline 16).
#define PK_NW 4    // waves per workgroup (k sub-slices)
#define PK_KPW 4   // 32-k pairs per wave
#define PK_SLICE (PK_NW * PK_KPW * 32)  // k per workgroup (512)

__device__ __forceinline__ void pk_store_sc1(__amdgpu_buffer_rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), r, off, 0, 16);  // aux 16 = sc1
}
__device__ __forceinline__ f32x4 pk_load_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

// !H3 (exact fp32, nd_set_exact_fp32): the same tiles and slices on the fp32 P16 weight (16-k blocks, 4
// v_mfma_f32_16x16x4f32 per block and output block), no range guard, no weight scale
template <bool H3, bool RESID>
__global__ void __launch_bounds__(PK_NW * 64) gemm_p16k_kernel(const GemmArgs g) {
  // ONE shared array: the waves' partial blocks, then the last-arriver word
  __shared__ __attribute__((aligned(16))) f32x4 red[PK_NW * 4 * 64 + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int S = g.K / PK_SLICE, NBT = g.N >> 5;  // slices; 32-column tiles across N
  const int tile = blockIdx.x / S, sl = blockIdx.x % S;
  const int mb0 = 2 * (tile / NBT), nb0 = 2 * (tile % NBT);
  const int MB = (g.M + 15) >> 4, KB = g.K >> 4, KP = g.K >> 5, NB = g.N >> 4;
  const f32x4* __restrict__ A4 = reinterpret_cast<const f32x4*>(g.A);
  const f32x4* __restrict__ W4 = reinterpret_cast<const f32x4*>(H3 ? (const void*)g.Wh : (const void*)g.W);
  // this wave's k pairs: sl * 16 + wave * 4 .. + 3; loads in order of use, straight-line
  const int kp0 = sl * (PK_NW * PK_KPW) + wave * PK_KPW;
  f32x4 a[2][2 * PK_KPW], w[2][2 * PK_KPW];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int f = 0; f < 2 * PK_KPW; ++f) a[r][f] = A4[((size_t)min(mb0 + r, MB - 1) * KB + 2 * kp0 + f) * 64 + lane];
  // H3: the P16H image's hi / lo planes of each k pair; fp32: the P16 blocks 2 kp0 .. + 7, as A
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int f = 0; f < 2 * PK_KPW; ++f)
      w[c][f] = H3 ? W4[(((size_t)(nb0 + c) * KP + kp0) * 2 + f) * 64 + lane]
                   : W4[((size_t)(nb0 + c) * KB + 2 * kp0 + f) * 64 + lane];
  // the epilogue operands of the block this wave finishes (rb, cb) = (wave >> 1, wave & 1)
  const int rb = wave >> 1, cb = wave & 1, mb = mb0 + rb, nb = nb0 + cb;
  const size_t ct = ((size_t)min(mb, MB - 1) * NB + nb) * 64 + lane;
  const f32x4 bv = ld4((g.bias ? g.bias + nb * 16 : nd_zero16) + 4 * (lane >> 4));
  f32x4 rv = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RESID) rv = reinterpret_cast<const f32x4*>(g.R)[ct];
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc0[4], acc1[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) acc0[b] = acc1[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (H3) {
    float amax = 0.f;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int f = 0; f < 2 * PK_KPW; ++f) amax = fmaxf(amax, absmax4(a[r][f]));
    flag_overflow(g.ovf, amax);
#pragma unroll
    for (int p = 0; p < PK_KPW; ++p) {
      h8 ah[2], al[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) split8(a[r][2 * p], a[r][2 * p + 1], ah[r], al[r]);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const h8 wh = __builtin_bit_cast(h8, w[b & 1][2 * p]), wl = __builtin_bit_cast(h8, w[b & 1][2 * p + 1]);
        acc0[b] = mfma16h(wh, ah[b >> 1], acc0[b]);
        acc1[b] = mfma16h(wh, al[b >> 1], acc1[b]);
        acc1[b] = mfma16h(wl, ah[b >> 1], acc1[b]);
      }
    }
  } else {
#pragma unroll
    for (int f = 0; f < 2 * PK_KPW; ++f)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const f32x4 wv = w[b & 1][f], av = a[b >> 1][f];
        acc0[b] = mfma16(wv[0], av[0], acc0[b]);
        acc1[b] = mfma16(wv[1], av[1], acc1[b]);
        acc0[b] = mfma16(wv[2], av[2], acc0[b]);
        acc1[b] = mfma16(wv[3], av[3], acc1[b]);
      }
  }
  // the workgroup's slice: block b summed over the 4 waves in wave order, by wave b
#pragma unroll
  for (int b = 0; b < 4; ++b) red[(wave * 4 + b) * 64 + lane] = acc0[b] + acc1[b];
  lds_barrier();
  f32x4 v = red[(0 * 4 + wave) * 64 + lane];
#pragma unroll
  for (int w2 = 1; w2 < PK_NW; ++w2) v += red[(w2 * 4 + wave) * 64 + lane];
  if (S > 1) {
    // slab [tile][slice][block][64 lanes] f32x4, write-through
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        g.sk_slab + (size_t)tile * S * 4 * 256, 0, S * 4 * 1024, 0x00020000);
    pk_store_sc1(rs, ((sl * 4 + wave) * 64 + lane) * 16, v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, before the ticket
    __syncthreads();
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(g.sk_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      reinterpret_cast<int*>(&red[PK_NW * 4 * 64])[0] = t;
    }
    __syncthreads();
    if (reinterpret_cast<const int*>(&red[PK_NW * 4 * 64])[0] != S - 1) return;  // not the last slice
    // the last arriver: every slice of block `wave` (S <= 4), all loads in flight at once (sc1; its own
    // from registers), summed in slice order
    f32x4 pp[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) pp[s2] = pk_load_sc1(rs, ((min(s2, S - 1) * 4 + wave) * 64 + lane) * 16);
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2)
      if (s2 < S) sum += s2 == sl ? v : pp[s2];
    v = sum;
    if (tid == 0) __hip_atomic_store(g.sk_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (H3) v *= g.wscale;
  v += bv;
  if constexpr (RESID) v += rv;
  if (mb >= MB) return;
  reinterpret_cast<f32x4*>(g.C)[ct] = v;
  if (g.part_out) {
    const float m_ = xor32_sum(xor16_sum(v.x + v.y + v.z + v.w)) * (1.0f / 16.0f);
    const f32x4 d = v - m_;
    const float q = xor32_sum(xor16_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w));
    if (lane < 16) {
      float* pp = g.part_out + ((size_t)(mb * 16 + lane) * ND_PART_LD + nb) * 2;
      pp[0] = m_;
      pp[1] = q;
    }
  }
}

// row-major [M, N] (leading dim ld) -> P16 packed, one thread per float4
__global__ void __launch_bounds__(256)
pack_p16_kernel(const float* __restrict__ src, int ld, float* __restrict__ dst, int M, int N) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)M * (N / 4)) return;
  const int m = (int)(i / (N / 4)), n = (int)(i % (N / 4)) * 4;
  st4(dst + pk(m, n, N), ld4(src + (size_t)m * ld + n));
}

hipError_t launch_pack_p16(const float* src, int ld, float* dst, int M, int N, hipStream_t s) {
  if (M % 16 || N % 16 || ld < N) return hipErrorInvalidValue;
  const size_t n4 = (size_t)M * (N / 4);
  hipLaunchKernelGGL(pack_p16_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, src, ld, dst, M, N);
  return hipGetLastError();
}

// max |W| as float bits (non-negative floats order like their bit patterns)
__global__ void __launch_bounds__(256) absmax_kernel(const float* __restrict__ W, size_t n, unsigned* __restrict__ out) {
  float m = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) m = fmaxf(m, fabsf(W[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

// one thread per 8-k group of a row: 8 hi halves then 8 lo halves (32 bytes)
__global__ void __launch_bounds__(256)
split_weight_kernel(const float* __restrict__ W, int ld, int K, size_t groups, float scale,
                    uint16_t* __restrict__ Wh) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= groups) return;
  const size_t n = i / (K / 8), k = (i % (K / 8)) * 8;
  const f32x4 v0 = ld4(W + n * ld + k) * scale, v1 = ld4(W + n * ld + k + 4) * scale;
  h4 h0, l0, h1, l1;
  split4(v0, h0, l0);
  split4(v1, h1, l1);
  h4* o = reinterpret_cast<h4*>(Wh + 16 * i);
  o[0] = h0;
  o[1] = h1;
  o[2] = l0;
  o[3] = l1;
}

hipError_t launch_split_weight(const float* W, int N, int K, uint16_t* Wh, float* wscale, hipStream_t s, int ld);

// P16H image (see mfma16h): thread = (column block, k pair, lane)
__global__ void __launch_bounds__(256) pack_p16h_kernel(const float* __restrict__ W, int ld, int N, int K, float scale,
                                                        uint16_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int KP = K / 32;
  if (i >= (size_t)(N / 16) * KP * 64) return;
  const int lane = (int)(i & 63), kp = (int)((i >> 6) % KP), nb = (int)((i >> 6) / KP);
  const float* r = W + (size_t)(nb * 16 + (lane & 15)) * ld + kp * 32 + 4 * (lane >> 4);
  h8 hi, lo;
  split8(ld4(r) * scale, ld4(r + 16) * scale, hi, lo);
  f32x4* o = reinterpret_cast<f32x4*>(out) + ((size_t)(nb * KP + kp) * 2) * 64 + lane;
  o[0] = __builtin_bit_cast(f32x4, hi);
  o[64] = __builtin_bit_cast(f32x4, lo);
}

// power-of-two exponent s with max|W| 2^s in [2^13, 2^14) (0 for an all-zero
// or non-finite W); synchronises the stream
static hipError_t weight_scale_exp(const float* W, int ld, int N, int K, hipStream_t s, int* s_exp) {
  unsigned* d = nullptr;
  hipError_t e = hipMallocAsync((void**)&d, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  unsigned bits = 0;
  if ((e = hipMemsetAsync(d, 0, sizeof(unsigned), s)) == hipSuccess) {
    for (int n = 0; n < N && e == hipSuccess; n += 1024) {  // rows in slabs: ld may exceed K
      const size_t cnt = (size_t)std::min(1024, N - n) * ld - (ld - K);
      hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)std::min<size_t>((cnt + 255) / 256, 1024)), dim3(256), 0, s,
                         W + (size_t)n * ld, cnt, d);
      e = hipGetLastError();
    }
    if (e == hipSuccess && (e = hipMemcpyAsync(&bits, d, 4, hipMemcpyDeviceToHost, s)) == hipSuccess)
      e = hipStreamSynchronize(s);
  }
  (void)hipFreeAsync(d, s);
  if (e != hipSuccess) return e;
  float mx;
  memcpy(&mx, &bits, 4);
  *s_exp = 0;
  if (mx > 0.f && std::isfinite(mx)) {
    int ex;
    (void)std::frexp(mx, &ex);  // mx in [2^(ex-1), 2^ex)
    *s_exp = 14 - ex;
  }
  return hipSuccess;
}

hipError_t launch_pack_p16h(const float* W, int ld, int N, int K, uint16_t* out, float* wscale, hipStream_t s) {
  if (N % 16 || K % 32 || ld < K || !W || !out || !wscale) return hipErrorInvalidValue;
  int s_exp = 0;
  hipError_t e = weight_scale_exp(W, ld, N, K, s, &s_exp);
  if (e != hipSuccess) return e;
  const size_t n = (size_t)(N / 16) * (K / 32) * 64;
  hipLaunchKernelGGL(pack_p16h_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, ld, N, K,
                     std::ldexp(1.0f, s_exp), out);
  *wscale = std::ldexp(1.0f, -s_exp);
  return hipGetLastError();
}

// 2^s puts max|W| 2^s in [2^13, 2^14): hi stays far from the fp16 maximum
// (65504) and lo (about 2^-11 of its element) stays normal for elements
// above about 2^-14 of the largest.
hipError_t launch_split_weight(const float* W, int N, int K, uint16_t* Wh, float* wscale, hipStream_t s, int ld) {
  if (ld == 0) ld = K;
  if (N <= 0 || K % 32 != 0 || ld < K || ld % 4 || !W || !Wh || !wscale) return hipErrorInvalidValue;
  int s_exp = 0;
  hipError_t e = weight_scale_exp(W, ld, N, K, s, &s_exp);
  if (e != hipSuccess) return e;
  const size_t groups = (size_t)N * K / 8;
  hipLaunchKernelGGL(split_weight_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, W, ld, K, groups,
                     std::ldexp(1.0f, s_exp), Wh);
  *wscale = std::ldexp(1.0f, -s_exp);
  return hipGetLastError();
}

// LayerNorm affine folded into the following Linear (done once per weight
// set): W'[n][k] = W[n][k] g[k], b'[n] = b[n] + sum_k W[n][k] beta[k]
// (accumulated in f64).  One wave per output row.
__global__ void __launch_bounds__(256)
fold_layernorm_kernel(const float* __restrict__ W, const float* __restrict__ bias, const float* __restrict__ lg,
                      const float* __restrict__ lb, float* __restrict__ Wo, float* __restrict__ bo, int N, int K) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  double s = 0.0;
  for (int k = lane; k < K; k += 64) {
    const float w = W[(size_t)n * K + k];
    Wo[(size_t)n * K + k] = w * lg[k];
    s += (double)w * (double)lb[k];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) bo[n] = (float)((bias ? (double)bias[n] : 0.0) + s);
}

hipError_t launch_fold_layernorm(const float* W, const float* bias, const float* ln_g, const float* ln_b,
                                 float* W_out, float* b_out, int N, int K, hipStream_t s) {
  if (N <= 0 || K <= 0 || !W || !ln_g || !ln_b || !W_out || !b_out) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fold_layernorm_kernel, dim3((N + 3) / 4), dim3(256), 0, s, W, bias, ln_g, ln_b, W_out, b_out, N,
                     K);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
#define ND_DISPATCH_FLAGS(KERNEL, ...)                                                          \
  do {                                                                                          \
    const bool ln_ = g.norm, re_ = g.relu, rs_ = g.R != nullptr;                     \
    if (!ln_ && !re_ && !rs_) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, false, false>), grid, block, 0, s, g); \
    if (!ln_ && !re_ && rs_) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, false, true>), grid, block, 0, s, g);   \
    if (!ln_ && re_ && !rs_) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, true, false>), grid, block, 0, s, g);   \
    if (!ln_ && re_ && rs_) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, true, true>), grid, block, 0, s, g);     \
    if (ln_ && !re_ && !rs_) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, false, false>), grid, block, 0, s, g);   \
    if (ln_ && !re_ && rs_) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, false, true>), grid, block, 0, s, g);     \
    if (ln_ && re_ && !rs_) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, true, false>), grid, block, 0, s, g);     \
    if (ln_ && re_ && rs_) hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, true, true>), grid, block, 0, s, g);       \
  } while (0)

// kernel routes taken (include/nanodec.h ND_ROUTE_*), counted at enqueue time
static std::atomic<long long> g_routes[ND_ROUTE_N];
static void count_route(int r) { g_routes[r].fetch_add(1, std::memory_order_relaxed); }

long long gemm_route_count(int r, bool reset) {
  if (r < 0 || r >= ND_ROUTE_N) return 0;
  return reset ? g_routes[r].exchange(0) : g_routes[r].load();
}

template <int BM, int BN, int WM, int WN, int BK = 32>
static hipError_t launch_cfg(GemmArgs& g, hipStream_t s) {
  if (g.K % BK != 0) return hipErrorInvalidValue;
  count_route(BM == 256 ? ND_ROUTE_TILE256 : BM == 128 ? ND_ROUTE_TILE128 : ND_ROUTE_TILE64);  // (32 counts as 64)
  const int nmb = (g.M + BM - 1) / BM;
  g.xcd_map = nmb % 8 == 0;
  dim3 grid((g.N / BN) * nmb), block(WM * WN * 64);
  g.part_n_out = g.N / BN;
  if (g.Wh)
    ND_DISPATCH_FLAGS(gemm_f32_kernel, BM, BN, WM, WN, BK, true);
  else
    ND_DISPATCH_FLAGS(gemm_f32_kernel, BM, BN, WM, WN, BK, false);
  return hipGetLastError();
}

// gemm_f32d_kernel: fp32 weights, row-major A / C, 256 x 256 tiles, at least FD_SLOTS k steps
static bool f32d_eligible(const GemmArgs& g, long t256) {
  return ND_F32D && !g.Wh && !g.p16io && !g.q24 && g.N % 256 == 0 && t256 >= 256 && g.K % FD_BK == 0 &&
         g.K >= FD_SLOTS * FD_BK;
}
static hipError_t launch_f32d(GemmArgs& g, hipStream_t s) {
  count_route(ND_ROUTE_TILE256);
  const int nmb = (g.M + 255) / 256;
  g.xcd_map = nmb % 8 == 0;
  dim3 grid((g.N / 256) * nmb), block(512);
  g.part_n_out = g.N / 256;
  const bool ln = g.norm, re = g.relu, rs = g.R != nullptr;
  if (!ln && !re && !rs) hipLaunchKernelGGL((gemm_f32d_kernel<false, false, false>), grid, block, 0, s, g);
  if (!ln && !re && rs) hipLaunchKernelGGL((gemm_f32d_kernel<false, false, true>), grid, block, 0, s, g);
  if (!ln && re && !rs) hipLaunchKernelGGL((gemm_f32d_kernel<false, true, false>), grid, block, 0, s, g);
  if (!ln && re && rs) hipLaunchKernelGGL((gemm_f32d_kernel<false, true, true>), grid, block, 0, s, g);
  if (ln && !re && !rs) hipLaunchKernelGGL((gemm_f32d_kernel<true, false, false>), grid, block, 0, s, g);
  if (ln && !re && rs) hipLaunchKernelGGL((gemm_f32d_kernel<true, false, true>), grid, block, 0, s, g);
  if (ln && re && !rs) hipLaunchKernelGGL((gemm_f32d_kernel<true, true, false>), grid, block, 0, s, g);
  if (ln && re && rs) hipLaunchKernelGGL((gemm_f32d_kernel<true, true, true>), grid, block, 0, s, g);
  return hipGetLastError();
}

// Row split a (a x 8/a rectangle of XCDs) that minimises the operand blocks
// each XCD's L2 fetches: GY / a row blocks of A plus GX / (8 / a) column
// groups of W (NT column blocks each); 0 when no split divides the grid.
static int p16_xcd_rows(int GX, int GY, int NT) {
  int best = 0;
  long cost = 0;
  for (int a = 1; a <= 8; a *= 2) {
    const int b = 8 / a;
    if (GY % a || GX % b) continue;
    const long c = (long)GY / a + (long)NT * GX / b;
    if (!best || c < cost) best = a, cost = c;
  }
  return best;
}

template <int NT, int KS, int KW>
static hipError_t launch_p16(GemmArgs& g, hipStream_t s) {
  if (g.N % (NT * 16) != 0 || g.K != KS * KW) return hipErrorInvalidValue;
  dim3 grid(g.N / (NT * 16), (g.M + 15) / 16), block(NT * KS * 64);
  count_route(g.K != 256 ? ND_ROUTE_P16_LONGK : NT == 1 ? ND_ROUTE_P16_SMALL : NT == 4 ? ND_ROUTE_P16_N64
                                                                                        : ND_ROUTE_P16_LN128);
  g.xcd_a = p16_xcd_rows((int)grid.x, (int)grid.y, NT);
  g.part_n_out = g.N / 16;
  if (g.Wh)
    ND_DISPATCH_FLAGS(gemm_p16_kernel, NT, KS, KW, true);
  else
    ND_DISPATCH_FLAGS(gemm_p16_kernel, NT, KS, KW, false);
  return hipGetLastError();
}

template <int BMB, int BNB>
static constexpr size_t p16s_lds() {
  return (size_t)(BMB + BNB) * (ND_D / 16) * 64 * sizeof(f32x4);
}

template <int BMB, int BNB>
static hipError_t launch_p16s(GemmArgs& g, hipStream_t s) {
  if (g.K != ND_D || g.N % (BNB * 16) != 0) return hipErrorInvalidValue;
  dim3 grid(g.N / (BNB * 16), (g.M + 16 * BMB - 1) / (16 * BMB)), block(BMB * BNB * 64);
  count_route(BNB == 4 ? ND_ROUTE_P16S_2X4 : ND_ROUTE_P16S_2X2);
  g.part_n_out = g.N / 16;
  const size_t lds = p16s_lds<BMB, BNB>();
  const bool h3_ = g.Wh != nullptr, ln_ = g.norm, re_ = g.relu, rs_ = g.R != nullptr;
#define ND_P16S(H, L, RE, RS)                                        \
  if (h3_ == H && ln_ == L && re_ == RE && rs_ == RS)                \
    hipLaunchKernelGGL((gemm_p16s_kernel<BMB, BNB, H, L, RE, RS>), grid, block, lds, s, g);
#define ND_P16S_H(H)                                                                                   \
  ND_P16S(H, false, false, false) ND_P16S(H, false, false, true) ND_P16S(H, false, true, false)        \
  ND_P16S(H, false, true, true) ND_P16S(H, true, false, false) ND_P16S(H, true, false, true)           \
  ND_P16S(H, true, true, false) ND_P16S(H, true, true, true)
  ND_P16S_H(false) ND_P16S_H(true)
#undef ND_P16S_H
#undef ND_P16S
  return hipGetLastError();
}

template <int BMB, int BNB, bool H>
static hipError_t set_p16s_attr_h() {
  const void* fns[] = {(const void*)gemm_p16s_kernel<BMB, BNB, H, false, false, false>,
                       (const void*)gemm_p16s_kernel<BMB, BNB, H, false, false, true>,
                       (const void*)gemm_p16s_kernel<BMB, BNB, H, false, true, false>,
                       (const void*)gemm_p16s_kernel<BMB, BNB, H, false, true, true>,
                       (const void*)gemm_p16s_kernel<BMB, BNB, H, true, false, false>,
                       (const void*)gemm_p16s_kernel<BMB, BNB, H, true, false, true>,
                       (const void*)gemm_p16s_kernel<BMB, BNB, H, true, true, false>,
                       (const void*)gemm_p16s_kernel<BMB, BNB, H, true, true, true>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p16s_lds<BMB, BNB>());
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int BMB, int BNB>
static hipError_t set_p16s_attr() {
  hipError_t e = set_p16s_attr_h<BMB, BNB, false>();
  return e != hipSuccess ? e : set_p16s_attr_h<BMB, BNB, true>();
}

hipError_t init_gemm_attributes() {
  hipError_t e = set_p16s_attr<2, 4>();
  return e != hipSuccess ? e : set_p16s_attr<2, 2>();
}

static bool gemm_f32_only() {
  static const bool f32only = [] {
    const char* e = getenv("ND_GEMM_F32");  // 1: fp32 MFMA kernels even where a split weight exists
    return e && atoi(e) != 0;
  }();
  return f32only;
}

bool gemm_f32_forced() { return gemm_f32_only(); }

static hipError_t check_args(const GemmArgs& g) {
  if (g.K % 32 != 0 || (g.norm && g.K != ND_D)) return hipErrorInvalidValue;
  if (g.part_in && (g.part_n_in < 1 || g.part_n_in > ND_PART_LD || (ND_D % g.part_n_in) != 0))
    return hipErrorInvalidValue;
  if (g.part_out && g.N != ND_D) return hipErrorInvalidValue;  // statistics of whole 256-wide rows
  return hipSuccess;
}

hipError_t launch_gemm(GemmArgs& g, hipStream_t s) {
  if (g.M <= 0) return hipSuccess;
  if (gemm_f32_only() && g.W) g.Wh = nullptr;
  if (!g.W && !g.Wh) return hipErrorInvalidValue;
  hipError_t e = check_args(g);
  if (e != hipSuccess) return e;
  // the 24-bit context K/V image: the 256 x 256 tiles (a wave holds one row's 256 columns = k or v of a layer)
  if (g.q24) {
    if (g.N % (2 * ND_D) || g.p16io || g.R || g.relu || g.q24_plane < (size_t)g.M * CTXQ_ROW)
      return hipErrorInvalidValue;
    return launch_cfg<256, 256, 2, 4>(g, s);
  }
  // 256x256 tiles, 8 waves of 128x64: half the global->LDS bytes per flop and
  // half the per-tile prologue/epilogue share of the 128x128 tile
  const long t256 = (long)((g.M + 255) / 256) * (g.N / 256);
  if (f32d_eligible(g, t256)) return launch_f32d(g, s);
  if (g.N % 256 == 0 && t256 >= 256) return launch_cfg<256, 256, 2, 4>(g, s);
  const long t128 = (long)((g.M + 127) / 128) * (g.N / 128);
  if (g.N % 128 == 0 && t128 >= 512) return launch_cfg<128, 128, 2, 2>(g, s);
  if (g.N % 64 != 0) return hipErrorInvalidValue;
  // long K on few small tiles (the beam decoder's K = 2048 products at M = 5120):
  // deeper k steps keep more of the next step's operands in flight.  Measured
  // at M = 5120, N = 256, K = 2048: BK 32 / 64 / 128 = 49.1 / 45.8 / 71.7 us
  // (128: 135 KB of LDS, one workgroup per CU); beam B = 1024 168.9 -> 164.7 ms.
  // 32 x 64 tiles there (two waves, twice the workgroups): 76.2 -> 78.2 ms per
  // pooled configs[3] call (round 4), dropped.
  if (g.K >= 1024 && g.K % 64 == 0) return launch_cfg<64, 64, 2, 2, 64>(g, s);
  return launch_cfg<64, 64, 2, 2>(g, s);
}

hipError_t launch_gemm_p16(GemmArgs& g, hipStream_t s) {
  if (g.M <= 0) return hipSuccess;
  if (gemm_f32_only() && g.W) g.Wh = nullptr;
  if (!g.W && !g.Wh) return hipErrorInvalidValue;
  hipError_t e = check_args(g);
  if (e != hipSuccess) return e;
  constexpr int big_min = 2048;  // rows from which the LDS-tiled kernel takes P16 GEMMs
  if (g.M >= big_min && !g.prefer_p16 && !g.c_rm && g.Wh_rm && !gemm_f32_only() && g.N % 64 == 0 &&
      (g.N >= 512 || g.K >= 1024)) {
    // many rows (beam search over large batches): the encoder's LDS-tiled
    // split-fp16 kernel on P16 activations, with the row-major weight image
    // (measured at M = 5120: QKV 25 -> 18 us, FFN1 59 -> 50, FFN2 71 -> 50;
    // the 256 x 256, K = 256 shapes stay on gemm_p16s, 8 -> 10 us there)
    count_route(ND_ROUTE_P16_BIG);  // the tile it runs on is counted too
    GemmArgs r = g;
    r.W = nullptr;
    r.Wh = g.Wh_rm;
    r.wscale = g.wscale_rm;
    r.p16io = 1;
    r.lda = r.ldr = r.ldc = 0;
    e = launch_gemm(r, s);
    g.part_n_out = r.part_n_out;
    return e;
  }
  if (g.N % 16 != 0 || (g.norm && !g.part_in)) return hipErrorInvalidValue;
  if (g.K == 256) {
    // LN consumers share the row statistics across many column blocks
    // LDS-staged tiles when they still give >= 128 workgroups (measured on
    // the decoder shapes: FFN1 / query-projection 7.2 -> 5.7 us, QKV 5.3 -> 4.3 us at M = 256)
    const long mb32 = (g.M + 31) / 32;
    if (g.N % 64 == 0 && (long)(g.N / 64) * mb32 >= 128) return launch_p16s<2, 4>(g, s);
    if (g.N % 32 == 0 && (long)(g.N / 32) * mb32 >= 128) return launch_p16s<2, 2>(g, s);
    if (g.norm && g.N % 128 == 0 && (long)(g.N / 128) * ((g.M + 15) / 16) >= 128) return launch_p16<8, 1, 256>(g, s);
    if (g.N % 64 == 0 && (long)(g.N / 64) * ((g.M + 15) / 16) >= 128) return launch_p16<4, 2, 128>(g, s);
    return launch_p16<1, 4, 64>(g, s);
  }
  // split over workgroups (gemm_p16k_kernel): 32 x 32 tiles x K / 512 slices, when the tiles x slices fill
  // the chip at least half (M from 128 rows) and the context gave the slab / tickets for that many tiles
  // (exact fp32: the fp32 P16 weight, same tiles and slices)
  if (!g.skip && !g.c_rm && !g.relu && (g.K == 2048 || g.K == 1024) && g.N % 32 == 0 && g.sk_slab && g.sk_cnt) {
    const int tiles = ((g.M + 31) / 32) * (g.N / 32), S = g.K / PK_SLICE;
    if (g.M > 128 && tiles <= g.sk_tiles) {
      count_route(ND_ROUTE_P16_SPLITK);
      g.part_n_out = g.N / 16;
      const dim3 grid(tiles * S), block(PK_NW * 64);
      if (g.Wh) {
        if (g.R)
          hipLaunchKernelGGL((gemm_p16k_kernel<true, true>), grid, block, 0, s, g);
        else
          hipLaunchKernelGGL((gemm_p16k_kernel<true, false>), grid, block, 0, s, g);
      } else if (g.R) {
        hipLaunchKernelGGL((gemm_p16k_kernel<false, true>), grid, block, 0, s, g);
      } else {
        hipLaunchKernelGGL((gemm_p16k_kernel<false, false>), grid, block, 0, s, g);
      }
      return hipGetLastError();
    }
  }
  // K = 2048 on 8 K-slice waves of 256 (16 waves of 128: pooled greedy 16.30 -> 16.63 ms, round 4, dropped)
  if (g.K == 2048) return launch_p16<1, 8, 256>(g, s);
  if (g.K == 1024) return launch_p16<1, 8, 128>(g, s);
  if (g.K == 512) return launch_p16<1, 8, 64>(g, s);
  return hipErrorInvalidValue;
}

}  // namespace nd
