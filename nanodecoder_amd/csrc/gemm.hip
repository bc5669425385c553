// fp32 MFMA GEMM for gfx950 with fused LayerNorm prologue and
// bias / ReLU / residual epilogue.
//
// Replaces the reference's nn.Linear addmm calls and the LayerNorm that
// precedes them (onmt/modules/multi_headed_attn.py:59-67,155-157,179;
// onmt/modules/position_ffn.py:20-22,38-40; encoder/transformer.py:50;
// decoder/transformer.py:75,88).  The reference computes in fp32, and gfx950
// has no xf32 MFMA, so the product runs on v_mfma_f32_32x32x2_f32 (exact f32
// FMA chains, 64 FLOP/clk/SIMD = the fp32 peak).
//
//   C[M,N] = epi( pro(A)[M,K] . W[N,K]^T + bias[N] )
//   pro(A) = LN(A) = (A - mean) * rstd * g + b over K      (when LN)
//   epi(v) = relu(v) (RELU); v + R[M,N] (RESID)
//
// Tiling: BM x BN x 32, WM x WN waves each owning (BM/WM) x (BN/WN) as
// 32x32 MFMA blocks.  A and W tiles are staged global -> registers -> LDS
// (double-buffered, one barrier per K step); row stride 36 floats makes the
// per-lane ds_read_b128 fragment loads bank-conflict free.  Inside an 8-wide
// k block, lane half h reads k = 4h..4h+3 with one ds_read_b128 and feeds them
// to 4 consecutive MFMAs, so MFMA step i sums over k = {i, 4+i} — a fixed
// permutation of the K order that A and W share.
#include "common.hpp"
#include "kernels.hpp"

namespace nd {

template <int BM, int BN, int WM, int WN, bool LN, bool RELU, bool RESID>
__global__ void __launch_bounds__(WM* WN * 64)
gemm_f32_kernel(const float* __restrict__ A, int lda, const float* __restrict__ W, int ldw,
                const float* __restrict__ bias, const float* __restrict__ R, int ldr, float* __restrict__ C,
                int ldc, const float* __restrict__ ln_g, const float* __restrict__ ln_b, int M, int N, int K) {
  constexpr int NT = WM * WN * 64;
  constexpr int BK = 32, LDK = BK + 4;
  constexpr int FM = BM / WM / 32, FN = BN / WN / 32;
  constexpr int A4 = BM * BK / 4 / NT;
  constexpr int W4 = BN * BK / 4 / NT;
  static_assert(A4 >= 1 && W4 >= 1, "tile too small for the thread count");
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) float Ws[2][BN * LDK];
  __shared__ float s_mu[LN ? BM : 1], s_rs[LN ? BM : 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;

  if constexpr (LN) {
    // two-pass row statistics, one wave per row, K == 256 (host-checked);
    // 8 rows' loads are issued together so their L2 latencies overlap
    constexpr int NW = NT / 64, RPW = BM / NW, G = RPW < 8 ? RPW : 8;
    for (int r0 = 0; r0 < RPW; r0 += G) {
      f32x4 v[G];
#pragma unroll
      for (int i = 0; i < G; ++i) v[i] = ld4(A + (size_t)min(m0 + wave + (r0 + i) * NW, M - 1) * lda + lane * 4);
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int r = wave + (r0 + i) * NW;
        const float mu = wave_sum(v[i].x + v[i].y + v[i].z + v[i].w) * (1.0f / 256.0f);
        const f32x4 d = v[i] - mu;
        const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / 256.0f);
        if (lane == 0) {
          s_mu[r] = mu;
          s_rs[r] = 1.0f / sqrtf(var + ND_LN_EPS);
        }
      }
    }
    __syncthreads();
  }

  f32x4 ra[A4], rw[W4];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int f = tid + i * NT, row = f >> 3, c = (f & 7) * 4;
      const int gr = m0 + row;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (gr < M) {
        v = ld4(A + (size_t)gr * lda + k0 + c);
        if constexpr (LN) {
          const f32x4 g = ld4(ln_g + k0 + c), b = ld4(ln_b + k0 + c);
          v = (v - s_mu[row]) * s_rs[row] * g + b;
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < W4; ++i) {
      const int f = tid + i * NT, row = f >> 3, c = (f & 7) * 4;
      rw[i] = ld4(W + (size_t)(n0 + row) * ldw + k0 + c);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int f = tid + i * NT, row = f >> 3, c = (f & 7) * 4;
      st4(&As[buf][row * LDK + c], ra[i]);
    }
#pragma unroll
    for (int i = 0; i < W4; ++i) {
      const int f = tid + i * NT, row = f >> 3, c = (f & 7) * 4;
      st4(&Ws[buf][row * LDK + c], rw[i]);
    }
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int KT = K / BK;

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) load_tile((kt + 1) * BK);
#pragma unroll
    for (int kb = 0; kb < BK / 8; ++kb) {
      f32x4 af[FM], bf[FN];
#pragma unroll
      for (int a = 0; a < FM; ++a) af[a] = ld4(&As[buf][(wm * FM * 32 + a * 32 + lr) * LDK + kb * 8 + lh * 4]);
#pragma unroll
      for (int b = 0; b < FN; ++b) bf[b] = ld4(&Ws[buf][(wn * FN * 32 + b * 32 + lr) * LDK + kb * 8 + lh * 4]);
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

#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) {
      const int col = n0 + wn * FN * 32 + b * 32 + lr;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * FM * 32 + a * 32 + mfma32_row(r, lane);
        if (row < M) {
          float v = acc[a][b][r] + bv;
          if constexpr (RELU) v = fmaxf(v, 0.f);
          if constexpr (RESID) v += R[(size_t)row * ldr + col];
          C[(size_t)row * ldc + col] = v;
        }
      }
    }
}

// Small-M variant (decoder steps: M = rows of the batch, 256 for greedy).
// One workgroup = one 16x16 output tile on v_mfma_f32_16x16x4_f32; its WAVES
// waves split K.  Each wave issues ALL of its A/W fragment loads up front
// (straight from L2 into registers: every fragment is used by exactly one
// wave, so LDS staging would only add latency), runs two interleaved
// accumulator chains (40-cycle dependent latency vs 32-cycle issue), and the
// partial tiles are summed through LDS before the epilogue.  A 256-row
// decoder GEMM becomes (M/16)*(N/16) >= 256 workgroups, filling every CU.
//
// 16x16x4 fragments: lane l supplies A[l&15][k = l>>4] and B[k = l>>4][l&15];
// lane l holds D[(l>>4)*4 + r][l&15].  With one float4 per lane covering
// k0 + 4*(l>>4) + {0..3}, MFMA step s sums k in {k0+s, k0+4+s, k0+8+s, k0+12+s}.
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int WAVES, int KW, bool LN, bool RELU, bool RESID>
__global__ void __launch_bounds__(WAVES * 64)
gemm_f32_small_kernel(const float* __restrict__ A, int lda, const float* __restrict__ W, int ldw,
                      const float* __restrict__ bias, const float* __restrict__ R, int ldr, float* __restrict__ C,
                      int ldc, const float* __restrict__ ln_g, const float* __restrict__ ln_b, int M, int N) {
  // KW = K per wave (K = WAVES * KW); KW % 16 == 0
  constexpr int NF = KW / 16;  // float4 fragments per lane per operand
  __shared__ float red[WAVES][256];
  __shared__ float s_mu[16], s_rs[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, m0 = blockIdx.y * 16;
  const int li = lane & 15, lq = lane >> 4;
  const int row = m0 + li;
  const bool row_ok = row < M;
  const int kb = wave * KW + 4 * lq;
  const float* arow = A + (size_t)(row_ok ? row : 0) * lda + kb;
  const float* wrow = W + (size_t)(n0 + li) * ldw + kb;
  f32x4 a[NF], w[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    a[f] = ld4(arow + 16 * f);
    w[f] = ld4(wrow + 16 * f);
  }
  if constexpr (LN) {
    // 16 rows' statistics: every wave loads its rows at once, then reduces
    constexpr int RPW = (16 + WAVES - 1) / WAVES;
    f32x4 v[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = wave + i * WAVES;
      v[i] = ld4(A + (size_t)min(m0 + min(r, 15), M - 1) * lda + lane * 4);
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int r = wave + i * WAVES;
      const float mu = wave_sum(v[i].x + v[i].y + v[i].z + v[i].w) * (1.0f / 256.0f);
      const f32x4 d = v[i] - mu;
      const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / 256.0f);
      if (lane == 0 && r < 16) {
        s_mu[r] = mu;
        s_rs[r] = 1.0f / sqrtf(var + ND_LN_EPS);
      }
    }
    __syncthreads();
    const float mu = s_mu[li], rs = s_rs[li];
#pragma unroll
    for (int f = 0; f < NF; ++f) a[f] = (a[f] - mu) * rs * ld4(ln_g + kb + 16 * f) + ld4(ln_b + kb + 16 * f);
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    acc0 = mfma16(a[f][0], w[f][0], acc0);
    acc1 = mfma16(a[f][1], w[f][1], acc1);
    acc0 = mfma16(a[f][2], w[f][2], acc0);
    acc1 = mfma16(a[f][3], w[f][3], acc1);
  }
  const f32x4 acc = acc0 + acc1;
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][r * 64 + lane] = acc[r];
  __syncthreads();
  if (tid < 256) {
    float v = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < WAVES; ++w2) v += red[w2][tid];
    const int r = tid >> 6, ln = tid & 63;
    const int orow = m0 + (ln >> 4) * 4 + r, col = n0 + (ln & 15);
    if (orow < M) {
      v += bias ? bias[col] : 0.f;
      if constexpr (RELU) v = fmaxf(v, 0.f);
      if constexpr (RESID) v += R[(size_t)orow * ldr + col];
      C[(size_t)orow * ldc + col] = v;
    }
  }
}

template <int WAVES, int KW>
static hipError_t launch_small(const GemmArgs& g, hipStream_t s) {
  dim3 grid(g.N / 16, (g.M + 15) / 16), block(WAVES * 64);
  const bool ln = g.ln_g != nullptr, relu = g.relu, res = g.R != nullptr;
#define ND_SM_CASE(L, Rl, Rs)                                                                                    \
  if (ln == L && relu == Rl && res == Rs) {                                                                      \
    hipLaunchKernelGGL((gemm_f32_small_kernel<WAVES, KW, L, Rl, Rs>), grid, block, 0, s, g.A, g.lda, g.W, g.ldw, \
                       g.bias, g.R, g.ldr, g.C, g.ldc, g.ln_g, g.ln_b, g.M, g.N);                                \
    return hipGetLastError();                                                                                    \
  }
  ND_SM_CASE(false, false, false)
  ND_SM_CASE(false, false, true)
  ND_SM_CASE(false, true, false)
  ND_SM_CASE(false, true, true)
  ND_SM_CASE(true, false, false)
  ND_SM_CASE(true, false, true)
  ND_SM_CASE(true, true, false)
  ND_SM_CASE(true, true, true)
#undef ND_SM_CASE
  return hipErrorInvalidValue;
}

template <int BM, int BN, int WM, int WN>
static hipError_t launch_cfg(const GemmArgs& g, hipStream_t s) {
  dim3 grid(g.N / BN, (g.M + BM - 1) / BM), block(WM * WN * 64);
  const bool ln = g.ln_g != nullptr, relu = g.relu, res = g.R != nullptr;
#define ND_GEMM_CASE(L, Rl, Rs)                                                                              \
  if (ln == L && relu == Rl && res == Rs) {                                                                  \
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, L, Rl, Rs>), grid, block, 0, s, g.A, g.lda, g.W, g.ldw, \
                       g.bias, g.R, g.ldr, g.C, g.ldc, g.ln_g, g.ln_b, g.M, g.N, g.K);                       \
    return hipGetLastError();                                                                                \
  }
  ND_GEMM_CASE(false, false, false)
  ND_GEMM_CASE(false, false, true)
  ND_GEMM_CASE(false, true, false)
  ND_GEMM_CASE(false, true, true)
  ND_GEMM_CASE(true, false, false)
  ND_GEMM_CASE(true, false, true)
  ND_GEMM_CASE(true, true, false)
  ND_GEMM_CASE(true, true, true)
#undef ND_GEMM_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_gemm(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0) return hipSuccess;
  if (g.K % 32 != 0 || (g.ln_g && g.K != ND_D)) return hipErrorInvalidValue;
  const long t128 = (long)((g.M + 127) / 128) * (g.N / 128);
  const long t64 = (long)((g.M + 63) / 64) * (g.N / 64);
  if (g.N % 128 == 0 && t128 >= 512) return launch_cfg<128, 128, 2, 2>(g, s);
  if (g.N % 64 == 0 && t64 >= 256) return launch_cfg<64, 64, 2, 2>(g, s);
  if (g.N % 16 != 0) return hipErrorInvalidValue;
  if (g.K == 256) return launch_small<4, 64>(g, s);
  if (g.K == 2048) return launch_small<8, 256>(g, s);
  if (g.K % 64 == 0 && g.K <= 1024) {
    if (g.K == 64) return launch_small<1, 64>(g, s);
    if (g.K == 128) return launch_small<2, 64>(g, s);
    if (g.K == 512) return launch_small<8, 64>(g, s);
    if (g.K == 1024) return launch_small<8, 128>(g, s);
  }
  return launch_cfg<64, 64, 2, 2>(g, s);
}

}  // namespace nd
