// NanoEncoder BiLSTM recurrence on gfx950 (encoder/nano_encoder.py:79-124,
// nn.LSTM through onmt/utils/rnn_factory.py:8-17, packed sequences).
//
// One workgroup = NS sequences (16, 8 or 4; default 4, ND_LSTM_SEQ) x one
// direction, for ALL time steps: the recurrence never leaves the CU, so a
// step costs one 16x512x128 product + one LDS exchange of h instead of a
// kernel launch.  W_hh^T (512 x 128) is held in REGISTERS across the waves:
// with 16 waves, wave w owns the four gates (i, f, g, o) of units
// 8w .. 8w + 7 as two 16-column tiles (i | f, g | o) of MFMA B operands (8
// waves: 16 units, four tiles), split-fp16 hi/lo on v_mfma_f32_16x16x32_f16
// (or fp32 on v_mfma_f32_16x16x4_f32 with ND_LSTM_F32=1, NS = 16).  h_{t-1}
// is the A operand, read from LDS (rows NS..15 zero).  A lane finds the other
// half of its unit's gates in lane ^ 8 (one DPP move); with NS < 16 the gate
// sums then fan out to the lanes of the padding rows (permlane swaps), and
// each lane applies the PyTorch cell (i, f, g, o order) to 1 (NS < 16) or 2
// (sequence, unit) pairs and writes h to LDS: one workgroup barrier per step.

// Packing semantics (pack_padded_sequence / pad_packed_sequence):
// sequence b only processes its valid steps; the reverse direction starts
// at t = len_b - 1.  Outputs at t >= len_b are left as the caller zeroed them.
//
// The input projection x_t W_ih^T + b_ih + b_hh is precomputed for all t by a
// GEMM (layers 1, 2) or computed in-kernel from the scalar sample (layer 0,
// input_size 1).  When `bn_scale` is set the kernel writes the eval-mode
// BatchNorm of h (the next layer's input, nano_encoder.py:108); otherwise the
// raw h (the last layer: memory = W . h, its BatchNorm is unused, :113-115).
#include "common.hpp"
#include "kernels.hpp"

#include <cstdlib>
#include <type_traits>

namespace nd {

__device__ __forceinline__ f32x4 mfma16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
// the cell's activations on the hardware exp (v_exp_f32) and reciprocal
// (v_rcp_f32, 1 ulp; __frcp_rn lowers to the ~10-instruction IEEE division
// sequence, and five of them sat on every step's dependent chain); a few ulp
// from the libm forms; ND_LSTM_LIBM=1 keeps expf / tanhf
__device__ __forceinline__ float sigm_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) {
  const float t = __expf(-2.0f * fabsf(x));
  return copysignf((1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t), x);
}
template <bool FAST>
__device__ __forceinline__ float act_sig(float x) { return FAST ? sigm_fast(x) : sigm(x); }
template <bool FAST>
__device__ __forceinline__ float act_tanh(float x) { return FAST ? tanh_fast(x) : tanhf(x); }

typedef _Float16 lh8 __attribute__((ext_vector_type(8)));
// split-fp16 (gemm.hip): hi = fp16(x), lo = fp16(x - hi), 22 significant bits
__device__ __forceinline__ void lsplit8(const float (&x)[8], lh8& hi, lh8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = (_Float16)x[j];
    lo[j] = (_Float16)(x[j] - (float)hi[j]);
  }
}
__device__ __forceinline__ f32x4 mfma16x32h(lh8 a, lh8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
#define LSTM_HSCALE 1024.0f  // h (|h| < 1) enters the split at 2^10: lo stays clear of the fp16 subnormals

#define LSTM_H 128
#define LSTM_G 512
#define LSTM_HS_LD (LSTM_H + 4)
#define LSTM_HP_LD (LSTM_H + 8)  // halves
#define LSTM_DPP_ROR8 0x128  // DPP row_ror:8: lane ^ 8 within a 16-lane row

// H3: the recurrent product on v_mfma_f32_16x16x32_f16 in the split-fp16
// form (hi*lo + lo*hi + hi*hi), W_hh scaled by a power of two per direction
// (max |W| in [2^13, 2^14)) and h by 2^10; otherwise fp32 16x16x4 MFMAs.
// NS < 16 (H3 only): fewer sequences per workgroup, more workgroups.  MFMA
// rows NS..15 are zero padding, so only the lanes of the first NS/4 16-lane
// rows hold gate sums; they hand them to the other rows by
// v_permlane16/32_swap, and every lane runs ONE cell per step instead of two.
//  NS = 8: 16 waves x 8 units; a lower lane keeps its row 2 (li / 8) and
//          hands row 2 (li / 8) + 1 to lane + 32.
//  NS = 4: 8 waves x 16 units (four tiles: i|f, g|o of units 0-7, then 8-15);
//          row-0 lane li holds all 8 (unit group, sequence) combinations of
//          unit li % 8 and sends combination k to 16-lane row k >> 1.
template <bool LAYER0, bool H3, bool FAST = false, int NS = 16>
__global__ void __launch_bounds__(NS == 4 ? 512 : 1024)
lstm_dir_kernel(const float* __restrict__ xp,      // [B*T, 1024] input projections (fwd | bwd), !LAYER0
                const float* __restrict__ signal,  // [B, T] (LAYER0)
                const float* __restrict__ wih0,    // [2][512] (LAYER0, input_size 1)
                const float* __restrict__ bsum,    // [2][512] b_ih + b_hh (LAYER0)
                const float* __restrict__ whh,     // [2][512][128]
                const int* __restrict__ len, int B, int T, float* __restrict__ out,  // [B*T, 256]
                const float* __restrict__ bn_scale, const float* __restrict__ bn_shift) {
  __shared__ __attribute__((aligned(16))) float hs[H3 ? 1 : 2][16 * LSTM_HS_LD];
  // H3: h_{t-1} 2^10 as split-fp16 planes, written once by the lane that
  // produced it (the 16 waves read it without re-splitting); row stride 136
  // halves = 68 banks, so the 16 rows a ds_read_b128 group reads are disjoint
  __shared__ __attribute__((aligned(16))) _Float16 hp[H3 ? 2 : 1][2][16 * LSTM_HP_LD];
  __shared__ int s_len[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int dir = blockIdx.y;
  static_assert(H3 || NS == 16, "NS < 16 is a split-fp16 mapping");
  static_assert(NS == 16 || NS == 8 || NS == 4, "sequences per workgroup");
  constexpr int NWAVE = NS == 4 ? 8 : 16, NTH = NWAVE * 64;
  constexpr int UPW = LSTM_H / NWAVE, NT = UPW / 4;  // units and 16-column tiles per wave
  constexpr int NP = NS == 16 ? 2 : 1;               // cells per lane
  const int b0 = blockIdx.x * NS;
  const int li = lane & 15, lq = lane >> 4;

  // W_hh^T fragments for this wave's two 16-column tiles, k order matching
  // the A fragment: fp32, block kb, step s <-> k = 16*kb + 4*lq + s; H3,
  // block kb (32 k), slot j <-> k = 32*kb + 8*lq + j
  float wr[2][32];
  lh8 whi[NT][4], wlo[NT][4];
  float unscale = 1.f;
  {
    const float* W = whh + (size_t)dir * LSTM_G * LSTM_H;
    float wsc = 1.f;
    if constexpr (H3) {
      __shared__ float s_max[16];
      float m = 0.f;
      for (int e = tid; e < LSTM_G * LSTM_H; e += NTH) m = fmaxf(m, fabsf(W[e]));
      m = wave_max(m);
      if (lane == 0) s_max[wave] = m;
      __syncthreads();
      m = 0.f;
#pragma unroll
      for (int w = 0; w < NWAVE; ++w) m = fmaxf(m, s_max[w]);
      int ex = 0;
      frexpf(m, &ex);  // m = f * 2^ex, f in [0.5, 1)
      const int sh = m > 0.f ? 14 - ex : 0;
      wsc = ldexpf(1.f, sh);
      unscale = ldexpf(1.f, -sh) / LSTM_HSCALE;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      // gate 2 (t % 2) + li / 8 of unit UPW w + 8 (t / 2) + li % 8
      const int n = (2 * (t & 1) + (li >> 3)) * LSTM_H + wave * UPW + 8 * (t >> 1) + (li & 7);
      if constexpr (H3) {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const f32x4 v0 = ld4(W + (size_t)n * LSTM_H + kb * 32 + 8 * lq);
          const f32x4 v1 = ld4(W + (size_t)n * LSTM_H + kb * 32 + 8 * lq + 4);
          const float x[8] = {v0.x * wsc, v0.y * wsc, v0.z * wsc, v0.w * wsc,
                              v1.x * wsc, v1.y * wsc, v1.z * wsc, v1.w * wsc};
          lsplit8(x, whi[t][kb], wlo[t][kb]);
        }
      } else {
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
          const f32x4 v = ld4(W + (size_t)n * LSTM_H + kb * 16 + 4 * lq);
          wr[t][kb * 4 + 0] = v.x;
          wr[t][kb * 4 + 1] = v.y;
          wr[t][kb * 4 + 2] = v.z;
          wr[t][kb * 4 + 3] = v.w;
        }
      }
    }
  }
  if (tid < 16) s_len[tid] = (tid < NS && b0 + tid < B) ? len[b0 + tid] : 0;
  // eval BatchNorm of the next layer's input, per unit, kept in LDS (registers
  // are the limit here); filled before the barrier below, which publishes it
  // to every wave before the first step's output
  __shared__ float s_bn[2][LSTM_H];
  if (bn_scale && tid < LSTM_H) {
    s_bn[0][tid] = bn_scale[dir * LSTM_H + tid];
    s_bn[1][tid] = bn_shift[dir * LSTM_H + tid];
  }
  if constexpr (H3) {
    for (int e = tid; e < 16 * LSTM_HP_LD; e += NTH) hp[0][0][e] = hp[0][1][e] = (_Float16)0.f;
  } else {
    for (int e = tid; e < 16 * LSTM_HS_LD; e += NTH) hs[0][e] = 0.f;
  }
  __syncthreads();
  int maxlen = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) maxlen = max(maxlen, s_len[q]);

  // cell ownership: the lane's accumulator rows 2 (li / 8) + u (sequences
  // 4 lq + 2 (li / 8) + u) of unit 8 wave + li % 8, whose four gates this wave
  // produced (i | f in tile 0, g | o in tile 1; the partner lane li ^ 8 holds
  // the other half of each), so the cell needs no exchange through LDS
  int pseq[2], punit[2];
  float c[2] = {0.f, 0.f};
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    if constexpr (NS == 16) {
      pseq[u] = 4 * lq + 2 * (li >> 3) + u;
      punit[u] = wave * 8 + (li & 7);
    } else if constexpr (NS == 8) {  // lane x < 32 owns its row pair's first row, lane x + 32 the second
      pseq[u] = 4 * ((lane & 31) >> 4) + 2 * (li >> 3) + (lane >> 5);
      punit[u] = wave * 8 + (li & 7);
    } else {  // 16-lane row k >> 1 = lq: combination k = 2 lq + li / 8
      pseq[u] = 2 * (lq & 1) + (li >> 3);
      punit[u] = wave * UPW + 8 * (lq >> 1) + (li & 7);
    }
  }
  float w0[2][4], bb[2][4];
  if constexpr (LAYER0) {
#pragma unroll
    for (int u = 0; u < NP; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        w0[u][g] = wih0[dir * LSTM_G + g * LSTM_H + punit[u]];
        bb[u][g] = bsum[dir * LSTM_G + g * LSTM_H + punit[u]];
      }
  }
  // lengths in registers (the step loop's raw barrier clobbers LDS-held values)
  int mylen[2];
#pragma unroll
  for (int u = 0; u < NP; ++u) mylen[u] = s_len[pseq[u]];
  // Global traffic inside the step loop is straight-line: every x load and
  // every h store is issued unconditionally (clamped rows; past a sequence's
  // end the lane re-writes 0 into a padding row), so the compiler's vmcnt
  // waits count exactly and a step waits only for its own x, which was
  // loaded PD steps earlier.  A branch around any of them made it wait
  // vmcnt(0), i.e. for this step's h store and the prefetch, every step.
  // Workgroups with fewer than NS live sequences run a second copy of the
  // loop with the guarded forms (FULL = false).
  auto pos_of = [&](int u, int step) { return dir == 0 ? step : mylen[u] - 1 - step; };
  auto load_x = [&](int step, float (&x)[2][4]) {
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int q = pseq[u];
      const bool act = step < mylen[u];
      const int pos = act ? pos_of(u, step) : 0;
      const size_t row = (size_t)min(b0 + q, B - 1) * T + pos;
      if constexpr (LAYER0) {
        x[u][0] = signal[row];  // the sample; its projection is formed at use
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) x[u][g] = xp[row * 1024 + dir * LSTM_G + g * LSTM_H + punit[u]];
      }
    }
  };

  // PD named x buffers (the step loop unrolled by PD): NS = 16 has no
  // registers to spare and keeps one
  constexpr int PD = NS == 16 ? 1 : 2;
  float xa[2][4], xb[2][4];
  load_x(0, xa);
  if (PD > 1) load_x(1, xb);
  auto step_body = [&](auto full_c, const int step, float (&xn)[2][4]) {
    constexpr bool FULL = decltype(full_c)::value;
    const int cur = step & 1;
    float xc[2][4];
#pragma unroll
    for (int u = 0; u < NP; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) xc[u][g] = LAYER0 ? xn[u][0] * w0[u][g] + bb[u][g] : xn[u][g];

    // gates = h_{t-1} W_hh^T on MFMA
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (H3) {
      const _Float16* hhi = &hp[cur][0][li * LSTM_HP_LD + 8 * lq];
      const _Float16* hlo = &hp[cur][1][li * LSTM_HP_LD + 8 * lq];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const lh8 ah = *reinterpret_cast<const lh8*>(hhi + kb * 32);
        const lh8 al = *reinterpret_cast<const lh8*>(hlo + kb * 32);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x32h(ah, wlo[t][kb], acc[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x32h(al, whi[t][kb], acc[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x32h(ah, whi[t][kb], acc[t]);
      }
      // (the 2^-s / 2^10 unscale is applied to the four gate sums a lane keeps,
      // in the cell: 4 FMAs instead of 4 NT multiplies here)
    } else {
      const float* hrow = &hs[cur][li * LSTM_HS_LD + 4 * lq];
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        const f32x4 a = ld4(hrow + kb * 16);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc[0] = mfma16x4(a[s], wr[0][kb * 4 + s], acc[0]);
          acc[1] = mfma16x4(a[s], wr[1][kb * 4 + s], acc[1]);
        }
      }
    }
    // the partner lane's half of each tile (row_ror:8 within 16 lanes = lane ^ 8)
    f32x4 pt[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) pt[t][r] = dpp_mov<LSTM_DPP_ROR8>(acc[t][r]);
    const bool lo = li < 8;
    // gate sums (i, f, g, o) of accumulator row r of this lane's unit in unit group ug
    auto gates_g = [&](int ug, int r, float (&z)[4]) {
      z[0] = lo ? acc[2 * ug][r] : pt[2 * ug][r];
      z[1] = lo ? pt[2 * ug][r] : acc[2 * ug][r];
      z[2] = lo ? acc[2 * ug + 1][r] : pt[2 * ug + 1][r];
      z[3] = lo ? pt[2 * ug + 1][r] : acc[2 * ug + 1][r];
    };
    auto gates = [&](int r, float (&z)[4]) { gates_g(0, r, z); };
    float zg[NP][4];
    if constexpr (NS == 4) {
      // row-0 lane li: v_q = the gate sums 16-lane row q will own
      float v0[4], v1[4], v2[4], v3[4], t_[4];
      gates_g(0, 0, v0);  // per target row q: (ug = q >> 1, r = 2 (q & 1) + li / 8)
      gates_g(0, 1, t_);
#pragma unroll
      for (int g = 0; g < 4; ++g) v0[g] = lo ? v0[g] : t_[g];
      gates_g(0, 2, v1);
      gates_g(0, 3, t_);
#pragma unroll
      for (int g = 0; g < 4; ++g) v1[g] = lo ? v1[g] : t_[g];
      gates_g(1, 0, v2);
      gates_g(1, 1, t_);
#pragma unroll
      for (int g = 0; g < 4; ++g) v2[g] = lo ? v2[g] : t_[g];
      gates_g(1, 2, v3);
      gates_g(1, 3, t_);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        v3[g] = lo ? v3[g] : t_[g];
        float a1, b1, a3, b3, a23, b23;
        lane_swap<false>(v1[g], a1, b1);  // odd rows: the value of the row below
        lane_swap<false>(v3[g], a3, b3);
        lane_swap<true>(lq == 0 ? v2[g] : a3, a23, b23);  // upper half: rows 0, 1 -> 2, 3
        zg[0][g] = lq == 0 ? v0[g] : lq == 1 ? a1 : a23;
      }
    } else if constexpr (NS == 8) {
      // lower lane: row 2 (li / 8) itself, row 2 (li / 8) + 1 to lane + 32
      float za[4], zb[4];
      gates(0, za);
      gates(2, zb);
      float zc[4], zd[4];
      gates(1, zc);
      gates(3, zd);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float own = lo ? za[g] : zb[g], send = lo ? zc[g] : zd[g];
        float a_, b_;
        lane_swap<true>(send, a_, b_);  // upper lanes: a_ = the lower partner's send
        zg[0][g] = (lane >> 5) ? a_ : own;
      }
    } else {
#pragma unroll
      for (int u = 0; u < NP; ++u) gates(2 * (li >> 3) + u, zg[u]);
    }
    // PyTorch LSTM cell (gates i, f, g, o)
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int q = pseq[u], j = punit[u];
      const bool act = step < mylen[u];
      float h = 0.f;
      if (act) {
        const float ig = act_sig<FAST>(fmaf(zg[u][0], unscale, xc[u][0]));
        const float fg = act_sig<FAST>(fmaf(zg[u][1], unscale, xc[u][1]));
        const float gg = act_tanh<FAST>(fmaf(zg[u][2], unscale, xc[u][2]));
        const float og = act_sig<FAST>(fmaf(zg[u][3], unscale, xc[u][3]));
        c[u] = fg * c[u] + ig * gg;
        h = og * act_tanh<FAST>(c[u]);
        if constexpr (H3) {
          // the split the consumers used to form from the fp32 h (lsplit8 of h 2^10)
          const float x = h * LSTM_HSCALE;
          const _Float16 hi = (_Float16)x;
          hp[cur ^ 1][0][q * LSTM_HP_LD + j] = hi;
          hp[cur ^ 1][1][q * LSTM_HP_LD + j] = (_Float16)(x - (float)hi);
        }
      } else if constexpr (H3) {  // past the sequence's end: h carries over
        hp[cur ^ 1][0][q * LSTM_HP_LD + j] = hp[cur][0][q * LSTM_HP_LD + j];
        hp[cur ^ 1][1][q * LSTM_HP_LD + j] = hp[cur][1][q * LSTM_HP_LD + j];
      } else {
        h = hs[cur][q * LSTM_HS_LD + j];
      }
      if constexpr (!H3) hs[cur ^ 1][q * LSTM_HS_LD + j] = h;
      const float ov = act ? (bn_scale ? h * s_bn[0][j] + s_bn[1][j] : h) : 0.f;
      if constexpr (FULL) {  // unconditional: past the end, 0 into padding row `step`
        const size_t row = (size_t)(b0 + q) * T + (act ? pos_of(u, step) : step);
        out[row * 2 * LSTM_H + dir * LSTM_H + j] = ov;
      } else if (act) {
        const size_t row = (size_t)(b0 + q) * T + pos_of(u, step);
        out[row * 2 * LSTM_H + dir * LSTM_H + j] = ov;
      }
    }
    load_x(step + PD, xn);  // this buffer's next use: step + PD (past maxlen: a clamped, unused load)
    // publish h_t (LDS) to every wave: a raw barrier behind an LDS-only wait
    // (__syncthreads() would also wait vmcnt(0): the h stores and the x
    // prefetch, one global round trip every step)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  auto run = [&](auto full_c) {
    if constexpr (PD == 1) {
      for (int step = 0; step < maxlen; ++step) step_body(full_c, step, xa);
    } else {
      for (int step = 0; step < maxlen; step += 2) {
        step_body(full_c, step, xa);
        if (step + 1 < maxlen) step_body(full_c, step + 1, xb);
      }
    }
  };
  if constexpr (NS == 16) {  // (registers: one guarded copy of the loop)
    run(std::false_type{});
  } else {
    if (b0 + NS <= B)
      run(std::true_type{});
    else
      run(std::false_type{});
  }
}

hipError_t launch_lstm_layer(const float* xp, const float* signal, const float* wih0, const float* bsum,
                             const float* whh, const int* len, int B, int T, float* out, const float* bn_scale,
                             const float* bn_shift, bool layer0, hipStream_t s, bool exact) {
  static const bool f32_env = [] {
    const char* e = getenv("ND_LSTM_F32");  // 1: fp32 MFMAs for the recurrence
    const char* g = getenv("ND_GEMM_F32");
    return (e && atoi(e) != 0) || (g && atoi(g) != 0);
  }();
  const bool f32 = f32_env || exact;
  // split-fp16: 4 sequences per workgroup (measured: 0.95 ms per layer at 4, 1.04 at 8, 1.52 at 16), the
  // cell's sigmoid / tanh on the hardware exp and reciprocal; fp32 MFMAs: 16 sequences per workgroup
  const int ns = f32 ? 16 : 4;
  dim3 grid((B + ns - 1) / ns, 2), block(ns == 4 ? 512 : 1024);
#define ND_LSTM_GO(L0, H, F, S)                                                                                       \
  hipLaunchKernelGGL((lstm_dir_kernel<L0, H, F, S>), grid, block, 0, s, xp, signal, wih0, bsum, whh, len, B, T, out, \
                     bn_scale, bn_shift)
  if (f32) {
    if (layer0)
      ND_LSTM_GO(true, false, false, 16);
    else
      ND_LSTM_GO(false, false, false, 16);
  } else if (layer0) {
    ND_LSTM_GO(true, true, true, 4);
  } else {
    ND_LSTM_GO(false, true, true, 4);
  }
#undef ND_LSTM_GO
  return hipGetLastError();
}

}  // namespace nd
