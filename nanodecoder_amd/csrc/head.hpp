// Per-row device pieces of the greedy output head (gfx950), shared by the
// standalone head kernel (search.hip) and the layer-0 self-attention kernel
// that runs the previous step's head in its own launch (attention.hip):
// final LayerNorm + generator + log_softmax (models/model_builder.py:326-334),
// argmax / sampling (translate/translator.py:371-394,455-483) and the next
// step's embedded input (onmt/modules/embeddings.py:189-207).
#pragma once
#include "common.hpp"
#include "kernels.hpp"

namespace nd {

// LN + generator + log_softmax for row `row` of the P16-packed decoder
// output x, held by one wave (lane owns dims 4*lane..4*lane+3).  Writes
// logp[0..V) to `lp` (LDS; every lane writes the same values).  The
// generator rows are read 8 at a time, all loads issued together and the 8
// cross-lane sums interleaved, so a step pays one load latency, not V.
__device__ __forceinline__ void head_row(const float* __restrict__ x, int row, const float* __restrict__ ln_g,
                                         const float* __restrict__ ln_b, const float* __restrict__ gw,
                                         const float* __restrict__ gb, int V, int lane, float* lp) {
  f32x4 wr[8];
  float br[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {  // first 8 rows in flight with x
    wr[k] = ld4(gw + (size_t)min(k, V - 1) * ND_D + lane * 4);
    br[k] = gb[min(k, V - 1)];
  }
  f32x4 v = ld4(x + pk(row, lane * 4, ND_D));
  const f32x4 g = ld4(ln_g + lane * 4), bt = ld4(ln_b + lane * 4);
  const float mu = wave_sum(v.x + v.y + v.z + v.w) * (1.0f / ND_D);
  const f32x4 d = v - mu;
  const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.0f / ND_D);
  const float rs = ln_rsqrt(var + ND_LN_EPS);
  const f32x4 y = d * rs * g + bt;
  float mx = -INFINITY;
  for (int k0 = 0; k0 < V; k0 += 8) {
    if (k0 > 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        wr[k] = ld4(gw + (size_t)min(k0 + k, V - 1) * ND_D + lane * 4);
        br[k] = gb[min(k0 + k, V - 1)];
      }
    }
    float dt[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) dt[k] = y.x * wr[k].x + y.y * wr[k].y + y.z * wr[k].z + y.w * wr[k].w;
#pragma unroll
    for (int k = 0; k < 8; ++k) dt[k] = wave_sum(dt[k]);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k0 + k < V) {
        const float logit = dt[k] + br[k];
        lp[k0 + k] = logit;
        mx = fmaxf(mx, logit);
      }
  }
  // torch log_softmax: (x - max) - log(sum(exp(x - max)))
  float s = 0.f;
  for (int k = 0; k < V; ++k) s += expf(lp[k] - mx);
  const float ls = logf(s);
  for (int k = 0; k < V; ++k) lp[k] = (lp[k] - mx) - ls;
}

// Writes the embedded input row of step `step_next` for token `tk` (one wave;
// onmt/modules/embeddings.py:189-207, PositionalEncoding :36-43).
__device__ __forceinline__ void embed_row(const NextEmbed& ne, int tk, int step_next, int row, int lane,
                                          const f32x4* pre = nullptr, int npre = 0) {
  // pre: the lane's slice of embedding rows 0..npre-1, loaded ahead of the
  // argmax (greedy) so the chosen row needs no dependent load
  f32x4 e = tk < npre ? pre[0] : ld4(ne.emb + (size_t)tk * ND_D + lane * 4);
  if (tk < npre) {
#pragma unroll
    for (int k = 1; k < 8; ++k)
      if (k == tk) e = pre[k];
  }
  if (ne.pe) e = e * 16.0f + ld4(ne.pe + (size_t)step_next * ND_D + lane * 4);  // sqrt(256) = 16
  st4(ne.x + pk(row, lane * 4, ND_D), e);
  if (ne.tok && lane == 0) ne.tok[row] = tk;
  const float mu = wave_sum(e.x + e.y + e.z + e.w) * (1.0f / ND_D);
  const f32x4 d = e - mu;
  const float q = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w);
  if (lane == 0) {
    ne.part[(size_t)row * ND_PART_LD * 2] = mu;  // one partial per row
    ne.part[(size_t)row * ND_PART_LD * 2 + 1] = q;
  }
}

// counter-based uniform in [0, 1) for (seed, row, step): splitmix64 finaliser
__device__ __forceinline__ float draw_uniform(unsigned long long seed, int row, int step) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (((unsigned long long)row << 32) + (unsigned)step + 1ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);  // 24 random bits
}

// sample_with_temperature (translate/translator.py:371-394) for one row's
// log-probs lp[0..V) (EOS already masked): l = lp / temp; with topk > 0 the
// logits below the k-th largest become -10000 (keep * l + (1 - keep) * -10000);
// one draw from softmax(l); the score is l at the drawn token.  Every lane
// computes the same draw (deterministic), so no broadcast is needed.
__device__ int sample_token(const float* lp, int V, float temp, int topk, float u, float& score) {
  float l[ND_MAXV];
  for (int k = 0; k < V; ++k) l[k] = lp[k] / temp;
  if (topk > 0) {
    // k-th largest value (torch.topk(...)[0][:, -1]); ties at it are kept (torch.ge)
    float kth = INFINITY;
    for (int q = 0; q < topk; ++q) {
      float m = -INFINITY;
      int cnt = 0;
      for (int k = 0; k < V; ++k)
        if (l[k] < kth) m = fmaxf(m, l[k]);
      for (int k = 0; k < V; ++k) cnt += l[k] == m ? 1 : 0;
      kth = m;
      q += cnt - 1;  // a tie block counts once per member
    }
    for (int k = 0; k < V; ++k) l[k] = l[k] >= kth ? l[k] : -10000.0f;
  }
  float mx = -INFINITY;
  for (int k = 0; k < V; ++k) mx = fmaxf(mx, l[k]);
  float sum = 0.f;
  for (int k = 0; k < V; ++k) sum += __expf(l[k] - mx);
  const float target = u * sum;
  float acc = 0.f;
  int pick = V - 1;
  for (int k = 0; k < V; ++k) {
    acc += __expf(l[k] - mx);
    if (target < acc) {
      pick = k;
      break;
    }
  }
  score = l[pick];
  return pick;
}

// One row of the greedy head for step `step`, run by one wave: log-probs into
// lp (LDS, ND_MAXV floats), the token written to h.tok / h.out_tokens (and
// the score, the optional logp dump), the row's input of step + 1 embedded.
// Returns the token (every lane holds it).
__device__ __forceinline__ int greedy_head_row(const GreedyHead& h, int r, int step, int lane, float* lp) {
  const int V = h.V;
  // the embedding rows of tokens 0..7, in flight with the head's own loads
  f32x4 er[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) er[k] = ld4(h.ne.emb + (size_t)min(k, V - 1) * ND_D + lane * 4);
  head_row(h.x, r, h.ln_g, h.ln_b, h.gw, h.gb, V, lane, lp);
  if (lane == 0 && h.logp_dump)
    for (int k = 0; k < V; ++k) h.logp_dump[((size_t)r * h.S + step) * V + k] = lp[k];
  // every lane runs the (tiny) argmax so the token needs no broadcast
  const bool no_eos = step < h.min_len;
  int best = 0;
  float bv;
  if (h.smp.seed) {  // random sampling (translator.py:469-475)
    float m[ND_MAXV];
    for (int k = 0; k < V; ++k) m[k] = (no_eos && k == h.eos) ? -1e20f : lp[k];
    best = sample_token(m, V, h.smp.temp, h.smp.topk, draw_uniform(*h.smp.seed, r, step), bv);
  } else {
    bv = (no_eos && h.eos == 0) ? -1e20f : lp[0];
    for (int k = 1; k < V; ++k) {
      const float v = (no_eos && k == h.eos) ? -1e20f : lp[k];
      if (v > bv) {  // first index wins ties (topk(1))
        bv = v;
        best = k;
      }
    }
  }
  if (lane == 0) {
    h.tok[r] = best;
    h.out_tokens[(size_t)r * h.S + step] = best;
    h.score[r] = bv;
  }
  if (step + 1 < h.S) embed_row(h.ne, best, step + 1, r, lane, er, min(V, 8));
  return best;
}

}  // namespace nd
