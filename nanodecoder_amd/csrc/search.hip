// Decoder output head and search (gfx950): final LayerNorm + generator
// (Linear + LogSoftmax, models/model_builder.py:326-334) fused with greedy
// argmax (translate/translator.py:371-394,455-483) or with one --fast beam
// step (translate/translator.py:701-823) including the finished-hypothesis
// bookkeeping the reference does on the host.  Every step stays on the
// device; the host only polls a one-int "chunks alive" counter.
#include "common.hpp"
#include "head.hpp"
#include "kernels.hpp"

namespace nd {

__global__ void __launch_bounds__(256) greedy_head_kernel(GreedyHead h, int step, int R) {
  __shared__ float lps[4][ND_MAXV];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + w;
  if (r >= R) return;
  greedy_head_row(h, r, step, lane, lps[w]);
}

GreedyHead make_greedy_head(const float* x, const float* ln_g, const float* ln_b, const float* gw, const float* gb,
                            int V, int S, int min_len, int eos, int* tok, int* out_tokens, float* score,
                            float* logp_dump, const NextEmbed& ne, const Sampling& smp) {
  GreedyHead h;
  h.x = x;
  h.ln_g = ln_g;
  h.ln_b = ln_b;
  h.gw = gw;
  h.gb = gb;
  h.V = V;
  h.S = S;
  h.min_len = min_len;
  h.eos = eos;
  h.tok = tok;
  h.out_tokens = out_tokens;
  h.score = score;
  h.logp_dump = logp_dump;
  h.ne = ne;
  h.smp = smp;
  return h;
}

hipError_t check_greedy_head(const GreedyHead& h) {
  if (h.V > ND_MAXV || h.V < 1 || !h.ne.emb || !h.ne.x || !h.ne.part) return hipErrorInvalidValue;
  if (h.smp.seed && (h.smp.temp == 0.f || h.smp.topk == 1 || h.smp.topk > h.V)) return hipErrorInvalidValue;
  return hipSuccess;
}

hipError_t launch_dec_greedy_head(const float* x, const float* ln_g, const float* ln_b, const float* gw,
                                  const float* gb, int V, int step, int S, int min_len, int eos, int* tok,
                                  int* out_tokens, float* score, float* logp_dump, const NextEmbed& ne, int R,
                                  hipStream_t s, const Sampling& smp) {
  const GreedyHead h = make_greedy_head(x, ln_g, ln_b, gw, gb, V, S, min_len, eos, tok, out_tokens, score, logp_dump,
                                        ne, smp);
  const hipError_t e = check_greedy_head(h);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(greedy_head_kernel, dim3((R + 3) / 4), dim3(256), 0, s, h, step, R);
  return hipGetLastError();
}

// ------------------------------------------------------------------ beam
#define BEAM_MAX 8

__global__ void __launch_bounds__(64)
beam_init_kernel(BeamState st, int C, int beam, int bos) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= C) return;
  for (int j = 0; j < beam; ++j) {
    st.cum[c * beam + j] = j == 0 ? 0.f : -INFINITY;  // translator.py:691-693
    st.tok[c * beam + j] = bos;
  }
  st.done[c] = 0;
  st.top_fin[c] = 0;
  st.n_hyp[c] = 0;
  st.steps_run[c] = 0;
  if (c == 0) *st.n_alive = C;
}

hipError_t launch_beam_init(const BeamState& st, int C, int beam, int n_best, int S, int bos, hipStream_t s) {
  (void)n_best;
  (void)S;
  hipLaunchKernelGGL(beam_init_kernel, dim3((C + 63) / 64), dim3(64), 0, s, st, C, beam, bos);
  return hipGetLastError();
}

// One workgroup (256 threads = 4 waves) per chunk.
__global__ void __launch_bounds__(256)
beam_step_kernel(NextEmbed ne, const float* __restrict__ x, const float* __restrict__ ln_g, const float* __restrict__ ln_b,
                 const float* __restrict__ gw, const float* __restrict__ gb, int V, BeamState st, int beam,
                 int n_best, int step, int S, int min_len, int eos, float lenpen, const int* __restrict__ clist) {
  __shared__ float lp[BEAM_MAX][ND_MAXV];
  __shared__ float tsc[BEAM_MAX];
  __shared__ int tid_sel[BEAM_MAX];
  __shared__ int fin[BEAM_MAX];
  const int c = clist ? clist[blockIdx.x] : (int)blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  if (c < 0 || st.done[c]) return;  // finished batches are dropped (translator.py:793-810); tail list: -1 = none
  const int cur = step & 1, nxt = cur ^ 1;
  const int row0 = c * beam;
  for (int j = w; j < beam; j += 4) {
    head_row(x, row0 + j, ln_g, ln_b, gw, gb, V, lane, lp[j]);
    if (lane == 0) {
      if (step < min_len) lp[j][eos] = -1e20f;          // :712-713
      const float cj = st.cum[row0 + j];
      for (int k = 0; k < V; ++k) lp[j][k] = (lp[j][k] + cj) / lenpen;  // :718-724
    }
  }
  __syncthreads();
  if (w == 0) {
    // top-`beam` over the flattened beam*V candidates, ties -> lower index
    const int n = beam * V;
    unsigned long long taken = 0ull;  // n <= 256; track per lane below
    bool tk[4] = {false, false, false, false};
    for (int sel = 0; sel < beam; ++sel) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int q = 0; q < 4; ++q) {
        const int idx = lane + 64 * q;
        if (idx < n && !tk[q]) {
          const float v = lp[idx / V][idx % V];
          if (v > bv || (v == bv && idx < bi)) {
            bv = v;
            bi = idx;
          }
        }
      }
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      if (bi != 0x7fffffff && (bi & 63) == lane) tk[bi >> 6] = true;
      if (lane == 0) {
        tsc[sel] = bv;
        tid_sel[sel] = bi;
      }
    }
    (void)taken;
  }
  __syncthreads();
  // reorder alive_seq / ancestry (index_select by origin beam, :737-744, :812-823)
  for (int e = tid; e < beam * (step + 1); e += 256) {
    const int j = e / (step + 1), t = e - j * (step + 1);
    const int par = tid_sel[j] / V;
    const int src = row0 + par, dst = row0 + j;
    if (t < step) {
      st.seq[nxt][(size_t)dst * S + t] = st.seq[cur][(size_t)src * S + t];
      st.anc[nxt][(size_t)dst * S + t] = st.anc[cur][(size_t)src * S + t];
    } else {
      st.seq[nxt][(size_t)dst * S + t] = tid_sel[j] % V;
      st.anc[nxt][(size_t)dst * S + t] = src;  // row `src` wrote this step's self K/V
    }
  }
  if (tid < beam) {
    const int tok = tid_sel[tid] % V;
    fin[tid] = (tok == eos || step + 1 == S) ? 1 : 0;  // :750-752
    st.tok[row0 + tid] = tok;
    st.cum[row0 + tid] = fin[tid] ? -1e10f : tsc[tid] * lenpen;  // :728, :756
  }
  // next step's input rows (x was fully read by head_row before the first barrier)
  if (step + 1 < S)
    for (int j = w; j < beam; j += 4) embed_row(ne, tid_sel[j] % V, step + 1, row0 + j, lane);
  __syncthreads();
  if (tid == 0) {
    bool any = false;
    for (int j = 0; j < beam; ++j) any |= fin[j] != 0;
    if (any) {
      if (fin[0]) st.top_fin[c] = 1;  // :758
      int nh = st.n_hyp[c];
      for (int j = 0; j < beam; ++j) {
        if (!fin[j]) continue;
        // stable insert into the best-first list (sorted(..., reverse=True), :784-786)
        const float sc = tsc[j];
        const int kept = min(nh, n_best);
        int pos = 0;
        while (pos < kept && st.hyp_score[c * n_best + pos] >= sc) ++pos;
        if (pos < n_best) {
          const int last = min(kept, n_best - 1);
          for (int q = last; q > pos; --q) {
            st.hyp_score[c * n_best + q] = st.hyp_score[c * n_best + q - 1];
            st.hyp_len[c * n_best + q] = st.hyp_len[c * n_best + q - 1];
            for (int t = 0; t < S; ++t) {
              st.hyp_tok[((size_t)c * n_best + q) * S + t] = st.hyp_tok[((size_t)c * n_best + q - 1) * S + t];
              st.hyp_anc[((size_t)c * n_best + q) * S + t] = st.hyp_anc[((size_t)c * n_best + q - 1) * S + t];
            }
          }
          st.hyp_score[c * n_best + pos] = sc;
          st.hyp_len[c * n_best + pos] = step + 1;
          for (int t = 0; t <= step; ++t) {
            st.hyp_tok[((size_t)c * n_best + pos) * S + t] = st.seq[nxt][(size_t)(row0 + j) * S + t];
            st.hyp_anc[((size_t)c * n_best + pos) * S + t] = st.anc[nxt][(size_t)(row0 + j) * S + t];
          }
        }
        ++nh;
      }
      st.n_hyp[c] = nh;
      if (st.top_fin[c] && nh >= n_best) {  // :780
        st.done[c] = 1;
        st.steps_run[c] = step + 1;  // dropped after this step (the alive set the attention cut reads)
        if (atomicSub(st.n_alive, 1) == 1) *st.steps_done = step + 1;
      }
    }
  }
}

hipError_t launch_beam_step(const NextEmbed& ne, const float* x, const float* ln_g, const float* ln_b, const float* gw, const float* gb,
                            int V, const BeamState& st, int C, int beam, int n_best, int step, int S, int min_len,
                            int eos, float lenpen, hipStream_t s, const int* clist, int ccap) {
  if (beam > BEAM_MAX || beam * V > 256 || V > ND_MAXV || !ne.emb || !ne.x || !ne.part) return hipErrorInvalidValue;
  if (clist && (ccap < 1 || ccap > C)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(beam_step_kernel, dim3(clist ? ccap : C), dim3(256), 0, s, ne, x, ln_g, ln_b, gw, gb, V, st, beam,
                     n_best, step, S, min_len, eos, lenpen, clist);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256)
beam_finish_kernel(BeamState st, int n_best, int S, int* __restrict__ tokens, float* __restrict__ scores,
                   int* __restrict__ lens) {
  const int c = blockIdx.x;
  for (int e = threadIdx.x; e < n_best * S; e += 256) {
    const int nb = e / S, t = e - nb * S;
    const int len = st.hyp_len[c * n_best + nb];
    tokens[((size_t)c * n_best + nb) * S + t] = t < len ? st.hyp_tok[((size_t)c * n_best + nb) * S + t] : -1;
  }
  if (threadIdx.x < n_best) {
    scores[c * n_best + threadIdx.x] = st.hyp_score[c * n_best + threadIdx.x];
    lens[c * n_best + threadIdx.x] = st.hyp_len[c * n_best + threadIdx.x];
  }
}

hipError_t launch_beam_finish(const BeamState& st, int C, int n_best, int S, int* tokens, float* scores, int* lens,
                              hipStream_t s) {
  hipLaunchKernelGGL(beam_finish_kernel, dim3(C), dim3(256), 0, s, st, n_best, S, tokens, scores, lens);
  return hipGetLastError();
}

// ------------------------------------------------------------ classic Beam
// onmt/translate/beam.py:6-178 driven by translate/translator.py:827-926:
// scores start at 0 for every beam, step 0 expands beam 0 only, EOS beams get
// -1e20 rows (no children), every EOS is a finished hypothesis scored by the
// GNMT global scorer (length penalty none / wu / avg, coverage penalty none /
// wu / summary, at scoring time or stepwise), n-gram repeats block a beam
// (-10e20 rows), and a reference batch advances all its beams until each is
// done (eos_top && finished >= n_best).  Finished lists keep the n_best best
// entries in stable order, which is what sort_finished's stable sort reads.

// global scorer divisor for len(next_ys) = n_ys (penalties.py:57-78); the
// Python float the reference computes is rounded to fp32 by torch.
__device__ __forceinline__ float classic_lp_div(int kind, int n_ys, float alpha) {
  if (kind == 1) return (float)(pow(5.0 + n_ys, (double)alpha) / pow(6.0, (double)alpha));
  if (kind == 2) return (float)n_ys;
  return 1.0f;
}

// cov_penalty(coverage [+ add]) of one beam over its first `cut` keys, one
// wave (penalties.py:34-53): wu = beta * -sum log(min(c, 1)),
// summary = beta * (sum max(c, 1) - cut)
__device__ float classic_cov_pen(const float* __restrict__ cov, const float* __restrict__ add, int cut, int kind,
                                 float beta, int lane) {
  float acc = 0.f;
  for (int t = lane; t < cut; t += 64) {
    float v = cov ? cov[t] : 0.f;
    if (add) v = cov ? v + add[t] : add[t];
    acc += kind == 1 ? logf(fminf(v, 1.f)) : fmaxf(v, 1.f);
  }
  acc = wave_sum(acc);
  return kind == 1 ? beta * -acc : beta * (acc - (float)cut);
}

// stable insertion of (sc, tokens src[0..len), rows anc[0..len)) into chunk c's best-first list
__device__ void classic_insert(const BeamState& st, int c, int n_best, int S, float sc, int len, const int* src,
                               const int* anc) {
  const int nh = st.n_hyp[c];
  const int kept = min(nh, n_best);
  int pos = 0;
  while (pos < kept && st.hyp_score[c * n_best + pos] >= sc) ++pos;
  if (pos < n_best) {
    const int last = min(kept, n_best - 1);
    for (int q = last; q > pos; --q) {
      st.hyp_score[c * n_best + q] = st.hyp_score[c * n_best + q - 1];
      st.hyp_len[c * n_best + q] = st.hyp_len[c * n_best + q - 1];
      for (int t = 0; t < S; ++t) {
        st.hyp_tok[((size_t)c * n_best + q) * S + t] = st.hyp_tok[((size_t)c * n_best + q - 1) * S + t];
        st.hyp_anc[((size_t)c * n_best + q) * S + t] = st.hyp_anc[((size_t)c * n_best + q - 1) * S + t];
      }
    }
    st.hyp_score[c * n_best + pos] = sc;
    st.hyp_len[c * n_best + pos] = len;
    for (int t = 0; t < len; ++t) {
      st.hyp_tok[((size_t)c * n_best + pos) * S + t] = src[t];
      st.hyp_anc[((size_t)c * n_best + pos) * S + t] = anc[t];
    }
  }
  st.n_hyp[c] = nh + 1;
}

// GNMTGlobalScorer.score(beam, beam.scores)[i] (beam.py:200-212).  With
// length penalty none, length_none hands back beam.scores itself and the
// in-place `normalized_probs -= penalty` lowers every live score: each call
// (one per finished beam, one per sort_finished top-up) moves them all.
__device__ float classic_score(const BeamState& st, int row0, int beam, int i, const ClassicOpts& o, float div) {
  const bool cov = o.cov_kind != 0 && !o.stepwise;
  if (cov && o.lp_kind == 0) {
    for (int j = 0; j < beam; ++j) st.cum[row0 + j] -= st.pen[row0 + j];
    return st.cum[row0 + i];
  }
  const float v = st.cum[row0 + i] / div;
  return cov ? v - st.pen[row0 + i] : v;
}

__global__ void __launch_bounds__(64)
beam_classic_init_kernel(BeamState st, const int* __restrict__ group, int C, int beam, int bos) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= C) return;
  for (int j = 0; j < beam; ++j) {
    st.cum[c * beam + j] = 0.f;  // beam.py:34
    // beams 1.. start from <blank> (:41-43); their step-0 output is never
    // read (step 0 expands beam 0 only and every beam then descends from it)
    st.tok[c * beam + j] = bos;
  }
  st.done[c] = 0;
  st.top_fin[c] = 0;
  st.n_hyp[c] = 0;
  st.steps_run[c] = 0;
  st.group[c] = group[c];
  st.grp_done[c] = 0;
  if (atomicAdd(&st.grp_left[group[c]], 1) == 0) atomicAdd(st.n_alive, 1);  // first chunk of its batch
}

hipError_t launch_beam_classic_init(const BeamState& st, const int* group, int C, int beam, int bos, hipStream_t s) {
  hipError_t e = hipMemsetAsync(st.grp_left, 0, (size_t)C * sizeof(int), s);
  if (e == hipSuccess) e = hipMemsetAsync(st.n_alive, 0, sizeof(int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(beam_classic_init_kernel, dim3((C + 63) / 64), dim3(64), 0, s, st, group, C, beam, bos);
  return hipGetLastError();
}

// One workgroup (256 threads = 4 waves) per chunk.
__global__ void __launch_bounds__(256)
beam_classic_step_kernel(NextEmbed ne, const float* __restrict__ x, const float* __restrict__ ln_g,
                         const float* __restrict__ ln_b, const float* __restrict__ gw, const float* __restrict__ gb,
                         int V, BeamState st, int beam, int n_best, int step, int S, int min_len, int eos,
                         ClassicOpts o) {
  __shared__ float lp[BEAM_MAX][ND_MAXV];
  __shared__ float tsc[BEAM_MAX];
  __shared__ int tid_sel[BEAM_MAX];
  __shared__ int fin[BEAM_MAX];
  const int c = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int g = st.group[c];
  if (st.grp_done[g]) return;  // translator.py:884-885: the whole batch is done
  const int cur = step & 1, nxt = cur ^ 1;
  const int row0 = c * beam;
  const bool cov_on = o.cov_kind != 0 && st.attn;
  const int cut = cov_on ? min(st.cut[c], st.T) : 0;
  const size_t aS = (size_t)S * st.T;  // attention row stride per decoder row
  for (int j = w; j < beam; j += 4) {
    // stepwise penalty: GNMTGlobalScorer.update_score (beam.py:80-81, :214-223)
    if (o.stepwise && cov_on && step > 0) {
      const float pen = classic_cov_pen(st.cov[cur] + (size_t)(row0 + j) * st.T,
                                        st.attn + (row0 + j) * aS + (size_t)step * st.T, cut, o.cov_kind, o.beta,
                                        lane);
      if (lane == 0) st.cum[row0 + j] = (st.cum[row0 + j] + st.prev_pen[row0 + j]) - pen;
    }
    head_row(x, row0 + j, ln_g, ln_b, gw, gb, V, lane, lp[j]);
    if (lane == 0) {
      if (step + 1 < min_len) lp[j][eos] = -1e20f;  // beam.py:88-91 (cur_len = step + 1)
      if (step > 0) {                               // :93-99
        const float cj = st.cum[row0 + j];
        const bool dead = st.tok[row0 + j] == eos;  // EOS has no children
        for (int k = 0; k < V; ++k) lp[j][k] = dead ? -1e20f : lp[j][k] + cj;
        if (o.ngram > 0 && st.blk[cur][row0 + j])   // :101-119 (-10e20)
          for (int k = 0; k < V; ++k) lp[j][k] = -10e20f;
      }
    }
  }
  __syncthreads();
  if (w == 0) {
    // topk(beam) over beam*V candidates (step 0: beam 0's V), ties -> lower index
    const int n = step == 0 ? V : beam * V;
    bool tk[4] = {false, false, false, false};
    for (int sel = 0; sel < beam; ++sel) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int q = 0; q < 4; ++q) {
        const int idx = lane + 64 * q;
        if (idx < n && !tk[q]) {
          const float v = lp[idx / V][idx % V];
          if (v > bv || (v == bv && idx < bi)) {
            bv = v;
            bi = idx;
          }
        }
      }
      for (int off = 32; off > 0; off >>= 1) {
        const float ov = __shfl_xor(bv, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      if (bi != 0x7fffffff && (bi & 63) == lane) tk[bi >> 6] = true;
      if (lane == 0) {
        tsc[sel] = bv;
        tid_sel[sel] = bi;
      }
    }
  }
  __syncthreads();
  // next_ys / prev_ks (beam.py:125-131) as the reordered histories
  for (int e = tid; e < beam * (step + 1); e += 256) {
    const int j = e / (step + 1), t = e - j * (step + 1);
    const int par = tid_sel[j] / V;
    const int src = row0 + par, dst = row0 + j;
    if (t < step) {
      st.seq[nxt][(size_t)dst * S + t] = st.seq[cur][(size_t)src * S + t];
      st.anc[nxt][(size_t)dst * S + t] = st.anc[cur][(size_t)src * S + t];
    } else {
      st.seq[nxt][(size_t)dst * S + t] = tid_sel[j] % V;
      st.anc[nxt][(size_t)dst * S + t] = src;
    }
  }
  if (tid < beam) {
    const int tok = tid_sel[tid] % V;
    fin[tid] = tok == eos ? 1 : 0;
    st.tok[row0 + tid] = tok;
    st.cum[row0 + tid] = tsc[tid];  // self.scores = best_scores (:126)
  }
  if (step + 1 < S)
    for (int j = w; j < beam; j += 4) embed_row(ne, tid_sel[j] % V, step + 1, row0 + j, lane);
  __syncthreads();
  for (int j = w; j < beam; j += 4) {
    const int par = tid_sel[j] / V, src = row0 + par, dst = row0 + j;
    // update_global_state (beam.py:132, :225-243): coverage of the new beam =
    // the parent's coverage + the parent's attention of this step
    if (cov_on) {
      const float* a = st.attn + src * aS + (size_t)step * st.T;
      const float* cp = st.cov[cur] + (size_t)src * st.T;
      float* cn = st.cov[nxt] + (size_t)dst * st.T;
      float acc = 0.f;
      for (int t = lane; t < cut; t += 64) {
        const float v = step == 0 ? a[t] : cp[t] + a[t];
        cn[t] = v;
        acc += o.cov_kind == 1 ? logf(fminf(v, 1.f)) : fmaxf(v, 1.f);
      }
      acc = wave_sum(acc);
      const float pen = o.cov_kind == 1 ? o.beta * -acc : o.beta * (acc - (float)cut);
      if (lane == 0) {
        st.pen[dst] = pen;
        st.prev_pen[dst] = step == 0 ? 0.f : pen;
      }
    }
    // n-gram blocking state of the new hypothesis (its step + 1 tokens): the
    // parent's, or its last n-gram (free of excluded tokens) seen earlier in it
    if (o.ngram > 0) {
      const int* h = st.seq[nxt] + (size_t)dst * S;
      const int n = o.ngram, L = step + 1;
      bool rep = false;
      if (L >= n) {
        bool excl = false;
        for (int k = 0; k < n; ++k) excl |= ((o.excl >> h[L - n + k]) & 1u) != 0;
        if (!excl)
          for (int e = n - 1 + lane; e < L - 1; e += 64) {
            bool same = true;
            for (int k = 0; k < n; ++k) same &= h[e - n + 1 + k] == h[L - n + k];
            rep |= same;
          }
      }
      rep = __any(rep);
      if (lane == 0) st.blk[nxt][dst] = (step > 0 && st.blk[cur][src]) || rep;
    }
  }
  __syncthreads();
  if (tid == 0) {
    const float div = classic_lp_div(o.lp_kind, step + 2, o.alpha);  // len(next_ys) after the append
    for (int j = 0; j < beam; ++j)                                   // :135-139
      if (fin[j])
        classic_insert(st, c, n_best, S, classic_score(st, row0, beam, j, o, div), step + 1,
                       st.seq[nxt] + (size_t)(row0 + j) * S, st.anc[nxt] + (size_t)(row0 + j) * S);
    if (fin[0]) st.top_fin[c] = 1;  // eos_top (:142-144)
    st.steps_run[c] = step + 1;
    if (!st.done[c] && st.top_fin[c] && st.n_hyp[c] >= n_best) {  // done() (:146-147)
      st.done[c] = 1;
      if (atomicSub(&st.grp_left[g], 1) == 1) {
        st.grp_done[g] = 1;
        if (atomicSub(st.n_alive, 1) == 1) *st.steps_done = step + 1;
      }
    }
  }
}

hipError_t launch_beam_classic_step(const NextEmbed& ne, const float* x, const float* ln_g, const float* ln_b,
                                    const float* gw, const float* gb, int V, const BeamState& st, int C, int beam,
                                    int n_best, int step, int S, int min_len, int eos, const ClassicOpts& o,
                                    hipStream_t s) {
  if (beam > BEAM_MAX || beam * V > 256 || V > ND_MAXV || V < beam || !ne.emb || !ne.x || !ne.part)
    return hipErrorInvalidValue;
  if (o.cov_kind != 0 && (!st.attn || !st.cut || !st.cov[0] || !st.cov[1])) return hipErrorInvalidValue;
  if (o.ngram < 0 || o.ngram > S || (o.ngram > 0 && (!st.blk[0] || !st.blk[1]))) return hipErrorInvalidValue;
  hipLaunchKernelGGL(beam_classic_step_kernel, dim3(C), dim3(256), 0, s, ne, x, ln_g, ln_b, gw, gb, V, st, beam,
                     n_best, step, S, min_len, eos, o);
  return hipGetLastError();
}

// sort_finished(minimum=n_best) (beam.py:149-161): beams still alive top the
// list up in beam order, scored at the chunk's last step; then the n_best
// best (score, tokens) go out like the --fast path's.
__global__ void __launch_bounds__(256)
beam_classic_finish_kernel(BeamState st, int beam, int n_best, int S, ClassicOpts o, int* __restrict__ tokens,
                           float* __restrict__ scores, int* __restrict__ lens) {
  const int c = blockIdx.x;
  if (threadIdx.x == 0 && st.n_hyp[c] < n_best) {
    const int t = st.steps_run[c], fb = t & 1;
    const float div = classic_lp_div(o.lp_kind, t + 1, o.alpha);
    for (int i = 0; st.n_hyp[c] < n_best; ++i)
      classic_insert(st, c, n_best, S, classic_score(st, c * beam, beam, i, o, div), t,
                     st.seq[fb] + (size_t)(c * beam + i) * S, st.anc[fb] + (size_t)(c * beam + i) * S);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n_best * S; e += 256) {
    const int nb = e / S, t = e - nb * S;
    const int len = st.hyp_len[c * n_best + nb];
    tokens[((size_t)c * n_best + nb) * S + t] = t < len ? st.hyp_tok[((size_t)c * n_best + nb) * S + t] : -1;
  }
  if (threadIdx.x < n_best) {
    scores[c * n_best + threadIdx.x] = st.hyp_score[c * n_best + threadIdx.x];
    lens[c * n_best + threadIdx.x] = st.hyp_len[c * n_best + threadIdx.x];
  }
}

hipError_t launch_beam_classic_finish(const BeamState& st, int C, int beam, int n_best, int S, const ClassicOpts& o,
                                      int* tokens, float* scores, int* lens, hipStream_t s) {
  if (n_best > beam) return hipErrorInvalidValue;
  hipLaunchKernelGGL(beam_classic_finish_kernel, dim3(C), dim3(256), 0, s, st, beam, n_best, S, o, tokens, scores,
                     lens);
  return hipGetLastError();
}

// ------------------------------------------------------- attention capture
// -attn_debug / coverage: the last layer's head-0 context scores of one step
// -> probabilities (multi_headed_attn.py:175), one wave per decoder row
__global__ void __launch_bounds__(256)
attn_step_softmax_kernel(float* __restrict__ a, size_t ld, const int* __restrict__ span, int R, int rpc, int T) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  const int L = min(span[r / rpc], T);
  float* p = a + (size_t)r * ld;
  float mx = -INFINITY;
  for (int t = lane; t < L; t += 64) mx = fmaxf(mx, p[t]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int t = lane; t < L; t += 64) sum += __expf(p[t] - mx);
  sum = wave_sum(sum);
  for (int t = lane; t < T; t += 64) p[t] = t < L ? __expf(p[t] - mx) / sum : 0.f;
}

hipError_t launch_attn_step_softmax(float* a, size_t ld, const int* span, int R, int rpc, int T, hipStream_t s) {
  if (R < 1 || rpc < 1 || T < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(attn_step_softmax_kernel, dim3((R + 3) / 4), dim3(256), 0, s, a, ld, span, R, rpc, T);
  return hipGetLastError();
}

// one workgroup per (chunk, hypothesis); a wave per step row
__global__ void __launch_bounds__(256)
beam_attn_gather_kernel(BeamState st, int n_best, int S, int max_len, int T, float* __restrict__ out) {
  const int ck = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int len = st.hyp_len[ck];
  for (int t = w; t < max_len; t += 4) {
    float* o = out + ((size_t)ck * max_len + t) * T;
    if (t < len) {
      const float* a = st.attn + ((size_t)st.hyp_anc[(size_t)ck * S + t] * S + t) * st.T;
      for (int x = lane; x < T; x += 64) o[x] = a[x];
    } else {
      for (int x = lane; x < T; x += 64) o[x] = 0.f;
    }
  }
}

hipError_t launch_beam_attn_gather(const BeamState& st, int C, int n_best, int S, int max_len, int T, float* out,
                                   hipStream_t s) {
  if (!st.attn || T > st.T || max_len > S) return hipErrorInvalidValue;
  hipLaunchKernelGGL(beam_attn_gather_kernel, dim3(C * n_best), dim3(256), 0, s, st, n_best, S, max_len, T, out);
  return hipGetLastError();
}

}  // namespace nd
