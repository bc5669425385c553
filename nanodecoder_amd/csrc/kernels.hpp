// Host-side launchers of the gfx950 kernels (one definition per .hip file).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nd {

struct GemmArgs {
  const float* A = nullptr;
  int lda = 0;
  const float* W = nullptr;  // [N, K] row-major (torch Linear layout)
  int ldw = 0;
  const float* bias = nullptr;
  const float* R = nullptr;  // residual [M, N]
  int ldr = 0;
  float* C = nullptr;
  int ldc = 0;
  // LayerNorm prologue over K (K == 256): rows of A are normalised,
  // (a - mean) * rstd; the LayerNorm's affine (gamma, beta) is folded into
  // W and bias once at load time (launch_fold_layernorm).
  bool norm = false;
  int M = 0, N = 0, K = 0;
  bool relu = false;
  // Row statistics hand-off (LayerNorm fusion across kernels):
  //  part_out: the producer writes, per output row and per column tile j of
  //            width N/part_n, {mean_j, M2_j} (M2 = sum of squared deviations)
  //            at part_out[(row*16 + j)*2]; launch_gemm reports part_n.
  //  part_in:  the LN consumer merges part_n_in such partials per row (Chan's
  //            formula) instead of re-reading and reducing the row.
  float* part_out = nullptr;
  const float* part_in = nullptr;
  int part_n_in = 0;
  int part_n_out = 0;  // set by launch_gemm
  // split-fp16 operand path (row-major kernel only): W pre-split by
  // launch_split_weight into fp16 hi/lo planes scaled by 2^s; the product is
  // computed as hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_f16 and the
  // accumulator scaled back by wscale = 2^-s (exact).
  const uint16_t* Wh = nullptr;
  float wscale = 1.0f;
  // P16 GEMMs: the weight's row-major split image too (large-M route through
  // the LDS-tiled kernel, launch_gemm_p16), and the P16 operand mode of the
  // row-major kernel (A, R, C in P16; lda / ldr / ldc unused)
  const uint16_t* Wh_rm = nullptr;
  float wscale_rm = 1.0f;
  int p16io = 0;
  int xcd_map = 0;     // row-major kernel: XCD-aware tile order (set by launch_gemm)
  int xcd_a = 0;       // P16 kernel: row-block split over the 8 XCDs (0: grid order; set by launch_p16)
  // split-fp16 range guard (common.hpp flag_overflow): set to 1 when a split
  // activation operand (no LN prologue) reaches |x| >= 65504; nullable
  int* ovf = nullptr;
  // --fast beam: row r belongs to chunk r / skip_rpc; a tile whose rows all
  // belong to finished chunks (skip[chunk] != 0) exits without work; nullable
  const int* skip = nullptr;
  int skip_rpc = 1;
  // P16 GEMMs: stay on the small-M kernels at any M (the beam loop's tail,
  // when few chunks are alive: a 16-row block's latency, not a 64-row tile's)
  int prefer_p16 = 0;
  // P16 GEMMs: C written row-major [M16][N] instead of P16 (the memory-bank
  // kernel's q': its one-row-per-chunk loads then read whole 1 KB runs, not
  // 16 B of every 64 B line; PMC: 4x over-fetch of q' in the P16 layout)
  int c_rm = 0;
  // row-major LDS-tiled kernel, N = layers * 512 (the beam's context K / V):
  // write the 24-bit image instead of C: layer l's row r at q24 + l *
  // q24_plane + r * CTXQ_ROW (layer-major planes, launch_ctx_pack_q24); nullable
  uint8_t* q24 = nullptr;
  size_t q24_plane = 0;
  // P16 GEMMs at K >= 1024: the split-K form's fp32 slab and per-tile tickets
  // (zero before the first launch; the last arriver of a tile resets its
  // ticket), sized for sk_tiles 32 x 32 tiles; null: the one-workgroup form
  float* sk_slab = nullptr;
  int* sk_cnt = nullptr;
  int sk_tiles = 0;
};
#define ND_PART_LD 16  // partial-stat slots per row (max column tiles of a 256-wide row)
// row-major operands (encoder, large M): LDS-tiled MFMA kernel
hipError_t launch_gemm(GemmArgs& g, hipStream_t s);
// P16-packed operands (decoder steps, small M; common.hpp pk()): A, W, R, C
// packed, lda/ldw/ldr/ldc ignored, rows padded to a multiple of 16 in every
// buffer (part buffers included); LN requires part_in.
hipError_t launch_gemm_p16(GemmArgs& g, hipStream_t s);
// W [N, K] fp32 (leading dimension ld, 0 = K) -> Wh (split-fp16, [N][K/8][hi 8 | lo 8] halves) with the
// power-of-two scale that puts max|W| just under 2^14; returns 2^-s in
// *wscale (synchronises the stream: load-time only).  K % 32 == 0.
hipError_t launch_split_weight(const float* W, int N, int K, uint16_t* Wh, float* wscale, hipStream_t s, int ld = 0);
// P16H image of a row-major weight [N, K] (leading dim ld) for the split-fp16
// P16 kernels: [N/16][K/32][hi | lo][64 lanes][8 halves] of W * 2^s (scale as
// launch_split_weight; synchronises the stream).  N % 16 == 0, K % 32 == 0.
hipError_t launch_pack_p16h(const float* W, int ld, int N, int K, uint16_t* out, float* wscale, hipStream_t s);
// ND_GEMM_F32=1: the fp32-MFMA kernels everywhere (split images unused)
bool gemm_f32_forced();
// launches per GEMM route (include/nanodec.h ND_ROUTE_*) since the last reset
long long gemm_route_count(int route, bool reset);
// raises the dynamic-LDS limit of the LDS-staged GEMM kernels (once per process)
hipError_t init_gemm_attributes();
// row-major [M, N] with leading dimension ld -> P16 (M, N multiples of 16)
hipError_t launch_pack_p16(const float* src, int ld, float* dst, int M, int N, hipStream_t s);
// W_out[n][k] = W[n][k] * ln_g[k];  b_out[n] = bias[n] + sum_k W[n][k] * ln_b[k]
// (LayerNorm(x) W^T + b == xhat (W diag(g))^T + (W beta + b)); bias may be null.
hipError_t launch_fold_layernorm(const float* W, const float* bias, const float* ln_g, const float* ln_b,
                                 float* W_out, float* b_out, int N, int K, hipStream_t s);

// ---- encoder -------------------------------------------------------------
// Layer 0 of the Transformer encoder reads x = s w + b (Linear(1, d) of the
// sample s): with w' = w - mean(w), b' = b - mean(b) its LayerNorm'd
// projection is the rank-2 form
//   LN(x) W'^T + b'' = (s a + c) / sqrt(s^2 m_ww + 2 s m_wb + m_bb + eps) + b''
// a = W' w', c = W' b', m_.. the means of w'^2, w'b', b'^2 (W', b'': the
// LN-folded QKV weight and bias), so the layer's QKV GEMM becomes a write of
// the [M, 768] rows beside the embedding's.
struct EmbedQkv {
  const float* ac = nullptr;  // [2][768]: a, c
  const float* bias = nullptr;
  float mww = 0.f, mwb = 0.f, mbb = 0.f;
  float* qkv = nullptr;       // [M, 768] row-major
};
// Layer 0's attention in the same closed form: per head h the query, key
// and value of position t are u_h y_t + v_h r_t + w_h (y = s r, r the LN
// scale of the row), so a score is y_u alpha_t + r_u beta_t + (a constant
// of t that cancels in the softmax) with alpha_t, beta_t linear in
// (y_t, r_t, 1) (coef [8 heads][6], log2 units), and the output is
// a_v E[y] + c_v E[r] + b_v over the softmax: out [M, 256] row-major.
struct R2Args {
  const float* signal = nullptr;
  const int* span = nullptr;
  EmbedQkv eq;
  const float* coef = nullptr;
  float* out = nullptr;
};
hipError_t launch_enc_attention_rank2(const float* signal, const int* span, const EmbedQkv& eq, const float* coef,
                                      float* out, int B, int T, hipStream_t s);
// ac and the three means (double scal[3]) from the LN-folded weight [768, 256]
hipError_t launch_embed_qkv_prep(const float* w_in, const float* b_in, const float* nwqkv, float* ac, double* scal,
                                 hipStream_t s);
// x[b*T+t][:] = signal[b][t] * w_in + b_in (Linear(1, d)); part: full-row stats;
// eq: also layer 0's q | k | v rows (EmbedQkv)
hipError_t launch_enc_embed(const float* signal, const float* w_in, const float* b_in, float* x, float* part, int B,
                            int T, hipStream_t s, const EmbedQkv* eq = nullptr);
// flash attention over qkv [B*T, 768]; mask signal==0; keys >= span excluded
// exact: the fp32-MFMA kernel instead of split-fp16 (also forced by ND_ENC_ATTN_F32=1);
// ovf: split-fp16 range guard word (nullable)
hipError_t launch_enc_attention(const float* qkv, const float* signal, const int* span, float* out, int B, int T,
                                hipStream_t s, bool exact = false, int* ovf = nullptr);
// NanoEncoder BiLSTM layer (both directions): xp [B*T, 1024] projections
// (or, layer0, computed from signal with wih0/bsum [2][512]); whh [2][512][128];
// out [B*T, 256] (h, or BatchNorm(h) when bn_scale != nullptr).
hipError_t launch_lstm_layer(const float* xp, const float* signal, const float* wih0, const float* bsum,
                             const float* whh, const int* len, int B, int T, float* out, const float* bn_scale,
                             const float* bn_shift, bool layer0, hipStream_t s, bool exact = false);
// fused encoder FFN block (ffn.hip): x = y + W2 relu(W1' LN(y) + b1') + b2 with
// the LN affine folded into W1' / b1'; w1h = P16H image of W1' [F, 256], w2h =
// P16H image of W2 [256, F] (launch_pack_p16h), w*s their scales; xpart gets
// each row's exact {mean, M2} in slot 0 (one partial).  F % 32 == 0, F <= 2048.
// wo (nullable): the attention block's output projection folded in front,
// y = x + att Wo^T + bo with y the residual argument (x may alias it), woh
// the P16H image of Wo [256, 256], wos its scale.
struct EncWo {
  const float* att = nullptr;
  const uint16_t* woh = nullptr;
  float wos = 1.f;
  const float* bo = nullptr;
};
// qk (nullable): the NEXT layer's QKV projection folded behind, out = LN(x)
// W'^T + b' (wh: P16H image of the LN-folded W' [768, 256], ws its scale;
// out row-major [M, 768])
struct EncQkv {
  const uint16_t* wh = nullptr;
  float ws = 1.f;
  const float* bias = nullptr;
  float* out = nullptr;
};
hipError_t launch_enc_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h,
                          float w2s, const float* b2, float* x, float* xpart, int M, int F, int* ovf, hipStream_t s,
                          const EncWo* wo = nullptr, const EncQkv* qk = nullptr);
// The same block for the beam's decoder rows (P16-packed y and x, the layer's
// position_ffn.py:27-40 at decoder/transformer.py:92): the d_ff walk split
// over nsplit workgroups per 128-row block (blockIdx.y), whose partial
// accumulators meet in an fp32 slab; the workgroup that draws a row block's
// last ticket sums them in split order (deterministic), adds nothing else
// (b2 and the residual are split 0's initial value) and writes x and the
// rows' exact statistics.  Row blocks whose chunks are all done (skip) exit.
struct DecFfn {
  int nsplit = 1;
  float* slab = nullptr;    // [row block][split][16 tiles][512 threads] f32x4
  int* tickets = nullptr;   // [row block], zero between launches
  const int* skip = nullptr;
  int skip_rpc = 1;
};
size_t dec_ffn_slab_floats(int M, int nsplit);
hipError_t launch_dec_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h,
                          float w2s, const float* b2, float* x, float* xpart, int M, int F, int* ovf,
                          const DecFfn& df, hipStream_t s);
// out[r] = LN(x[r]) (rows of 256)
hipError_t launch_layernorm(const float* x, const float* g, const float* b, float* out, int rows, hipStream_t s);

// ---- decoder -------------------------------------------------------------
// Layer 0's self-attention reads its row's q | k | v from a per-call table
// QKV0[step][token] (P16 [S * V, 768]; launch_dec_embed_table + one GEMM)
// instead of a per-step GEMM: its input LN(emb[tok] * 16 + pe[step]) takes
// only V values per step.  tok == nullptr: the per-step qkv matrix.
struct QkvRows {
  const int* tok = nullptr;  // row -> token of this step (steps > 0)
  int V = 0;
  int tok0 = 0;  // every row's step-0 token (BOS)
  // q | k | v (the table or the per-step matrix) row-major [rows][768]
  // instead of P16: a workgroup reads ONE row, which in P16 is 16 B of every
  // 128 B line (GemmArgs.c_rm)
  int rm = 0;
};
// rows s * V + v (s < S, v < V) of the layer-0 QKV table's input, P16, with
// one row-statistics partial per row; rows S * V .. rows_alloc - 1 zero
hipError_t launch_dec_embed_table(const float* emb, const float* pe, int V, int S, float* x, float* part, int rows_alloc,
                                  hipStream_t s);
struct DecStepArgs;
hipError_t launch_dec_embed(const int* tok, const float* emb, const float* pe, int step, float* x, float* part,
                            int R, hipStream_t s);
// self attention: writes k,v of this step into cache[slot=r][step], attends
// over the row's history cache[anc[r][t]][t] (anc == nullptr: identity).
// skip (nullable): per chunk (row / rpc), nonzero = finished, its rows do nothing.
// head (greedy, table mode, step > 0, no anc / skip): the workgroup of row r first
// runs the previous step's greedy head for r (its token is this step's input),
// so the standalone head kernel runs only after the last step
struct GreedyHead;
hipError_t launch_dec_self_attention(const float* qkv, float* cache, const int* anc, int anc_ld, int step,
                                     int max_steps, float* out, int R, hipStream_t s, int rpc = 1,
                                     const int* skip = nullptr, const QkvRows& qr = QkvRows(),
                                     const GreedyHead* head = nullptr, const int* clist = nullptr, int ccap = 0,
                                     bool q24 = false);
// q24: the cache holds 1600-B 24-bit rows (attention.hip SELF_Q24_ROW) instead of [512] floats
// context attention: rows r = c*rpc + j attend over ctxkv rows of chunk c
// (K at kv[(c*T+t)*ld + koff], V at +256), mask signal == pad_val, keys < span.
// q24: kv is the 24-bit image of launch_ctx_pack_q24 (ld, koff in bytes).
hipError_t launch_dec_ctx_attention(const float* q, const void* kv, int ld, int koff, const float* signal,
                                    const int* span, float pad_val, float* out, int C, int rpc, int T,
                                    hipStream_t s, unsigned long long* stamp = nullptr, float* attn_dbg = nullptr,
                                    size_t dbg_stride = 0, const int* skip = nullptr, bool q24 = false,
                                    const int* clist = nullptr, int ccap = 0, int nsplit = 1, float* part = nullptr);
// part: nsplit > 1 (with clist): scratch of ccap * nsplit * rpc * (256 + 16) floats
// --fast beam tail: clist (nullable) lists the chunks the self / context
// attention and the beam step run (ccap entries, -1 = none); launch_alive_list
// builds it from the done flags (*ovf = 1 when more than cap are alive)
hipError_t launch_alive_list(const int* done, int C, int* list, int cap, int* ovf, hipStream_t s);
// 24-bit context K/V (beam rows): per (key row, layer) CTXQ_ROW bytes = k's 256
// integers (3 bytes each, lane i's 12 bytes = dims 4i..4i+3) | v's | per head
// {k scale, v scale} (powers of two, f32).  Image [Ld][B*T][CTXQ_ROW] (layer-
// major: one layer's keys of a chunk are one contiguous 819 KB run, round 5)
// from the fp32 [B*T][ld] K/V (layer l at column l*512); rows t >= span not
// written.
#define CTXQ_V 768
#define CTXQ_S 1536
#define CTXQ_ROW 1600
hipError_t launch_ctx_pack_q24(const float* kv, int ld, int Ld, uint8_t* out, const int* span, int B, int T,
                               hipStream_t s);
// Next step's decoder input, written by the search kernel that picks the
// token (the embedding of step+1 fused into the head: one launch fewer per
// step): x[row] = emb[tok] (* 16 + pe[step+1] with position encoding) and
// its row statistics.  Skipped after the last step.
struct NextEmbed {
  const float* emb = nullptr;
  const float* pe = nullptr;  // null: no position encoding (and no sqrt(d) scale)
  float* x = nullptr;
  float* part = nullptr;
  int* tok = nullptr;  // optional: the row's token (the layer-0 QKV table's row index)
};
// memory-bank context attention (greedy, one row per chunk: rpc == 1):
// qp = Q' [C, 8*256] P16 (column block h = head h's 256-dim query in memory
// space), mem = row-major memory bank [C * ldT, 256] (chunk c's position t at
// row c*ldT + t, t < T <= ldT); out = U [C, 8*256] P16 (head h's
// softmax-weighted memory sum).
hipError_t launch_dec_mem_attention(const float* qp, const float* mem, const float* signal, const int* span,
                                    float pad_val, float* out, int C, int rpc, int T, int ldT, hipStream_t s,
                                    unsigned long long* stamp = nullptr, float* attn_dbg = nullptr,
                                    size_t dbg_stride = 0, int grid = 0);
// -attn_debug: raw head-0 score rows [B*S][T] (keys < span[c]) -> probabilities
hipError_t launch_attn_rows_softmax(float* a, const int* span, int B, int S, int T, hipStream_t s);
// stamp pairs (earliest start, latest end) <- (UINT64_MAX, 0)
hipError_t launch_stamp_reset(unsigned long long* stamps, int pairs, hipStream_t s);
// encoder output rows x[b*T+t] -> memory bank rows b*ldT+t, row-major (LN when
// ln_g; rows t >= T of each chunk zero)
// the 24-bit digit bank serves T in [1, 512] (the context's bank buffer holds 512 rows per chunk)
bool bank_eligible(int T, int ldT);
hipError_t launch_memory_pack(const float* x, const float* ln_g, const float* ln_b, float* out, int B, int T, int ldT,
                              hipStream_t s);
hipError_t init_mem_attributes();
// 24-bit fixed-point memory bank (bank8.hip): digits in bank (B * 512 * 256 * 3
// bytes), per-row scales kscale [B * 512], per-chunk biased max exponent kemax [B]
hipError_t launch_bank_pack_d8(const float* x, const float* ln_g, const float* ln_b, void* bank, float* kscale,
                               int* kemax, const int* span, int B, int T, int* ovf, hipStream_t s);
hipError_t launch_dec_bank_d8(const float* qp, const void* bank, const float* kscale, const int* kemax,
                              const float* signal, const int* span, float pad_val, float* out, int C, int T,
                              hipStream_t s, unsigned long long* stamp, float* attn_dbg, size_t dbg_stride, int* ovf,
                              bool nt = false, int grid = 0);
hipError_t init_bank8_attributes();
// signal front end (frontend.hip): per-read normalisation (method 0 none, 1
// median/MAD, 2 median/std; fp64 math, float32 out) of reads concatenated at
// off[0..R], and windowing of chunks (read, start, len) into a [C, T] batch
hipError_t launch_read_normalize(const double* raw, const long long* off, int R, int method, float* out,
                                 hipStream_t s);
hipError_t launch_read_window(const float* sig, const long long* off, const int* rd, const int* start,
                              const int* len, int C, int T, float* out, hipStream_t s);
// average self-attention (aan.hip): xn = LN_1(x), avg = (xn + step prev) / (step + 1)
// (prev from hist[anc[r][step-1]][step-1], avg stored at hist[r][step]), avg's
// row statistics (one partial); then q1 = sig(g_in) xn + sig(g_f) a + x (+ stats)
hipError_t launch_aan_prep(const float* x, const float* ln_g, const float* ln_b, float* hist, const int* anc,
                           int anc_ld, int step, int max_steps, float* xn, float* avg, float* avg_part, int R,
                           hipStream_t s);
hipError_t launch_aan_gate(const float* g, const float* xn, const float* a, const float* x, float* out, float* part,
                           int R, hipStream_t s);
// random sampling (translate/translator.py:371-394): temperature, top-k
// (-1: the full distribution), and the draw's seed (device word, so one
// captured graph serves every seed); temp == 0 or topk == 1 is argmax
struct Sampling {
  float temp = 1.f;
  int topk = 1;
  const unsigned long long* seed = nullptr;
};
// One greedy head (search.hip / head.hpp greedy_head_row): LN_dec ->
// generator -> log_softmax -> argmax (or a sample) for a row, its token into
// tok / out_tokens[row][step], score, optional logp dump [R][S][V], and the
// next step's embedded input (ne).  Run by greedy_head_kernel, or by the
// layer-0 self-attention of the next step (launch_dec_self_attention's head).
struct GreedyHead {
  const float* x = nullptr;
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
  const float* gw = nullptr;
  const float* gb = nullptr;
  int V = 0, S = 0, min_len = 0, eos = 0;
  int* tok = nullptr;
  int* out_tokens = nullptr;
  float* score = nullptr;
  float* logp_dump = nullptr;
  NextEmbed ne;
  Sampling smp;
};
GreedyHead make_greedy_head(const float* x, const float* ln_g, const float* ln_b, const float* gw, const float* gb,
                            int V, int S, int min_len, int eos, int* tok, int* out_tokens, float* score,
                            float* logp_dump, const NextEmbed& ne, const Sampling& smp);
hipError_t check_greedy_head(const GreedyHead& h);
// greedy head: LN_dec -> generator -> log_softmax -> argmax (or a sample);
// writes token (next input + output [R, S] at column step), score, optional
// logp dump, and the next step's embedded input (ne).
hipError_t launch_dec_greedy_head(const float* x, const float* ln_g, const float* ln_b, const float* gw,
                                  const float* gb, int V, int step, int S, int min_len, int eos, int* tok,
                                  int* out_tokens, float* score, float* logp_dump, const NextEmbed& ne, int R,
                                  hipStream_t s, const Sampling& smp = Sampling());

struct BeamState {
  float* cum;        // [C, beam] topk_log_probs
  int* seq[2];       // [C*beam, S] alive_seq (without BOS), double buffered
  int* anc[2];       // [C*beam, S] self-attn cache slot ancestry, double buffered
  int* tok;          // [C*beam] next decoder input
  int* done;         // [C]
  int* top_fin;      // [C]
  int* n_hyp;        // [C] hypotheses found so far
  float* hyp_score;  // [C, n_best]
  int* hyp_len;      // [C, n_best]
  int* hyp_tok;      // [C, n_best, S]
  int* n_alive;      // [1] chunks (classic: reference batches) not done
  int* steps_done;   // [1] decoder steps until the last chunk finished
  // classic onmt Beam (translate/translator.py:827-926): the reference batch
  // each chunk belongs to; a batch keeps advancing all of its beams until
  // every one of them is done
  int* group;        // [C] reference batch id
  int* grp_left;     // [C] chunks of the batch not done yet
  int* grp_done;     // [C] batch finished (its beams stop advancing)
  int* steps_run;    // [C] advance() calls made on the chunk's beam (--fast: the step count when it was dropped)
  int* hyp_anc;      // [C, n_best, S] decoder row that ran each step of the hypothesis (its attention rows)
  // classic Beam: GNMTGlobalScorer state (onmt/translate/beam.py:181-243) and n-gram blocking (:100-119)
  float* cov[2];     // [C*beam, T] coverage = sum of the hypothesis' attention rows, double buffered
  float* pen;        // [C*beam] cov_penalty(coverage) of the live beams (score(), sort_finished)
  float* prev_pen;   // [C*beam] global_state["prev_penalty"] (stepwise penalty)
  int* blk[2];       // [C*beam] the hypothesis repeats an n-gram, double buffered
  const float* attn; // [C*beam][S][T] head-0 context attention probabilities, null when not captured
  const int* cut;    // [C] attention length of the chunk's beams (memory_lengths[j], translator.py:902-907)
  int T;             // attention row stride
};
// classic Beam options (translate/translator.py:113-173, onmt/translate/beam.py, penalties.py)
struct ClassicOpts {
  int lp_kind;     // length penalty: 0 none, 1 wu, 2 avg
  float alpha;
  float beta;
  int cov_kind;    // coverage penalty: 0 none, 1 wu, 2 summary
  int stepwise;    // -stepwise_penalty
  int ngram;       // -block_ngram_repeat (0: off)
  unsigned excl;   // -ignore_when_blocking token ids as a bit mask
};
hipError_t launch_beam_init(const BeamState& st, int C, int beam, int n_best, int S, int bos, hipStream_t s);
hipError_t launch_beam_step(const NextEmbed& ne, const float* x, const float* ln_g, const float* ln_b, const float* gw, const float* gb,
                            int V, const BeamState& st, int C, int beam, int n_best, int step, int S, int min_len,
                            int eos, float lenpen, hipStream_t s, const int* clist = nullptr, int ccap = 0);
hipError_t launch_beam_finish(const BeamState& st, int C, int n_best, int S, int* tokens, float* scores, int* lens,
                              hipStream_t s);
// classic Beam: length_penalty 0 none, 1 wu, 2 avg (onmt/translate/penalties.py)
hipError_t launch_beam_classic_init(const BeamState& st, const int* group, int C, int beam, int bos, hipStream_t s);
hipError_t launch_beam_classic_step(const NextEmbed& ne, const float* x, const float* ln_g, const float* ln_b,
                                    const float* gw, const float* gb, int V, const BeamState& st, int C, int beam,
                                    int n_best, int step, int S, int min_len, int eos, const ClassicOpts& o,
                                    hipStream_t s);
hipError_t launch_beam_classic_finish(const BeamState& st, int C, int beam, int n_best, int S, const ClassicOpts& o,
                                      int* tokens, float* scores, int* lens, hipStream_t s);
// per-step softmax of the captured head-0 scores of R rows (row r belongs to
// chunk r / rpc; keys t < span), in place at a[r * ld + t], zero for t >= span
hipError_t launch_attn_step_softmax(float* a, size_t ld, const int* span, int R, int rpc, int T, hipStream_t s);
// attention of each hypothesis along its ancestry: out[c][k][t][:] =
// attn[hyp_anc[c][k][t]][t][:] for t < hyp_len[c][k], zero after
hipError_t launch_beam_attn_gather(const BeamState& st, int C, int n_best, int S, int max_len, int T, float* out,
                                   hipStream_t s);

}  // namespace nd
