/*
 * nanodec.h — C-ABI of libnanodec_hip.so, the MI355X (gfx950) engine for
 * NanoDecoder's translate path.
 *
 * The reference has no native boundary: its path is PyTorch modules driven by
 * translate/translator.py.  Each entry point below replaces the reference
 * interface named in its comment (file:line in achilles1989/NanoDecoder).
 * Plain pointers and sizes only; device pointers are HIP device memory owned
 * by the caller (PyTorch-ROCm tensors' data_ptr()).  Every function returns
 * 0 on success; on failure a nonzero ND_* code and a thread-local message in
 * nd_last_error().
 *
 * Threading: one context is bound to one device and must not be called
 * concurrently; every call sets the device first (the reference drives the
 * GPU from a multiprocessing.Pool result thread, translate.py:100-161).
 * All work is enqueued on the caller's stream; no hidden device-wide syncs.
 */
#ifndef NANODEC_H
#define NANODEC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ND_OK 0
#define ND_ERR_ARG 1      /* bad argument / shape / config */
#define ND_ERR_WEIGHT 2   /* unknown / missing / mis-shaped weight */
#define ND_ERR_HIP 3      /* HIP runtime error */
#define ND_ERR_STATE 4    /* call order (e.g. translate before finalize) */

#define ND_ENC_TRANSFORMER 0  /* encoder/transformer.py */
#define ND_ENC_NANO 1         /* encoder/nano_encoder.py (3x BiLSTM) */
#define ND_SELF_SCALED_DOT 0
#define ND_SELF_AVERAGE 1

typedef struct nd_ctx nd_ctx;

/* Architecture + capacity.  Mirrors the checkpoint ``opt`` the reference
 * builds its model from (models/model_builder.py:236-334). */
typedef struct nd_config {
  int32_t encoder_type;       /* ND_ENC_* */
  int32_t enc_layers;         /* 3 */
  int32_t dec_layers;         /* 3 */
  int32_t d_model;            /* 256 (only value compiled) */
  int32_t heads;              /* 8   (d_model / heads == 32) */
  int32_t d_ff;               /* 2048 (multiple of 128) */
  int32_t vocab;              /* |tgt vocab|, <= 32 */
  int32_t rnn_hidden;         /* 128 per direction (NanoEncoder) */
  int32_t position_encoding;  /* decoder sinusoidal PE (embeddings.py:36-43) */
  int32_t pad_idx, bos_idx, eos_idx;
  int32_t max_batch;          /* chunks per call */
  int32_t max_src_len;        /* 512 (src_seq_length) */
  int32_t max_steps;          /* max_length (100), at most 512 */
  int32_t max_beam;           /* beam_size upper bound (1 = greedy only) */
  int32_t device;             /* HIP device ordinal */
  int32_t self_attn_type;     /* decoder self-attention: ND_SELF_SCALED_DOT | ND_SELF_AVERAGE
                                 (decoder/transformer.py:33-37, onmt/modules/average_attn.py) */
} nd_config;

/* Replaces models/model_builder.py:load_test_model (:217-233) +
 * build_base_model (:236-382): allocate the engine for one device. */
int nd_create(const nd_config* cfg, nd_ctx** out);

/* Replaces model.load_state_dict (models/model_builder.py:356-357) for one
 * tensor.  ``name`` is the reference state-dict key (after the a_2/b_2 fix,
 * :345-353); generator keys are "generator.0.weight"/"generator.0.bias".
 * Unknown names and shape mismatches are errors (the reference's strict=False
 * silent fallback is deliberately NOT reproduced); decoder ``*.mask`` buffers
 * and BatchNorm ``num_batches_tracked`` are accepted and ignored. */
int nd_load_weight(nd_ctx* ctx, const char* name, const float* host, const int64_t* shape, int ndim);

/* Checks that every required weight was loaded and builds derived packed
 * weights.  Must be called once before any translate call.  The first call
 * also rebalances the decoder attentions' key / query and value / output
 * projections by exact powers of two per dimension (the model's function is
 * unchanged; a dimension far larger than the rest of its head would otherwise
 * cost the 24-bit K/V forms their bits); a weight loaded afterwards gets the
 * same scales. */
int nd_finalize(nd_ctx* ctx);

/* ctx (just created, no weight loaded, the same model configuration as src)
 * reads src's weights and every image nd_finalize derived from them instead
 * of holding its own; ctx is finalized by this call.  src must be finalized,
 * on the same device, and outlive ctx.  ND_ERR_STATE if a weight was loaded
 * into ctx; nd_load_weight on ctx afterwards returns ND_ERR_STATE.  ctx's own
 * raw weight buffers from nd_create stay allocated and unread.  For several contexts of one model on
 * one GPU (EnginePool lanes): one copy of the weights in the caches they
 * share (L2 per XCD, the Infinity Cache).  No reference counterpart (the
 * reference holds one model per process). */
int nd_share_weights(nd_ctx* ctx, const nd_ctx* src);

/* Greedy translate of a batch of chunks: encoder forward + max_len decoder
 * steps with argmax selection.  Replaces Translator.translate_batch ->
 * _translate_random_sampling (translate/translator.py:396-540) for
 * beam_size == 1 (keep_topk == 1): all max_len steps always run (no EOS
 * early exit, :455-483) and the score is the last step's top log-prob
 * (:491-499).
 *   d_signal  [B, T] f32 row-major, zero padded (make_nano, inputters/inputter.py:86-95)
 *   d_len     [B] i32 valid samples per chunk (src_lengths)
 *   d_span    [B] i32 padded length the reference batch would have had
 *             (= longest chunk of the reference batch; len <= span <= T).
 *             Positions >= span do not exist for that chunk.
 *   d_tokens  [B, max_len] i32 out;  d_score [B] f32 out
 *   d_logp    nullable [B, max_len, V] f32 out: per-step log-probs (pre min_len mask)
 *   stream    hipStream_t of the caller (void* here to keep HIP out of the ABI) */
int nd_translate_greedy(nd_ctx* ctx, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                        int32_t B, int32_t T, int32_t max_len, int32_t min_len,
                        int32_t* d_tokens, float* d_score, float* d_logp, void* stream);

/* Greedy decode that also returns -attn_debug attention (translate/
 * translator.py:285-336, return_attention at :396-503): d_attn [B, max_len, T]
 * = per step the last decoder layer's context attention of head 0
 * (attn["std"], onmt/modules/multi_headed_attn.py:187-192) over source
 * positions t < span (zero beyond).  Otherwise as nd_translate_greedy. */
int nd_translate_greedy_attn(nd_ctx* ctx, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                             int32_t B, int32_t T, int32_t max_len, int32_t min_len, int32_t* d_tokens, float* d_score,
                             float* d_logp, float* d_attn, void* stream);

/* Random sampling: Translator._translate_random_sampling with
 * sample_with_temperature (translate/translator.py:371-503).  Every step
 * draws the next token from softmax(log_probs / temp), restricted to the
 * keep_topk most likely tokens when keep_topk > 0 (the others set to -10000);
 * the score is the tempered (masked) value of the drawn token.  temp == 0 or
 * keep_topk == 1 is the argmax of nd_translate_greedy.  The draws come from a
 * counter-based generator keyed by (seed, chunk, step): equal seeds give
 * equal outputs (the reference draws from torch's global generator).
 * Outputs as nd_translate_greedy; d_attn nullable as nd_translate_greedy_attn. */
int nd_translate_sample(nd_ctx* ctx, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B,
                        int32_t T, int32_t max_len, int32_t min_len, float temp, int32_t keep_topk, uint64_t seed,
                        int32_t* d_tokens, float* d_score, float* d_logp, float* d_attn, void* stream);

/* --fast beam search.  Replaces Translator._fast_translate_batch
 * (translate/translator.py:619-825) with GNMTGlobalScorer.alpha
 * (onmt/translate/beam.py:181-199; beta must be 0).  Per chunk the n_best
 * finished hypotheses, best first:
 *   d_tokens [B, n_best, max_len] i32 (EOS included when emitted; -1 padded)
 *   d_scores [B, n_best] f32, d_lens [B, n_best] i32
 *   d_steps  nullable [1] i32: decoder steps actually executed */
int nd_translate_beam(nd_ctx* ctx, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                      int32_t B, int32_t T, int32_t beam, int32_t n_best, float alpha, int32_t max_len,
                      int32_t min_len, int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps,
                      void* stream);

/* Classic beam search: replaces Translator._translate_batch with the onmt
 * Beam (translate/translator.py:827-926, onmt/translate/beam.py:6-199; the
 * path the reference takes for beam_size > 1 without --fast).  d_group [B]
 * is the reference batch of every chunk (translate() batches batch_size
 * consecutive chunks of one read): a batch advances all its beams until each
 * is done, exactly as the reference loop does, however the chunks are packed
 * into this call.  length_penalty: 0 none, 1 wu, 2 avg (alpha for wu);
 * coverage penalty none.  Outputs as nd_translate_beam: tokens [B, n_best,
 * max_len] (-1 padded, EOS included when the hypothesis finished), scores
 * and lens [B, n_best]; d_steps (nullable) = steps run. */
int nd_translate_beam_classic(nd_ctx* ctx, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                              const int32_t* d_group, int32_t B, int32_t T, int32_t beam, int32_t n_best,
                              int32_t length_penalty, float alpha, int32_t max_len, int32_t min_len,
                              int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps, void* stream);

/* --fast beam search with -attn_debug (translate/translator.py:745-751,
 * :780-790): as nd_translate_beam, plus
 *   d_attn      [B, n_best, max_len, T] f32: row t of hypothesis k = the
 *               last layer's head-0 context attention of the decoder row
 *               that produced its token t (probabilities over keys < span,
 *               zero after), zero rows past the hypothesis length
 *   d_done_step [B] i32: the number of steps the chunk ran before it was
 *               dropped as finished (the caller derives the reference's
 *               memory_lengths[i] cut from the alive set of each step) */
int nd_translate_beam_attn(nd_ctx* ctx, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                           int32_t B, int32_t T, int32_t beam, int32_t n_best, float alpha, int32_t max_len,
                           int32_t min_len, int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps,
                           float* d_attn, int32_t* d_done_step, void* stream);

/* Options of the classic onmt Beam (translate/translator.py:127-173,
 * onmt/translate/beam.py:6-243, onmt/translate/penalties.py). */
typedef struct nd_classic_opts {
  int32_t length_penalty;     /* 0 none, 1 wu, 2 avg */
  float alpha;                /* -alpha */
  float beta;                 /* -beta (coverage weight) */
  int32_t coverage_penalty;   /* 0 none, 1 wu, 2 summary */
  int32_t stepwise_penalty;   /* -stepwise_penalty */
  int32_t block_ngram_repeat; /* -block_ngram_repeat (0: off) */
  uint32_t ignore_mask;       /* -ignore_when_blocking: bit i = token id i */
} nd_classic_opts;

/* Classic beam search with the full option set: as nd_translate_beam_classic,
 * plus coverage penalties (wu / summary, at scoring time or stepwise) and
 * n-gram blocking, and optionally the hypotheses' attention.
 *   d_cut  [B] i32, required when coverage_penalty != 0: the attention length
 *          of the chunk's beams, memory_lengths[j] as the reference indexes
 *          its beam-tiled lengths (translate/translator.py:902-907)
 *   d_attn nullable [B, n_best, max_len, T] f32: as nd_translate_beam_attn
 * With coverage_penalty != 0 the attention is captured every step whether or
 * not d_attn is given. */
int nd_translate_beam_classic_ex(nd_ctx* ctx, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                                 const int32_t* d_group, const int32_t* d_cut, int32_t B, int32_t T, int32_t beam,
                                 int32_t n_best, const nd_classic_opts* opts, int32_t max_len, int32_t min_len,
                                 int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps, float* d_attn,
                                 void* stream);

/* Signal front end (utils/labelop.py:194-243, extract_fast5_raw): R raw
 * reads concatenated in d_raw (float64, read r at d_offsets[r] ..
 * d_offsets[r+1]) normalised per read into d_out (float32, same offsets).
 * method: 0 none, 1 median (x - median) / MAD with statsmodels' robust.mad
 * (median(|x - median| / 0.6744897501960817)), 2 mean ((x - median) / std,
 * as the reference centres it).  fp64 arithmetic and exact medians, so the
 * float32 chunks equal the reference's (method 2: within 1 ulp, the std is a
 * reduction).  No context needed. */
int nd_normalize_reads(const double* d_raw, const int64_t* d_offsets, int32_t R, int32_t method, float* d_out,
                       void* stream);

/* Windowing (utils/labelop.py:225-233) straight into a signal batch: chunk c
 * = d_len[c] samples of read d_read[c] from d_start[c], zero padded to T, is
 * row c of d_signal [C, T].  The caller lists the windows (stride, length). */
int nd_window_reads(const float* d_sig, const int64_t* d_offsets, const int32_t* d_read, const int32_t* d_start,
                    const int32_t* d_len, int32_t C, int32_t T, float* d_signal, void* stream);

/* Encoder forward only; writes the memory bank [B, T, d_model] (rows
 * t >= span are unspecified).  Replaces Translator._run_encoder
 * (translate/translator.py:542-559).  Used by parity tests. */
int nd_encode(nd_ctx* ctx, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B,
              int32_t T, float* d_memory, void* stream);

/* The context's own HIP stream (non-blocking; the translate graphs run on
 * it).  A caller that enqueues its inputs and reads
 * its outputs on this stream needs no cross-stream join per call. */
void* nd_stream(nd_ctx* ctx);

/* Enables/disables hipGraph capture of the translate calls (default on). */
int nd_set_graphs(nd_ctx* ctx, int enable);

/* Context-attention form: 0 (default) = the memory-bank form for greedy
 * decoding (ctx K/V projections folded into the query / output GEMMs, one
 * shared 256-float memory row per source position) and the per-layer K/V
 * form for beam search; 1 = the K/V form always.  Same results to fp32
 * rounding; replaces decoder/transformer.py:82-86 + multi_headed_attn.py:
 * 142-177's context path. */
int nd_set_ctx_path(nd_ctx* ctx, int path);

/* Arithmetic of the products: 0 (default) = split-fp16 (each fp32 operand as
 * an fp16 hi/lo pair, 22 significant bits, three fp16 MFMA products summed in
 * fp32 accumulators); 1 = exact fp32 (fp32-MFMA kernels for every GEMM, the
 * encoder attention and the BiLSTM recurrence), the reference's own fp32
 * arithmetic (nn.Linear / bmm in fp32).  Default from ND_GEMM_F32.  The
 * captured graphs of both forms are kept (keyed by it). */
int nd_set_exact_fp32(nd_ctx* ctx, int enable);

/* Cache policy of the greedy memory bank: nontemporal != 0 streams it with
 * non-temporal loads (it then does not stay in the Infinity Cache).  For
 * several contexts on one GPU (EnginePool) whose banks together exceed the
 * cache.  Default 0.  No reference counterpart. */
int nd_set_bank_policy(nd_ctx* ctx, int nontemporal);

/* Workgroups of the greedy memory-bank kernel at most: 0 (default) = one per
 * chunk, i.e. every CU while it streams; n > 0 = n workgroups walking the
 * chunks.  The kernel holds 137 KB of a CU's 160 KB LDS, so while it runs no
 * other context's LDS-staged GEMM fits beside it; EnginePool lanes cap it at
 * half the CUs (measured, 3 lanes x 256 chunks: 18.3 -> 17.6 ms per call).
 * Same results (each chunk is one workgroup's work either way).  No reference
 * counterpart. */
int nd_set_bank_grid(nd_ctx* ctx, int32_t workgroups);

/* The decoder step's K = 2048 products (W_vo, FFN2 at 256 rows) split over
 * workgroups (gemm_p16k_kernel, partial slabs + arrival tickets) instead of
 * one workgroup per output tile.  Default 0 (off): a lone call is faster
 * without; several calls in flight (EnginePool lanes) gain from it (DESIGN.md
 * section 3).  Results differ from the unsplit kernel's in fp32 rounding of
 * the K sum only.  No reference counterpart. */
int nd_set_gemm_splitk(nd_ctx* ctx, int32_t on);

/* Split-fp16 range guard.  An activation operand the split form carries as
 * fp16 hi/lo leaves the fp16 range from |x| = 65504 on, where the
 * reference's fp32 arithmetic is still finite.  Every kernel that splits an
 * activation it does not normalise itself (GEMMs without a LayerNorm
 * prologue, the encoder attention's Q/K/V) raises the context's overflow
 * word when it sees one.  nd_take_overflow enqueues, on `stream`, a copy of
 * that word to d_out (one int32: nonzero = some product of the calls
 * enqueued since the last take saw an out-of-range operand) and clears it.
 * Call it right after each translate call, as the Python Translator does,
 * and rerun a flagged call after nd_set_exact_fp32(ctx, 1).  No reference
 * counterpart: the reference computes in fp32 (nn.Linear / bmm). */
int nd_take_overflow(nd_ctx* ctx, int32_t* d_out, void* stream);

/* Launch-duration stamps of the decoder's context attention (the bench's
 * roofline kernel: dec_mem_attention_kernel for greedy, dec_ctx_attention_kernel
 * for beam), taken inside the kernels with the constant-rate wall clock while
 * enable != 0 (part of the captured graphs, so they time graph replays).
 * nd_kernel_stamps waits for the context's stream and returns the mean
 * duration (first workgroup start to last workgroup end) of the launches of
 * the last call. */
int nd_set_kernel_stamps(nd_ctx* c, int enable);
int nd_kernel_stamps(nd_ctx* c, float* avg_us, int32_t* launches);

/* Kernel statistics of the last translate call (ms of device time per
 * phase, measured with HIP events on the engine stream when enabled). */
int nd_set_timing(nd_ctx* ctx, int enable);
int nd_last_timing(nd_ctx* ctx, float* encode_ms, float* decode_ms);

void nd_destroy(nd_ctx* ctx);
const char* nd_last_error(void);
const char* nd_version(void);

/* ---- diagnostics (no reference counterpart) ----------------------------- */

/* GEMM kernel routes, counted per process each time a GEMM is enqueued (a
 * graph capture enqueues once; replays are not counted).  Lets a test check
 * which kernels a workload of a given size runs (gemm.hip launch_gemm_p16 /
 * launch_gemm pick the kernel from M, N, K). */
#define ND_ROUTE_P16_SMALL 0   /* gemm_p16_kernel<1,4,64>  (K = 256, few row blocks) */
#define ND_ROUTE_P16_N64 1     /* gemm_p16_kernel<4,2,128> (K = 256) */
#define ND_ROUTE_P16_LN128 2   /* gemm_p16_kernel<8,1,256> (K = 256, LN prologue) */
#define ND_ROUTE_P16S_2X4 3    /* gemm_p16s_kernel<2,4>    (K = 256, LDS-staged, 32-row blocks) */
#define ND_ROUTE_P16S_2X2 4    /* gemm_p16s_kernel<2,2> */
#define ND_ROUTE_P16_LONGK 5   /* gemm_p16_kernel<1,8,*>   (K = 512 / 1024 / 2048) */
#define ND_ROUTE_P16_BIG 6     /* P16 operands on the LDS-tiled row-major kernel (large M) */
#define ND_ROUTE_TILE256 7     /* gemm_f32_kernel 256x256 tiles */
#define ND_ROUTE_TILE128 8     /* gemm_f32_kernel 128x128 tiles */
#define ND_ROUTE_TILE64 9      /* gemm_f32_kernel 64x64 tiles */
#define ND_ROUTE_P16_SPLITK 10 /* gemm_p16k_kernel (K = 1024 / 2048, 32 x 32 tiles split over K, 128 < M) */
#define ND_ROUTE_N 11
/* counts[0 .. min(n, ND_ROUTE_N) - 1] <- launches per route since the last
 * reset; reset != 0 zeroes the counters afterwards. */
int nd_gemm_routes(int64_t* counts, int32_t n, int32_t reset);

/* The library's run-time switches (ND_* environment variables read by the
 * kernels' launchers, A/B timing knobs): writes "NAME=value" pairs separated
 * by ';' for every switch whose environment value differs from its default
 * into buf (NUL-terminated, truncated to len) and returns their number. */
int nd_switches(char* buf, int32_t len);

/* ---- op-level entry points (unit tests of individual kernels) ---------- */

/* C[M,N] = epilogue(prologue(A)[M,K] . W[N,K]^T + bias):
 * prologue row normalisation (A - mean) / sqrt(var + 1e-6) over K when
 * norm != 0 (a LayerNorm whose affine was folded into W / bias by
 * nd_op_fold_layernorm); relu when relu != 0; + R[M,N] when R != NULL.
 * All fp32, row-major, dense.  Replaces nn.Linear (+ the LayerNorm before it):
 * onmt/modules/multi_headed_attn.py:155-157, onmt/modules/position_ffn.py:38-40,
 * decoder/transformer.py:75,88, encoder/transformer.py:50. */
int nd_op_gemm(const float* A, const float* W, const float* bias, const float* R, float* C, int32_t M,
               int32_t N, int32_t K, int32_t norm, int32_t relu, void* stream);

/* Split-fp16 image of a weight for nd_op_gemm_split (the engine's encoder
 * GEMMs): Wh [N][K/8][hi 8 | lo 8] fp16 halves of W * 2^s with hi = fp16(x),
 * lo = fp16(x - hi); *wscale receives 2^-s.  K % 32 == 0.  Synchronises the
 * stream (load-time operation). */
int nd_op_split_weight(const float* W, int32_t N, int32_t K, uint16_t* Wh, float* wscale, void* stream);

/* nd_op_gemm on a split weight: A is split the same way as it is staged and
 * the product summed as hi*hi + hi*lo + lo*hi on fp16 MFMAs with fp32
 * accumulation (22-bit operands; fp32-class results). */
int nd_op_gemm_split(const float* A, const uint16_t* Wh, float wscale, const float* bias, const float* R, float* C,
                     int32_t M, int32_t N, int32_t K, int32_t norm, int32_t relu, void* stream);

/* The decoder-step form of the same GEMM, on the fragment-packed "P16"
 * layout the engine keeps decoder activations and step weights in: an
 * [M, N] matrix (M, N multiples of 16) stored as 16x16 blocks in row-major
 * block order, each block 64 float4 entries, entry e = (m%16) + 16*((n%16)/4)
 * holding columns n&~3..+3 of row m (nd_op_pack_p16 converts).  A, W, R, C
 * packed.  LayerNorm prologue when part_in != NULL: per-row partial
 * statistics {mean_j, M2_j} of part_n_in equal column tiles at
 * part_in[(row*16 + j)*2]; part_out (nullable, N == 256) receives this
 * GEMM's output row partials, their count in *part_n_out. */
int nd_op_gemm_p16(const float* A, const float* W, const float* bias, const float* R, float* C, int32_t M,
                   int32_t N, int32_t K, const float* part_in, int32_t part_n_in, float* part_out, int32_t relu,
                   int32_t* part_n_out, void* stream);

/* Split-fp16 decoder-step GEMM: W as its P16H image (nd_op_pack_p16h:
 * [N/16][K/32][hi | lo][64 lanes][8 halves] of W * 2^s, *wscale = 2^-s from
 * a row-major W [N, K]; synchronises the stream), A split on the fly, the
 * product hi*hi + hi*lo + lo*hi on 16x16x32 f16 MFMAs into fp32.  Otherwise
 * exactly nd_op_gemm_p16. */
int nd_op_pack_p16h(const float* W, int32_t N, int32_t K, uint16_t* out, float* wscale, void* stream);
/* The encoder's fused position-wise FFN block (onmt/modules/position_ffn.py:
 * 27-40 as encoder/transformer.py:36-54 runs it): x = y + W2 relu(W1' LN(y)
 * + b1') + b2 over M rows of 256, y and x row-major [M, 256] (x != y), with
 * the LayerNorm affine folded into W1' / b1' (nd_op_fold_layernorm).  w1h /
 * w2h: P16H images (nd_op_pack_p16h) of W1' [F, 256] and W2 [256, F] with
 * their scales; F % 32 == 0, F <= 2048.  xpart (nullable) gets each row's
 * {mean, M2} at xpart[row * 32]; overflow (nullable) is set to 1 when a
 * hidden value leaves the fp16 range. */
int nd_op_enc_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h, float w2s,
                  const float* b2, float* x, float* xpart, int32_t M, int32_t F, int32_t* overflow, void* stream);
/* The same block over the beam's decoder rows (decoder/transformer.py:92,
 * position_ffn.py:27-40): y and x P16-packed [M, 256] (M % 16 == 0, x != y),
 * the d_ff walk split over nsplit workgroups per 128-row block whose partial
 * sums meet in slab (nd_op_dec_ffn_slab_floats(M, nsplit) floats) and are
 * added in split order by the block's last workgroup (tickets: one int per
 * row block, zero before the launch and zero again after it).  skip
 * (nullable): per chunk of skip_rpc rows, nonzero = finished; a row block of
 * finished chunks is left as it was.  xpart: each row's {mean, M2} in one
 * partial.  Replaces the FFN1 + FFN2 GEMM pair of nd_translate_beam*'s step. */
int nd_op_dec_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h, float w2s,
                  const float* b2, float* x, float* xpart, int32_t M, int32_t F, int32_t nsplit, float* slab,
                  int32_t* tickets, const int32_t* skip, int32_t skip_rpc, int32_t* overflow, void* stream);
int64_t nd_op_dec_ffn_slab_floats(int32_t M, int32_t nsplit);
/* The same block with the attention's output projection folded in front
 * (encoder/transformer.py:45-54, one launch for the rest of the layer):
 * y = x_in + att Wo^T + bo, then x = y + W2 relu(W1' LN(y) + b1') + b2.
 * woh: P16H image of Wo [256, 256] with its scale wos.  x may alias x_in
 * (the engine updates the layer's rows in place); att must not.  With qkvh
 * (nullable) the next layer's projection follows in the same launch:
 * qkv = LN(x) Wq'^T + qkvb (row-major [M, 768]; qkvh the P16H image of the
 * LN-folded Wq' [768, 256], qkvs its scale). */
int nd_op_enc_ffn_wo(const float* att, const float* x_in, const uint16_t* woh, float wos, const float* bo,
                     const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h, float w2s, const float* b2,
                     float* x, float* xpart, const uint16_t* qkvh, float qkvs, const float* qkvb, float* qkv,
                     int32_t M, int32_t F, int32_t* overflow, void* stream);

int nd_op_gemm_p16_split(const float* A, const uint16_t* Wh, float wscale, const float* bias, const float* R, float* C,
                         int32_t M, int32_t N, int32_t K, const float* part_in, int32_t part_n_in, float* part_out,
                         int32_t relu, int32_t* part_n_out, void* stream);
/* The split-K form of the long-K decoder products (gemm_p16k_kernel: 32 x 32
 * tiles, K / 512 slices over workgroups, the slices summed in slice order by
 * the last arriving workgroup; the engine's route for W_vo and FFN2 at
 * 128 < rows <= 1024; decoder/transformer.py:88-93, position_ffn.py:38-40):
 * operands as nd_op_gemm_p16_split (no LN, no relu).  slab: >= tiles * 4096
 * floats; tickets: >= tiles int32, zero before the first call (each tile's
 * last arriver resets its own); tiles >= ceil(M / 32) * N / 32.  Fails if the
 * route is not taken. */
int nd_op_gemm_p16_splitk(const float* A, const uint16_t* Wh, float wscale, const float* bias, const float* R,
                          float* C, int32_t M, int32_t N, int32_t K, float* part_out, float* slab, int32_t* tickets,
                          int32_t tiles, int32_t* part_n_out, void* stream);

/* The same split-K route in exact fp32 (nd_set_exact_fp32: the pool lanes'
 * form of W_vo / FFN2 there): W is the fp32 weight [N, K] in the P16 layout
 * (as A), products on v_mfma_f32_16x16x4f32, no weight scale. */
int nd_op_gemm_p16_splitk_f32(const float* A, const float* W, const float* bias, const float* R, float* C,
                              int32_t M, int32_t N, int32_t K, float* part_out, float* slab, int32_t* tickets,
                              int32_t tiles, int32_t* part_n_out, void* stream);

/* The same GEMM with the weight's row-major split image too (nd_op_split_weight
 * of the row-major W): from M >= 2048 rows (beam search over large batches)
 * the engine runs it on the LDS-tiled kernel with P16 operands. */
int nd_op_gemm_p16_split_rm(const float* A, const uint16_t* Wh, float wscale, const uint16_t* Wh_rm, float wscale_rm,
                            const float* bias, const float* R, float* C, int32_t M, int32_t N, int32_t K,
                            const float* part_in, int32_t part_n_in, float* part_out, int32_t relu,
                            int32_t* part_n_out, void* stream);

/* row-major [M, N] -> P16 packed (M, N multiples of 16). */
int nd_op_pack_p16(const float* src, float* dst, int32_t M, int32_t N, void* stream);

/* Fold a LayerNorm's affine into the Linear that consumes it:
 * W_out = W diag(ln_g), b_out = bias + W ln_b (bias may be NULL), so that
 * Linear(LayerNorm(x)) == nd_op_gemm(x, W_out, b_out, norm = 1).  W [N,K]. */
int nd_op_fold_layernorm(const float* W, const float* bias, const float* ln_g, const float* ln_b, float* W_out,
                         float* b_out, int32_t N, int32_t K, void* stream);

/* Encoder self-attention over qkv [B*T, 3*d] (q | k | v) with the key mask
 * signal == 0.0 and keys >= span excluded; out [B*T, d]. */
int nd_op_enc_attention(const float* qkv, const float* signal, const int32_t* span, float* out, int32_t B,
                        int32_t T, void* stream);

/* Decoder self-attention for one step (multi_headed_attn.py:124-141):
 * qkv [R, 3*d] and out [R, d] P16-packed (R padded to a multiple of 16);
 * cache [R, max_steps, 2*d] row-major (this step's k|v is appended at
 * [r][step]); anc nullable [R, anc_ld] slot ancestry (NULL = identity). */
int nd_op_dec_self_attention(const float* qkv, float* cache, const int32_t* anc, int32_t anc_ld, int32_t step,
                             int32_t max_steps, float* out, int32_t R, void* stream);
/* The same for beam rows, rpc (2..6) consecutive rows per chunk (R a
 * multiple of rpc) on the chunk-per-workgroup kernel the engine runs for
 * them: anc [R, anc_ld] required (each row's slots), done nullable [R / rpc]
 * (rows of chunks with done != 0 untouched, translate/translator.py:793-823). */
int nd_op_dec_self_attention_beam(const float* qkv, float* cache, const int32_t* anc, int32_t anc_ld, int32_t step,
                                  int32_t max_steps, float* out, int32_t R, int32_t rpc, const int32_t* done,
                                  void* stream);
/* The engine's form for beam rows outside exact fp32 (greedy rows keep the fp32 history above): the
 * cache holds each (slot, t) as 1600 bytes, k's 256 values as 24-bit
 * integers | v's | per head {k scale, v scale} (the layout of
 * nd_op_ctx_pack_q24's rows), [R, max_steps, 1600] bytes; this step's k|v
 * is quantised and appended.  rpc 1: the per-row kernel (anc nullable), 2..6:
 * the chunk kernel (anc required). */
int nd_op_dec_self_attention_q24(const float* qkv, void* cache, const int32_t* anc, int32_t anc_ld, int32_t step,
                                 int32_t max_steps, float* out, int32_t R, int32_t rpc, const int32_t* done,
                                 void* stream);

/* Memory-bank context attention (greedy form, engine.hip
 * derive_memory_bank_weights; replaces the context MultiHeadedAttention of
 * decoder/transformer.py:88-92 for one row per chunk, rpc == 1): row c of
 * qp = Q' [C, 8*256] (P16; column block h = head h's query mapped into
 * memory space) attends over the row-major memory bank mem (chunk c's
 * position t at row c*ldT + t, T <= ldT) with keys t < span[c] and key mask
 * signal[c*T+t] == pad_val; out = U [C, 8*256] P16 (head h: the
 * softmax-weighted sum of memory rows).  grid > 0: that many workgroups walk
 * the chunks (the form nd_set_bank_grid selects for pool lanes). */
int nd_op_dec_mem_attention(const float* qp, const float* mem, const float* signal, const int32_t* span, float pad_val,
                            float* out, int32_t C, int32_t rpc, int32_t T, int32_t ldT, int32_t grid, void* stream);

/* One NanoEncoder BiLSTM layer, both directions (encoder/nano_encoder.py:92-111,
 * nn.LSTM(in, 128, bidirectional) over packed sequences): out [B*T, 256]
 * (fwd | bwd per row b*T + t) for t < len[b]; rows t >= len[b] are left as
 * the caller set them (pad_packed_sequence zeros).  layer0 != 0: input_size
 * 1, xp unused, the projection signal[b*T+t] * wih0[dir][g] + bsum[dir][g]
 * ([2][512] each) is formed in-kernel; otherwise xp [B*T, 1024] holds
 * x W_ih^T + b_ih + b_hh (fwd | bwd).  whh [2][512][128] (gates i, f, g, o).
 * bn_scale/bn_shift ([2][128], nullable): eval BatchNorm applied to the
 * written h. */
int nd_op_lstm_layer(const float* xp, const float* signal, const float* wih0, const float* bsum, const float* whh,
                     const int32_t* len, int32_t B, int32_t T, float* out, const float* bn_scale,
                     const float* bn_shift, int32_t layer0, void* stream);

/* Encoder output x [B*T, 256] row-major -> memory bank, row-major with ldT
 * rows per chunk (LayerNorm with ln_g/ln_b when ln_g != NULL,
 * encoder/transformer.py:125; rows t >= T zero). */
int nd_op_memory_pack(const float* x, const float* ln_g, const float* ln_b, float* out, int32_t B, int32_t T,
                      int32_t ldT, void* stream);

/* 24-bit fixed-point memory bank (the greedy decoder's context attention at
 * every chunk length T <= 512; multi_headed_attn.py:142-177 in the memory-bank form of
 * nd_op_dec_mem_attention).  nd_op_bank_pack_d8: x [B*T, 256] row-major -> the
 * digit bank (B x 512 rows; every row t as s_t times an integer of at most
 * 126 * 2^16 in magnitude in three signed 8-bit digit planes, B * 512 * 256 *
 * 3 bytes in the v_mfma_i32_16x16x64_i8 A-operand fragment order), kscale
 * [B * 512] floats (s_t) and kemax [B] (each chunk's largest s_t, float bits);
 * LayerNorm with ln_g/ln_b when set; rows t >= T, and rows t >= span[c] when
 * span (nullable, [B]) is given, zero with scale 0 (the engine passes the
 * call's spans: rows past a chunk's span are never attended and must not set
 * its largest scale).  nd_op_dec_bank_d8: qp [C, 2048] ROW-MAJOR (one row
 * per chunk), T in [1, 512] (the first ceil(T / 128) key blocks of each wave
 * streamed); out U [C16, 2048] P16.  grid: workgroups at
 * most (0 = one per chunk; fewer walk the chunks, as nd_set_bank_grid).  ovf
 * (nullable): set to 1 on a non-finite operand. */
int nd_op_bank_pack_d8(const float* x, const float* ln_g, const float* ln_b, void* bank, float* kscale,
                       int32_t* kemax, const int32_t* span, int32_t B, int32_t T, int32_t* ovf, void* stream);
int nd_op_dec_bank_d8(const float* qp, const void* bank, const float* kscale, const int32_t* kemax,
                      const float* signal, const int32_t* span, float pad_val, float* out, int32_t C, int32_t T,
                      int32_t* ovf, int32_t grid, void* stream);

/* Which memory bank the context's last call streamed (diagnostics, the
 * bench's roofline accounting): 0 fp32 bank, or fp32 K/V (a beam call in
 * exact fp32), 2 24-bit digits (nd_op_dec_bank_d8), 3 the 24-bit context K/V
 * of a beam call (nd_op_dec_ctx_attention_q24).  (1, the split-fp16 bank of
 * rounds 2-3, is retired.) */
int nd_bank_form(nd_ctx* ctx);

/* Decoder context attention (multi_headed_attn.py:142-177): rows r = c*rpc+j
 * of q [C*rpc, d] attend over K at kv[(c*T+t)*ld + koff] and V at +d, keys
 * t < span[c], key mask signal == pad_val; out [C*rpc, d].  q and out are
 * P16-packed (rows padded to a multiple of 16), kv row-major. */
int nd_op_dec_ctx_attention(const float* q, const float* kv, int32_t ld, int32_t koff, const float* signal,
                            const int32_t* span, float pad_val, float* out, int32_t C, int32_t rpc, int32_t T,
                            void* stream);

/* The beam's context K/V in 24-bit fixed point (the default for beam rows
 * outside exact fp32; the same attention as nd_op_dec_ctx_attention,
 * multi_headed_attn.py:142-177, on 0.78x the bytes).  nd_op_ctx_pack_q24:
 * fp32 K/V kv [B*T, ld] (layer l's k at column l*512, v at l*512+256; the
 * reference's linear_keys / linear_values outputs, multi_headed_attn.py:
 * 142-150) -> image out [layers][B*T][1600 B] (layer-major: one layer's
 * keys of a chunk are contiguous): per (layer, key) k's 256
 * values as 24-bit integers (3 bytes each; the 12 bytes at 12*i hold dims
 * 4i..4i+3), v's at byte 768, then per head h {2^(e_k - 23), 2^(e_v - 23)}
 * as floats at byte 1536 + 8h, with e the head's exponent (max|x| < 2^e); an
 * element's error is at most 2^-23 of its head's largest |x|.  Rows t >=
 * span[c] are not written.  nd_op_dec_ctx_attention_q24: as
 * nd_op_dec_ctx_attention with K/V of layer `layer` from that image (C*T
 * rows per layer plane). */
int nd_op_ctx_pack_q24(const float* kv, int32_t ld, int32_t layers, void* out, const int32_t* span, int32_t B,
                       int32_t T, void* stream);
/* The engine's form: the memory's K / V projection (split-fp16, as
 * nd_op_gemm_split, N = layers * 512) whose epilogue writes that image
 * (layer planes of plane_rows >= M rows) instead of fp32 K / V; every row
 * is written. */
int nd_op_gemm_split_q24(const float* A, const uint16_t* Wh, float wscale, const float* bias, void* img,
                         int32_t plane_rows, int32_t M, int32_t N, int32_t K, int32_t norm, void* stream);
int nd_op_dec_ctx_attention_q24(const float* q, const void* kvq, int32_t layers, int32_t layer, const float* signal,
                                const int32_t* span, float pad_val, float* out, int32_t C, int32_t rpc, int32_t T,
                                void* stream);

/* The --fast beam tail's forms (translate/translator.py:793-823 drops
 * finished batches; the engine launches over the alive chunks only once at
 * most a sixteenth of them remain).  nd_op_alive_list: chunks c < C with
 * done[c] == 0, ascending, into list[0 .. cap), the rest -1; more than cap
 * alive sets *ovf (nullable) to 1.  nd_op_dec_ctx_attention_list: the context
 * attention (fp32 K/V, or one layer plane of the 24-bit image when q24 != 0,
 * ld = 1600 and koff = 0 bytes) for the listed chunks only (list entries -1 and chunks with done[c]
 * != 0 untouched), each chunk's keys in nsplit workgroups (1..64) whose
 * partial softmax states go to part (ccap * nsplit * rpc * 272 floats) and
 * are combined by a second launch. */
int nd_op_alive_list(const int32_t* done, int32_t C, int32_t* list, int32_t cap, int32_t* ovf, void* stream);
int nd_op_dec_ctx_attention_list(const float* q, const void* kv, int32_t ld, int32_t koff, int32_t q24,
                                 const float* signal, const int32_t* span, float pad_val, float* out, int32_t C,
                                 int32_t rpc, int32_t T, const int32_t* clist, int32_t ccap, int32_t nsplit,
                                 float* part, const int32_t* done, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NANODEC_H */
