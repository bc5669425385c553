// libnanodec_hip.so — engine context, weight registry, launch sequences,
// hipGraph capture and the C-ABI of include/nanodec.h.
//
// One nd_ctx per device.  It owns:
//   * the packed fp32 weights (QKV of each attention fused into one [768,256]
//     matrix; the three decoder layers' context K/V projections fused into one
//     [3*512, 256] matrix so the memory bank is projected by ONE GEMM),
//   * encoder/decoder workspaces sized for (max_batch, max_src_len,
//     max_steps, max_beam),
//   * instantiated hipGraphs of whole translate calls, keyed by shape.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/nanodec.h"
#include "common.hpp"
#include "kernels.hpp"

namespace nd {
hipError_t init_kernel_attributes();
hipError_t launch_fill_i32(int* p, int v, int n, hipStream_t s);
}  // namespace nd

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      return fail(ND_ERR_HIP, std::string(#expr) + " failed: " + hipGetErrorString(e_));      \
  } while (0)

struct Slot {
  float* dst = nullptr;
  std::vector<int64_t> shape;  // expected shape
  size_t numel = 0;
  bool loaded = false;
  bool required = true;
  int copy_rows = -1;  // >= 0: copy only the first copy_rows rows (pe table)
};

// n* = LayerNorm-folded copies (gamma into the weight columns, beta into the
// bias; derived at finalize): the GEMM prologue only normalises rows.
struct EncLayer {
  float *ln_g, *ln_b, *wqkv, *bqkv, *wo, *bo, *fln_g, *fln_b, *w1, *b1, *w2, *b2;
  float *nwqkv, *nbqkv, *nw1, *nb1;
  // P16H images of W1' (LN folded) and W2 for the fused FFN block (ffn.hip)
  uint16_t *w1h = nullptr, *w2h = nullptr;
  float w1s = 1.f, w2s = 1.f;
  // P16H image of Wo, folded into the FFN block's launch (ffn.hip WO)
  uint16_t* woh = nullptr;
  float wos = 1.f;
  // P16H image of the LN-folded W_qkv, folded into the previous layer's FFN launch (ffn.hip QK)
  uint16_t* qkvh = nullptr;
  float qkvs = 1.f;
};
struct DecLayer {
  float *ln1_g, *ln1_b, *wqkv, *bqkv, *wo, *bo, *ln2_g, *ln2_b, *cwq, *cbq, *cwo, *cbo, *fln_g, *fln_b, *w1, *b1,
      *w2, *b2;
  float *nwqkv, *nbqkv, *ncwq, *ncbq, *nw1, *nb1;
  // P16-packed step weights (kernels.hpp launch_gemm_p16), derived at finalize
  float *pwqkv, *pwo, *pcwq, *pcwo, *pw1, *pw2;
  // memory-bank context attention (greedy): ctx K folded into the query
  // projection, ctx V into the output projection (derived at finalize, f64)
  float *pwqk, *bqk, *pwvo, *bvo;
  // average self-attention (onmt/modules/average_attn.py): average_layer FFN
  // (LN + 256 -> 256 -> 256) and gating Linear(512, 512); derived: LN-folded
  // P16 w_1, P16 w_2, the gate's xn / a column halves P16
  float *aln_g = nullptr, *aln_b = nullptr, *aw1 = nullptr, *ab1 = nullptr, *aw2 = nullptr, *ab2 = nullptr,
        *gw = nullptr, *gb = nullptr;
  float *naw1 = nullptr, *nab1 = nullptr, *paw1 = nullptr, *paw2 = nullptr, *pgwx = nullptr, *pgwa = nullptr;
};
struct NanoLayer {
  float *wih, *bih, *bhh, *whh, *bn_g, *bn_b, *bn_rm, *bn_rv;  // raw
  float *bsum, *bn_scale, *bn_shift;                             // derived at finalize
  int in;
};

struct GraphKey {
  int mode, B, T, S, min_len, beam, n_best, seg, logp;
  float alpha;
  int stamp = 0;
  // attention capture and the classic Beam's options
  int attn = 0, cov = 0, stepwise = 0, ngram = 0;
  unsigned excl = 0;
  float beta = 0.f;
  // random sampling (greedy path): top-k (1 = argmax) and temperature
  int topk = 1;
  float temp = 0.f;
  int exact = 0;  // exact fp32 products (set by run_graph from the ctx)
  int bank_nt = 0;  // memory bank streamed non-temporally (set by run_graph from the ctx)
  int bank_grid = 0;  // the bank kernel's workgroup cap (set by run_graph from the ctx)
  int splitk = 0;     // long-K step GEMMs split over workgroups (set by run_graph from the ctx)
  int tail = 0;   // --fast beam tail segments (nd_ctx.beam_tail)
  bool operator<(const GraphKey& o) const {
    return std::tie(mode, B, T, S, min_len, beam, n_best, seg, logp, alpha, stamp, attn, cov, stepwise, ngram, excl,
                    beta, topk, temp, exact, tail, bank_nt, bank_grid, splitk) <
           std::tie(o.mode, o.B, o.T, o.S, o.min_len, o.beam, o.n_best, o.seg, o.logp, o.alpha, o.stamp, o.attn,
                    o.cov, o.stepwise, o.ngram, o.excl, o.beta, o.topk, o.temp, o.exact, o.tail, o.bank_nt,
                    o.bank_grid, o.splitk);
  }
};

struct nd_ctx {
  nd_config cfg{};
  int D = ND_D, F = 2048, V = 8, H = 128;
  std::map<std::string, Slot> slots;
  std::vector<void*> allocs;
  bool finalized = false;
  bool shares = false;  // reads another context's weights (nd_share_weights)
  bool use_graphs = true;
  int ctx_path = 0;  // 0: memory-bank form for greedy, K/V form for beam; 1: always K/V
  bool kstamp_on = false;                 // stamp every context-attention launch (bench roofline)
  unsigned long long* kstamp = nullptr;   // [dec_layers * max_steps][2] (start, end) wall-clock ticks
  bool timing = false;
  float t_enc = 0.f, t_dec = 0.f;
  // exact fp32: plain fp32-MFMA kernels everywhere (no split-fp16 products);
  // nd_set_exact_fp32, default from ND_GEMM_F32
  bool exact = false;
  // split-fp16 range guard word (common.hpp flag_overflow), read and cleared
  // per call by nd_take_overflow
  int* ovf = nullptr;
  // --fast beam: few chunks alive (seen at a segment poll): the decoder GEMMs
  // stay on the small-M P16 kernels (GraphKey.tail)
  bool beam_tail = false;
  // stream the memory bank with non-temporal loads (nd_set_bank_policy): an
  // EnginePool lane whose bank should not displace another lane's from the
  // Infinity Cache
  bool bank_nt = false;
  // workgroups of the bank kernel at most (nd_set_bank_grid; 0 = one per chunk)
  int bank_grid = 0;
  // the K = 2048 step GEMMs split over workgroups (gemm_p16k_kernel, nd_set_gemm_splitk).  Off by default:
  // a lone call is faster on the one-workgroup-per-tile long-K kernel; EnginePool lanes (several calls in
  // flight) turn it on ("Decoder GEMMs at 256 rows")
  bool splitk = false;

  // weights
  float *enc_lin_w = nullptr, *enc_lin_b = nullptr, *enc_ln_g = nullptr, *enc_ln_b = nullptr;
  // the memory bank's LayerNorm affine divided by its per-dimension power-of-two
  // scales (derive_bank_dim_scales; transformer encoder), and the scales
  float *bank_ln_g = nullptr, *bank_ln_b = nullptr;
  std::vector<float> bank_dim_scale;
  // per-dimension power-of-two rebalancing of the decoder attentions' key / query and value / output
  // projections (rebalance_attention): for a weight buffer, the scale of each of its rows (or columns), which
  // nd_load_weight applies to a tensor loaded into it later so the set stays consistent
  struct Rescale {
    std::vector<float> s;
    bool cols = false;
  };
  std::map<const float*, Rescale> rescale;
  bool rebalanced = false;
  // encoder layer 0's QKV in the rank-2 form (kernels.hpp EmbedQkv): a | c on
  // the device, the three means on the host (kernel arguments); set at finalize
  float* eq_ac = nullptr;
  double* eq_scal = nullptr;
  float eq_m[3] = {0.f, 0.f, 0.f};
  bool eq_ready = false;
  // layer 0's attention in the same closed form: per head the 6 coefficients
  // of alpha_t, beta_t (launch_enc_attention_rank2), on the device
  float* eq_coef = nullptr;
  std::vector<EncLayer> enc;
  std::vector<NanoLayer> nano;
  float* nano_W = nullptr;
  std::vector<DecLayer> dec;
  float *ctxkv_w = nullptr, *ctxkv_b = nullptr, *nctxkv_w = nullptr, *nctxkv_b = nullptr;
  float *emb = nullptr, *pe = nullptr, *dec_ln_g = nullptr, *dec_ln_b = nullptr, *gen_w = nullptr, *gen_b = nullptr;
  // split-fp16 images of the row-major GEMM weights (gemm.hip, H3), keyed by
  // the fp32 weight they were made from (built at finalize)
  std::map<const float*, std::pair<uint16_t*, float>> split;
  // row-major split images of the P16 step weights (large-M route), keyed by the P16 weight
  std::map<const float*, std::pair<uint16_t*, float>> split_rm;

  // workspaces
  float* sig = nullptr;
  int *len = nullptr, *span = nullptr;
  float *x = nullptr, *y = nullptr, *att = nullptr, *big = nullptr, *ctxkv = nullptr;
  float* mem_p = nullptr;                 // memory bank [B * T, 256] row-major (LN'd encoder output)
  const float* mem = nullptr;             // the bank the decoder reads: mem_p, or x (NanoEncoder)
  bool bank_d8 = false;                   // mem_p holds the 24-bit digit bank (dec_bank_d8_kernel; bank8.hip)
  bool ctx_q24 = false;                   // beam rows read the 24-bit context K/V image (ctxq), not fp32 ctxkv
  int* clist = nullptr;                   // --fast beam tail: the alive chunks (launch_alive_list), ceil(B/16)
  float* ctx_part = nullptr;              // ... and the split context attention's partial states
  uint8_t* ctxq = nullptr;                // [layers][B * T][CTXQ_ROW] (attention.hip ctx_pack_q24_kernel)
  float* bank_ks = nullptr;               // digit bank: per-row scales 2^e_t [B * 512]
  int* bank_em = nullptr;                 // digit bank: per-chunk max e_t (biased) [B]
  int last_bank_form = 0;                 // nd_bank_form
  float *dqk = nullptr, *dU = nullptr;    // [R, 8*256] P16 (memory-bank path)
  float* sk_slab = nullptr;               // split-K P16 GEMMs: fp32 partial slabs (gemm_p16k_kernel)
  int* sk_cnt = nullptr;                  // ... and their per-tile tickets (zeroed per call)
  int sk_tiles = 0;                       // 32 x 32 tiles the slab serves
  float* dffn_slab = nullptr;             // beam rows' split fused FFN (ffn.hip DecFfn): partial slabs
  int* dffn_cnt = nullptr;                // ... and per-row-block tickets (zeroed per call)
  int dffn_rb = 0;                        // 128-row blocks they serve
  // average self-attention step buffers (P16): xn, avg (+ its row stats), the
  // average_layer hidden, a = FFN(avg), the gate pre-activations [R, 512]
  float *axn = nullptr, *aavg = nullptr, *aavg_part = nullptr, *ah = nullptr, *aa = nullptr, *ag = nullptr;
  float *nano_xp = nullptr, *nano_h = nullptr;
  float *x_part = nullptr, *y_part = nullptr, *dx_part = nullptr, *dq1_part = nullptr, *dmid_part = nullptr;
  int x_pn = 1;
  float *dx = nullptr, *dq1 = nullptr, *dmid = nullptr, *dcq = nullptr, *datt = nullptr, *dqkv = nullptr,
        *dhid = nullptr, *cache = nullptr;
  int *tok = nullptr, *gtok = nullptr;
  // layer-0 QKV table (QkvRows): input rows, their statistics, the table
  // [round16(max_steps * V), 768] P16, and each row's token of the step
  float *qtab_x = nullptr, *qtab_part = nullptr, *qtab = nullptr;
  int* rtok = nullptr;
  float *gscore = nullptr, *glogp = nullptr;
  nd::BeamState bs{};
  int* steps_done = nullptr;
  int* group_in = nullptr;  // classic Beam: staged reference-batch ids
  int* cut_in = nullptr;    // classic Beam: staged attention lengths (coverage penalties)
  unsigned long long* seed_dev = nullptr;  // random sampling: the call's seed (read by the captured graph)
  // -attn_debug / coverage: [decoder rows][max_steps][max_src_len] head-0 context scores -> probabilities
  float* attn_raw = nullptr;
  bool attn_on = false;       // set while a call that captures the attention is enqueued
  int* h_alive = nullptr;  // pinned

  hipStream_t es = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr, ev_a = nullptr, ev_b = nullptr, ev_c = nullptr;
  std::map<GraphKey, hipGraphExec_t> graphs;
};

// ------------------------------------------------------------------ helpers
template <typename T>
static hipError_t dalloc(nd_ctx* c, T** p, size_t n) {
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, n * sizeof(T) + 256);
  if (e != hipSuccess) return e;
  e = hipMemset(q, 0, n * sizeof(T) + 256);
  c->allocs.push_back(q);
  *p = reinterpret_cast<T*>(q);
  return e;
}

static void add_slot(nd_ctx* c, const std::string& name, float* dst, std::vector<int64_t> shape, bool required = true,
                     int copy_rows = -1) {
  Slot s;
  s.dst = dst;
  s.shape = shape;
  s.numel = 1;
  for (auto d : shape) s.numel *= (size_t)d;
  s.required = required;
  s.copy_rows = copy_rows;
  c->slots[name] = s;
}

static int build_registry(nd_ctx* c) {
  const int D = c->D, F = c->F, V = c->V;
  const auto& cfg = c->cfg;
  hipError_t e;
#define AL(ptr, n)                                          \
  if ((e = dalloc(c, &(ptr), (size_t)(n))) != hipSuccess) \
    return fail(ND_ERR_HIP, std::string("hipMalloc weights: ") + hipGetErrorString(e));
  if (cfg.encoder_type == ND_ENC_TRANSFORMER) {
    AL(c->enc_lin_w, D);
    AL(c->enc_lin_b, D);
    AL(c->enc_ln_g, D);
    AL(c->enc_ln_b, D);
    add_slot(c, "encoder.linear.weight", c->enc_lin_w, {D, 1});
    add_slot(c, "encoder.linear.bias", c->enc_lin_b, {D});
    add_slot(c, "encoder.layer_norm.weight", c->enc_ln_g, {D});
    add_slot(c, "encoder.layer_norm.bias", c->enc_ln_b, {D});
    c->enc.resize(cfg.enc_layers);
    for (int i = 0; i < cfg.enc_layers; ++i) {
      EncLayer& L = c->enc[i];
      AL(L.ln_g, D); AL(L.ln_b, D); AL(L.wqkv, 3 * D * D); AL(L.bqkv, 3 * D); AL(L.wo, D * D); AL(L.bo, D);
      AL(L.fln_g, D); AL(L.fln_b, D); AL(L.w1, (size_t)F * D); AL(L.b1, F); AL(L.w2, (size_t)D * F); AL(L.b2, D);
      AL(L.nwqkv, 3 * D * D); AL(L.nbqkv, 3 * D); AL(L.nw1, (size_t)F * D); AL(L.nb1, F);
      const std::string p = "encoder.transformer." + std::to_string(i);
      add_slot(c, p + ".layer_norm.weight", L.ln_g, {D});
      add_slot(c, p + ".layer_norm.bias", L.ln_b, {D});
      const char* qkv[3] = {"linear_query", "linear_keys", "linear_values"};
      for (int k = 0; k < 3; ++k) {
        add_slot(c, p + ".self_attn." + qkv[k] + ".weight", L.wqkv + (size_t)k * D * D, {D, D});
        add_slot(c, p + ".self_attn." + qkv[k] + ".bias", L.bqkv + k * D, {D});
      }
      add_slot(c, p + ".self_attn.final_linear.weight", L.wo, {D, D});
      add_slot(c, p + ".self_attn.final_linear.bias", L.bo, {D});
      add_slot(c, p + ".feed_forward.layer_norm.weight", L.fln_g, {D});
      add_slot(c, p + ".feed_forward.layer_norm.bias", L.fln_b, {D});
      add_slot(c, p + ".feed_forward.w_1.weight", L.w1, {F, D});
      add_slot(c, p + ".feed_forward.w_1.bias", L.b1, {F});
      add_slot(c, p + ".feed_forward.w_2.weight", L.w2, {D, F});
      add_slot(c, p + ".feed_forward.w_2.bias", L.b2, {D});
    }
  } else {
    const int Hh = c->H;
    c->nano.resize(cfg.enc_layers);
    for (int l = 0; l < cfg.enc_layers; ++l) {
      NanoLayer& L = c->nano[l];
      L.in = l == 0 ? 1 : 2 * Hh;
      AL(L.wih, (size_t)8 * Hh * L.in); AL(L.bih, 8 * Hh); AL(L.bhh, 8 * Hh); AL(L.whh, (size_t)8 * Hh * Hh);
      AL(L.bn_g, 2 * Hh); AL(L.bn_b, 2 * Hh); AL(L.bn_rm, 2 * Hh); AL(L.bn_rv, 2 * Hh);
      AL(L.bsum, 8 * Hh); AL(L.bn_scale, 2 * Hh); AL(L.bn_shift, 2 * Hh);
      const std::string p = "encoder.rnn_" + std::to_string(l);
      const char* sfx[2] = {"", "_reverse"};
      for (int d = 0; d < 2; ++d) {
        add_slot(c, p + ".weight_ih_l0" + sfx[d], L.wih + (size_t)d * 4 * Hh * L.in, {4 * Hh, L.in});
        add_slot(c, p + ".weight_hh_l0" + sfx[d], L.whh + (size_t)d * 4 * Hh * Hh, {4 * Hh, Hh});
        add_slot(c, p + ".bias_ih_l0" + sfx[d], L.bih + d * 4 * Hh, {4 * Hh});
        add_slot(c, p + ".bias_hh_l0" + sfx[d], L.bhh + d * 4 * Hh, {4 * Hh});
      }
      const std::string b = "encoder.batchnorm_" + std::to_string(l);
      add_slot(c, b + ".weight", L.bn_g, {2 * Hh});
      add_slot(c, b + ".bias", L.bn_b, {2 * Hh});
      add_slot(c, b + ".running_mean", L.bn_rm, {2 * Hh});
      add_slot(c, b + ".running_var", L.bn_rv, {2 * Hh});
    }
    AL(c->nano_W, (size_t)D * 2 * Hh);
    add_slot(c, "encoder.W.weight", c->nano_W, {D, 2 * Hh});
  }
  c->dec.resize(cfg.dec_layers);
  AL(c->ctxkv_w, (size_t)cfg.dec_layers * 2 * D * D);
  AL(c->ctxkv_b, (size_t)cfg.dec_layers * 2 * D);
  if (cfg.encoder_type == ND_ENC_TRANSFORMER) {
    AL(c->nctxkv_w, (size_t)cfg.dec_layers * 2 * D * D);
    AL(c->nctxkv_b, (size_t)cfg.dec_layers * 2 * D);
  }
  for (int i = 0; i < cfg.dec_layers; ++i) {
    DecLayer& L = c->dec[i];
    AL(L.ln1_g, D); AL(L.ln1_b, D); AL(L.wqkv, 3 * D * D); AL(L.bqkv, 3 * D); AL(L.wo, D * D); AL(L.bo, D);
    AL(L.ln2_g, D); AL(L.ln2_b, D); AL(L.cwq, D * D); AL(L.cbq, D); AL(L.cwo, D * D); AL(L.cbo, D);
    AL(L.fln_g, D); AL(L.fln_b, D); AL(L.w1, (size_t)F * D); AL(L.b1, F); AL(L.w2, (size_t)D * F); AL(L.b2, D);
    AL(L.nwqkv, 3 * D * D); AL(L.nbqkv, 3 * D); AL(L.ncwq, D * D); AL(L.ncbq, D); AL(L.nw1, (size_t)F * D);
    AL(L.nb1, F);
    AL(L.pwqkv, 3 * D * D); AL(L.pwo, D * D); AL(L.pcwq, D * D); AL(L.pcwo, D * D); AL(L.pw1, (size_t)F * D);
    AL(L.pw2, (size_t)D * F);
    AL(L.pwqk, (size_t)ND_H * D * D); AL(L.bqk, ND_H * D); AL(L.pwvo, (size_t)D * ND_H * D); AL(L.bvo, D);
    const std::string p = "decoder.transformer_layers." + std::to_string(i);
    add_slot(c, p + ".layer_norm_1.weight", L.ln1_g, {D});
    add_slot(c, p + ".layer_norm_1.bias", L.ln1_b, {D});
    add_slot(c, p + ".layer_norm_2.weight", L.ln2_g, {D});
    add_slot(c, p + ".layer_norm_2.bias", L.ln2_b, {D});
    if (cfg.self_attn_type == ND_SELF_AVERAGE) {
      AL(L.aln_g, D); AL(L.aln_b, D); AL(L.aw1, D * D); AL(L.ab1, D); AL(L.aw2, D * D); AL(L.ab2, D);
      AL(L.gw, 4 * D * D); AL(L.gb, 2 * D);
      AL(L.naw1, D * D); AL(L.nab1, D); AL(L.paw1, D * D); AL(L.paw2, D * D); AL(L.pgwx, 2 * D * D);
      AL(L.pgwa, 2 * D * D);
      const std::string a = p + ".self_attn.";
      add_slot(c, a + "average_layer.layer_norm.weight", L.aln_g, {D});
      add_slot(c, a + "average_layer.layer_norm.bias", L.aln_b, {D});
      add_slot(c, a + "average_layer.w_1.weight", L.aw1, {D, D});
      add_slot(c, a + "average_layer.w_1.bias", L.ab1, {D});
      add_slot(c, a + "average_layer.w_2.weight", L.aw2, {D, D});
      add_slot(c, a + "average_layer.w_2.bias", L.ab2, {D});
      add_slot(c, a + "gating_layer.weight", L.gw, {2 * D, 2 * D});
      add_slot(c, a + "gating_layer.bias", L.gb, {2 * D});
    } else {
      const char* qkv[3] = {"linear_query", "linear_keys", "linear_values"};
      for (int k = 0; k < 3; ++k) {
        add_slot(c, p + ".self_attn." + qkv[k] + ".weight", L.wqkv + (size_t)k * D * D, {D, D});
        add_slot(c, p + ".self_attn." + qkv[k] + ".bias", L.bqkv + k * D, {D});
      }
      add_slot(c, p + ".self_attn.final_linear.weight", L.wo, {D, D});
      add_slot(c, p + ".self_attn.final_linear.bias", L.bo, {D});
    }
    add_slot(c, p + ".context_attn.linear_query.weight", L.cwq, {D, D});
    add_slot(c, p + ".context_attn.linear_query.bias", L.cbq, {D});
    add_slot(c, p + ".context_attn.linear_keys.weight", c->ctxkv_w + (size_t)(2 * i) * D * D, {D, D});
    add_slot(c, p + ".context_attn.linear_keys.bias", c->ctxkv_b + (2 * i) * D, {D});
    add_slot(c, p + ".context_attn.linear_values.weight", c->ctxkv_w + (size_t)(2 * i + 1) * D * D, {D, D});
    add_slot(c, p + ".context_attn.linear_values.bias", c->ctxkv_b + (2 * i + 1) * D, {D});
    add_slot(c, p + ".context_attn.final_linear.weight", L.cwo, {D, D});
    add_slot(c, p + ".context_attn.final_linear.bias", L.cbo, {D});
    add_slot(c, p + ".feed_forward.layer_norm.weight", L.fln_g, {D});
    add_slot(c, p + ".feed_forward.layer_norm.bias", L.fln_b, {D});
    add_slot(c, p + ".feed_forward.w_1.weight", L.w1, {F, D});
    add_slot(c, p + ".feed_forward.w_1.bias", L.b1, {F});
    add_slot(c, p + ".feed_forward.w_2.weight", L.w2, {D, F});
    add_slot(c, p + ".feed_forward.w_2.bias", L.b2, {D});
  }
  AL(c->emb, (size_t)V * D);
  add_slot(c, "decoder.embeddings.make_embedding.emb_luts.0.weight", c->emb, {V, D});
  if (cfg.position_encoding) {
    AL(c->pe, (size_t)cfg.max_steps * D);
    add_slot(c, "decoder.embeddings.make_embedding.pe.pe", c->pe, {-1, 1, D}, true, cfg.max_steps);
  }
  AL(c->dec_ln_g, D);
  AL(c->dec_ln_b, D);
  add_slot(c, "decoder.layer_norm.weight", c->dec_ln_g, {D});
  add_slot(c, "decoder.layer_norm.bias", c->dec_ln_b, {D});
  AL(c->gen_w, (size_t)V * D);
  AL(c->gen_b, V);
  add_slot(c, "generator.0.weight", c->gen_w, {V, D});
  add_slot(c, "generator.0.bias", c->gen_b, {V});
#undef AL
  return ND_OK;
}

static int alloc_ctx_kv(nd_ctx* c) {
  if (c->ctxkv) return ND_OK;
  const auto& cfg = c->cfg;
  const size_t B = cfg.max_batch, T = cfg.max_src_len, D = c->D, Ld = cfg.dec_layers;
  hipError_t e;
#define WSK(ptr, n)                                         \
  if ((e = dalloc(c, &(ptr), (size_t)(n))) != hipSuccess) \
    return fail(ND_ERR_HIP, std::string("hipMalloc workspace " #ptr ": ") + hipGetErrorString(e));
  WSK(c->ctxkv, B * T * Ld * 2 * D);
  float* q = nullptr;
  WSK(q, B * T * Ld * (CTXQ_ROW / 4));
  c->ctxq = reinterpret_cast<uint8_t*>(q);
  float* l = nullptr;
  WSK(l, B);
  c->clist = reinterpret_cast<int*>(l);
  // ceil(B/16) listed chunks x up to 32 splits x rows x {num[256], max[8], den[8]}
  WSK(c->ctx_part, (B + 15) / 16 * 32 * std::max(1, cfg.max_beam) * (D + 16));
  {
    // the beam's split fused FFN: up to 8 splits per 128-row block
    const int R = (int)((B * (size_t)std::max(1, cfg.max_beam) + 15) / 16 * 16);
    c->dffn_rb = (R + 127) / 128;
    WSK(c->dffn_slab, nd::dec_ffn_slab_floats(R, 8));
    float* t = nullptr;
    WSK(t, (size_t)(c->dffn_rb + 3) / 4 * 4);
    c->dffn_cnt = reinterpret_cast<int*>(t);
    if ((e = hipMemset(c->dffn_cnt, 0, (size_t)(c->dffn_rb + 3) / 4 * 16)) != hipSuccess)
      return fail(ND_ERR_HIP, std::string("hipMemset FFN tickets: ") + hipGetErrorString(e));
  }
#undef WSK
  return ND_OK;
}

static int alloc_workspaces(nd_ctx* c) {
  const auto& cfg = c->cfg;
  const size_t B = cfg.max_batch, T = cfg.max_src_len, S = cfg.max_steps;
  // decoder rows, padded to whole 16-row P16 blocks
  const size_t R = (B * (size_t)std::max(1, cfg.max_beam) + 15) / 16 * 16;
  const size_t D = c->D, F = c->F, Ld = cfg.dec_layers;
  hipError_t e;
#define WS(ptr, n)                                          \
  if ((e = dalloc(c, &(ptr), (size_t)(n))) != hipSuccess) \
    return fail(ND_ERR_HIP, std::string("hipMalloc workspace " #ptr ": ") + hipGetErrorString(e));
  WS(c->sig, B * T);
  WS(c->len, B);
  WS(c->span, B);
  WS(c->x, B * T * D);
  WS(c->y, B * T * D);
  WS(c->att, B * T * D);
  WS(c->big, B * T * std::max(F, 3 * D));
  // the per-layer context K/V (fp32 and the 24-bit image) and the beam tail's buffers: beam-capable
  // contexts only (a greedy context allocates them on nd_set_ctx_path(1)); ADVICE r04: 1.4 GB per
  // greedy lane at B = 256
  if (cfg.max_beam > 1) {
    const int rc = alloc_ctx_kv(c);
    if (rc != ND_OK) return rc;
  }
  {
    // split-K P16 GEMMs (K = 2048 / 1024 at 128 < R <= 1024): 32 x 32 tiles x 4 slices x 4 KB
    const int tiles = (int)std::min<size_t>((R + 31) / 32, 32) * (int)(D / 32);
    WS(c->sk_slab, (size_t)tiles * 4 * 1024);
    float* t = nullptr;
    WS(t, (size_t)(tiles + 3) / 4 * 4);
    c->sk_cnt = reinterpret_cast<int*>(t);
    c->sk_tiles = tiles;
    if ((e = hipMemset(c->sk_cnt, 0, (size_t)(tiles + 3) / 4 * 16)) != hipSuccess)
      return fail(ND_ERR_HIP, std::string("hipMemset split-K tickets: ") + hipGetErrorString(e));
  }
  // the fp32 bank [B * T, 256], or the digit bank: 512 rows per chunk whatever T is (B * 512 * 256 * 3 bytes)
  WS(c->mem_p, std::max(B * T * D, B * 512 * ND_D * 3 / 4));
  WS(c->bank_ks, B * 512);
  {
    float* em = nullptr;
    WS(em, B);
    c->bank_em = reinterpret_cast<int*>(em);
  }
  WS(c->x_part, B * T * ND_PART_LD * 2);
  WS(c->y_part, B * T * ND_PART_LD * 2);
  WS(c->dx_part, R * ND_PART_LD * 2);
  WS(c->dq1_part, R * ND_PART_LD * 2);
  WS(c->dmid_part, R * ND_PART_LD * 2);
  if (cfg.encoder_type == ND_ENC_NANO) {
    WS(c->nano_xp, B * T * 8 * (size_t)c->H);
    WS(c->nano_h, B * T * 2 * (size_t)c->H);
  }
  WS(c->dx, R * D);
  WS(c->dq1, R * D);
  WS(c->dmid, R * D);
  WS(c->dcq, R * D);
  WS(c->datt, R * D);
  WS(c->dqkv, R * 3 * D);
  WS(c->dhid, R * F);
  WS(c->dqk, R * ND_H * D);
  WS(c->dU, R * ND_H * D);
  if (cfg.self_attn_type == ND_SELF_AVERAGE) {
    WS(c->axn, R * D);
    WS(c->aavg, R * D);
    WS(c->aavg_part, R * ND_PART_LD * 2);
    WS(c->ah, R * D);
    WS(c->aa, R * D);
    WS(c->ag, R * 2 * D);
  }
  WS(c->cache, Ld * R * S * 2 * D);
  WS(c->tok, R);
  if (cfg.self_attn_type != ND_SELF_AVERAGE) {
    const size_t QR = (S * (size_t)c->V + 15) / 16 * 16;
    WS(c->qtab_x, QR * D);
    WS(c->qtab_part, QR * ND_PART_LD * 2);
    WS(c->qtab, QR * 3 * D);
    WS(c->rtok, R);
  }
  WS(c->gtok, B * S);
  WS(c->gscore, B);
  WS(c->glogp, B * S * (size_t)c->V);
  WS(c->bs.cum, R);
  WS(c->bs.seq[0], R * S);
  WS(c->bs.seq[1], R * S);
  WS(c->bs.anc[0], R * S);
  WS(c->bs.anc[1], R * S);
  c->bs.tok = c->tok;
  WS(c->bs.done, B);
  WS(c->bs.top_fin, B);
  WS(c->bs.n_hyp, B);
  const size_t NB = (size_t)std::max(1, cfg.max_beam);
  WS(c->bs.hyp_score, B * NB);
  WS(c->bs.hyp_len, B * NB);
  WS(c->bs.hyp_tok, B * NB * S);
  WS(c->bs.n_alive, 4);
  WS(c->steps_done, 4);
  c->bs.steps_done = c->steps_done;
  WS(c->bs.group, B);
  WS(c->bs.grp_left, B);
  WS(c->bs.grp_done, B);
  WS(c->bs.steps_run, B);
  WS(c->bs.hyp_anc, B * NB * S);
  WS(c->bs.cov[0], R * T);
  WS(c->bs.cov[1], R * T);
  WS(c->bs.pen, R);
  WS(c->bs.prev_pen, R);
  WS(c->bs.blk[0], R);
  WS(c->bs.blk[1], R);
  c->bs.T = (int)T;
  WS(c->group_in, B);
  WS(c->cut_in, B);
  WS(c->seed_dev, 2);
  WS(c->kstamp, Ld * S * 2);
  WS(c->ovf, 4);
#undef WS
  if ((e = hipHostMalloc((void**)&c->h_alive, 16, hipHostMallocDefault)) != hipSuccess)
    return fail(ND_ERR_HIP, std::string("hipHostMalloc: ") + hipGetErrorString(e));
  return ND_OK;
}

// ------------------------------------------------------------ launch sequences
#define LCHK(expr)                                                                    \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) {                                                           \
      g_err = std::string(#expr) + ": " + hipGetErrorString(e_);                      \
      return e_;                                                                      \
    }                                                                                 \
  } while (0)

static hipError_t gemm(const float* A, int lda, const float* W, int N, int K, const float* bias, float* C, int ldc,
                       int M, hipStream_t s, bool norm = false, bool relu = false, const float* R = nullptr,
                       int ldr = 0) {
  nd::GemmArgs g;
  g.A = A; g.lda = lda; g.W = W; g.ldw = K; g.bias = bias; g.R = R; g.ldr = ldr; g.C = C; g.ldc = ldc;
  g.norm = norm; g.M = M; g.N = N; g.K = K; g.relu = relu;
  return nd::launch_gemm(g, s);
}

// Fluent GEMM launch: G(...).ln(...).res(...).stats(...).run(s, &part_n)
struct G {
  nd::GemmArgs a;
  G(const float* A, int lda, const float* W, int N, int K, const float* bias, float* C, int ldc, int M) {
    a.A = A; a.lda = lda; a.W = W; a.ldw = K; a.bias = bias; a.C = C; a.ldc = ldc; a.M = M; a.N = N; a.K = K;
  }
  // LayerNorm prologue (affine already folded into W / bias)
  G& ln(const float* part, int pn) {
    a.norm = true; a.part_in = part; a.part_n_in = pn;
    return *this;
  }
  G& relu() { a.relu = true; return *this; }
  // use the weight's split-fp16 image when finalize made one
  G& h3(const nd_ctx* c) {
    if (c->exact) return *this;  // fp32 weights only: the fp32-MFMA kernels
    auto it = c->split.find(a.W);
    if (it != c->split.end()) {
      a.Wh = it->second.first;
      a.wscale = it->second.second;
      a.ovf = c->ovf;
    }
    auto jt = c->split_rm.find(a.W);
    if (jt != c->split_rm.end()) {
      a.Wh_rm = jt->second.first;
      a.wscale_rm = jt->second.second;
    }
    return *this;
  }
  G& res(const float* R, int ldr) { a.R = R; a.ldr = ldr; return *this; }
  G& stats(float* part) { a.part_out = part; return *this; }
  G& skip(const int* done, int rpc) { a.skip = done; a.skip_rpc = rpc; return *this; }
  G& small_m(bool on) { a.prefer_p16 = on ? 1 : 0; return *this; }
  G& c_rowmajor(bool on) { a.c_rm = on ? 1 : 0; return *this; }  // P16 GEMMs: C row-major
  G& q24(uint8_t* img, size_t plane) { a.q24 = img; a.q24_plane = plane; return *this; }  // the 24-bit image, not C
  // long-K P16 products may split over workgroups (gemm_p16k_kernel) into the context's slab
  G& splitk(const nd_ctx* c) {
    if (!c->splitk) return *this;
    a.sk_slab = c->sk_slab;
    a.sk_cnt = c->sk_cnt;
    a.sk_tiles = c->sk_tiles;
    return *this;
  }
  bool packed = false;
  G& p16() { packed = true; return *this; }  // decoder-step operands in the P16 layout
  hipError_t run(hipStream_t s, int* pn_out = nullptr) {
    hipError_t e = packed ? nd::launch_gemm_p16(a, s) : nd::launch_gemm(a, s);
    if (pn_out) *pn_out = a.part_n_out;
    return e;
  }
};

// Encoder forward (transformer): x <- memory before the final LayerNorm (its
// row statistics in x_part); the final LN is the ctx-K/V GEMM's prologue.
// fused FFN block (ffn.hip) on the split-fp16 path (exact fp32 keeps the two
// GEMMs; same arithmetic)
static bool enc_ffn_fused(const nd_ctx* c, const EncLayer& L) {
  constexpr bool on = true;
  return on && !c->exact && L.w1h != nullptr && !nd::gemm_f32_forced();
}

// the attention's output projection folded into the fused FFN block's launch
// (y never written)
static bool enc_wo_fused(const nd_ctx* c, const EncLayer& L) {
  constexpr bool on = true;
  return on && enc_ffn_fused(c, L) && L.woh != nullptr;
}

// layer 0's QKV from the embedding in the rank-2 form (EmbedQkv)
static bool enc_qkv0_rank2(const nd_ctx* c) {
  constexpr bool on = true;
  return on && c->eq_ready;
}

// the next layer's QKV projection folded into the FFN block's launch (q | k | v
// from the block's registers)
static bool enc_qkv_folded(const nd_ctx* c, const EncLayer& next) {
  constexpr bool on = true;
  return on && next.qkvh != nullptr;
}

// layer 0's attention in closed form (launch_enc_attention_rank2): no q | k | v
// rows at all for layer 0 (encoder 3.65 -> 3.40 ms per 256-chunk call).  On by
// default since its LDS is exactly 64 KB: the round-3 layout (67,584 B, wave 7's
// E[y] / E[r] rows read and written past byte 65,536 by ds_read2 / ds_write2)
// returned wrong chunks whenever another engine's decoder GEMMs shared the CU;
// every layout whose accesses stay below 65,536 is clean (tools/r2_lds.sh,
// DESIGN.md section 5).  ND_ENC_ATTN0=0 keeps the attention kernel for layer 0.
static bool enc_attn0_rank2(const nd_ctx* c) {
  static const bool on = [] {
    const char* e = getenv("ND_ENC_ATTN0");
    return !(e && atoi(e) == 0);
  }();
  return on && c->eq_ready && c->eq_coef != nullptr;
}

static hipError_t enqueue_encode_transformer(nd_ctx* c, int B, int T, hipStream_t s) {
  const int M = B * T, D = c->D, F = c->F;
  nd::EmbedQkv eq;
  const bool r2 = enc_qkv0_rank2(c), a0 = r2 && enc_attn0_rank2(c);
  if (r2) {
    eq.ac = c->eq_ac;
    eq.bias = c->enc[0].nbqkv;
    eq.mww = c->eq_m[0];
    eq.mwb = c->eq_m[1];
    eq.mbb = c->eq_m[2];
    eq.qkv = c->big;
  }
  LCHK(nd::launch_enc_embed(c->sig, c->enc_lin_w, c->enc_lin_b, c->x, c->x_part, B, T, s,
                            r2 && !a0 ? &eq : nullptr));
  int pnx = 1, pny = 0;
  bool qkv_done = r2;  // this layer's q | k | v already in c->big
  for (size_t li = 0; li < c->enc.size(); ++li) {
    EncLayer& L = c->enc[li];
    // encoder/transformer.py:36-54
    if (!qkv_done) LCHK(G(c->x, D, L.nwqkv, 3 * D, D, L.nbqkv, c->big, 3 * D, M).h3(c).ln(c->x_part, pnx).run(s));
    qkv_done = false;
    if (a0 && li == 0)
      LCHK(nd::launch_enc_attention_rank2(c->sig, c->span, eq, c->eq_coef, c->att, B, T, s));
    else
      LCHK(nd::launch_enc_attention(c->big, c->sig, c->span, c->att, B, T, s, c->exact, c->ovf));
    if (enc_wo_fused(c, L)) {  // Wo + residual, LN, FFN in one launch; the layer's rows updated in place
      nd::EncWo wo;
      wo.att = c->att;
      wo.woh = L.woh;
      wo.wos = L.wos;
      wo.bo = L.bo;
      nd::EncQkv qk;
      if (li + 1 < c->enc.size() && enc_qkv_folded(c, c->enc[li + 1])) {
        const EncLayer& N = c->enc[li + 1];
        qk.wh = N.qkvh;
        qk.ws = N.qkvs;
        qk.bias = N.nbqkv;
        qk.out = c->big;
        qkv_done = true;
      }
      LCHK(nd::launch_enc_ffn(c->x, L.w1h, L.w1s, L.nb1, L.w2h, L.w2s, L.b2, c->x, c->x_part, M, F, c->ovf, s, &wo,
                              qkv_done ? &qk : nullptr));
      pnx = 1;
      continue;
    }
    LCHK(G(c->att, D, L.wo, D, D, L.bo, c->y, D, M).h3(c).res(c->x, D).stats(c->y_part).run(s, &pny));
    if (enc_ffn_fused(c, L)) {  // position_ffn.py:27-40 in one launch: the hidden stays on chip
      LCHK(nd::launch_enc_ffn(c->y, L.w1h, L.w1s, L.nb1, L.w2h, L.w2s, L.b2, c->x, c->x_part, M, F, c->ovf, s));
      pnx = 1;
      continue;
    }
    LCHK(G(c->y, D, L.nw1, F, D, L.nb1, c->big, F, M).h3(c).ln(c->y_part, pny).relu().run(s));
    LCHK(G(c->big, F, L.w2, D, F, L.b2, c->x, D, M).h3(c).res(c->y, D).stats(c->x_part).run(s, &pnx));
  }
  c->x_pn = pnx;
  return hipSuccess;
}

// q24: the GEMM's epilogue writes the 24-bit image (ctxq) instead of fp32 K/V
static hipError_t enqueue_ctxkv(nd_ctx* c, int B, int T, hipStream_t s, bool q24 = false) {
  const int M = B * T, D = c->D, N = (int)c->dec.size() * 2 * D;
  uint8_t* img = q24 ? c->ctxq : nullptr;
  const size_t plane = (size_t)M * CTXQ_ROW;  // one layer's keys of the call (enqueue_dec_step reads the same)
  if (c->cfg.encoder_type == ND_ENC_TRANSFORMER)
    return G(c->x, D, c->nctxkv_w, N, D, c->nctxkv_b, c->ctxkv, N, M).h3(c).ln(c->x_part, c->x_pn).q24(img, plane).run(s);
  return G(c->x, D, c->ctxkv_w, N, D, c->ctxkv_b, c->ctxkv, N, M).h3(c).q24(img, plane).run(s);
}

// the 24-bit image straight from the K/V GEMM's epilogue (fp32-forced GEMMs: fp32 K/V, then the pack kernel)
static bool use_ctx_q24_fuse() {
  constexpr bool on = true;
  return on;
}

static hipError_t enqueue_encode(nd_ctx* c, int B, int T, hipStream_t s);

// Layer 0 of a scaled-dot decoder reads q | k | v from the per-call table
// QKV0[step][token] (kernels.hpp, QkvRows) instead of running its QKV GEMM
// every step (average-attention decoders keep the per-step GEMM).
static bool use_qkv_table(const nd_ctx* c) {
  constexpr bool on = true;
  return on && c->qtab != nullptr;
}

// the greedy head fused into the next step's layer-0 self-attention (table
// mode, scaled-dot layer 0)
static bool head_fused(const nd_ctx* c) {
  constexpr bool on = true;
  return on && use_qkv_table(c) && c->cfg.self_attn_type != ND_SELF_AVERAGE && c->V <= 8;  // SELF_TABV
}

static nd::NextEmbed next_embed(nd_ctx* c) {
  nd::NextEmbed ne;
  ne.emb = c->emb;
  ne.pe = c->cfg.position_encoding ? c->pe : nullptr;
  ne.x = c->dx;
  ne.part = c->dx_part;
  ne.tok = use_qkv_table(c) ? c->rtok : nullptr;
  return ne;
}

// QKV0[s][v] = LN(emb[v] (* 16 + pe[s])) W_qkv + b for the S steps of the
// call: the layer-0 projection of every input a step can see (V of them),
// through the same split-fp16 GEMM the step would run (decoder/transformer.py:
// 76-78, the embedding as onmt/modules/embeddings.py:189-207)
static hipError_t enqueue_qkv_table(nd_ctx* c, int S, hipStream_t s) {
  if (!use_qkv_table(c)) return hipSuccess;
  if (S < 1 || S > c->cfg.max_steps) return hipErrorInvalidValue;
  const int D = c->D, rows = (S * c->V + 15) / 16 * 16;
  LCHK(nd::launch_dec_embed_table(c->emb, c->cfg.position_encoding ? c->pe : nullptr, c->V, S, c->qtab_x,
                                  c->qtab_part, rows, s));
  const DecLayer& L = c->dec[0];
  // row-major: the self-attention reads one table row per workgroup (QkvRows.rm)
  return G(c->qtab_x, D, L.pwqkv, 3 * D, D, L.nbqkv, c->qtab, 3 * D, rows)
      .p16()
      .h3(c)
      .ln(c->qtab_part, 1)
      .c_rowmajor(true)
      .run(s);
}

// Step-0 decoder input (later steps' inputs are written by the search
// kernel that picks their token).
static hipError_t enqueue_first_embed(nd_ctx* c, int R, hipStream_t s) {
  return nd::launch_dec_embed(c->tok, c->emb, c->cfg.position_encoding ? c->pe : nullptr, 0, c->dx, c->dx_part, R, s);
}

// One decoder step for R = C*rpc rows: dx (embedded input, row stats in
// dx_part) -> dx (pre final LN).
// greedy rows always take the memory-bank form (ctx path 0); beam rows read
// the per-layer context K/V
static bool use_memory_bank(nd_ctx* c, int rpc) { return c->ctx_path == 0 && rpc == 1; }

// The decoder's view of the encoder output: a pure function of (ctx path,
// exact, T, rpc, encoder type).  Set on the host before every call's graphs
// run or are captured: a replayed encoder graph does not re-enter
// enqueue_memory, but the step graphs captured after it read these fields.
// beam rows' context K/V in 24-bit fixed point (attention.hip ctx_pack_q24_kernel: 0.78x the bytes of
// the HBM-bound context attention).  Exact fp32 keeps fp32 K/V
static bool use_ctx_q24() {
  constexpr bool on = true;
  return on;
}

// --fast beam tail launches over the alive chunks (launch_alive_list); ND_BEAM_COMPACT=0: over all B
static bool use_beam_compact() {
  static const bool on = [] {
    const char* e = getenv("ND_BEAM_COMPACT");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// --fast beam tail: the context attention over a chunk's keys in this many workgroups (one per CU: a lone
// chunk's 512 keys are latency-bound on one workgroup, ~150 us); ND_CTX_SPLIT=1 keeps one per chunk
static int ctx_split() {
  static const int n = [] {
    const char* e = getenv("ND_CTX_SPLIT");
    const int v = e ? atoi(e) : 16;
    return std::min(32, std::max(1, v));
  }();
  return n;
}

static void set_memory_view(nd_ctx* c, int T, int rpc) {
  c->bank_d8 = false;
  c->mem = nullptr;
  c->last_bank_form = 0;
  c->ctx_q24 = !use_memory_bank(c, rpc) && !c->exact && use_ctx_q24();
  if (c->ctx_q24) c->last_bank_form = 3;
  if (!use_memory_bank(c, rpc)) return;
  const bool tf = c->cfg.encoder_type == ND_ENC_TRANSFORMER;
  // 512-sample chunks: the 24-bit digit bank (LN'd for the transformer, the
  // NanoEncoder's output as it stands)
  c->bank_d8 = !c->exact && nd::bank_eligible(T, c->cfg.max_src_len);
  c->mem = (c->bank_d8 || tf) ? c->mem_p : c->x;  // the NanoEncoder's fp32 output is the bank as it stands
  c->last_bank_form = c->bank_d8 ? 2 : 0;
}

// The beam's decoder FFN as one fused launch (ffn.hip launch_dec_ffn) at
// R >= 1024 rows outside the tail: d_ff split so that about 160 workgroups
// (one per CU, 128 KB of LDS each) run at once, at most 8 splits per row
// block (the last arriver reads the others' 128 KB partials).  Measured at
// R = 5120 (40 row blocks, configs[3], same box, two reps each): 3 / 4 / 5 /
// 6 / 8 splits = 70.3-71.0 / 70.1-70.6 / 71.8-72.0 / 71.0-71.2 / 71.4-72.0 ms
// per pooled call (one call: 89.5 / 88.2 / 87.2 / 87.0 / 91.1 ms); the two
// GEMMs 74.0 / 92.6.  0: the two GEMMs (greedy rows, the tail, exact fp32,
// no split images).
// ND_DEC_FFN=0 keeps the GEMMs, ND_DEC_FFN=n > 1 forces n splits (A/B).
static int dec_ffn_splits(const nd_ctx* c, int R) {
  static const int knob = [] {
    const char* e = getenv("ND_DEC_FFN");
    return e ? atoi(e) : 1;
  }();
  if (knob == 0 || c->exact || c->beam_tail || !c->dffn_slab || R < 1024 || R % 16 || nd::gemm_f32_forced()) return 0;
  const int F = c->F;
  const DecLayer& L = c->dec[0];
  if (F % 32 || F > 2048 || !c->split.count(L.pw1) || !c->split.count(L.pw2)) return 0;
  const int rb = (R + 127) / 128;
  if (rb > c->dffn_rb) return 0;
  if (knob > 1) return std::min({knob, 8, F / 32});
  return std::max(1, std::min({8, 160 / rb, F / 32}));
}

// done: per chunk, nonzero = finished (--fast beam; null otherwise): its rows'
// tiles and attention workgroups exit without work
static hipError_t enqueue_dec_step(nd_ctx* c, int C, int rpc, int T, int step, const int* anc, int anc_ld,
                                   hipStream_t s, const int* done = nullptr, const nd::GreedyHead* head = nullptr,
                                   const int* clist = nullptr, int ccap = 0) {
  const int R = C * rpc, D = c->D, F = c->F, S = c->cfg.max_steps;
  const int Ld = (int)c->dec.size();
  const bool mb = use_memory_bank(c, rpc);
  int pnx = 1, pnq = 0, pnm = 0;
  // a decoder-step GEMM over the R rows: P16 operands, split-fp16 weights, dead chunks skipped
  auto dg = [&](const float* A, int lda, const float* W, int N, int K, const float* bias, float* out, int ldc) {
    return G(A, lda, W, N, K, bias, out, ldc, R).p16().h3(c).skip(done, rpc).small_m(c->beam_tail).splitk(c);
  };
  for (int i = 0; i < Ld; ++i) {
    DecLayer& L = c->dec[i];
    // the self-attention history: beam rows keep 24-bit rows (1600 B per key, attention.hip
    // SELF_Q24_ROW) outside exact fp32; greedy rows, exact fp32 and the average-attention layers keep
    // fp32 k | v (2 KB).  Same box, two reps (profiles/r05_self_q24_ab.txt): configs[3] pooled
    // 67.71 / 67.78 -> 67.28 / 67.17 ms; greedy configs[1] pooled 15.55 / 15.53 -> 15.70 / 15.74 (the
    // row's own history is 100 keys at most: the dequantise costs more than the bytes it saves)
    const bool sq24 = anc && !c->exact && c->cfg.self_attn_type != ND_SELF_AVERAGE;
    float* cache = sq24 ? reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(c->cache) + (size_t)i * R * S * CTXQ_ROW)
                        : c->cache + (size_t)i * R * S * 2 * D;
    unsigned long long* stamp = c->kstamp_on ? c->kstamp + 2 * ((size_t)step * Ld + i) : nullptr;
    // -attn_debug (greedy): the last layer's head-0 context scores, [B][S][T]
    float* dbg = (c->attn_on && i == Ld - 1) ? c->attn_raw + (size_t)step * T : nullptr;
    const size_t dbg_stride = (size_t)S * T;
    // decoder/transformer.py:53-95
    // all step activations are P16-packed (kernels.hpp)
    if (c->cfg.self_attn_type == ND_SELF_AVERAGE) {
      // average_attn.py:55-106 + the layer residual (decoder/transformer.py:82-86)
      LCHK(nd::launch_aan_prep(c->dx, L.ln1_g, L.ln1_b, cache, anc, anc_ld, step, S, c->axn, c->aavg, c->aavg_part,
                               R, s));
      LCHK(dg(c->aavg, D, L.paw1, D, D, L.nab1, c->ah, D).ln(c->aavg_part, 1).relu().run(s));
      LCHK(dg(c->ah, D, L.paw2, D, D, L.ab2, c->aa, D).res(c->aavg, D).run(s));
      LCHK(dg(c->axn, D, L.pgwx, 2 * D, D, L.gb, c->ag, 2 * D).run(s));
      LCHK(dg(c->aa, D, L.pgwa, 2 * D, D, nullptr, c->ag, 2 * D).res(c->ag, 2 * D).run(s));
      LCHK(nd::launch_aan_gate(c->ag, c->axn, c->aa, c->dx, c->dq1, c->dq1_part, R, s));
      pnq = 1;
    } else {
      if (i == 0 && use_qkv_table(c)) {  // the row's q | k | v from the call's table
        nd::QkvRows qr;
        qr.tok = c->rtok;
        qr.V = c->V;
        qr.tok0 = c->cfg.bos_idx;
        qr.rm = 1;  // the table is row-major (enqueue_qkv_table)
        LCHK(nd::launch_dec_self_attention(c->qtab, cache, anc, anc_ld, step, S, c->datt, R, s, rpc, done, qr, head,
                                           clist, ccap, sq24));
      } else {
        // greedy rows (one workgroup each): q | k | v row-major; beam keeps P16 (its M = 5120 GEMMs
        // take the LDS-tiled route, which writes P16)
        nd::QkvRows q12;
        q12.rm = (rpc == 1 && !anc && !done) ? 1 : 0;
        LCHK(dg(c->dx, D, L.pwqkv, 3 * D, D, L.nbqkv, c->dqkv, 3 * D).ln(c->dx_part, pnx).c_rowmajor(q12.rm).run(s));
        LCHK(nd::launch_dec_self_attention(c->dqkv, cache, anc, anc_ld, step, S, c->datt, R, s, rpc, done, q12, nullptr,
                                           clist, ccap, sq24));
      }
      LCHK(dg(c->datt, D, L.pwo, D, D, L.bo, c->dq1, D).res(c->dx, D).stats(c->dq1_part).run(s, &pnq));
    }
    if (mb) {  // memory-bank form (attention.hip)
      const int HD = ND_H * D;
      // q' row-major for the digit-bank kernel (one row per chunk), P16 for the fp32 one
      LCHK(dg(c->dq1, D, L.pwqk, HD, D, L.bqk, c->dqk, HD).ln(c->dq1_part, pnq).c_rowmajor(c->bank_d8).run(s));
      if (c->bank_d8)
        LCHK(nd::launch_dec_bank_d8(c->dqk, c->mem_p, c->bank_ks, c->bank_em, c->sig, c->span, (float)c->cfg.pad_idx,
                                    c->dU, C, T, s, stamp, dbg, dbg_stride, c->ovf, c->bank_nt, c->bank_grid));
      else
        LCHK(nd::launch_dec_mem_attention(c->dqk, c->mem, c->sig, c->span, (float)c->cfg.pad_idx, c->dU, C, rpc, T,
                                          T, s, stamp, dbg, dbg_stride, c->bank_grid));
      LCHK(dg(c->dU, HD, L.pwvo, D, HD, L.bvo, c->dmid, D).res(c->dq1, D).stats(c->dmid_part).run(s, &pnm));
    } else {
      LCHK(dg(c->dq1, D, L.pcwq, D, D, L.ncbq, c->dcq, D).ln(c->dq1_part, pnq).run(s));
      if (c->ctx_q24)
        LCHK(nd::launch_dec_ctx_attention(c->dcq, c->ctxq + (size_t)i * C * T * CTXQ_ROW, CTXQ_ROW, 0, c->sig, c->span,
                                          (float)c->cfg.pad_idx, c->datt, C, rpc, T, s, stamp, dbg, dbg_stride, done,
                                          true, clist, ccap, ctx_split(), c->ctx_part));
      else
        LCHK(nd::launch_dec_ctx_attention(c->dcq, c->ctxkv, Ld * 2 * D, i * 2 * D, c->sig, c->span,
                                          (float)c->cfg.pad_idx, c->datt, C, rpc, T, s, stamp, dbg, dbg_stride, done,
                                          false, clist, ccap, ctx_split(), c->ctx_part));
      LCHK(dg(c->datt, D, L.pcwo, D, D, L.cbo, c->dmid, D).res(c->dq1, D).stats(c->dmid_part).run(s, &pnm));
    }
    if (const int ns = dec_ffn_splits(c, R)) {  // beam rows: the fused block, hidden on chip (ffn.hip)
      const auto& i1 = c->split.at(L.pw1);
      const auto& i2 = c->split.at(L.pw2);
      nd::DecFfn df;
      df.nsplit = ns;
      df.slab = c->dffn_slab;
      df.tickets = c->dffn_cnt;
      df.skip = done;
      df.skip_rpc = rpc;
      LCHK(nd::launch_dec_ffn(c->dmid, i1.first, i1.second, L.nb1, i2.first, i2.second, L.b2, c->dx, c->dx_part, R, F,
                              c->ovf, df, s));
      pnx = 1;  // each row's exact statistics in one partial
    } else {
      LCHK(dg(c->dmid, D, L.pw1, F, D, L.nb1, c->dhid, F).ln(c->dmid_part, pnm).relu().run(s));
      LCHK(dg(c->dhid, F, L.pw2, D, F, L.b2, c->dx, D).res(c->dmid, D).stats(c->dx_part).run(s, &pnx));
    }
  }
  return hipSuccess;
}

// The decoder's view of the encoder output: the memory bank (greedy) or the
// per-layer context K/V (beam).
static hipError_t enqueue_memory(nd_ctx* c, int B, int T, int rpc, hipStream_t s) {
  set_memory_view(c, T, rpc);
  if (!use_memory_bank(c, rpc)) {
    if (!c->ctxkv) return hipErrorInvalidValue;  // a beam call on a context created with max_beam 1
    // the fused form needs the split-fp16 weights (h3): exact fp32 never takes the image
    const bool fuse = c->ctx_q24 && use_ctx_q24_fuse() && !nd::gemm_f32_forced();
    LCHK(enqueue_ctxkv(c, B, T, s, fuse));
    if (!c->ctx_q24 || fuse) return hipSuccess;
    const int Ld = (int)c->dec.size();
    return nd::launch_ctx_pack_q24(c->ctxkv, Ld * 2 * c->D, Ld, c->ctxq, c->span, B, T, s);
  }
  const bool tf = c->cfg.encoder_type == ND_ENC_TRANSFORMER;
  if (c->bank_d8)
    return nd::launch_bank_pack_d8(c->x, tf ? c->bank_ln_g : nullptr, tf ? c->bank_ln_b : nullptr, c->mem_p, c->bank_ks,
                                   c->bank_em, c->span, B, T, c->ovf, s);
  if (!tf) return hipSuccess;  // the NanoEncoder's output is the bank as it stands
  return nd::launch_memory_pack(c->x, c->bank_ln_g, c->bank_ln_b, c->mem_p, B, T, T, s);
}

static hipError_t enqueue_greedy(nd_ctx* c, int B, int T, int S, int min_len, bool logp, hipStream_t s,
                                 const nd::Sampling& smp = nd::Sampling()) {
  if (c->kstamp_on) LCHK(nd::launch_stamp_reset(c->kstamp, (int)c->dec.size() * c->cfg.max_steps, s));
  LCHK(enqueue_encode(c, B, T, s));
  LCHK(enqueue_memory(c, B, T, 1, s));
  LCHK(nd::launch_fill_i32(c->tok, c->cfg.bos_idx, B, s));
  LCHK(enqueue_qkv_table(c, S, s));
  LCHK(enqueue_first_embed(c, B, s));
  const nd::NextEmbed ne = next_embed(c);
  // step k's head runs inside step k + 1's layer-0 self-attention (table
  // mode); only the last step's head is a launch of its own
  const bool fuse = head_fused(c);
  const nd::GreedyHead hd = nd::make_greedy_head(c->dx, c->dec_ln_g, c->dec_ln_b, c->gen_w, c->gen_b, c->V, S, min_len,
                                                 c->cfg.eos_idx, c->tok, c->gtok, c->gscore,
                                                 logp ? c->glogp : nullptr, ne, smp);
  for (int step = 0; step < S; ++step) {
    LCHK(enqueue_dec_step(c, B, 1, T, step, nullptr, 0, s, nullptr, fuse && step > 0 ? &hd : nullptr));
    if (!fuse || step == S - 1)
      LCHK(nd::launch_dec_greedy_head(c->dx, c->dec_ln_g, c->dec_ln_b, c->gen_w, c->gen_b, c->V, step, S, min_len,
                                      c->cfg.eos_idx, c->tok, c->gtok, c->gscore, logp ? c->glogp : nullptr, ne, B,
                                      s, smp));
  }
  if (c->attn_on) LCHK(nd::launch_attn_rows_softmax(c->attn_raw, c->span, B, c->cfg.max_steps, T, s));
  return hipSuccess;
}

// the beam paths' view of the search state: the attention rows are visible
// to the search kernels only while a capturing call is enqueued
static nd::BeamState beam_state(nd_ctx* c) {
  nd::BeamState st = c->bs;
  st.attn = c->attn_on ? c->attn_raw : nullptr;
  st.cut = c->cut_in;
  return st;
}

// -attn_debug / coverage: this step's captured scores -> probabilities
static hipError_t enqueue_attn_step(nd_ctx* c, int C, int rpc, int T, int step, hipStream_t s) {
  if (!c->attn_on) return hipSuccess;
  const size_t S = c->cfg.max_steps;
  return nd::launch_attn_step_softmax(c->attn_raw + (size_t)step * T, S * T, c->span, C * rpc, rpc, T, s);
}

static hipError_t enqueue_beam_steps(nd_ctx* c, int B, int T, int beam, int n_best, float alpha, int S, int min_len,
                                     int s0, int s1, hipStream_t s) {
  const nd::BeamState st = beam_state(c);
  // the tail (at most a sixteenth of the chunks alive, translate_beam): the attention and beam-step launches
  // run over the segment's alive chunks only (a list built at its start), not B chunks that exit at once
  const int ccap = (B + 15) / 16;
  const int* clist = nullptr;
  if (c->beam_tail && use_beam_compact()) {
    LCHK(nd::launch_alive_list(c->bs.done, B, c->clist, ccap, c->ovf, s));
    clist = c->clist;
  }
  for (int step = s0; step < s1; ++step) {
    const int cur = step & 1;
    LCHK(enqueue_dec_step(c, B, beam, T, step, c->bs.anc[cur], S, s, c->bs.done, nullptr, clist, ccap));
    LCHK(enqueue_attn_step(c, B, beam, T, step, s));
    const float lenpen = (float)std::pow((5.0 + (step + 1)) / 6.0, (double)alpha);
    LCHK(nd::launch_beam_step(next_embed(c), c->dx, c->dec_ln_g, c->dec_ln_b, c->gen_w, c->gen_b, c->V, st, B, beam,
                              n_best, step, S, min_len, c->cfg.eos_idx, lenpen, s, clist, ccap));
  }
  return hipSuccess;
}

static hipError_t enqueue_classic_steps(nd_ctx* c, int B, int T, int beam, int n_best, const nd::ClassicOpts& o, int S,
                                        int min_len, int s0, int s1, hipStream_t s) {
  const nd::BeamState st = beam_state(c);
  for (int step = s0; step < s1; ++step) {
    LCHK(enqueue_dec_step(c, B, beam, T, step, c->bs.anc[step & 1], S, s));
    LCHK(enqueue_attn_step(c, B, beam, T, step, s));
    LCHK(nd::launch_beam_classic_step(next_embed(c), c->dx, c->dec_ln_g, c->dec_ln_b, c->gen_w, c->gen_b, c->V, st,
                                      B, beam, n_best, step, S, min_len, c->cfg.eos_idx, o, s));
  }
  return hipSuccess;
}

// --------------------------------------------------------------- graphs
template <typename F>
static int run_graph(nd_ctx* c, const GraphKey& key, F&& enqueue) {
  if (!c->use_graphs) {
    hipError_t e = enqueue(c->es);
    if (e != hipSuccess) return fail(ND_ERR_HIP, g_err.empty() ? hipGetErrorString(e) : g_err);
    return ND_OK;
  }
  GraphKey k = key;
  k.exact = c->exact ? 1 : 0;  // both product forms keep their graphs (the overflow rerun switches)
  k.tail = c->beam_tail ? 1 : 0;
  k.bank_nt = c->bank_nt ? 1 : 0;
  k.bank_grid = c->bank_grid;
  k.splitk = c->splitk ? 1 : 0;
  auto it = c->graphs.find(k);
  if (it == c->graphs.end()) {
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(c->es, hipStreamCaptureModeRelaxed));
    hipError_t e = enqueue(c->es);
    hipError_t e2 = hipStreamEndCapture(c->es, &g);
    if (e != hipSuccess) {
      if (g) (void)hipGraphDestroy(g);
      return fail(ND_ERR_HIP, "capture: " + g_err);
    }
    if (e2 != hipSuccess) return fail(ND_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e2));
    hipGraphExec_t ex = nullptr;
    e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) return fail(ND_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    it = c->graphs.emplace(k, ex).first;
  }
  HIPCHK(hipGraphLaunch(it->second, c->es));
  return ND_OK;
}

// --------------------------------------------------------------- C-ABI
extern "C" {

const char* nd_last_error(void) { return g_err.c_str(); }
const char* nd_version(void) { return "nanodec_hip 0.1.0 gfx950 fp32-mfma"; }

// Engine streams are recycled, never destroyed: a caller may still hold HIP
// events recorded on a context's stream (EnginePool results carry one) after
// the context is gone, and destroying the stream under them leaves the
// events pointing at a freed queue.  nd_destroy parks its (synchronised)
// stream here; nd_create takes a parked one first.
static std::mutex g_streams_mu;
static std::vector<std::pair<int, hipStream_t>> g_spare_streams;  // (device, stream)

static hipError_t acquire_stream(int dev, hipStream_t* s) {
  {
    std::lock_guard<std::mutex> lk(g_streams_mu);
    for (size_t i = 0; i < g_spare_streams.size(); ++i)
      if (g_spare_streams[i].first == dev) {
        *s = g_spare_streams[i].second;
        g_spare_streams.erase(g_spare_streams.begin() + i);
        return hipSuccess;
      }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

static void release_stream(int dev, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_streams_mu);
  g_spare_streams.emplace_back(dev, s);
}

int nd_create(const nd_config* cfg, nd_ctx** out) {
  if (!cfg || !out) return fail(ND_ERR_ARG, "null argument");
  *out = nullptr;
  if (cfg->d_model != ND_D || cfg->heads != ND_H) return fail(ND_ERR_ARG, "only d_model=256, heads=8 are compiled");
  if (cfg->d_ff <= 0 || cfg->d_ff % 128) return fail(ND_ERR_ARG, "d_ff must be a positive multiple of 128");
  if (cfg->vocab < 4 || cfg->vocab > ND_MAXV) return fail(ND_ERR_ARG, "vocab must be in [4, 32]");
  if (cfg->max_src_len < 1 || cfg->max_src_len > 512) return fail(ND_ERR_ARG, "max_src_len must be in [1, 512]");
  if (cfg->max_steps < 1 || cfg->max_steps > 512) return fail(ND_ERR_ARG, "max_steps must be in [1, 512]");
  if (cfg->max_beam < 1 || cfg->max_beam > 8) return fail(ND_ERR_ARG, "max_beam must be in [1, 8]");
  if (cfg->max_batch < 1) return fail(ND_ERR_ARG, "max_batch must be >= 1");
  if (cfg->enc_layers < 1 || cfg->dec_layers < 1) return fail(ND_ERR_ARG, "layers must be >= 1");
  if (cfg->encoder_type != ND_ENC_TRANSFORMER && cfg->encoder_type != ND_ENC_NANO)
    return fail(ND_ERR_ARG, "unknown encoder_type");
  if (cfg->encoder_type == ND_ENC_NANO && cfg->rnn_hidden != 128) return fail(ND_ERR_ARG, "rnn_hidden must be 128");
  if (cfg->self_attn_type != ND_SELF_SCALED_DOT && cfg->self_attn_type != ND_SELF_AVERAGE)
    return fail(ND_ERR_ARG, "unknown self_attn_type");
  HIPCHK(hipSetDevice(cfg->device));
  nd_ctx* c = new nd_ctx();
  c->cfg = *cfg;
  {
    const char* e = getenv("ND_GEMM_F32");
    c->exact = e && atoi(e) != 0;
  }
  c->F = cfg->d_ff;
  c->V = cfg->vocab;
  c->H = cfg->rnn_hidden;
  int rc = build_registry(c);
  if (rc == ND_OK) rc = alloc_workspaces(c);
  if (rc != ND_OK) {
    nd_destroy(c);
    return rc;
  }
  hipError_t e = nd::init_kernel_attributes();
  if (e == hipSuccess) e = acquire_stream(cfg->device, &c->es);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreate(&c->ev_a);
  if (e == hipSuccess) e = hipEventCreate(&c->ev_b);
  if (e == hipSuccess) e = hipEventCreate(&c->ev_c);
  if (e != hipSuccess) {
    nd_destroy(c);
    return fail(ND_ERR_HIP, std::string("stream/event setup: ") + hipGetErrorString(e));
  }
  *out = c;
  return ND_OK;
}

int nd_load_weight(nd_ctx* c, const char* name, const float* host, const int64_t* shape, int ndim) {
  if (!c || !name || !host || (!shape && ndim > 0)) return fail(ND_ERR_ARG, "null argument");
  if (c->shares) return fail(ND_ERR_STATE, "nd_load_weight: the context reads another context's weights");
  const std::string n(name);
  auto it = c->slots.find(n);
  if (it == c->slots.end()) {
    auto ends = [&](const char* sfx) {
      const size_t k = strlen(sfx);
      return n.size() >= k && n.compare(n.size() - k, k, sfx) == 0;
    };
    if (ends(".mask") || ends("num_batches_tracked")) return ND_OK;  // buffers the engine does not use
    if (!c->cfg.position_encoding && n == "decoder.embeddings.make_embedding.pe.pe") return ND_OK;
    return fail(ND_ERR_WEIGHT, "unknown weight '" + n + "'");
  }
  Slot& s = it->second;
  if ((size_t)ndim != s.shape.size()) return fail(ND_ERR_WEIGHT, "rank mismatch for '" + n + "'");
  size_t numel = 1;
  for (int i = 0; i < ndim; ++i) {
    if (s.shape[i] >= 0 && shape[i] != s.shape[i]) return fail(ND_ERR_WEIGHT, "shape mismatch for '" + n + "'");
    numel *= (size_t)shape[i];
  }
  size_t copy = numel;
  if (s.copy_rows >= 0) {
    if (shape[0] < s.copy_rows) return fail(ND_ERR_WEIGHT, "'" + n + "' has fewer rows than max_steps");
    copy = (size_t)s.copy_rows * (numel / (size_t)shape[0]);
  }
  HIPCHK(hipSetDevice(c->cfg.device));
  auto rs = c->rescale.find(s.dst);
  if (rs != c->rescale.end()) {  // a weight the context already rebalanced: the same exact scales
    const auto& R = rs->second;
    const size_t cols = ndim >= 2 ? (size_t)shape[ndim - 1] : 1;
    std::vector<float> tmp(host, host + copy);
    for (size_t e = 0; e < copy; ++e) tmp[e] *= R.s[R.cols ? e % cols : e / cols];
    HIPCHK(hipMemcpy(s.dst, tmp.data(), copy * sizeof(float), hipMemcpyHostToDevice));
  } else {
    HIPCHK(hipMemcpy(s.dst, host, copy * sizeof(float), hipMemcpyHostToDevice));
  }
  s.loaded = true;
  c->finalized = false;
  return ND_OK;
}

// P16 step weight (fp32, for the fp32 kernels) and its split-fp16 P16H image
// (gemm.hip H3), registered under the P16 pointer for G::h3
static hipError_t pack_step_weight(nd_ctx* c, const float* src, int ld, float* dst, int rows, int cols) {
  hipError_t e = nd::launch_pack_p16(src, ld, dst, rows, cols, c->es);
  if (e != hipSuccess) return e;
  uint16_t* h = nullptr;
  auto it = c->split.find(dst);
  if (it != c->split.end()) h = it->second.first;  // finalize called again: refresh in place
  // hi and lo halves: two per element
  if (!h && (e = dalloc(c, &h, (size_t)2 * rows * cols)) != hipSuccess) return e;
  float sc = 1.f;
  if ((e = nd::launch_pack_p16h(src, ld, rows, cols, h, &sc, c->es)) != hipSuccess) return e;
  c->split[dst] = {h, sc};
  // and the row-major image for the LDS-tiled kernel (many rows)
  uint16_t* hr = nullptr;
  auto jt = c->split_rm.find(dst);
  if (jt != c->split_rm.end()) hr = jt->second.first;
  if (!hr && (e = dalloc(c, &hr, (size_t)2 * rows * cols)) != hipSuccess) return e;
  if ((e = nd::launch_split_weight(src, rows, cols, hr, &sc, c->es, ld)) != hipSuccess) return e;
  c->split_rm[dst] = {hr, sc};
  return hipSuccess;
}

// Per-dimension power-of-two rebalancing of the decoder's attentions (self
// and context, onmt/modules/multi_headed_attn.py:124-177).  The beam path
// stores keys and values as 24-bit integers with one scale per (key, head)
// (the context K/V image, the self-attention history), so a dimension far
// larger than the rest of its head -- an "outlier dimension", common in
// trained transformers -- would cost the head's other dimensions that many
// bits.  Scores q.k and the context W_o v are unchanged when key dimension j
// is divided by c_j and query dimension j multiplied by it (value dimension
// j divided, output column j multiplied), so with c_j a power of two the
// model's function is unchanged in exact arithmetic and in fp32 alike.  c_j =
// 2^clamp(floor(log2(a_j / median of a over j's head)), 0, 12), a_j the
// predicted magnitude of projection row j over its input (a LayerNorm output
// y = n g + b: mean b, variance g^2; the NanoEncoder's memory: 0, 1):
// sqrt(sum_i W_ji^2 g_i^2) + |bias_j + sum_i W_ji b_i|.  Applied in place to
// the loaded weights once (nd_finalize); a weight loaded into the context
// afterwards gets the same scales (nd_load_weight).
static void rebalance_scales(const std::vector<float>& W, const std::vector<float>& b, const float* mu,
                             const float* var, int D, std::vector<float>& c) {
  std::vector<double> a(D);
  for (int j = 0; j < D; ++j) {
    double v = 0.0, m = b[j];
    for (int i = 0; i < D; ++i) {
      const double w = W[(size_t)j * D + i];
      v += w * w * (var ? (double)var[i] : 1.0);
      m += mu ? w * mu[i] : 0.0;
    }
    a[j] = std::sqrt(v) + std::fabs(m);
  }
  c.assign(D, 1.f);
  for (int h = 0; h < ND_H; ++h) {
    std::vector<double> hd(a.begin() + h * ND_DH, a.begin() + (h + 1) * ND_DH);
    std::nth_element(hd.begin(), hd.begin() + ND_DH / 2, hd.end());
    const double med = hd[ND_DH / 2];
    for (int j = h * ND_DH; j < (h + 1) * ND_DH; ++j) {
      int k = 0;
      if (med > 0 && a[j] > 0 && std::isfinite(a[j])) k = (int)std::floor(std::log2(a[j] / med));
      c[j] = std::ldexp(1.f, std::min(std::max(k, 0), 12));
    }
  }
}

static int rebalance_attention(nd_ctx* c) {
  if (c->rebalanced) return ND_OK;
  const int D = c->D;
  auto down = [&](const float* d, size_t n, std::vector<float>& h) {
    h.resize(n);
    return hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
  };
  // scale rows (or columns) of a D x D buffer / a D vector by f(c_j), upload, record the scales
  auto apply = [&](float* dst, std::vector<float>& h, const std::vector<float>& cs, bool inv, bool cols,
                   size_t rows) -> hipError_t {
    nd_ctx::Rescale R;
    R.cols = cols;
    R.s.resize(cs.size());
    for (size_t j = 0; j < cs.size(); ++j) R.s[j] = inv ? 1.f / cs[j] : cs[j];
    const size_t ncol = h.size() / rows;
    for (size_t e = 0; e < h.size(); ++e) h[e] *= R.s[cols ? e % ncol : e / ncol];
    c->rescale[dst] = R;
    return hipMemcpy(dst, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  };
  std::vector<float> g, bb, Wq, bq, Wk, bk, Wv, bv, Wo, ck, cv;
  std::vector<float> mg, mb;  // the memory's LN affine (transformer encoder)
  const bool tf = c->cfg.encoder_type == ND_ENC_TRANSFORMER;
  if (tf) {
    HIPCHK(down(c->enc_ln_g, D, mg));
    HIPCHK(down(c->enc_ln_b, D, mb));
    for (auto& x : mg) x *= x;  // variance g^2
  }
  for (size_t i = 0; i < c->dec.size(); ++i) {
    DecLayer& L = c->dec[i];
    if (c->cfg.self_attn_type != ND_SELF_AVERAGE) {
      HIPCHK(down(L.ln1_g, D, g));
      HIPCHK(down(L.ln1_b, D, bb));
      for (auto& x : g) x *= x;
      HIPCHK(down(L.wqkv, (size_t)D * D, Wq));
      HIPCHK(down(L.bqkv, D, bq));
      HIPCHK(down(L.wqkv + (size_t)D * D, (size_t)D * D, Wk));
      HIPCHK(down(L.bqkv + D, D, bk));
      HIPCHK(down(L.wqkv + (size_t)2 * D * D, (size_t)D * D, Wv));
      HIPCHK(down(L.bqkv + 2 * D, D, bv));
      HIPCHK(down(L.wo, (size_t)D * D, Wo));
      rebalance_scales(Wk, bk, bb.data(), g.data(), D, ck);
      rebalance_scales(Wv, bv, bb.data(), g.data(), D, cv);
      HIPCHK(apply(L.wqkv, Wq, ck, false, false, D));
      HIPCHK(apply(L.bqkv, bq, ck, false, false, D));
      HIPCHK(apply(L.wqkv + (size_t)D * D, Wk, ck, true, false, D));
      HIPCHK(apply(L.bqkv + D, bk, ck, true, false, D));
      HIPCHK(apply(L.wqkv + (size_t)2 * D * D, Wv, cv, true, false, D));
      HIPCHK(apply(L.bqkv + 2 * D, bv, cv, true, false, D));
      HIPCHK(apply(L.wo, Wo, cv, false, true, D));
    }
    float* wk = c->ctxkv_w + (size_t)(2 * i) * D * D;
    float* wv = c->ctxkv_w + (size_t)(2 * i + 1) * D * D;
    float* bk_ = c->ctxkv_b + (size_t)(2 * i) * D;
    float* bv_ = c->ctxkv_b + (size_t)(2 * i + 1) * D;
    HIPCHK(down(L.cwq, (size_t)D * D, Wq));
    HIPCHK(down(L.cbq, D, bq));
    HIPCHK(down(wk, (size_t)D * D, Wk));
    HIPCHK(down(bk_, D, bk));
    HIPCHK(down(wv, (size_t)D * D, Wv));
    HIPCHK(down(bv_, D, bv));
    HIPCHK(down(L.cwo, (size_t)D * D, Wo));
    rebalance_scales(Wk, bk, tf ? mb.data() : nullptr, tf ? mg.data() : nullptr, D, ck);
    rebalance_scales(Wv, bv, tf ? mb.data() : nullptr, tf ? mg.data() : nullptr, D, cv);
    HIPCHK(apply(L.cwq, Wq, ck, false, false, D));
    HIPCHK(apply(L.cbq, bq, ck, false, false, D));
    HIPCHK(apply(wk, Wk, ck, true, false, D));
    HIPCHK(apply(bk_, bk, ck, true, false, D));
    HIPCHK(apply(wv, Wv, cv, true, false, D));
    HIPCHK(apply(bv_, bv, cv, true, false, D));
    HIPCHK(apply(L.cwo, Wo, cv, false, true, D));
  }
  c->rebalanced = true;
  return ND_OK;
}

// Per-dimension power-of-two scales of the memory bank (transformer encoder).
// The bank holds m_i / c_i with m = LN(x) g + b (encoder/transformer.py:127):
// a dimension whose LN affine makes it far larger than the rest (an "outlier
// dimension", common in trained transformers) would otherwise set every row's
// 24-bit scale (bank8.hip: one scale per key row) and cost the other
// dimensions that many bits.  c_i = 2^k_i, k_i = clamp(floor(log2(a_i /
// median a)), 0, 12), a_i = 3 |g_i| + |b_i| (a LayerNorm'd value lies mostly
// within +-3); c_i is folded back exactly into W_qk's rows and W_vo's
// columns (derive_memory_bank_weights), so scores and context vectors are
// unchanged in exact arithmetic.  The NanoEncoder's bank keeps c = 1.
static int derive_bank_dim_scales(nd_ctx* c) {
  const int D = c->D;
  c->bank_dim_scale.assign(D, 1.f);
  if (c->cfg.encoder_type != ND_ENC_TRANSFORMER) return ND_OK;
  std::vector<float> g(D), b(D);
  HIPCHK(hipMemcpy(g.data(), c->enc_ln_g, D * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(b.data(), c->enc_ln_b, D * 4, hipMemcpyDeviceToHost));
  std::vector<double> a(D);
  for (int i = 0; i < D; ++i) a[i] = 3.0 * std::fabs((double)g[i]) + std::fabs((double)b[i]);
  std::vector<double> srt(a);
  std::nth_element(srt.begin(), srt.begin() + D / 2, srt.end());
  const double med = srt[D / 2];
  for (int i = 0; i < D; ++i) {
    int k = 0;
    if (med > 0 && a[i] > 0 && std::isfinite(a[i])) k = (int)std::floor(std::log2(a[i] / med));
    k = std::min(std::max(k, 0), 12);
    c->bank_dim_scale[i] = std::ldexp(1.f, k);
    g[i] = std::ldexp(g[i], -k);
    b[i] = std::ldexp(b[i], -k);
  }
  if (!c->bank_ln_g && dalloc(c, &c->bank_ln_g, D) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
  if (!c->bank_ln_b && dalloc(c, &c->bank_ln_b, D) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
  HIPCHK(hipMemcpy(c->bank_ln_g, g.data(), D * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->bank_ln_b, b.data(), D * 4, hipMemcpyHostToDevice));
  return ND_OK;
}

// Memory-bank form of the context attention (attention.hip): per decoder
// layer, in f64 on the host from the reference weights,
//   W_qk[h*256+i][k] = sum_a W_k[32h+a][i] W_q'[32h+a][k] / sqrt(32)
//   b_qk[h*256+i]    = sum_a W_k[32h+a][i] b_q'[32h+a]     / sqrt(32)
//   W_vo[n][h*256+i] = sum_a W_o[n][32h+a] W_v[32h+a][i]
//   b_vo[n]          = W_o[n] . b_v + b_o[n]
// with W_q' = W_q diag(ln2_g), b_q' = W_q ln2_b + b_q (layer_norm_2 folded).
// q_h . b_k,h is constant over keys and drops out of the softmax exactly.
// Row h*256+i of W_qk / b_qk and column h*256+i of W_vo carry the bank's
// per-dimension scale c_i (derive_bank_dim_scales; powers of two: exact).
static int derive_memory_bank_weights(nd_ctx* c) {
  const int D = c->D, H = ND_H, DH = ND_DH, Ld = (int)c->dec.size();
  auto down = [&](const float* d, size_t n, std::vector<float>& h) {
    h.resize(n);
    return hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
  };
  float* scratch = nullptr;
  HIPCHK(hipMalloc(&scratch, (size_t)H * D * D * sizeof(float)));
  std::vector<float> Wq, bq, g2, b2, Wk, Wv, bv, Wo, bo;
  std::vector<float> wqk((size_t)H * D * D), bqk((size_t)H * D), wvo((size_t)D * H * D), bvo(D);
  int rc = ND_OK;
  for (int i = 0; i < Ld && rc == ND_OK; ++i) {
    DecLayer& L = c->dec[i];
    hipError_t e = hipSuccess;
    if ((e = down(L.cwq, (size_t)D * D, Wq)) != hipSuccess || (e = down(L.cbq, D, bq)) != hipSuccess ||
        (e = down(L.ln2_g, D, g2)) != hipSuccess || (e = down(L.ln2_b, D, b2)) != hipSuccess ||
        (e = down(c->ctxkv_w + (size_t)(2 * i) * D * D, (size_t)D * D, Wk)) != hipSuccess ||
        (e = down(c->ctxkv_w + (size_t)(2 * i + 1) * D * D, (size_t)D * D, Wv)) != hipSuccess ||
        (e = down(c->ctxkv_b + (size_t)(2 * i + 1) * D, D, bv)) != hipSuccess ||
        (e = down(L.cwo, (size_t)D * D, Wo)) != hipSuccess || (e = down(L.cbo, D, bo)) != hipSuccess) {
      rc = fail(ND_ERR_HIP, std::string("memory-bank weights: ") + hipGetErrorString(e));
      break;
    }
    const double inv = 1.0 / std::sqrt((double)DH);
    std::vector<double> wq2((size_t)D * D), bq2(D);
    for (int a = 0; a < D; ++a) {
      double sb = bq[a];
      for (int k = 0; k < D; ++k) {
        wq2[(size_t)a * D + k] = (double)Wq[(size_t)a * D + k] * g2[k];
        sb += (double)Wq[(size_t)a * D + k] * b2[k];
      }
      bq2[a] = sb;
    }
    std::vector<double> row(D);
    for (int h = 0; h < H; ++h)
      for (int ii = 0; ii < D; ++ii) {
        std::fill(row.begin(), row.end(), 0.0);
        double sb = 0.0;
        for (int a = 0; a < DH; ++a) {
          const double wk = Wk[(size_t)(h * DH + a) * D + ii];
          const double* wr = &wq2[(size_t)(h * DH + a) * D];
          for (int k = 0; k < D; ++k) row[k] += wk * wr[k];
          sb += wk * bq2[h * DH + a];
        }
        const double ci = c->bank_dim_scale[ii];
        for (int k = 0; k < D; ++k) wqk[((size_t)h * D + ii) * D + k] = (float)(row[k] * inv * ci);
        bqk[(size_t)h * D + ii] = (float)(sb * inv * ci);
      }
    for (int n = 0; n < D; ++n) {
      double sb = bo[n];
      for (int j = 0; j < D; ++j) sb += (double)Wo[(size_t)n * D + j] * bv[j];
      bvo[n] = (float)sb;
      for (int h = 0; h < H; ++h) {
        std::fill(row.begin(), row.end(), 0.0);
        for (int a = 0; a < DH; ++a) {
          const double wo = Wo[(size_t)n * D + h * DH + a];
          const float* vr = &Wv[(size_t)(h * DH + a) * D];
          for (int ii = 0; ii < D; ++ii) row[ii] += wo * vr[ii];
        }
        for (int ii = 0; ii < D; ++ii) wvo[(size_t)n * H * D + h * D + ii] = (float)(row[ii] * c->bank_dim_scale[ii]);
      }
    }
    if ((e = hipMemcpy(scratch, wqk.data(), wqk.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = pack_step_weight(c, scratch, D, L.pwqk, H * D, D)) != hipSuccess ||
        (e = hipStreamSynchronize(c->es)) != hipSuccess ||
        (e = hipMemcpy(scratch, wvo.data(), wvo.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = pack_step_weight(c, scratch, H * D, L.pwvo, D, H * D)) != hipSuccess ||
        (e = hipStreamSynchronize(c->es)) != hipSuccess ||
        (e = hipMemcpy(L.bqk, bqk.data(), bqk.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(L.bvo, bvo.data(), bvo.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
      rc = fail(ND_ERR_HIP, std::string("memory-bank weights: ") + hipGetErrorString(e));
  }
  (void)hipFree(scratch);
  return rc;
}

int nd_finalize(nd_ctx* c) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  std::string missing;
  for (auto& kv : c->slots)
    if (kv.second.required && !kv.second.loaded) missing += (missing.empty() ? "" : ", ") + kv.first;
  if (!missing.empty()) return fail(ND_ERR_WEIGHT, "missing weights: " + missing);
  HIPCHK(hipSetDevice(c->cfg.device));
  if (int rc = rebalance_attention(c)) return rc;
  if (c->cfg.encoder_type == ND_ENC_NANO) {
    // derived: b_ih + b_hh per gate; eval BatchNorm as scale/shift
    const int Hh = c->H;
    for (auto& L : c->nano) {
      std::vector<float> bih(8 * Hh), bhh(8 * Hh), g(2 * Hh), b(2 * Hh), rm(2 * Hh), rv(2 * Hh);
      HIPCHK(hipMemcpy(bih.data(), L.bih, bih.size() * 4, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(bhh.data(), L.bhh, bhh.size() * 4, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(g.data(), L.bn_g, g.size() * 4, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(b.data(), L.bn_b, b.size() * 4, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(rm.data(), L.bn_rm, rm.size() * 4, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(rv.data(), L.bn_rv, rv.size() * 4, hipMemcpyDeviceToHost));
      std::vector<float> bs(8 * Hh), sc(2 * Hh), sh(2 * Hh);
      for (int i = 0; i < 8 * Hh; ++i) bs[i] = bih[i] + bhh[i];
      for (int i = 0; i < 2 * Hh; ++i) {
        sc[i] = (float)(1.0 / std::sqrt((double)rv[i] + 1e-5)) * g[i];
        sh[i] = b[i] - rm[i] * sc[i];
      }
      HIPCHK(hipMemcpy(L.bsum, bs.data(), bs.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(L.bn_scale, sc.data(), sc.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(L.bn_shift, sh.data(), sh.size() * 4, hipMemcpyHostToDevice));
    }
  }
  // LayerNorm affines folded into the Linear that consumes them
  {
    const int D = c->D, F = c->F;
    auto fold = [&](const float* W, const float* b, const float* g, const float* be, float* Wo, float* bo, int N,
                    int K) { return nd::launch_fold_layernorm(W, b, g, be, Wo, bo, N, K, c->es); };
    for (auto& L : c->enc) {
      HIPCHK(fold(L.wqkv, L.bqkv, L.ln_g, L.ln_b, L.nwqkv, L.nbqkv, 3 * D, D));
      HIPCHK(fold(L.w1, L.b1, L.fln_g, L.fln_b, L.nw1, L.nb1, F, D));
    }
    if (c->cfg.encoder_type == ND_ENC_TRANSFORMER && !c->enc.empty()) {
      if (!c->eq_ac && dalloc(c, &c->eq_ac, (size_t)6 * D) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
      if (!c->eq_scal && dalloc(c, &c->eq_scal, 3) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
      HIPCHK(nd::launch_embed_qkv_prep(c->enc_lin_w, c->enc_lin_b, c->enc[0].nwqkv, c->eq_ac, c->eq_scal, c->es));
      double m[3];
      HIPCHK(hipMemcpyAsync(m, c->eq_scal, sizeof(m), hipMemcpyDeviceToHost, c->es));
      HIPCHK(hipStreamSynchronize(c->es));
      for (int i = 0; i < 3; ++i) c->eq_m[i] = (float)m[i];
      // per head h: alpha = k0 y + k1 r + k2, beta = k3 y + k4 r + k5 with
      // k = (a_q, c_q, b_q) . (a_k | c_k) log2(e) / sqrt(32), in double
      std::vector<float> ac(6 * D), nb(3 * D), coef(ND_H * 6);
      HIPCHK(hipMemcpyAsync(ac.data(), c->eq_ac, ac.size() * 4, hipMemcpyDeviceToHost, c->es));
      HIPCHK(hipMemcpyAsync(nb.data(), c->enc[0].nbqkv, nb.size() * 4, hipMemcpyDeviceToHost, c->es));
      HIPCHK(hipStreamSynchronize(c->es));
      const double sc = 1.4426950408889634 / std::sqrt((double)(D / ND_H));
      for (int h = 0; h < ND_H; ++h) {
        double k[6] = {0, 0, 0, 0, 0, 0};
        for (int d = 0; d < D / ND_H; ++d) {
          const int i = h * (D / ND_H) + d;
          const double aq = ac[i], ak = ac[D + i], cq = ac[3 * D + i], ck = ac[4 * D + i], bq = nb[i];
          k[0] += aq * ak;
          k[1] += cq * ak;
          k[2] += bq * ak;
          k[3] += aq * ck;
          k[4] += cq * ck;
          k[5] += bq * ck;
        }
        for (int j = 0; j < 6; ++j) coef[h * 6 + j] = (float)(k[j] * sc);
      }
      if (!c->eq_coef && dalloc(c, &c->eq_coef, coef.size()) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
      HIPCHK(hipMemcpy(c->eq_coef, coef.data(), coef.size() * 4, hipMemcpyHostToDevice));
      c->eq_ready = true;
    }
    if (c->nctxkv_w)
      HIPCHK(fold(c->ctxkv_w, c->ctxkv_b, c->enc_ln_g, c->enc_ln_b, c->nctxkv_w, c->nctxkv_b,
                  (int)c->dec.size() * 2 * D, D));
    for (auto& L : c->dec) {
      if (c->cfg.self_attn_type == ND_SELF_AVERAGE) {
        HIPCHK(fold(L.aw1, L.ab1, L.aln_g, L.aln_b, L.naw1, L.nab1, D, D));
        HIPCHK(pack_step_weight(c, L.naw1, D, L.paw1, D, D));
        HIPCHK(pack_step_weight(c, L.aw2, D, L.paw2, D, D));
        HIPCHK(pack_step_weight(c, L.gw, 2 * D, L.pgwx, 2 * D, D));      // gate columns of xn
        HIPCHK(pack_step_weight(c, L.gw + D, 2 * D, L.pgwa, 2 * D, D));  // gate columns of a
      } else {
        HIPCHK(fold(L.wqkv, L.bqkv, L.ln1_g, L.ln1_b, L.nwqkv, L.nbqkv, 3 * D, D));
        HIPCHK(pack_step_weight(c, L.nwqkv, D, L.pwqkv, 3 * D, D));
        HIPCHK(pack_step_weight(c, L.wo, D, L.pwo, D, D));
      }
      HIPCHK(fold(L.cwq, L.cbq, L.ln2_g, L.ln2_b, L.ncwq, L.ncbq, D, D));
      HIPCHK(fold(L.w1, L.b1, L.fln_g, L.fln_b, L.nw1, L.nb1, F, D));
      HIPCHK(pack_step_weight(c, L.ncwq, D, L.pcwq, D, D));
      HIPCHK(pack_step_weight(c, L.cwo, D, L.pcwo, D, D));
      HIPCHK(pack_step_weight(c, L.nw1, D, L.pw1, F, D));
      HIPCHK(pack_step_weight(c, L.w2, F, L.pw2, D, F));
    }
    HIPCHK(hipStreamSynchronize(c->es));
  }
  {
    // split-fp16 images of the encoder-side row-major GEMM weights
    // (gemm.hip H3); ND_GEMM_F32=1 at run time keeps the fp32 kernels
    const int D = c->D, F = c->F, L2 = (int)c->dec.size() * 2 * D;
    hipError_t e_ = hipSuccess;
    auto mk = [&](const float* W, int N, int K) -> hipError_t {
      uint16_t* h = nullptr;
      float sc = 1.f;
      auto it = c->split.find(W);
      if (it != c->split.end()) h = it->second.first;  // finalize called again: refresh in place
      hipError_t e = h ? hipSuccess : dalloc(c, &h, (size_t)2 * N * K);
      if (e == hipSuccess) e = nd::launch_split_weight(W, N, K, h, &sc, c->es);
      if (e == hipSuccess) c->split[W] = {h, sc};
      return e;
    };
    for (auto& L : c->enc) {
      HIPCHK(mk(L.nwqkv, 3 * D, D));
      HIPCHK(mk(L.wo, D, D));
      HIPCHK(mk(L.nw1, F, D));
      HIPCHK(mk(L.w2, D, F));
      if (F % 32 == 0 && F <= 2048) {  // the fused FFN block's weight images
        if (!L.w1h && (e_ = dalloc(c, &L.w1h, (size_t)2 * F * D)) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
        if (!L.w2h && (e_ = dalloc(c, &L.w2h, (size_t)2 * F * D)) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
        HIPCHK(nd::launch_pack_p16h(L.nw1, D, F, D, L.w1h, &L.w1s, c->es));
        HIPCHK(nd::launch_pack_p16h(L.w2, F, D, F, L.w2h, &L.w2s, c->es));
        if (!L.woh && (e_ = dalloc(c, &L.woh, (size_t)2 * D * D)) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
        HIPCHK(nd::launch_pack_p16h(L.wo, D, D, D, L.woh, &L.wos, c->es));
        if (!L.qkvh && (e_ = dalloc(c, &L.qkvh, (size_t)2 * 3 * D * D)) != hipSuccess) return fail(ND_ERR_HIP, "alloc");
        HIPCHK(nd::launch_pack_p16h(L.nwqkv, D, 3 * D, D, L.qkvh, &L.qkvs, c->es));
      }
    }
    HIPCHK(mk(c->cfg.encoder_type == ND_ENC_TRANSFORMER ? c->nctxkv_w : c->ctxkv_w, L2, D));
    for (size_t l = 1; l < c->nano.size(); ++l) HIPCHK(mk(c->nano[l].wih, 8 * c->H, 2 * c->H));
    if (c->nano_W) HIPCHK(mk(c->nano_W, D, 2 * c->H));
    HIPCHK(hipStreamSynchronize(c->es));
  }
  {
    int rc = derive_bank_dim_scales(c);
    if (!rc) rc = derive_memory_bank_weights(c);
    if (rc) return rc;
  }
  for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
  c->graphs.clear();
  c->finalized = true;
  return ND_OK;
}

int nd_share_weights(nd_ctx* c, const nd_ctx* src) {
  if (!c || !src) return fail(ND_ERR_ARG, "null ctx");
  if (!src->finalized) return fail(ND_ERR_STATE, "nd_share_weights: the source context is not finalized");
  if (c == src || c->finalized) return fail(ND_ERR_STATE, "nd_share_weights: the context already holds weights");
  for (const auto& kv : c->slots)
    if (kv.second.loaded) return fail(ND_ERR_STATE, "nd_share_weights: weights were loaded into the context");
  const nd_config &a = c->cfg, &b = src->cfg;
  if (a.encoder_type != b.encoder_type || a.self_attn_type != b.self_attn_type || a.enc_layers != b.enc_layers ||
      a.dec_layers != b.dec_layers || a.d_model != b.d_model || a.heads != b.heads || a.d_ff != b.d_ff ||
      a.vocab != b.vocab || a.rnn_hidden != b.rnn_hidden || a.position_encoding != b.position_encoding ||
      a.pad_idx != b.pad_idx || a.bos_idx != b.bos_idx || a.eos_idx != b.eos_idx || a.device != b.device)
    return fail(ND_ERR_ARG, "nd_share_weights: the model configurations differ");
  // every weight pointer and every image nd_finalize derived (the layer structs hold both; nothing in them is
  // a workspace).  The context's own raw weight buffers from nd_create stay allocated and are never read (a
  // few tens of MB at d_model 256): the derived images -- the split-fp16 and P16 forms, the memory-bank
  // products -- are what sharing saves, and every lane reads one copy.
  c->enc = src->enc;
  c->nano = src->nano;
  c->nano_W = src->nano_W;
  c->dec = src->dec;
  c->enc_lin_w = src->enc_lin_w;
  c->enc_lin_b = src->enc_lin_b;
  c->enc_ln_g = src->enc_ln_g;
  c->enc_ln_b = src->enc_ln_b;
  c->bank_ln_g = src->bank_ln_g;
  c->bank_ln_b = src->bank_ln_b;
  c->bank_dim_scale = src->bank_dim_scale;
  c->eq_ac = src->eq_ac;
  c->eq_scal = src->eq_scal;
  for (int i = 0; i < 3; ++i) c->eq_m[i] = src->eq_m[i];
  c->eq_ready = src->eq_ready;
  c->eq_coef = src->eq_coef;
  c->ctxkv_w = src->ctxkv_w;
  c->ctxkv_b = src->ctxkv_b;
  c->nctxkv_w = src->nctxkv_w;
  c->nctxkv_b = src->nctxkv_b;
  c->emb = src->emb;
  c->pe = src->pe;
  c->dec_ln_g = src->dec_ln_g;
  c->dec_ln_b = src->dec_ln_b;
  c->gen_w = src->gen_w;
  c->gen_b = src->gen_b;
  c->split = src->split;
  c->split_rm = src->split_rm;
  for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
  c->graphs.clear();
  c->shares = true;
  c->finalized = true;
  return ND_OK;
}

static int check_call(nd_ctx* c, int B, int T, int S) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  if (!c->finalized) return fail(ND_ERR_STATE, "nd_finalize has not been called");
  if (B < 1 || B > c->cfg.max_batch) return fail(ND_ERR_ARG, "B out of range [1, max_batch]");
  if (T < 1 || T > c->cfg.max_src_len) return fail(ND_ERR_ARG, "T out of range [1, max_src_len]");
  if (S < 1 || S > c->cfg.max_steps) return fail(ND_ERR_ARG, "max_len out of range [1, max_steps]");
  return ND_OK;
}

static int stage_inputs(nd_ctx* c, const float* sig, const int32_t* len, const int32_t* span, int B, int T,
                        hipStream_t cs) {
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(hipEventRecord(c->ev_in, cs));
  HIPCHK(hipStreamWaitEvent(c->es, c->ev_in, 0));
  HIPCHK(hipMemcpyAsync(c->sig, sig, (size_t)B * T * 4, hipMemcpyDeviceToDevice, c->es));
  HIPCHK(hipMemcpyAsync(c->len, len, (size_t)B * 4, hipMemcpyDeviceToDevice, c->es));
  HIPCHK(hipMemcpyAsync(c->span, span, (size_t)B * 4, hipMemcpyDeviceToDevice, c->es));
  return ND_OK;
}

static int release_to(nd_ctx* c, hipStream_t cs) {
  HIPCHK(hipEventRecord(c->ev_out, c->es));
  HIPCHK(hipStreamWaitEvent(cs, c->ev_out, 0));
  return ND_OK;
}

// the attention capture buffer, [decoder rows][max_steps][max_src_len], made on first use
static int ensure_attn(nd_ctx* c) {
  if (c->attn_raw) return ND_OK;
  const size_t R = ((size_t)c->cfg.max_batch * std::max(1, c->cfg.max_beam) + 15) / 16 * 16;
  hipError_t e = dalloc(c, &c->attn_raw, R * c->cfg.max_steps * c->cfg.max_src_len);
  if (e != hipSuccess) return fail(ND_ERR_HIP, std::string("hipMalloc attention capture: ") + hipGetErrorString(e));
  return ND_OK;
}

static int translate_greedy(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B,
                            int32_t T, int32_t max_len, int32_t min_len, int32_t* d_tokens, float* d_score,
                            float* d_logp, float* d_attn, void* stream, float temp = 0.f, int topk = 1,
                            unsigned long long seed = 0) {
  int rc = check_call(c, B, T, max_len);
  if (rc) return rc;
  if (!d_signal || !d_len || !d_span || !d_tokens || !d_score) return fail(ND_ERR_ARG, "null buffer");
  if (d_attn && (rc = ensure_attn(c))) return rc;
  hipStream_t cs = (hipStream_t)stream;
  if ((rc = stage_inputs(c, d_signal, d_len, d_span, B, T, cs))) return rc;
  const bool lp = d_logp != nullptr;
  GraphKey key{0, B, T, max_len, min_len, 1, 1, d_attn ? 1 : 0, lp ? 1 : 0, 0.f, c->kstamp_on ? 1 : 0};
  nd::Sampling smp;
  if (temp != 0.f && topk != 1) {  // sample_with_temperature's random branch (translator.py:376-393)
    smp.temp = temp;
    smp.topk = topk;
    smp.seed = c->seed_dev;
    key.topk = topk;
    key.temp = temp;
    // the seed travels as kernel arguments (captured at launch), not through host memory
    int* sw = reinterpret_cast<int*>(c->seed_dev);
    HIPCHK(nd::launch_fill_i32(sw, (int)(unsigned)(seed & 0xffffffffull), 1, c->es));
    HIPCHK(nd::launch_fill_i32(sw + 1, (int)(unsigned)(seed >> 32), 1, c->es));
  }
  if (c->timing) HIPCHK(hipEventRecord(c->ev_a, c->es));
  c->attn_on = d_attn != nullptr;
  set_memory_view(c, T, 1);
  rc = run_graph(c, key, [&](hipStream_t s) { return enqueue_greedy(c, B, T, max_len, min_len, lp, s, smp); });
  c->attn_on = false;
  if (rc) return rc;
  if (c->timing) HIPCHK(hipEventRecord(c->ev_b, c->es));
  HIPCHK(hipMemcpyAsync(d_tokens, c->gtok, (size_t)B * max_len * 4, hipMemcpyDeviceToDevice, c->es));
  HIPCHK(hipMemcpyAsync(d_score, c->gscore, (size_t)B * 4, hipMemcpyDeviceToDevice, c->es));
  if (lp) HIPCHK(hipMemcpyAsync(d_logp, c->glogp, (size_t)B * max_len * c->V * 4, hipMemcpyDeviceToDevice, c->es));
  if (d_attn)  // [B][max_steps][T] -> [B][max_len][T]
    HIPCHK(hipMemcpy2DAsync(d_attn, (size_t)max_len * T * 4, c->attn_raw, (size_t)c->cfg.max_steps * T * 4,
                            (size_t)max_len * T * 4, B, hipMemcpyDeviceToDevice, c->es));
  if (c->timing) {
    HIPCHK(hipEventSynchronize(c->ev_b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev_a, c->ev_b));
    c->t_enc = 0.f;
    c->t_dec = ms;
  }
  return release_to(c, cs);
}

int nd_translate_greedy(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B,
                        int32_t T, int32_t max_len, int32_t min_len, int32_t* d_tokens, float* d_score, float* d_logp,
                        void* stream) {
  return translate_greedy(c, d_signal, d_len, d_span, B, T, max_len, min_len, d_tokens, d_score, d_logp, nullptr,
                          stream);
}

int nd_translate_greedy_attn(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                             int32_t B, int32_t T, int32_t max_len, int32_t min_len, int32_t* d_tokens, float* d_score,
                             float* d_logp, float* d_attn, void* stream) {
  if (!d_attn) return fail(ND_ERR_ARG, "null attention buffer");
  return translate_greedy(c, d_signal, d_len, d_span, B, T, max_len, min_len, d_tokens, d_score, d_logp, d_attn,
                          stream);
}

static int translate_beam(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B,
                          int32_t T, int32_t beam, int32_t n_best, float alpha, int32_t max_len, int32_t min_len,
                          int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps, float* d_attn,
                          int32_t* d_done_step, void* stream) {
  int rc = check_call(c, B, T, max_len);
  if (rc) return rc;
  if (beam < 1 || beam > c->cfg.max_beam) return fail(ND_ERR_ARG, "beam out of range [1, max_beam]");
  if (n_best < 1 || n_best > beam) return fail(ND_ERR_ARG, "n_best out of range [1, beam]");
  if (c->V < beam) return fail(ND_ERR_ARG, "vocab smaller than beam");
  if (!d_signal || !d_len || !d_span || !d_tokens || !d_scores || !d_lens) return fail(ND_ERR_ARG, "null buffer");
  if (d_attn && (rc = ensure_attn(c))) return rc;
  hipStream_t cs = (hipStream_t)stream;
  if ((rc = stage_inputs(c, d_signal, d_len, d_span, B, T, cs))) return rc;
  // n_best hypothesis storage is sized by max_beam
  const int SEG = 10;
  const int st = c->kstamp_on ? 1 : 0;
  GraphKey k0{1, B, T, max_len, min_len, beam, n_best, -1, 0, alpha, st};
  k0.attn = d_attn ? 1 : 0;
  if (c->timing) HIPCHK(hipEventRecord(c->ev_a, c->es));
  c->attn_on = d_attn != nullptr;
  set_memory_view(c, T, beam);
  rc = run_graph(c, k0, [&](hipStream_t s) -> hipError_t {
    if (c->kstamp_on) LCHK(nd::launch_stamp_reset(c->kstamp, (int)c->dec.size() * c->cfg.max_steps, s));
    LCHK(enqueue_encode(c, B, T, s));
    LCHK(enqueue_memory(c, B, T, beam, s));  // K/V per layer (memory bank at beam 1)
    LCHK(nd::launch_beam_init(c->bs, B, beam, n_best, max_len, c->cfg.bos_idx, s));
    LCHK(enqueue_qkv_table(c, max_len, s));
    LCHK(enqueue_first_embed(c, B * beam, s));
    LCHK(nd::launch_fill_i32(c->steps_done, max_len, 1, s));
    return hipSuccess;
  });
  if (rc) {
    c->attn_on = false;
    return rc;
  }
  if (c->timing) HIPCHK(hipEventRecord(c->ev_b, c->es));
  c->beam_tail = false;
  for (int s0 = 0; s0 < max_len; s0 += SEG) {
    const int s1 = std::min(max_len, s0 + SEG);
    GraphKey k{1, B, T, max_len, min_len, beam, n_best, s0, 0, alpha, st};
    k.attn = k0.attn;
    rc = run_graph(c, k, [&](hipStream_t s) {
      return enqueue_beam_steps(c, B, T, beam, n_best, alpha, max_len, min_len, s0, s1, s);
    });
    if (rc) break;
    if (s1 < max_len) {
      HIPCHK(hipMemcpyAsync(c->h_alive, c->bs.n_alive, 4, hipMemcpyDeviceToHost, c->es));
      HIPCHK(hipStreamSynchronize(c->es));
      if (*c->h_alive == 0) break;
      // a sixteenth of the chunks or fewer left (a trained model's stragglers):
      // the remaining segments' GEMMs run on the latency-bound small-M kernels
      c->beam_tail = (long)*c->h_alive * 16 <= (long)B;
    }
  }
  c->beam_tail = false;
  c->attn_on = false;
  if (rc) return rc;
  if (c->timing) HIPCHK(hipEventRecord(c->ev_c, c->es));
  HIPCHK(nd::launch_beam_finish(c->bs, B, n_best, max_len, d_tokens, d_scores, d_lens, c->es));
  if (d_steps) HIPCHK(hipMemcpyAsync(d_steps, c->steps_done, 4, hipMemcpyDeviceToDevice, c->es));
  if (d_attn) {
    nd::BeamState bst = c->bs;
    bst.attn = c->attn_raw;
    HIPCHK(nd::launch_beam_attn_gather(bst, B, n_best, c->cfg.max_steps, max_len, T, d_attn, c->es));
  }
  if (d_done_step) HIPCHK(hipMemcpyAsync(d_done_step, c->bs.steps_run, (size_t)B * 4, hipMemcpyDeviceToDevice, c->es));
  if (c->timing) {
    HIPCHK(hipEventSynchronize(c->ev_c));
    HIPCHK(hipEventElapsedTime(&c->t_enc, c->ev_a, c->ev_b));
    HIPCHK(hipEventElapsedTime(&c->t_dec, c->ev_b, c->ev_c));
  }
  return release_to(c, cs);
}

int nd_translate_sample(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B,
                        int32_t T, int32_t max_len, int32_t min_len, float temp, int32_t keep_topk, uint64_t seed,
                        int32_t* d_tokens, float* d_score, float* d_logp, float* d_attn, void* stream) {
  if (keep_topk > c->V) return fail(ND_ERR_ARG, "random_sampling_topk larger than the vocabulary");
  return translate_greedy(c, d_signal, d_len, d_span, B, T, max_len, min_len, d_tokens, d_score, d_logp, d_attn,
                          stream, temp, keep_topk, (unsigned long long)seed);
}

int nd_translate_beam(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B,
                      int32_t T, int32_t beam, int32_t n_best, float alpha, int32_t max_len, int32_t min_len,
                      int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps, void* stream) {
  return translate_beam(c, d_signal, d_len, d_span, B, T, beam, n_best, alpha, max_len, min_len, d_tokens, d_scores,
                        d_lens, d_steps, nullptr, nullptr, stream);
}

int nd_translate_beam_attn(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B,
                           int32_t T, int32_t beam, int32_t n_best, float alpha, int32_t max_len, int32_t min_len,
                           int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps, float* d_attn,
                           int32_t* d_done_step, void* stream) {
  if (!d_attn || !d_done_step) return fail(ND_ERR_ARG, "null attention buffer");
  return translate_beam(c, d_signal, d_len, d_span, B, T, beam, n_best, alpha, max_len, min_len, d_tokens, d_scores,
                        d_lens, d_steps, d_attn, d_done_step, stream);
}

static int translate_classic(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                             const int32_t* d_group, const int32_t* d_cut, int32_t B, int32_t T, int32_t beam,
                             int32_t n_best, const nd_classic_opts& op, int32_t max_len, int32_t min_len,
                             int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps, float* d_attn,
                             void* stream) {
  int rc = check_call(c, B, T, max_len);
  if (rc) return rc;
  if (beam < 1 || beam > c->cfg.max_beam) return fail(ND_ERR_ARG, "beam out of range [1, max_beam]");
  if (n_best < 1 || n_best > beam) return fail(ND_ERR_ARG, "n_best out of range [1, beam]");
  if (c->V < beam) return fail(ND_ERR_ARG, "vocab smaller than beam");
  if (op.length_penalty < 0 || op.length_penalty > 2)
    return fail(ND_ERR_ARG, "length_penalty must be 0 (none), 1 (wu), 2 (avg)");
  if (op.coverage_penalty < 0 || op.coverage_penalty > 2)
    return fail(ND_ERR_ARG, "coverage_penalty must be 0 (none), 1 (wu), 2 (summary)");
  if (op.block_ngram_repeat < 0 || op.block_ngram_repeat > max_len)
    return fail(ND_ERR_ARG, "block_ngram_repeat out of range [0, max_len]");
  if (!d_signal || !d_len || !d_span || !d_group || !d_tokens || !d_scores || !d_lens)
    return fail(ND_ERR_ARG, "null buffer");
  if (op.coverage_penalty != 0 && !d_cut) return fail(ND_ERR_ARG, "coverage penalty needs the attention lengths");
  const bool capture = d_attn != nullptr || op.coverage_penalty != 0;
  if (capture && (rc = ensure_attn(c))) return rc;
  hipStream_t cs = (hipStream_t)stream;
  if ((rc = stage_inputs(c, d_signal, d_len, d_span, B, T, cs))) return rc;
  HIPCHK(hipMemcpyAsync(c->group_in, d_group, (size_t)B * 4, hipMemcpyDeviceToDevice, c->es));
  if (d_cut) HIPCHK(hipMemcpyAsync(c->cut_in, d_cut, (size_t)B * 4, hipMemcpyDeviceToDevice, c->es));
  const nd::ClassicOpts o{op.length_penalty, op.alpha, op.beta,          op.coverage_penalty,
                          op.stepwise_penalty, op.block_ngram_repeat, op.ignore_mask};
  const int SEG = 10;
  const int st = c->kstamp_on ? 1 : 0;
  // graph keys: mode 2, the length penalty kind in the logp slot
  GraphKey k0{2, B, T, max_len, min_len, beam, n_best, -1, op.length_penalty, op.alpha, st};
  k0.attn = capture ? 1 : 0;
  k0.cov = op.coverage_penalty;
  k0.stepwise = op.stepwise_penalty;
  k0.ngram = op.block_ngram_repeat;
  k0.excl = op.ignore_mask;
  k0.beta = op.beta;
  c->attn_on = capture;
  set_memory_view(c, T, beam);
  rc = run_graph(c, k0, [&](hipStream_t s) -> hipError_t {
    if (c->kstamp_on) LCHK(nd::launch_stamp_reset(c->kstamp, (int)c->dec.size() * c->cfg.max_steps, s));
    LCHK(enqueue_encode(c, B, T, s));
    LCHK(enqueue_memory(c, B, T, beam, s));  // K/V per layer (memory bank at beam 1)
    LCHK(nd::launch_beam_classic_init(c->bs, c->group_in, B, beam, c->cfg.bos_idx, s));
    LCHK(enqueue_qkv_table(c, max_len, s));
    LCHK(enqueue_first_embed(c, B * beam, s));
    LCHK(nd::launch_fill_i32(c->steps_done, max_len, 1, s));
    return hipSuccess;
  });
  if (rc) {
    c->attn_on = false;
    return rc;
  }
  for (int s0 = 0; s0 < max_len; s0 += SEG) {
    const int s1 = std::min(max_len, s0 + SEG);
    GraphKey k = k0;
    k.seg = s0;
    rc = run_graph(c, k, [&](hipStream_t s) {
      return enqueue_classic_steps(c, B, T, beam, n_best, o, max_len, min_len, s0, s1, s);
    });
    if (rc) break;
    if (s1 < max_len) {
      HIPCHK(hipMemcpyAsync(c->h_alive, c->bs.n_alive, 4, hipMemcpyDeviceToHost, c->es));
      HIPCHK(hipStreamSynchronize(c->es));
      if (*c->h_alive == 0) break;
    }
  }
  c->attn_on = false;
  if (rc) return rc;
  HIPCHK(nd::launch_beam_classic_finish(c->bs, B, beam, n_best, max_len, o, d_tokens, d_scores, d_lens, c->es));
  if (d_steps) HIPCHK(hipMemcpyAsync(d_steps, c->steps_done, 4, hipMemcpyDeviceToDevice, c->es));
  if (d_attn) {
    nd::BeamState bst = c->bs;
    bst.attn = c->attn_raw;
    HIPCHK(nd::launch_beam_attn_gather(bst, B, n_best, c->cfg.max_steps, max_len, T, d_attn, c->es));
  }
  return release_to(c, cs);
}

int nd_translate_beam_classic(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                              const int32_t* d_group, int32_t B, int32_t T, int32_t beam, int32_t n_best,
                              int32_t length_penalty, float alpha, int32_t max_len, int32_t min_len,
                              int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps, void* stream) {
  nd_classic_opts op{};
  op.length_penalty = length_penalty;
  op.alpha = alpha;
  return translate_classic(c, d_signal, d_len, d_span, d_group, nullptr, B, T, beam, n_best, op, max_len, min_len,
                           d_tokens, d_scores, d_lens, d_steps, nullptr, stream);
}

int nd_translate_beam_classic_ex(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span,
                                 const int32_t* d_group, const int32_t* d_cut, int32_t B, int32_t T, int32_t beam,
                                 int32_t n_best, const nd_classic_opts* opts, int32_t max_len, int32_t min_len,
                                 int32_t* d_tokens, float* d_scores, int32_t* d_lens, int32_t* d_steps, float* d_attn,
                                 void* stream) {
  if (!opts) return fail(ND_ERR_ARG, "null options");
  return translate_classic(c, d_signal, d_len, d_span, d_group, d_cut, B, T, beam, n_best, *opts, max_len, min_len,
                           d_tokens, d_scores, d_lens, d_steps, d_attn, stream);
}

int nd_encode(nd_ctx* c, const float* d_signal, const int32_t* d_len, const int32_t* d_span, int32_t B, int32_t T,
              float* d_memory, void* stream) {
  int rc = check_call(c, B, T, 1);
  if (rc) return rc;
  hipStream_t cs = (hipStream_t)stream;
  if ((rc = stage_inputs(c, d_signal, d_len, d_span, B, T, cs))) return rc;
  hipError_t e = enqueue_encode(c, B, T, c->es);
  if (e != hipSuccess) return fail(ND_ERR_HIP, g_err);
  if (c->cfg.encoder_type == ND_ENC_TRANSFORMER) {
    e = nd::launch_layernorm(c->x, c->enc_ln_g, c->enc_ln_b, d_memory, B * T, c->es);
    if (e != hipSuccess) return fail(ND_ERR_HIP, hipGetErrorString(e));
  } else {
    HIPCHK(hipMemcpyAsync(d_memory, c->x, (size_t)B * T * c->D * 4, hipMemcpyDeviceToDevice, c->es));
  }
  return release_to(c, cs);
}

void* nd_stream(nd_ctx* c) { return c ? (void*)c->es : nullptr; }

int nd_gemm_routes(int64_t* counts, int32_t n, int32_t reset) {
  if (!counts || n < 0) return fail(ND_ERR_ARG, "null argument");
  for (int r = 0; r < ND_ROUTE_N; ++r) {
    const long long v = nd::gemm_route_count(r, reset != 0);
    if (r < n) counts[r] = v;
  }
  return ND_OK;
}

// the A/B switches the launchers read (name, default); nd_switches reports the
// ones set to something else
static const struct {
  const char* name;
  int def;
} kSwitches[] = {{"ND_GEMM_F32", 0},  {"ND_ENC_ATTN_F32", 0}, {"ND_LSTM_F32", 0},
                 {"ND_ENC_ATTN0", 1}, {"ND_BEAM_COMPACT", 1}, {"ND_CTX_SPLIT", 16},
                 {"ND_DEC_FFN", 1}};

int nd_switches(char* buf, int32_t len) {
  std::string out;
  int n = 0;
  for (const auto& sw : kSwitches) {
    const char* e = getenv(sw.name);
    if (!e || atoi(e) == sw.def) continue;
    out += (n ? ";" : "") + std::string(sw.name) + "=" + e;
    ++n;
  }
  if (buf && len > 0) {
    const size_t k = std::min(out.size(), (size_t)len - 1);
    memcpy(buf, out.data(), k);
    buf[k] = 0;
  }
  return n;
}

int nd_set_graphs(nd_ctx* c, int enable) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  c->use_graphs = enable != 0;
  return ND_OK;
}

int nd_set_ctx_path(nd_ctx* c, int path) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  if (path < 0 || path > 1) return fail(ND_ERR_ARG, "path must be 0 (auto) or 1 (K/V form)");
  if (path == 1) {  // a greedy-only context allocates the context K/V now (beam contexts have it)
    HIPCHK(hipSetDevice(c->cfg.device));
    const int rc = alloc_ctx_kv(c);
    if (rc != ND_OK) return rc;
  }
  if (c->ctx_path != path) {
    for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
    c->graphs.clear();
  }
  c->ctx_path = path;
  return ND_OK;
}

int nd_set_bank_policy(nd_ctx* c, int nontemporal) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  c->bank_nt = nontemporal != 0;  // graphs are keyed by it
  return ND_OK;
}

int nd_set_bank_grid(nd_ctx* c, int32_t workgroups) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  if (workgroups < 0) return fail(ND_ERR_ARG, "bank grid: workgroups must be >= 0");
  c->bank_grid = workgroups;  // graphs are keyed by it
  return ND_OK;
}

int nd_set_gemm_splitk(nd_ctx* c, int32_t on) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  c->splitk = on != 0;  // graphs are keyed by it
  return ND_OK;
}

int nd_set_exact_fp32(nd_ctx* c, int enable) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  c->exact = enable != 0;  // graphs are keyed by it
  return ND_OK;
}

int nd_take_overflow(nd_ctx* c, int32_t* d_out, void* stream) {
  if (!c || !d_out) return fail(ND_ERR_ARG, "null argument");
  HIPCHK(hipSetDevice(c->cfg.device));
  const hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipMemcpyAsync(d_out, c->ovf, sizeof(int), hipMemcpyDeviceToDevice, s));
  HIPCHK(hipMemsetAsync(c->ovf, 0, sizeof(int), s));
  return ND_OK;
}

int nd_set_timing(nd_ctx* c, int enable) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  c->timing = enable != 0;
  return ND_OK;
}

int nd_set_kernel_stamps(nd_ctx* c, int enable) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  c->kstamp_on = enable != 0;
  return ND_OK;
}

int nd_kernel_stamps(nd_ctx* c, float* avg_us, int32_t* launches) {
  if (!c || !avg_us || !launches) return fail(ND_ERR_ARG, "null argument");
  const size_t n = c->dec.size() * (size_t)c->cfg.max_steps;
  std::vector<unsigned long long> h(2 * n);
  HIPCHK(hipSetDevice(c->cfg.device));
  HIPCHK(hipStreamSynchronize(c->es));
  HIPCHK(hipMemcpy(h.data(), c->kstamp, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  int rate_khz = 0;
  HIPCHK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->cfg.device));
  double sum = 0.0;
  int cnt = 0;
  for (size_t i = 0; i < n; ++i)
    if (h[2 * i] != ~0ull && h[2 * i + 1] >= h[2 * i]) {
      sum += (double)(h[2 * i + 1] - h[2 * i]);
      ++cnt;
    }
  *launches = cnt;
  *avg_us = cnt && rate_khz > 0 ? (float)(sum / cnt / rate_khz * 1e3) : 0.f;
  return ND_OK;
}

int nd_last_timing(nd_ctx* c, float* encode_ms, float* decode_ms) {
  if (!c) return fail(ND_ERR_ARG, "null ctx");
  if (encode_ms) *encode_ms = c->t_enc;
  if (decode_ms) *decode_ms = c->t_dec;
  return ND_OK;
}

void nd_destroy(nd_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  if (c->es) (void)hipStreamSynchronize(c->es);
  for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->h_alive) (void)hipHostFree(c->h_alive);
  for (hipEvent_t e : {c->ev_in, c->ev_out, c->ev_a, c->ev_b, c->ev_c})
    if (e) (void)hipEventDestroy(e);
  if (c->es) release_stream(c->cfg.device, c->es);  // synchronised above; recycled, not destroyed
  delete c;
}

int nd_op_gemm(const float* A, const float* W, const float* bias, const float* R, float* C, int32_t M, int32_t N,
               int32_t K, int32_t norm, int32_t relu, void* stream) {
  hipError_t e = gemm(A, K, W, N, K, bias, C, N, M, (hipStream_t)stream, norm != 0, relu != 0, R, N);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("gemm: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_split_weight(const float* W, int32_t N, int32_t K, uint16_t* Wh, float* wscale, void* stream) {
  hipError_t e = nd::launch_split_weight(W, N, K, Wh, wscale, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("split_weight: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_gemm_split(const float* A, const uint16_t* Wh, float wscale, const float* bias, const float* R, float* C,
                     int32_t M, int32_t N, int32_t K, int32_t norm, int32_t relu, void* stream) {
  if (!Wh) return fail(ND_ERR_ARG, "gemm_split: null Wh");
  G g(A, K, nullptr, N, K, bias, C, N, M);
  g.a.Wh = Wh;
  g.a.wscale = wscale;
  g.a.norm = norm != 0;
  g.a.relu = relu != 0;
  if (R) g.res(R, N);
  hipError_t e = g.run((hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("gemm_split: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_gemm_split_q24(const float* A, const uint16_t* Wh, float wscale, const float* bias, void* img,
                         int32_t plane_rows, int32_t M, int32_t N, int32_t K, int32_t norm, void* stream) {
  if (!Wh || !img || plane_rows < M) return fail(ND_ERR_ARG, "gemm_split_q24: null Wh / image, or plane_rows < M");
  G g(A, K, nullptr, N, K, bias, nullptr, N, M);
  g.a.Wh = Wh;
  g.a.wscale = wscale;
  g.a.norm = norm != 0;
  g.q24(static_cast<uint8_t*>(img), (size_t)plane_rows * CTXQ_ROW);
  hipError_t e = g.run((hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("gemm_split_q24: ") + hipGetErrorString(e));
  return ND_OK;
}

static int ensure_attributes() {
  static hipError_t e = nd::init_kernel_attributes();
  return e == hipSuccess ? ND_OK : fail(ND_ERR_HIP, "hipFuncSetAttribute failed");
}

int nd_op_dec_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h, float w2s,
                  const float* b2, float* x, float* xpart, int32_t M, int32_t F, int32_t nsplit, float* slab,
                  int32_t* tickets, const int32_t* skip, int32_t skip_rpc, int32_t* overflow, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  nd::DecFfn df;
  df.nsplit = nsplit;
  df.slab = slab;
  df.tickets = tickets;
  df.skip = skip;
  df.skip_rpc = skip_rpc;
  hipError_t e = nd::launch_dec_ffn(y, w1h, w1s, b1, w2h, w2s, b2, x, xpart, M, F, overflow, df, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_ffn: ") + hipGetErrorString(e));
  return ND_OK;
}

int64_t nd_op_dec_ffn_slab_floats(int32_t M, int32_t nsplit) {
  return M > 0 && nsplit > 0 ? (int64_t)nd::dec_ffn_slab_floats(M, nsplit) : 0;
}

int nd_op_gemm_p16(const float* A, const float* W, const float* bias, const float* R, float* C, int32_t M,
                   int32_t N, int32_t K, const float* part_in, int32_t part_n_in, float* part_out, int32_t relu,
                   int32_t* part_n_out, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  nd::GemmArgs g;
  g.A = A; g.W = W; g.bias = bias; g.R = R; g.C = C; g.M = M; g.N = N; g.K = K; g.relu = relu != 0;
  g.norm = part_in != nullptr; g.part_in = part_in; g.part_n_in = part_n_in; g.part_out = part_out;
  hipError_t e = nd::launch_gemm_p16(g, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("gemm_p16: ") + hipGetErrorString(e));
  if (part_n_out) *part_n_out = g.part_n_out;
  return ND_OK;
}

int nd_op_pack_p16h(const float* W, int32_t N, int32_t K, uint16_t* out, float* wscale, void* stream) {
  hipError_t e = nd::launch_pack_p16h(W, K, N, K, out, wscale, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("pack_p16h: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_enc_ffn(const float* y, const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h, float w2s,
                  const float* b2, float* x, float* xpart, int32_t M, int32_t F, int32_t* overflow, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  hipError_t e = nd::launch_enc_ffn(y, w1h, w1s, b1, w2h, w2s, b2, x, xpart, M, F, overflow, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("enc_ffn: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_enc_ffn_wo(const float* att, const float* x_in, const uint16_t* woh, float wos, const float* bo,
                     const uint16_t* w1h, float w1s, const float* b1, const uint16_t* w2h, float w2s, const float* b2,
                     float* x, float* xpart, const uint16_t* qkvh, float qkvs, const float* qkvb, float* qkv,
                     int32_t M, int32_t F, int32_t* overflow, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  nd::EncWo wo;
  wo.att = att;
  wo.woh = woh;
  wo.wos = wos;
  wo.bo = bo;
  nd::EncQkv qk;
  qk.wh = qkvh;
  qk.ws = qkvs;
  qk.bias = qkvb;
  qk.out = qkv;
  hipError_t e = nd::launch_enc_ffn(x_in, w1h, w1s, b1, w2h, w2s, b2, x, xpart, M, F, overflow, (hipStream_t)stream,
                                    &wo, qkvh ? &qk : nullptr);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("enc_ffn_wo: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_gemm_p16_split(const float* A, const uint16_t* Wh, float wscale, const float* bias, const float* R, float* C,
                         int32_t M, int32_t N, int32_t K, const float* part_in, int32_t part_n_in, float* part_out,
                         int32_t relu, int32_t* part_n_out, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  if (!Wh) return fail(ND_ERR_ARG, "gemm_p16_split: null Wh");
  nd::GemmArgs g;
  g.A = A; g.Wh = Wh; g.wscale = wscale; g.bias = bias; g.R = R; g.C = C; g.M = M; g.N = N; g.K = K;
  g.relu = relu != 0; g.norm = part_in != nullptr; g.part_in = part_in; g.part_n_in = part_n_in;
  g.part_out = part_out;
  hipError_t e = nd::launch_gemm_p16(g, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("gemm_p16_split: ") + hipGetErrorString(e));
  if (part_n_out) *part_n_out = g.part_n_out;
  return ND_OK;
}

static int gemm_p16_splitk(const float* A, const uint16_t* Wh, const float* W, float wscale, const float* bias,
                           const float* R, float* C, int32_t M, int32_t N, int32_t K, float* part_out, float* slab,
                           int32_t* tickets, int32_t tiles, int32_t* part_n_out, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  if (!A || (!Wh && !W) || !C || !slab || !tickets || tiles < 1)
    return fail(ND_ERR_ARG, "gemm_p16_splitk: bad arguments");
  if ((K != 1024 && K != 2048) || N % 32 || M <= 128 || ((M + 31) / 32) * (N / 32) > tiles)
    return fail(ND_ERR_ARG, "gemm_p16_splitk: needs K 1024 / 2048, N % 32 == 0, M > 128 and enough tiles");
  nd::GemmArgs g;
  g.A = A; g.Wh = Wh; g.W = W; g.wscale = wscale; g.bias = bias; g.R = R; g.C = C; g.M = M; g.N = N; g.K = K;
  g.part_out = part_out;
  g.sk_slab = slab; g.sk_cnt = tickets; g.sk_tiles = tiles;
  const long long before = nd::gemm_route_count(ND_ROUTE_P16_SPLITK, false);
  hipError_t e = nd::launch_gemm_p16(g, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("gemm_p16_splitk: ") + hipGetErrorString(e));
  if (nd::gemm_route_count(ND_ROUTE_P16_SPLITK, false) == before) return fail(ND_ERR_ARG, "gemm_p16_splitk: not taken");
  if (part_n_out) *part_n_out = g.part_n_out;
  return ND_OK;
}

int nd_op_gemm_p16_splitk(const float* A, const uint16_t* Wh, float wscale, const float* bias, const float* R,
                          float* C, int32_t M, int32_t N, int32_t K, float* part_out, float* slab, int32_t* tickets,
                          int32_t tiles, int32_t* part_n_out, void* stream) {
  if (!Wh) return fail(ND_ERR_ARG, "gemm_p16_splitk: null Wh");
  return gemm_p16_splitk(A, Wh, nullptr, wscale, bias, R, C, M, N, K, part_out, slab, tickets, tiles, part_n_out,
                         stream);
}

int nd_op_gemm_p16_splitk_f32(const float* A, const float* W, const float* bias, const float* R, float* C,
                              int32_t M, int32_t N, int32_t K, float* part_out, float* slab, int32_t* tickets,
                              int32_t tiles, int32_t* part_n_out, void* stream) {
  if (!W) return fail(ND_ERR_ARG, "gemm_p16_splitk_f32: null W");
  return gemm_p16_splitk(A, nullptr, W, 1.0f, bias, R, C, M, N, K, part_out, slab, tickets, tiles, part_n_out,
                         stream);
}

int nd_op_gemm_p16_split_rm(const float* A, const uint16_t* Wh, float wscale, const uint16_t* Wh_rm, float wscale_rm,
                            const float* bias, const float* R, float* C, int32_t M, int32_t N, int32_t K,
                            const float* part_in, int32_t part_n_in, float* part_out, int32_t relu,
                            int32_t* part_n_out, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  if (!Wh || !Wh_rm) return fail(ND_ERR_ARG, "gemm_p16_split_rm: null weight image");
  nd::GemmArgs g;
  g.A = A; g.Wh = Wh; g.wscale = wscale; g.Wh_rm = Wh_rm; g.wscale_rm = wscale_rm; g.bias = bias; g.R = R; g.C = C;
  g.M = M; g.N = N; g.K = K; g.relu = relu != 0; g.norm = part_in != nullptr; g.part_in = part_in;
  g.part_n_in = part_n_in; g.part_out = part_out;
  hipError_t e = nd::launch_gemm_p16(g, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("gemm_p16_split_rm: ") + hipGetErrorString(e));
  if (part_n_out) *part_n_out = g.part_n_out;
  return ND_OK;
}

int nd_op_pack_p16(const float* src, float* dst, int32_t M, int32_t N, void* stream) {
  hipError_t e = nd::launch_pack_p16(src, N, dst, M, N, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("pack_p16: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_fold_layernorm(const float* W, const float* bias, const float* ln_g, const float* ln_b, float* W_out,
                         float* b_out, int32_t N, int32_t K, void* stream) {
  hipError_t e = nd::launch_fold_layernorm(W, bias, ln_g, ln_b, W_out, b_out, N, K, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("fold_layernorm: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_enc_attention(const float* qkv, const float* signal, const int32_t* span, float* out, int32_t B, int32_t T,
                        void* stream) {
  hipError_t e = nd::launch_enc_attention(qkv, signal, span, out, B, T, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("enc_attention: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_dec_self_attention(const float* qkv, float* cache, const int32_t* anc, int32_t anc_ld, int32_t step,
                             int32_t max_steps, float* out, int32_t R, void* stream) {
  hipError_t e = nd::launch_dec_self_attention(qkv, cache, anc, anc_ld, step, max_steps, out, R, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_self_attention: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_dec_self_attention_beam(const float* qkv, float* cache, const int32_t* anc, int32_t anc_ld, int32_t step,
                                  int32_t max_steps, float* out, int32_t R, int32_t rpc, const int32_t* done,
                                  void* stream) {
  if (!qkv || !cache || !anc || !out || rpc < 2 || rpc > 8 || R % rpc)
    return fail(ND_ERR_ARG, "dec_self_attention_beam: bad arguments");
  hipError_t e = nd::launch_dec_self_attention(qkv, cache, anc, anc_ld, step, max_steps, out, R, (hipStream_t)stream,
                                               rpc, done);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_self_attention_beam: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_dec_self_attention_q24(const float* qkv, void* cache, const int32_t* anc, int32_t anc_ld, int32_t step,
                                 int32_t max_steps, float* out, int32_t R, int32_t rpc, const int32_t* done,
                                 void* stream) {
  if (!qkv || !cache || !out || rpc < 1 || rpc > 8 || R % rpc || (rpc > 1 && !anc))
    return fail(ND_ERR_ARG, "dec_self_attention_q24: bad arguments");
  hipError_t e = nd::launch_dec_self_attention(qkv, static_cast<float*>(cache), anc, anc_ld, step, max_steps, out, R,
                                               (hipStream_t)stream, rpc, done, nd::QkvRows(), nullptr, nullptr, 0,
                                               true);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_self_attention_q24: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_dec_mem_attention(const float* qp, const float* mem, const float* signal, const int32_t* span, float pad_val,
                            float* out, int32_t C, int32_t rpc, int32_t T, int32_t ldT, int32_t grid, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  hipError_t e = nd::launch_dec_mem_attention(qp, mem, signal, span, pad_val, out, C, rpc, T, ldT, (hipStream_t)stream,
                                              nullptr, nullptr, 0, grid);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_mem_attention: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_lstm_layer(const float* xp, const float* signal, const float* wih0, const float* bsum, const float* whh,
                     const int32_t* len, int32_t B, int32_t T, float* out, const float* bn_scale,
                     const float* bn_shift, int32_t layer0, void* stream) {
  if (B < 1 || T < 1 || !whh || !len || !out || (layer0 ? (!signal || !wih0 || !bsum) : !xp))
    return fail(ND_ERR_ARG, "lstm_layer: bad arguments");
  if ((bn_scale == nullptr) != (bn_shift == nullptr))
    return fail(ND_ERR_ARG, "lstm_layer: bn_scale and bn_shift must both be set or both be null");
  hipError_t e = nd::launch_lstm_layer(xp, signal, wih0, bsum, whh, len, B, T, out, bn_scale, bn_shift, layer0 != 0,
                                       (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("lstm_layer: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_normalize_reads(const double* d_raw, const int64_t* d_offsets, int32_t R, int32_t method, float* d_out,
                       void* stream) {
  hipError_t e = nd::launch_read_normalize(d_raw, (const long long*)d_offsets, R, method, d_out, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("normalize_reads: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_window_reads(const float* d_sig, const int64_t* d_offsets, const int32_t* d_read, const int32_t* d_start,
                    const int32_t* d_len, int32_t C, int32_t T, float* d_signal, void* stream) {
  hipError_t e = nd::launch_read_window(d_sig, (const long long*)d_offsets, d_read, d_start, d_len, C, T, d_signal,
                                        (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("window_reads: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_memory_pack(const float* x, const float* ln_g, const float* ln_b, float* out, int32_t B, int32_t T,
                      int32_t ldT, void* stream) {
  hipError_t e = nd::launch_memory_pack(x, ln_g, ln_b, out, B, T, ldT, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("memory_pack: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_bank_pack_d8(const float* x, const float* ln_g, const float* ln_b, void* bank, float* kscale,
                       int32_t* kemax, const int32_t* span, int32_t B, int32_t T, int32_t* ovf, void* stream) {
  if (!x || !bank || !kscale || !kemax || (ln_g == nullptr) != (ln_b == nullptr))
    return fail(ND_ERR_ARG, "bank_pack_d8: bad arguments");
  hipError_t e = nd::launch_bank_pack_d8(x, ln_g, ln_b, bank, kscale, kemax, span, B, T, ovf, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("bank_pack_d8: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_dec_bank_d8(const float* qp, const void* bank, const float* kscale, const int32_t* kemax,
                      const float* signal, const int32_t* span, float pad_val, float* out, int32_t C, int32_t T,
                      int32_t* ovf, int32_t grid, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  if (!qp || !bank || !kscale || !kemax || !signal || !span || !out || grid < 0)
    return fail(ND_ERR_ARG, "dec_bank_d8: bad arguments");
  hipError_t e = nd::launch_dec_bank_d8(qp, bank, kscale, kemax, signal, span, pad_val, out, C, T,
                                        (hipStream_t)stream, nullptr, nullptr, 0, ovf, false, grid);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_bank_d8: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_bank_form(nd_ctx* c) { return c ? c->last_bank_form : 0; }

int nd_op_dec_ctx_attention(const float* q, const float* kv, int32_t ld, int32_t koff, const float* signal,
                            const int32_t* span, float pad_val, float* out, int32_t C, int32_t rpc, int32_t T,
                            void* stream) {
  if (int rc = ensure_attributes()) return rc;
  hipError_t e = nd::launch_dec_ctx_attention(q, kv, ld, koff, signal, span, pad_val, out, C, rpc, T,
                                              (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_ctx_attention: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_ctx_pack_q24(const float* kv, int32_t ld, int32_t layers, void* out, const int32_t* span, int32_t B,
                       int32_t T, void* stream) {
  if (!kv || !out || !span) return fail(ND_ERR_ARG, "ctx_pack_q24: bad arguments");
  hipError_t e = nd::launch_ctx_pack_q24(kv, ld, layers, static_cast<uint8_t*>(out), span, B, T, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("ctx_pack_q24: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_dec_ctx_attention_list(const float* q, const void* kv, int32_t ld, int32_t koff, int32_t q24,
                                 const float* signal, const int32_t* span, float pad_val, float* out, int32_t C,
                                 int32_t rpc, int32_t T, const int32_t* clist, int32_t ccap, int32_t nsplit,
                                 float* part, const int32_t* done, void* stream) {
  if (int rc = ensure_attributes()) return rc;
  if (!q || !kv || !signal || !span || !out || !clist || (nsplit > 1 && !part))
    return fail(ND_ERR_ARG, "dec_ctx_attention_list: bad arguments");
  hipError_t e = nd::launch_dec_ctx_attention(q, kv, ld, koff, signal, span, pad_val, out, C, rpc, T,
                                              (hipStream_t)stream, nullptr, nullptr, 0, done, q24 != 0, clist, ccap,
                                              nsplit, part);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_ctx_attention_list: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_alive_list(const int32_t* done, int32_t C, int32_t* list, int32_t cap, int32_t* ovf, void* stream) {
  if (!done || !list) return fail(ND_ERR_ARG, "alive_list: bad arguments");
  hipError_t e = nd::launch_alive_list(done, C, list, cap, ovf, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("alive_list: ") + hipGetErrorString(e));
  return ND_OK;
}

int nd_op_dec_ctx_attention_q24(const float* q, const void* kvq, int32_t layers, int32_t layer, const float* signal,
                                const int32_t* span, float pad_val, float* out, int32_t C, int32_t rpc, int32_t T,
                                void* stream) {
  if (int rc = ensure_attributes()) return rc;
  if (!q || !kvq || !signal || !span || !out || layer < 0 || layer >= layers)
    return fail(ND_ERR_ARG, "dec_ctx_attention_q24: bad arguments");
  const uint8_t* plane = static_cast<const uint8_t*>(kvq) + (size_t)layer * C * T * CTXQ_ROW;
  hipError_t e = nd::launch_dec_ctx_attention(q, plane, CTXQ_ROW, 0, signal, span, pad_val, out, C, rpc, T,
                                              (hipStream_t)stream, nullptr, nullptr, 0, nullptr, true);
  if (e != hipSuccess) return fail(ND_ERR_ARG, std::string("dec_ctx_attention_q24: ") + hipGetErrorString(e));
  return ND_OK;
}

}  // extern "C"

// NanoEncoder (encoder/nano_encoder.py:79-124): 3x BiLSTM; layers 0-1 emit
// BatchNorm(h) for the next layer, layer 2 emits raw h (zeros at padded
// steps, as pad_packed_sequence does); memory = h W^T -> c->x.
static hipError_t enqueue_encode_nano(nd_ctx* c, int B, int T, hipStream_t s) {
  const int M = B * T, D = c->D, Lz = (int)c->nano.size();
  float* bufs[2] = {c->y, c->att};
  for (int l = 0; l < Lz; ++l) {
    NanoLayer& L = c->nano[l];
    float* out = bufs[l & 1];
    const bool last = l == Lz - 1;
    if (l > 0)
      LCHK(G(bufs[(l - 1) & 1], 2 * c->H, L.wih, 8 * c->H, 2 * c->H, L.bsum, c->nano_xp, 8 * c->H, M).h3(c).run(s));
    if (last) LCHK(hipMemsetAsync(out, 0, (size_t)M * 2 * c->H * sizeof(float), s));
    LCHK(nd::launch_lstm_layer(c->nano_xp, c->sig, L.wih, L.bsum, L.whh, c->len, B, T, out,
                               last ? nullptr : L.bn_scale, last ? nullptr : L.bn_shift, l == 0, s, c->exact));
  }
  return G(bufs[(Lz - 1) & 1], 2 * c->H, c->nano_W, D, 2 * c->H, nullptr, c->x, D, M).h3(c).run(s);
}

static hipError_t enqueue_encode(nd_ctx* c, int B, int T, hipStream_t s) {
  // every call starts with the split-K tickets at zero (a memset node in the call's graph): each tile's last
  // arriver resets its own, this repairs a ticket left by an aborted call (cdna_hip_programming.md §6,
  // Guideline 16 "Re-initialise every call")
  if (c->sk_cnt) LCHK(hipMemsetAsync(c->sk_cnt, 0, (size_t)(c->sk_tiles + 3) / 4 * 16, s));
  if (c->dffn_cnt) LCHK(hipMemsetAsync(c->dffn_cnt, 0, (size_t)(c->dffn_rb + 3) / 4 * 16, s));
  if (c->cfg.encoder_type == ND_ENC_TRANSFORMER) return enqueue_encode_transformer(c, B, T, s);
  return enqueue_encode_nano(c, B, T, s);
}
