"""CPU restatement of NanoDecoder's translate hot path — TEST INFRASTRUCTURE.

This is the oracle: the parity checker for the HIP engine and the timed CPU
baseline in ``bench.py``.  It is plain PyTorch fp32 on the CPU, written from the
reference's semantics, each function citing the
reference file:line it follows.  It is pinned against golden vectors produced
by the reference's own modules (``oracle/make_golden.py`` →
``tests/golden/*.npz``; ``tests/test_oracle.py`` checks it to <=1e-5).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module.  The product path (``nanodecoder_amd``) never does.

Layouts: ``src`` is [B, T] float32 (chunk-major, zero padded), ``lengths`` [B].
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

EPS_LN = 1e-6    # nn.LayerNorm(d, eps=1e-6): encoder/transformer.py:32,103; position_ffn.py:22
EPS_BN = 1e-5    # nn.BatchNorm1d default eps: encoder/nano_encoder.py:56,64
MASK_FILL = -1e18  # onmt/modules/multi_headed_attn.py:172


def _t(x):
    return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float32)


class RefModel:
    """Weights (reference state-dict names) + architecture (synth.ModelConfig)."""

    def __init__(self, cfg, W: Dict[str, np.ndarray]):
        self.cfg = cfg
        self.W = {k: _t(v) for k, v in W.items()}
        self.d = cfg.d_model
        self.h = cfg.heads
        self.dh = cfg.d_model // cfg.heads

    # ----------------------------------------------------------- primitives
    def lin(self, x, name, bias=True):
        y = x @ self.W[name + ".weight"].t()
        return y + self.W[name + ".bias"] if bias else y

    def ln(self, x, name):
        return torch.nn.functional.layer_norm(x, (x.shape[-1],), self.W[name + ".weight"],
                                              self.W[name + ".bias"], EPS_LN)

    def ffn(self, x, p):
        """onmt/modules/position_ffn.py:27-40: x + W2 relu(W1 LN(x) + b1) + b2."""
        inter = torch.relu(self.lin(self.ln(x, p + ".layer_norm"), p + ".w_1"))
        return self.lin(inter, p + ".w_2") + x

    def _heads(self, x):       # [B, L, d] -> [B, h, L, dh]   (multi_headed_attn.py:113-116)
        B = x.shape[0]
        return x.view(B, -1, self.h, self.dh).transpose(1, 2)

    def _unheads(self, x):     # [B, h, L, dh] -> [B, L, d]  (multi_headed_attn.py:118-121)
        B = x.shape[0]
        return x.transpose(1, 2).contiguous().view(B, -1, self.d)

    def attend(self, q, k, v, key_mask=None):
        """multi_headed_attn.py:166-177: (q/sqrt(dh)) k^T, masked_fill(-1e18),
        softmax, @ v.  q,k,v are [B, h, L, dh]; key_mask [B, 1, Lk] bool."""
        q = q / math.sqrt(self.dh)
        s = torch.matmul(q, k.transpose(2, 3))
        if key_mask is not None:
            s = s.masked_fill(key_mask.unsqueeze(1), MASK_FILL)
        p = torch.softmax(s, dim=-1)
        return torch.matmul(p, v), p

    # -------------------------------------------------------------- encoders
    def encode_transformer(self, src):
        """encoder/transformer.py:106-127.  src [B, T] -> memory [B, T, d]."""
        # Linear(1, d) (:104,113)
        x = src.unsqueeze(-1) @ self.W["encoder.linear.weight"].t() + self.W["encoder.linear.bias"]
        mask = (src == 0.0).unsqueeze(1)                          # [B,1,T] (:117-121)
        for i in range(self.cfg.enc_layers):                      # (:123-124) -> :36-54
            p = f"encoder.transformer.{i}"
            h = self.ln(x, p + ".layer_norm")
            a = p + ".self_attn"
            ctx, _ = self.attend(self._heads(self.lin(h, a + ".linear_query")),
                                 self._heads(self.lin(h, a + ".linear_keys")),
                                 self._heads(self.lin(h, a + ".linear_values")), mask)
            y = self.lin(self._unheads(ctx), a + ".final_linear") + x
            x = self.ffn(y, p + ".feed_forward")
        return self.ln(x, "encoder.layer_norm")                  # (:125)

    def _lstm_dir(self, x, lengths, p, sfx, reverse):
        """PyTorch LSTM cell over the VALID steps of each sequence (packing,
        encoder/nano_encoder.py:97-99): gates i,f,g,o."""
        B, T, _ = x.shape
        H = self.cfg.rnn_hidden
        Wih, Whh = self.W[f"{p}.weight_ih_l0{sfx}"], self.W[f"{p}.weight_hh_l0{sfx}"]
        b = self.W[f"{p}.bias_ih_l0{sfx}"] + 0.0
        bh = self.W[f"{p}.bias_hh_l0{sfx}"]
        xp = x @ Wih.t() + b                                       # [B, T, 4H]
        out = torch.zeros(B, T, H)
        h = torch.zeros(B, H)
        c = torch.zeros(B, H)
        lens = torch.as_tensor(lengths)
        for s in range(T):
            # position processed by each sequence at iteration s
            if reverse:
                t = lens - 1 - s
            else:
                t = torch.full((B,), s, dtype=torch.long)
            active = (s < lens)
            if not bool(active.any()):
                break
            tt = t.clamp(min=0)
            g = xp[torch.arange(B), tt] + (h @ Whh.t() + bh)
            i_, f_, g_, o_ = g.chunk(4, dim=1)
            c_new = torch.sigmoid(f_) * c + torch.sigmoid(i_) * torch.tanh(g_)
            h_new = torch.sigmoid(o_) * torch.tanh(c_new)
            am = active.unsqueeze(1)
            c = torch.where(am, c_new, c)
            h = torch.where(am, h_new, h)
            rows = torch.nonzero(active).view(-1)
            out[rows, tt[rows]] = h_new[rows]
        return out

    def encode_nano(self, src, lengths):
        """encoder/nano_encoder.py:79-124.  3x (BiLSTM -> MaxPool1d(1) ->
        BatchNorm1d eval); memory = W . (last layer's pooled output, no BN)."""
        x = src.unsqueeze(-1)
        out = None
        for l in range(self.cfg.enc_layers):
            p = f"encoder.rnn_{l}"
            fwd = self._lstm_dir(x, lengths, p, "", False)
            bwd = self._lstm_dir(x, lengths, p, "_reverse", True)
            out = torch.cat([fwd, bwd], dim=-1)                    # unpacked, zeros at pads
            bn = f"encoder.batchnorm_{l}"
            x = (out - self.W[bn + ".running_mean"]) / torch.sqrt(self.W[bn + ".running_var"] + EPS_BN) \
                * self.W[bn + ".weight"] + self.W[bn + ".bias"]
        return out @ self.W["encoder.W.weight"].t()                 # (:113-115)

    def encode(self, src, lengths):
        if self.cfg.encoder_type == "transformer":
            return self.encode_transformer(src)
        return self.encode_nano(src, lengths)

    # --------------------------------------------------------------- decoder
    def decoder_state(self, memory, src, n_rows_per_chunk=1, max_len=100):
        """decoder/transformer.py:173-176,248-266 + context K/V projected at
        step 0 (multi_headed_attn.py:142-153)."""
        st = {"src": src, "memory": memory, "ctx_k": [], "ctx_v": [], "self_k": [], "self_v": [],
              "prev_g": [], "len": 0}
        for i in range(self.cfg.dec_layers):
            a = f"decoder.transformer_layers.{i}.context_attn"
            st["ctx_k"].append(self._heads(self.lin(memory, a + ".linear_keys")))
            st["ctx_v"].append(self._heads(self.lin(memory, a + ".linear_values")))
            st["self_k"].append(None)
            st["self_v"].append(None)
            # average self-attention cache (decoder/transformer.py:262-263)
            st["prev_g"].append(torch.zeros(memory.shape[0], 1, self.d))
        return st

    def average_attention(self, st, i, h, step):
        """onmt/modules/average_attn.py:55-106 with a layer cache:
        avg = (h + step * prev_g) / (step + 1); a = FFN(avg);
        out = sigmoid(g_in) * h + sigmoid(g_forget) * a, [g_in; g_forget] =
        gating_layer([h; a])."""
        a = f"decoder.transformer_layers.{i}.self_attn"
        avg = (h + step * st["prev_g"][i]) / (step + 1)
        st["prev_g"][i] = avg
        ao = self.ffn(avg, a + ".average_layer")
        g = self.lin(torch.cat((h, ao), -1), a + ".gating_layer")
        gi, gf = torch.chunk(g, 2, dim=2)
        return torch.sigmoid(gi) * h + torch.sigmoid(gf) * ao

    def decode_step(self, st, tok, step):
        """decoder/transformer.py:194-246 for one step + generator
        (models/model_builder.py:331-334).  tok [R] int64 -> logp [R, V]."""
        cfg = self.cfg
        emb = self.W["decoder.embeddings.make_embedding.emb_luts.0.weight"][tok]   # [R, d]
        if cfg.position_encoding:                                   # embeddings.py:36-43
            emb = emb * math.sqrt(self.d) + self.W["decoder.embeddings.make_embedding.pe.pe"][step]
        x = emb.unsqueeze(1)                                        # [R, 1, d]
        src_mask = (st["src"] == float(cfg.pad_idx)).unsqueeze(1)   # [R,1,T] (:220-221)
        for i in range(cfg.dec_layers):                             # :53-95
            p = f"decoder.transformer_layers.{i}"
            h = self.ln(x, p + ".layer_norm_1")
            a = p + ".self_attn"
            if cfg.self_attn_type == "average":                     # (:82-84)
                q1 = self.average_attention(st, i, h, step) + x
            else:
                q = self._heads(self.lin(h, a + ".linear_query"))
                k = self._heads(self.lin(h, a + ".linear_keys"))
                v = self._heads(self.lin(h, a + ".linear_values"))
                if st["self_k"][i] is not None:                     # cache cat (mha.py:132-141)
                    k = torch.cat([st["self_k"][i], k], dim=2)
                    v = torch.cat([st["self_v"][i], v], dim=2)
                st["self_k"][i], st["self_v"][i] = k, v
                c, _ = self.attend(q, k, v, None)
                q1 = self.lin(self._unheads(c), a + ".final_linear") + x
            h2 = self.ln(q1, p + ".layer_norm_2")
            ca = p + ".context_attn"
            qc = self._heads(self.lin(h2, ca + ".linear_query"))
            cc, pc = self.attend(qc, st["ctx_k"][i], st["ctx_v"][i], src_mask)
            st["attn"] = pc[:, 0, 0, :]   # attn["std"]: the last layer's head 0 (mha.py:187-192, :238-246)
            mid = self.lin(self._unheads(cc), ca + ".final_linear")
            x = self.ffn(mid + q1, p + ".feed_forward")
        out = self.ln(x, "decoder.layer_norm").squeeze(1)
        logits = self.lin(out, "generator.0")
        return torch.log_softmax(logits, dim=-1)

    def reorder(self, st, idx):
        """map_state(index_select) (decoder/transformer.py:178-189)."""
        st["src"] = st["src"].index_select(0, idx)
        for key in ("ctx_k", "ctx_v", "self_k", "self_v", "prev_g"):
            st[key] = [t.index_select(0, idx) if t is not None else None for t in st[key]]


# ---------------------------------------------------------------------------
# search
# ---------------------------------------------------------------------------

def greedy(model: RefModel, src, lengths, max_length=100, min_length=0):
    """translate/translator.py:396-503 with keep_topk=1: argmax every step, all
    ``max_length`` steps (no EOS early exit), score = last step's top logp."""
    src = _t(src)
    with torch.no_grad():
        memory = model.encode(src, lengths)
        st = model.decoder_state(memory, src)
        B = src.shape[0]
        tok = torch.full((B,), model.cfg.bos_idx, dtype=torch.long)
        toks, lps, attns = [], [], []
        score = None
        for step in range(max_length):
            lp = model.decode_step(st, tok, step)
            lps.append(lp.clone())                                # model output (parity surface)
            attns.append(st["attn"].clone())                      # return_attention (:491-501)
            if step < min_length:
                lp[:, model.cfg.eos_idx] = -1e20                  # (:469-470)
            score, tok = lp.topk(1, dim=-1)                       # (:375)
            score, tok = score[:, 0], tok[:, 0]
            toks.append(tok)
    return dict(tokens=torch.stack(toks, 1).numpy().astype(np.int32), scores=score.numpy(),
                logp=torch.stack(lps, 1).numpy(), memory=memory.numpy(), attn=torch.stack(attns, 1).numpy())


def sampling_logits(logp, temp, keep_topk):
    """translate/translator.py:376-389 (sample_with_temperature's random
    branch up to the draw): logits / temp, and with keep_topk > 0 every
    logit below the k-th largest replaced by -10000.  The draw is
    Multinomial(logits=...) (:391-393); the score is the returned logit of
    the drawn token."""
    logp = torch.as_tensor(logp, dtype=torch.float32)
    lg = torch.div(logp, temp)
    if keep_topk > 0:
        kth = torch.topk(lg, keep_topk, dim=1)[0][:, -1].view(-1, 1).repeat(1, lg.shape[1])
        keep = torch.ge(lg, kth).float()
        lg = (keep * lg) + ((1 - keep) * -10000)
    return lg


def tile(x, count, dim=0):
    """onmt/utils/misc.py:28-47 (batch-major repeat_interleave)."""
    return x.repeat_interleave(count, dim=dim)


def fast_beam(model: RefModel, src, lengths, beam_size=5, n_best=1, max_length=100, min_length=0,
              alpha=0.0, return_attention=False):
    """translate/translator.py:619-825 (``--fast``).  Returns per chunk a list
    of n_best (score, tokens) best-first; with ``return_attention`` each entry
    also carries the hypothesis' attention rows [steps, cut] (:745-751,
    :780-790), cut = memory_lengths[i] with i the chunk's index among the
    batches still alive (the reference indexes the beam-tiled lengths by it)."""
    src = _t(src)
    cfg = model.cfg
    V = cfg.vocab
    with torch.no_grad():
        memory = model.encode(src, lengths)
        B = src.shape[0]
        st = model.decoder_state(tile(memory, beam_size), tile(src, beam_size))
        memory_lengths = tile(torch.as_tensor(np.asarray(lengths), dtype=torch.long), beam_size)
        top_beam_finished = torch.zeros(B, dtype=torch.bool)
        batch_offset = torch.arange(B)
        beam_offset = torch.arange(0, B * beam_size, beam_size)
        alive_seq = torch.full((B * beam_size, 1), cfg.bos_idx, dtype=torch.long)
        alive_attn = None
        topk_log_probs = torch.tensor([0.0] + [float("-inf")] * (beam_size - 1)).repeat(B)
        hyps = [[] for _ in range(B)]
        results = [[] for _ in range(B)]
        for step in range(max_length):
            lp = model.decode_step(st, alive_seq[:, -1], step)
            attn = st["attn"].unsqueeze(0)                          # [1, R, T]
            if step < min_length:
                lp[:, cfg.eos_idx] = -1e20
            lp = lp + topk_log_probs.view(-1, 1)
            length_penalty = ((5.0 + (step + 1)) / 6.0) ** alpha
            curr = (lp / length_penalty).reshape(-1, beam_size * V)
            topk_scores, topk_ids = curr.topk(beam_size, dim=-1)
            topk_log_probs = topk_scores * length_penalty
            topk_beam_index = torch.div(topk_ids, V, rounding_mode="floor")
            topk_ids = topk_ids.fmod(V)
            batch_index = topk_beam_index + beam_offset[: topk_beam_index.size(0)].unsqueeze(1)
            select = batch_index.view(-1)
            alive_seq = torch.cat([alive_seq.index_select(0, select), topk_ids.view(-1, 1)], -1)
            if return_attention:                                    # (:745-751)
                cur_attn = attn.index_select(1, select)
                alive_attn = cur_attn if alive_attn is None else \
                    torch.cat([alive_attn.index_select(1, select), cur_attn], 0)
            is_finished = topk_ids.eq(cfg.eos_idx)
            if step + 1 == max_length:
                is_finished.fill_(True)
            if bool(is_finished.any()):
                topk_log_probs = topk_log_probs.masked_fill(is_finished, -1e10)
                top_beam_finished |= is_finished[:, 0]
                preds = alive_seq.view(-1, beam_size, alive_seq.size(-1))
                attention = (alive_attn.view(alive_attn.size(0), -1, beam_size, alive_attn.size(-1))
                             if alive_attn is not None else None)
                non_finished = []
                for i in range(is_finished.size(0)):
                    b = int(batch_offset[i])
                    for j in torch.nonzero(is_finished[i]).view(-1).tolist():
                        a = attention[:, i, j, : int(memory_lengths[i])].clone() if attention is not None else None
                        hyps[b].append((float(topk_scores[i, j]), preds[i, j, 1:].clone(), a))
                    if bool(top_beam_finished[i]) and len(hyps[b]) >= n_best:
                        best = sorted(hyps[b], key=lambda x: x[0], reverse=True)
                        results[b] = [(sc, p.numpy().astype(np.int32)) + ((a.numpy(),) if return_attention else ())
                                      for sc, p, a in best[:n_best]]
                    else:
                        non_finished.append(i)
                if not non_finished:
                    break
                nf = torch.tensor(non_finished, dtype=torch.long)
                top_beam_finished = top_beam_finished.index_select(0, nf)
                batch_offset = batch_offset.index_select(0, nf)
                topk_log_probs = topk_log_probs.index_select(0, nf)
                batch_index = batch_index.index_select(0, nf)
                select = batch_index.view(-1)
                alive_seq = preds.index_select(0, nf).view(-1, alive_seq.size(-1))
                if alive_attn is not None:
                    alive_attn = attention.index_select(1, nf).view(alive_attn.size(0), -1, alive_attn.size(-1))
            model.reorder(st, select)
            memory_lengths = memory_lengths.index_select(0, select)
    return results


def _length_penalty(kind, n_ys, alpha):
    """onmt/translate/penalties.py:57-78 (the divisor applied to log-probs;
    n_ys = len(beam.next_ys))."""
    if kind == "wu":
        return ((5 + n_ys) ** alpha) / ((5 + 1) ** alpha)
    if kind == "avg":
        return float(n_ys)
    return 1.0


def _coverage_penalty(kind, cov, beta):
    """onmt/translate/penalties.py:34-53: beta * penalty per beam, cov [beam, cut]."""
    if kind == "wu":
        return beta * (-torch.min(cov, cov.clone().fill_(1.0)).log().sum(1))
    if kind == "summary":
        return beta * (torch.max(cov, cov.clone().fill_(1.0)).sum(1) - cov.size(1))
    return torch.zeros(cov.size(0))


class ClassicBeam:
    """onmt/translate/beam.py:6-178 (``Beam``) with GNMTGlobalScorer
    (:181-243): length penalty none / wu / avg, coverage penalty none / wu /
    summary (at scoring time, or stepwise), n-gram blocking with exclusion
    tokens, per-step attention kept for get_hyp."""

    def __init__(self, size, pad, bos, eos, n_best, min_length, length_penalty, alpha, beta=0.0,
                 coverage_penalty="none", stepwise_penalty=False, block_ngram_repeat=0, exclusion_tokens=()):
        self.size, self._eos, self.n_best, self.min_length = size, eos, n_best, min_length
        self.lp, self.alpha = length_penalty, alpha
        self.beta, self.cov = beta, coverage_penalty
        self.stepwise_penalty = stepwise_penalty
        self.block_ngram_repeat = block_ngram_repeat
        self.exclusion_tokens = set(exclusion_tokens)
        self.scores = torch.zeros(size)                       # (:34)
        self.prev_ks = []
        self.next_ys = [torch.full((size,), pad, dtype=torch.long)]
        self.next_ys[0][0] = bos                              # (:41-43)
        self.attn = []
        self.eos_top = False
        self.finished = []
        self.global_state = {}

    def _cov_pen(self, cov):
        if self.cov == "none":                                # coverage_none: beam.scores zeros
            return torch.zeros(self.size)
        return _coverage_penalty(self.cov, cov, self.beta)

    def global_score(self, scores):                           # GNMTGlobalScorer.score (:200-212)
        """length_none returns ``scores`` itself (penalties.py:74-78), so the
        in-place ``normalized_probs -= penalty`` then also lowers beam.scores:
        with length penalty none and a coverage penalty at scoring time, every
        call (one per finished beam, and per top-up in sort_finished) moves
        the live scores."""
        if self.lp == "none":
            normalized = scores
        else:
            normalized = scores / _length_penalty(self.lp, len(self.next_ys), self.alpha)
        if not self.stepwise_penalty:
            normalized -= self._cov_pen(self.global_state["coverage"])
        return normalized

    def _update_score(self, attn):                            # (:214-223)
        if "prev_penalty" in self.global_state:
            self.scores.add_(self.global_state["prev_penalty"])
            self.scores.sub_(self._cov_pen(self.global_state["coverage"] + attn))

    def _update_global_state(self):                           # (:225-243)
        if len(self.prev_ks) == 1:
            self.global_state["prev_penalty"] = self.scores.clone().fill_(0.0)
            self.global_state["coverage"] = self.attn[-1]
        else:
            self.global_state["coverage"] = self.global_state["coverage"].index_select(
                0, self.prev_ks[-1]).add(self.attn[-1])
            self.global_state["prev_penalty"] = self._cov_pen(self.global_state["coverage"])

    def _blocked(self, j):                                    # (:100-119)
        le = len(self.next_ys)
        hyp = self.get_hyp(le - 1, j)
        ngrams, gram = set(), []
        for i in range(le - 1):
            gram = (gram + [hyp[i]])[-self.block_ngram_repeat:]
            if set(gram) & self.exclusion_tokens:
                continue
            if tuple(gram) in ngrams:
                return True
            ngrams.add(tuple(gram))
        return False

    def advance(self, word_probs, attn_out):                  # (:73-150)
        V = word_probs.size(1)
        word_probs = word_probs.clone()
        if self.stepwise_penalty:
            self._update_score(attn_out)
        if len(self.next_ys) < self.min_length:               # (:88-91)
            word_probs[:, self._eos] = -1e20
        if len(self.prev_ks) > 0:                             # (:93-99)
            beam_scores = word_probs + self.scores.unsqueeze(1)
            for i in range(self.next_ys[-1].size(0)):
                if int(self.next_ys[-1][i]) == self._eos:
                    beam_scores[i] = -1e20
            if self.block_ngram_repeat > 0:
                for j in range(self.next_ys[-1].size(0)):
                    if self._blocked(j):
                        beam_scores[j] = -10e20
        else:
            beam_scores = word_probs[0]
        best_scores, best_ids = beam_scores.reshape(-1).topk(self.size, 0, True, True)   # (:122-123)
        self.scores = best_scores
        prev_k = torch.div(best_ids, V, rounding_mode="floor")   # (:129, integer division in torch 1.0)
        self.prev_ks.append(prev_k)
        self.next_ys.append(best_ids - prev_k * V)
        self.attn.append(attn_out.index_select(0, prev_k))
        self._update_global_state()
        for i in range(self.next_ys[-1].size(0)):             # (:135-139)
            if int(self.next_ys[-1][i]) == self._eos:
                s = self.global_score(self.scores)[i]
                self.finished.append((float(s), len(self.next_ys) - 1, i))
        if int(self.next_ys[-1][0]) == self._eos:             # (:142-144)
            self.eos_top = True

    def done(self):                                           # (:146-147)
        return self.eos_top and len(self.finished) >= self.n_best

    def sort_finished(self, minimum=None):                    # (:149-161)
        if minimum is not None:
            i = 0
            while len(self.finished) < minimum:
                s = self.global_score(self.scores)[i]
                self.finished.append((float(s), len(self.next_ys) - 1, i))
                i += 1
        self.finished.sort(key=lambda a: -a[0])
        return [sc for sc, _, _ in self.finished], [(t, k) for _, t, k in self.finished]

    def get_hyp(self, timestep, k):                           # (:163-173)
        hyp = []
        for j in range(len(self.prev_ks[:timestep]) - 1, -1, -1):
            hyp.append(int(self.next_ys[j + 1][k]))
            k = int(self.prev_ks[j][k])
        return hyp[::-1]

    def get_hyp_attn(self, timestep, k):
        att = []
        for j in range(len(self.prev_ks[:timestep]) - 1, -1, -1):
            att.append(self.attn[j][k])
            k = int(self.prev_ks[j][k])
        return torch.stack(att[::-1])


def classic_beam(model: RefModel, src, lengths, beam_size=5, n_best=1, max_length=100, min_length=0,
                 alpha=0.0, length_penalty="none", beta=0.0, coverage_penalty="none", stepwise_penalty=False,
                 block_ngram_repeat=0, exclusion_tokens=(), return_attention=False):
    """translate/translator.py:827-926 (``_translate_batch``, beam_size > 1
    without --fast): one Beam per chunk, the whole batch advances until every
    beam is done.  Beam j's attention rows are cut at memory_lengths[j] of the
    beam-tiled lengths (:902-907), i.e. at lengths[j // beam_size].  Returns
    per chunk n_best (score, tokens[, attention [steps, cut]]) best-first."""
    src = _t(src)
    cfg = model.cfg
    with torch.no_grad():
        memory = model.encode(src, lengths)
        B = src.shape[0]
        beams = [ClassicBeam(beam_size, cfg.pad_idx, cfg.bos_idx, cfg.eos_idx, n_best, min_length,
                             length_penalty, alpha, beta, coverage_penalty, stepwise_penalty, block_ngram_repeat,
                             exclusion_tokens) for _ in range(B)]
        st = model.decoder_state(tile(memory, beam_size), tile(src, beam_size))
        memory_lengths = tile(torch.as_tensor(np.asarray(lengths), dtype=torch.long), beam_size)
        for i in range(max_length):
            if all(b.done() for b in beams):                   # (:884-885)
                break
            inp = torch.stack([b.next_ys[-1] for b in beams]).view(-1)
            lp = model.decode_step(st, inp, i).view(B, beam_size, -1)
            attn = st["attn"].view(B, beam_size, -1)
            sel = []
            for j, b in enumerate(beams):
                b.advance(lp[j], attn[j, :, : int(memory_lengths[j])])
                sel.append(b.prev_ks[-1] + j * beam_size)
            model.reorder(st, torch.cat(sel))
        out = []
        for b in beams:                                        # (:914-924)
            scores, ks = b.sort_finished(minimum=n_best)
            out.append([(scores[n], np.array(b.get_hyp(t, k), np.int32))
                        + ((b.get_hyp_attn(t, k).numpy(),) if return_attention else ())
                        for n, (t, k) in enumerate(ks[:n_best])])
    return out


# ---------------------------------------------------------------------------
# Translator.translate semantics (batching, ordering, EOS truncation)
# ---------------------------------------------------------------------------

def make_batch(chunks: Sequence[np.ndarray]):
    """inputters/inputter.py:86-95 (zero pad to the longest chunk in the batch)
    + OrderedIterator sort_within_batch (descending length, stable)."""
    order = sorted(range(len(chunks)), key=lambda i: len(chunks[i]), reverse=True)
    T = max(len(c) for c in chunks)
    src = np.zeros((len(chunks), T), np.float32)
    for j, i in enumerate(order):
        src[j, : len(chunks[i])] = chunks[i]
    lengths = np.array([len(chunks[i]) for i in order], np.int64)
    return src, lengths, order


def tokens_to_string(tokens, itos, eos_idx):
    """translate/translation.py:31-47: ids -> itos, cut at the first EOS;
    joined with spaces as translate/translator.py:271-273."""
    out = []
    for t in tokens:
        t = int(t)
        if t == eos_idx:
            break
        out.append(itos[t])
    return " ".join(out)


def translate(model: RefModel, chunks: Sequence[np.ndarray], batch_size: int, beam_size=1, n_best=1,
              max_length=100, min_length=0, alpha=0.0, fast=True, length_penalty="none"):
    """translate/translator.py:181-369: consecutive batches of ``batch_size``
    chunks (never across reads), results in input order.  Returns
    (all_scores, all_predictions) like the reference."""
    all_scores, all_preds = [], []
    itos, eos = model.cfg.itos, model.cfg.eos_idx
    for b0 in range(0, len(chunks), batch_size):
        part = list(chunks[b0: b0 + batch_size])
        src, lengths, order = make_batch(part)
        per = [None] * len(part)
        if beam_size == 1:
            r = greedy(model, src, lengths, max_length, min_length)
            for j, i in enumerate(order):
                per[i] = ([float(r["scores"][j])], [tokens_to_string(r["tokens"][j], itos, eos)])
        else:
            if fast:
                r = fast_beam(model, src, lengths, beam_size, n_best, max_length, min_length, alpha)
            else:
                r = classic_beam(model, src, lengths, beam_size, n_best, max_length, min_length, alpha,
                                 length_penalty)
            for j, i in enumerate(order):
                per[i] = ([s for s, _ in r[j]], [tokens_to_string(p, itos, eos) for _, p in r[j]])
        for s, p in per:
            all_scores.append(s[:n_best])
            all_preds.append(p[:n_best])
    return all_scores, all_preds
