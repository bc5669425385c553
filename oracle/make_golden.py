"""Generate golden vectors from the REFERENCE's own modules (this container only).

Test infrastructure.  Runs the reference's PyTorch translate path —
``encoder/transformer.py``, ``encoder/nano_encoder.py``, ``decoder/
transformer.py``, ``onmt/modules/*`` and ``translate/translator.py``'s own
``_translate_random_sampling`` (greedy, :396-503) and ``_fast_translate_batch``
(--fast beam, :619-825) — on seeded synthetic weights and synthetic signal
chunks, and writes small ``.npz`` fixtures to ``tests/golden/``.

The reference never travels to the GPU box; only these fixtures (data) do.
Regenerate with:  ``python oracle/make_golden.py``  (needs /root/reference).

Compat shims: integer ``Tensor.div`` is floor division while
the --fast beam runs (``translate/translator.py:732`` was written for torch 1.0).
"""
from __future__ import annotations

import argparse
import contextlib
import hashlib
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from nanodecoder_amd import synth  # noqa: E402
from oracle._refimport import load_reference  # noqa: E402

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")
MEM_STRIDE = 16  # memory-bank rows kept in the fixture: t = 0, 16, 32, ...


def weights_digest(W):
    h = hashlib.sha256()
    for k in sorted(W):
        h.update(k.encode())
        h.update(np.ascontiguousarray(W[k]).tobytes())
    return h.hexdigest()


def build_reference_model(ns, cfg: synth.ModelConfig, W):
    """Instantiate the reference modules (models/model_builder.py:65-214,
    :326-334) and load W into them."""
    d = cfg.d_model
    if cfg.encoder_type == "transformer":
        enc = ns.TransformerEncoder(cfg.enc_layers, d, cfg.heads, cfg.d_ff, 0.0, 1, None)
    else:
        enc = ns.NanoEncoder("LSTM", cfg.enc_layers, cfg.dec_layers, 2 * cfg.rnn_hidden, d, "1",
                             0.0, 4000, 0.075, 1)
    emb = ns.Embeddings(d, cfg.vocab, cfg.pad_idx, position_encoding=cfg.position_encoding)
    dec = ns.TransformerDecoder(cfg.dec_layers, d, cfg.heads, cfg.d_ff, "general", False,
                                cfg.self_attn_type, 0.0, emb)
    gen = nn.Sequential(nn.Linear(d, cfg.vocab), nn.LogSoftmax(dim=-1))
    model = nn.Module()
    model.encoder, model.decoder = enc, dec
    sd = {}
    for k, v in W.items():
        if k.startswith("generator."):
            continue
        sd[k] = torch.from_numpy(np.array(v))
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [m for m in missing if not m.endswith(".mask") and not m.endswith("num_batches_tracked")]
    assert not missing and not unexpected, (missing, unexpected)
    gen.load_state_dict({"0.weight": torch.from_numpy(W["generator.0.weight"]),
                         "0.bias": torch.from_numpy(W["generator.0.bias"])})
    model.generator = gen
    model.eval()
    return model


class _Field:
    def __init__(self, itos):
        self.vocab = types.SimpleNamespace(itos=list(itos), stoi={s: i for i, s in enumerate(itos)})
        self.init_token, self.eos_token = "<s>", "</s>"
        self.pad_token, self.unk_token = "<blank>", "<unk>"


def make_translator(ns, model, cfg, beam_size, n_best=1, max_length=100, min_length=0, alpha=0.0, fast=True,
                    length_penalty="none", beta=0.0, coverage_penalty="none", stepwise_penalty=False,
                    block_ngram_repeat=0, ignore_when_blocking=()):
    opt = types.SimpleNamespace(
        gpu=-1, n_best=n_best, max_length=max_length, beam_size=beam_size,
        random_sampling_temp=1.0, random_sampling_topk=1, min_length=min_length,
        stepwise_penalty=stepwise_penalty, dump_beam="", block_ngram_repeat=block_ngram_repeat,
        ignore_when_blocking=list(ignore_when_blocking),
        fft=False, sample_rate=4000, window_size=0.075, window_stride=0.015, window="hamming",
        replace_unk=False, data_type="nano", verbose=False, fast=fast)
    model_opt = types.SimpleNamespace(copy_attn=False)
    if fast:
        scorer = types.SimpleNamespace(alpha=alpha, beta=0.0)
    else:  # onmt/translate/beam.py:181-199 (the real scorer drives the classic Beam)
        scorer = ns.GNMTGlobalScorer(types.SimpleNamespace(alpha=alpha, beta=beta, coverage_penalty=coverage_penalty,
                                                           length_penalty=length_penalty))
    return ns.Translator(model, {"tgt": _Field(cfg.itos)}, opt, model_opt, global_scorer=scorer,
                         report_score=False, logger=None)


def make_batch(chunks):
    """inputters/inputter.py:86-95 (make_nano) + OrderedIterator sort_within_batch:
    zero-pad to the longest chunk, batch sorted by length descending (stable)."""
    order = sorted(range(len(chunks)), key=lambda i: len(chunks[i]), reverse=True)
    T = max(len(c) for c in chunks)
    src = torch.zeros(T, len(chunks), 1)
    for j, i in enumerate(order):
        src[: len(chunks[i]), j, 0] = torch.from_numpy(chunks[i])
    lengths = torch.tensor([len(chunks[i]) for i in order], dtype=torch.long)
    batch = types.SimpleNamespace(src=src, src_lengths=lengths, batch_size=len(chunks),
                                  indices=torch.tensor(order, dtype=torch.long))
    return batch, order


@contextlib.contextmanager
def floor_int_div():
    orig = torch.Tensor.div

    def div(self, other, *a, **k):
        if not self.is_floating_point() and isinstance(other, int) and not a and not k:
            return orig(self, other, rounding_mode="floor")
        return orig(self, other, *a, **k)

    torch.Tensor.div = div
    try:
        yield
    finally:
        torch.Tensor.div = orig


def run_greedy(ns, model, cfg, chunks, max_length=100, min_length=0, attention=False):
    tr = make_translator(ns, model, cfg, beam_size=1, max_length=max_length, min_length=min_length)
    batch, order = make_batch(chunks)
    rec = []
    orig = tr._decode_and_generate

    def wrapped(*a, **k):
        lp, attn = orig(*a, **k)
        rec.append(lp.detach().clone())
        return lp, attn

    tr._decode_and_generate = wrapped
    mem_box = {}
    enc_fwd = model.encoder.forward

    def enc_wrap(src, lengths=None):
        out = enc_fwd(src, lengths)
        mem_box["memory"] = out[1].detach().clone()
        return out

    model.encoder.forward = enc_wrap
    with torch.no_grad():
        res = tr._translate_random_sampling(batch, types.SimpleNamespace(data_type="nano"), max_length,
                                            min_length=min_length, sampling_temp=1.0, keep_topk=1,
                                            return_attention=attention)
    model.encoder.forward = enc_fwd
    B = len(chunks)
    inv = np.argsort(order)  # batch row j holds chunk order[j]
    logp = torch.stack(rec, 1).numpy()[inv]                     # [B, S, V]
    tokens = np.stack([res["predictions"][j][0].numpy() for j in range(B)])[inv].astype(np.int32)
    scores = np.array([float(res["scores"][j][0]) for j in range(B)], np.float32)[inv]
    memory = mem_box["memory"].numpy()[:, inv, :]              # [T, B, d]
    out = dict(logp=logp.astype(np.float32), tokens=tokens, scores=scores,
               memory_sub=np.ascontiguousarray(memory[::MEM_STRIDE]).astype(np.float32),
               T=np.int32(memory.shape[0]))
    if attention:
        # -attn_debug: results["attention"][b][0] = [steps, src_length of chunk b]
        T = memory.shape[0]
        att = np.zeros((B, max_length, T), np.float32)
        for j in range(B):
            a = res["attention"][j][0].numpy()
            att[j, :, : a.shape[1]] = a
        out["attn"] = att[inv]
    return out


def _hyp_attention(res, B, n_best, max_length, T):
    """results["attention"][b][n]: [steps, cut] rows along the hypothesis,
    cut = memory_lengths[i] as the reference indexes it -> zero-padded
    [B, n_best, max_length, T] plus the cut per hypothesis."""
    att = np.zeros((B, n_best, max_length, T), np.float32)
    cut = np.zeros((B, n_best), np.int32)
    for j in range(B):
        for n in range(n_best):
            a = res["attention"][j][n]
            a = a.numpy() if hasattr(a, "numpy") else np.asarray(a)
            att[j, n, : a.shape[0], : a.shape[1]] = a
            cut[j, n] = a.shape[1]
    return att, cut


def run_beam(ns, model, cfg, chunks, beam_size=5, n_best=1, max_length=100, min_length=0, alpha=0.0,
             attention=False):
    tr = make_translator(ns, model, cfg, beam_size=beam_size, n_best=n_best, max_length=max_length,
                         min_length=min_length, alpha=alpha)
    batch, order = make_batch(chunks)
    with torch.no_grad(), floor_int_div():
        res = tr._fast_translate_batch(batch, types.SimpleNamespace(data_type="nano"), max_length,
                                       min_length=min_length, n_best=n_best, return_attention=attention)
    B = len(chunks)
    inv = np.argsort(order)
    tokens = np.full((B, n_best, max_length), -1, np.int32)
    lens = np.zeros((B, n_best), np.int32)
    scores = np.zeros((B, n_best), np.float32)
    for j in range(B):
        for n in range(n_best):
            p = res["predictions"][j][n].numpy()
            tokens[j, n, : len(p)] = p
            lens[j, n] = len(p)
            scores[j, n] = float(res["scores"][j][n])
    out = dict(beam_tokens=tokens[inv], beam_lens=lens[inv], beam_scores=scores[inv])
    if attention:
        att, cut = _hyp_attention(res, B, n_best, max_length, batch.src.shape[0])
        out.update(beam_attn=att[inv], beam_attn_cut=cut[inv])
    return out


@contextlib.contextmanager
def floor_int_truediv():
    """onmt/translate/beam.py:129 divides LongTensors with '/', integer
    division in torch 1.0 (true division since torch 1.5)."""
    orig = torch.Tensor.__truediv__

    def truediv(self, other):
        if not self.is_floating_point() and isinstance(other, int):
            return torch.div(self, other, rounding_mode="floor")
        return orig(self, other)

    torch.Tensor.__truediv__ = truediv
    try:
        yield
    finally:
        torch.Tensor.__truediv__ = orig


def run_classic_beam(ns, model, cfg, chunks, beam_size=5, n_best=1, max_length=100, min_length=0, alpha=0.0,
                     length_penalty="none", attention=False, **extra):
    """translate/translator.py:827-926 (_translate_batch, the onmt Beam);
    ``extra``: beta, coverage_penalty, stepwise_penalty, block_ngram_repeat,
    ignore_when_blocking (token strings)."""
    tr = make_translator(ns, model, cfg, beam_size=beam_size, n_best=n_best, max_length=max_length,
                         min_length=min_length, alpha=alpha, fast=False, length_penalty=length_penalty, **extra)
    batch, order = make_batch(chunks)
    with torch.no_grad(), floor_int_div(), floor_int_truediv():
        res = tr._translate_batch(batch, types.SimpleNamespace(data_type="nano"))
    B = len(chunks)
    inv = np.argsort(order)
    tokens = np.full((B, n_best, max_length), -1, np.int32)
    lens = np.zeros((B, n_best), np.int32)
    scores = np.zeros((B, n_best), np.float32)
    for j in range(B):
        for n in range(n_best):
            p = np.array([int(t) for t in res["predictions"][j][n]], np.int32)
            tokens[j, n, : len(p)] = p
            lens[j, n] = len(p)
            scores[j, n] = float(res["scores"][j][n])
    out = dict(beam_tokens=tokens[inv], beam_lens=lens[inv], beam_scores=scores[inv])
    if attention:
        att, cut = _hyp_attention(res, B, n_best, max_length, batch.src.shape[0])
        out.update(beam_attn=att[inv], beam_attn_cut=cut[inv])
    return out


SCENARIOS = [
    # name, model config kwargs, weight seed, eos_bias, chunk spec, runs
    dict(name="transformer_greedy", cfg=dict(encoder_type="transformer"), seed=11, eos_bias=-3.0,
         chunks=dict(kind="mixed"), greedy=dict(max_length=100)),
    dict(name="transformer_pe_short", cfg=dict(encoder_type="transformer", position_encoding=True),
         seed=12, eos_bias=0.0, chunks=dict(kind="short"), greedy=dict(max_length=40, min_length=5, attention=True)),
    dict(name="transformer_beam", cfg=dict(encoder_type="transformer"), seed=13, eos_bias=2.5,
         chunks=dict(kind="mixed"), beam=dict(beam_size=5, n_best=1, max_length=100),
         beam2=dict(beam_size=5, n_best=3, max_length=60, min_length=10)),
    dict(name="nano_greedy", cfg=dict(encoder_type="nano"), seed=14, eos_bias=-2.0,
         chunks=dict(kind="mixed"), greedy=dict(max_length=60)),
    # -cpg models (models/opts.py:254): the methylated-C label 'M' is a fifth base, V = 9
    dict(name="transformer_cpg", cfg=dict(encoder_type="transformer",
                                          itos=["<unk>", "<blank>", "<s>", "</s>", "A", "C", "G", "T", "M"]),
         seed=19, eos_bias=-1.0, chunks=dict(kind="ragged"), greedy=dict(max_length=60, min_length=5),
         beam=dict(beam_size=5, n_best=2, max_length=50, min_length=5)),
    # decoder with average self-attention (onmt/modules/average_attn.py), greedy and --fast beam
    # the classic onmt Beam (no --fast): length penalties none / wu, n_best 1 and 3
    dict(name="transformer_classic_beam", cfg=dict(encoder_type="transformer"), seed=16, eos_bias=2.5,
         chunks=dict(kind="mixed"), classic=dict(beam_size=5, n_best=1, max_length=100),
         classic2=dict(beam_size=4, n_best=3, max_length=60, min_length=10, alpha=0.6, length_penalty="wu")),
    dict(name="transformer_classic_beam_mid", cfg=dict(encoder_type="transformer"), seed=17, eos_bias=1.0,
         chunks=dict(kind="mixed"), classic=dict(beam_size=5, n_best=2, max_length=60, min_length=8,
                                                 length_penalty="avg")),
    dict(name="transformer_aan", cfg=dict(encoder_type="transformer", self_attn_type="average"), seed=15,
         eos_bias=1.5, chunks=dict(kind="mixed"), greedy=dict(max_length=60),
         beam=dict(beam_size=4, n_best=2, max_length=50, min_length=5)),
    # -attn_debug with beam search (attention along each hypothesis, cut at
    # memory_lengths[i] as the reference indexes it) on a batch of six chunks
    # of distinct lengths, for --fast and for the classic Beam
    dict(name="transformer_beam_attn", cfg=dict(encoder_type="transformer"), seed=18, eos_bias=1.0,
         chunks=dict(kind="ragged"), beam=dict(beam_size=4, n_best=2, max_length=40, min_length=3, attention=True),
         classic=dict(beam_size=4, n_best=2, max_length=40, min_length=3, attention=True)),
    # the classic Beam's n-gram blocking (with an exclusion token, and without)
    dict(name="transformer_classic_ext", cfg=dict(encoder_type="transformer"), seed=18, eos_bias=1.0,
         chunks=dict(kind="mixed"),
         classic=dict(beam_size=4, n_best=2, max_length=40, min_length=3, attention=True,
                      block_ngram_repeat=4, ignore_when_blocking=["A"]),
         classic2=dict(beam_size=4, n_best=2, max_length=30, min_length=3, block_ngram_repeat=7)),
    # coverage penalties: wu at scoring time with length penalty none (the
    # scorer then subtracts in place from beam.scores, penalties.py:74-78 +
    # beam.py:200-212), summary stepwise, summary at scoring time with avg
    dict(name="transformer_classic_cov", cfg=dict(encoder_type="transformer"), seed=18, eos_bias=1.0,
         chunks=dict(kind="ragged"),
         classic=dict(beam_size=4, n_best=2, max_length=40, min_length=3, coverage_penalty="wu", beta=0.2),
         classic2=dict(beam_size=4, n_best=2, max_length=40, min_length=3, coverage_penalty="summary", beta=0.3,
                       stepwise_penalty=True, attention=True),
         classic3=dict(beam_size=4, n_best=3, max_length=40, min_length=3, coverage_penalty="summary", beta=0.1,
                       length_penalty="avg")),
]


def scenario_chunks(kind, seed):
    if kind == "mixed":
        # two full chunks, one short tail chunk (zero padded in the batch), one
        # all-zero chunk (every encoder key masked -> uniform attention rows).
        full = synth.synth_chunk_batch(2, 512, seed=seed, inject_masks=True)
        tail = synth.synth_read_chunks(seed + 500, 812)[-1]
        assert len(tail) == 300
        zero = np.zeros(512, np.float32)
        return [full[0], tail, full[1], zero]
    if kind == "ragged":
        # six chunks of distinct lengths in unsorted order (T_max = 512)
        full = synth.synth_chunk_batch(1, 512, seed=seed, inject_masks=False)[0]
        tails = {n: synth.synth_read_chunks(seed + 700 + n, 512 + n)[-1] for n in (300, 200, 150, 100, 77)}
        return [tails[150], full, tails[77], tails[300], tails[100], tails[200]]
    if kind == "short":
        # a batch made only of short chunks: T_max < 512 (reference batching quirk)
        return [synth.synth_read_chunks(seed + 600 + i, 512 + n)[-1] for i, n in enumerate((200, 150, 77))]
    raise ValueError(kind)


def make_sampling_fixture(ns, out_dir):
    """translate/translator.py:371-394, the random branch with keep_topk = -1
    (the top-k branch casts to torch.cuda.FloatTensor and cannot run on a
    CPU): the reference's own draws from seeded torch generators on the
    reference's step-0 log-probs of transformer_greedy (64 copies of each
    chunk's row)."""
    z = np.load(os.path.join(out_dir, "transformer_greedy.npz"))
    logits = torch.from_numpy(np.repeat(z["logp"][:, 0, :], 64, axis=0)).float()
    temps = np.array([1.0, 0.7, 1.6], np.float32)
    seeds = np.array([11, 12, 13], np.int64)
    ids, scores = [], []
    for t, sd in zip(temps, seeds):
        torch.manual_seed(int(sd))
        i, sc = ns.Translator.sample_with_temperature(None, logits.clone(), float(t), -1)
        ids.append(i[:, 0].numpy().astype(np.int32))
        scores.append(sc[:, 0].numpy().astype(np.float32))
    path = os.path.join(out_dir, "sampling.npz")
    np.savez_compressed(path, logits=logits.numpy(), temps=temps, seeds=seeds, ids=np.stack(ids),
                        scores=np.stack(scores), torch=np.frombuffer(torch.__version__.encode(), np.uint8))
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=GOLDEN_DIR)
    ap.add_argument("--only", nargs="*", help="regenerate only these scenarios (index.json is merged)")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    torch.manual_seed(0)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ns = load_reference()
    index = {}
    ipath = os.path.join(args.out, "index.json")
    if args.only and os.path.exists(ipath):
        with open(ipath) as f:
            index = json.load(f)
    for sc in SCENARIOS:
        if args.only and sc["name"] not in args.only:
            continue
        cfg = synth.ModelConfig(**sc["cfg"])
        W = synth.make_weights(cfg, seed=sc["seed"], eos_bias=sc["eos_bias"])
        model = build_reference_model(ns, cfg, W)
        chunks = scenario_chunks(sc["chunks"]["kind"], sc["seed"])
        out = {}
        lens = np.array([len(c) for c in chunks], np.int32)
        T = int(lens.max())
        src = np.zeros((len(chunks), T), np.float32)
        for i, c in enumerate(chunks):
            src[i, : len(c)] = c
        out["src"], out["lengths"] = src, lens
        if "greedy" in sc:
            g = run_greedy(ns, model, cfg, chunks, **sc["greedy"])
            out.update(g)
        if "beam" in sc:
            b = run_beam(ns, model, cfg, chunks, **sc["beam"])
            out.update(b)
        if "beam2" in sc:
            b = run_beam(ns, model, cfg, chunks, **sc["beam2"])
            out.update({k + "2": v for k, v in b.items()})
        for key in ("classic", "classic2", "classic3"):
            if key in sc:
                b = run_classic_beam(ns, model, cfg, chunks, **sc[key])
                out.update({k.replace("beam", key): v for k, v in b.items()})
        meta = dict(name=sc["name"], cfg=sc["cfg"], seed=sc["seed"], eos_bias=sc["eos_bias"],
                    greedy=sc.get("greedy"), beam=sc.get("beam"), beam2=sc.get("beam2"),
                    classic=sc.get("classic"), classic2=sc.get("classic2"), classic3=sc.get("classic3"),
                    mem_stride=MEM_STRIDE, weights_sha256=weights_digest(W),
                    torch=torch.__version__, numpy=np.__version__)
        out["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        path = os.path.join(args.out, sc["name"] + ".npz")
        np.savez_compressed(path, **out)
        index[sc["name"]] = meta
        print(f"wrote {path} ({os.path.getsize(path)} B)")
    with open(ipath, "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)
    if not args.only or "sampling" in args.only:
        make_sampling_fixture(ns, args.out)


if __name__ == "__main__":
    main()
