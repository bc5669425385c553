"""Host logic of the Translator drop-in (batching, spans, ordering, EOS cut,
errors) with a recording stand-in for the HIP engine.  CPU only."""
import types

import numpy as np
import pytest
import torch

from nanodecoder_amd import synth
from nanodecoder_amd.translator import Translator, parse_chunk


class FakeEngine:
    """Encodes each chunk's (len, span) into its tokens so tests can check
    what the Translator passed to the engine."""

    def __init__(self, max_batch=8, max_src_len=512):
        self.max_batch, self.max_src_len = max_batch, max_src_len
        self.calls = []

    def _tok(self, L, S, n):
        row = [4 + (L % 4), 4 + (S % 4), 5, 3] + [6] * (n - 4)
        return row[:n]

    def translate_greedy(self, sig, L, S, max_len, min_len=0, return_attn=False):
        self.calls.append(("greedy", sig.shape, L.copy(), S.copy()))
        tok = torch.tensor([self._tok(int(a), int(b), max_len) for a, b in zip(L, S)], dtype=torch.int32)
        out = {"tokens": tok, "scores": torch.tensor(L, dtype=torch.float32) * -0.01, "logp": None, "attn": None}
        if return_attn:  # row t: uniform over the first t + 1 positions
            a = torch.zeros(len(L), max_len, sig.shape[1])
            for t in range(max_len):
                a[:, t, : t + 1] = 1.0 / (t + 1)
            out["attn"] = a
        return out

    def translate_sample(self, sig, L, S, temp, keep_topk, seed, max_len, min_len=0, return_attn=False):
        out = self.translate_greedy(sig, L, S, max_len, min_len, return_attn)
        self.calls[-1] = ("sample", sig.shape, L.copy(), S.copy(), temp, keep_topk, seed)
        return out

    def translate_beam(self, sig, L, S, beam, n_best, alpha, max_len, min_len=0, return_attn=False,
                       done_step=None, hyp_len=4):
        self.calls.append(("beam", sig.shape, L.copy(), S.copy()))
        B = len(L)
        tok = torch.full((B, n_best, max_len), -1, dtype=torch.int32)
        lens = torch.zeros(B, n_best, dtype=torch.int32)
        sc = torch.zeros(B, n_best)
        for i in range(B):
            for k in range(n_best):
                t = self._tok(int(L[i]), int(S[i]) + k, hyp_len)
                n = hyp_len if done_step is None or done_step[i] == 0 else int(done_step[i])
                tok[i, k, :n] = torch.tensor(t[:n])
                lens[i, k] = n
                sc[i, k] = -float(k)
        out = {"tokens": tok, "scores": sc, "lens": lens, "steps": torch.tensor([4])}
        if return_attn:  # entry (t, x) = 1000 * t + x, so cuts are visible
            T = sig.shape[1]
            a = torch.arange(max_len).view(-1, 1) * 1000.0 + torch.arange(T).view(1, -1)
            out["attn"] = a.expand(B, n_best, max_len, T).clone()
            out["done_step"] = torch.as_tensor(np.zeros(B, np.int32) if done_step is None else done_step)
        return out

    def translate_beam_classic(self, sig, L, S, groups, beam, n_best, length_penalty, alpha, max_len, min_len=0,
                               return_attn=False, **opts):
        out = self.translate_beam(sig, L, S, beam, n_best, alpha, max_len, min_len, return_attn=return_attn)
        self.calls[-1] = ("classic", sig.shape, L.copy(), S.copy(), np.asarray(groups).copy(), length_penalty)
        self.classic_opts = opts
        return out


def make_tr(**over):
    opt = dict(gpu=0, n_best=1, max_length=10, min_length=0, beam_size=1, random_sampling_temp=1.0,
               random_sampling_topk=1, block_ngram_repeat=0, dump_beam="", replace_unk=False, verbose=False,
               fast=False, alpha=0.0, beta=0.0, batch_size=3)
    opt.update(over)
    eng = FakeEngine()
    return Translator(synth.ModelConfig(), None, types.SimpleNamespace(**opt), engine=eng), eng


def chunks(lens, seed=0):
    rng = np.random.default_rng(seed)
    return [rng.normal(size=n).astype(np.float32) for n in lens]


def test_parse_chunk_string_matches_float32_cast():
    x = np.random.default_rng(1).normal(size=20)
    s = " ".join(str(v) for v in x)      # utils/labelop.py:231 str() round trip
    np.testing.assert_array_equal(parse_chunk(s), x.astype(np.float32))


def test_reference_batching_spans_and_order():
    tr, eng = make_tr()
    lens = [512, 512, 512, 512, 300]           # batches of 3: [512x3], [512, 300]
    sc, preds = tr.translate(chunks(lens), batch_size=3)
    assert len(preds) == 5 and all(len(p) == 1 for p in preds)
    # every chunk's span is its own reference batch's longest chunk (512 here)
    for i, L in enumerate(lens):
        assert preds[i][0] == " ".join(synth.DEFAULT_ITOS[t] for t in (4 + L % 4, 4 + 512 % 4, 5))
    # a reference batch made only of short chunks has a short span
    tr, eng = make_tr()
    sc, preds = tr.translate(chunks([512, 512, 512, 200, 150]), batch_size=3)
    assert preds[3][0].split()[1] == synth.DEFAULT_ITOS[4 + 200 % 4]
    assert preds[4][0].split()[1] == synth.DEFAULT_ITOS[4 + 200 % 4]


def test_eos_truncation_and_scores():
    tr, eng = make_tr()
    sc, preds = tr.translate(chunks([100]), batch_size=3)
    assert preds[0][0].count(" ") == 2          # 3 tokens then EOS
    assert abs(sc[0][0] - (-1.0)) < 1e-6


def test_pack_across_reads_equals_per_read():
    reads = [chunks([512, 512, 77], seed=1), chunks([512, 300], seed=2), chunks([60], seed=3)]
    tr, eng = make_tr()
    packed = tr.translate_reads(reads, batch_size=2)
    for r, exp in zip(reads, packed):
        tr2, _ = make_tr()
        assert tr2.translate(r, batch_size=2) == exp
    # packing fills engine batches across reads
    assert len(eng.calls) == 1 and eng.calls[0][1][0] >= 6


def test_beam_n_best():
    tr, eng = make_tr(beam_size=5, fast=True, n_best=2)
    sc, preds = tr.translate(chunks([512, 300]), batch_size=2)
    assert [len(p) for p in preds] == [2, 2]
    assert sc[0] == [0.0, -1.0]


def test_attn_debug_dump_format():
    """-attn_debug (translate/translator.py:285-336): '>' + the source samples
    and '|' + the prediction + '</s>' as one header line, then one row of
    weights per step, cut at the chunk length."""
    import io
    tr, eng = make_tr(max_length=6)
    f = io.StringIO()
    tr.setAttnFile(f)
    src = chunks([5, 3])
    sc, preds = tr.translate(src, batch_size=2, attn_debug=True)
    lines = f.getvalue().split("\n")
    assert lines[0].startswith("       > ") and "       | " in lines[0]
    assert lines[0].split("|")[1].split() == preds[0][0].split() + ["</s>"]
    assert lines[0].split()[1] == str(src[0][0])[:7]
    rows = lines[1:7]
    assert [len(r.split()) for r in rows] == [5] * 6
    assert rows[1].split() == ["{:.5f}".format(0.5)] * 2 + ["{:.5f}".format(0.0)] * 3
    assert len(lines[7].split("|")[0].split()) == 1 + 3       # second chunk: 3 samples


def _batch_of(src):
    return types.SimpleNamespace(
        src=torch.from_numpy(np.stack([np.pad(c, (0, 512 - len(c))) for c in src], 1)[:, :, None]),
        src_lengths=torch.tensor([len(c) for c in src]), batch_size=len(src))


def test_attn_debug_beam_cuts():
    """-attn_debug with beam search: each hypothesis' rows (one per token, EOS
    included), cut at memory_lengths[i] as the reference indexes its
    beam-tiled lengths: the classic Beam at lengths[j // beam] of the sorted
    batch; --fast by the same rule over the batches still alive at the
    hypothesis' last step.  The dump file rows keep the source width (the
    reference's row format has one field per source sample)."""
    import io
    src = chunks([150, 512, 77, 300, 100, 200])   # sorted: 512 300 200 150 100 77
    tr, eng = make_tr(beam_size=4, fast=False, max_length=6, batch_size=6)
    res = tr.translate_batch(_batch_of(src), None, True)
    # sorted positions 0..5 -> cut = sorted[pos // 4]: 512 for the first four, 300 for 100 and 77
    assert [a[0].shape for a in res["attention"]] == [(4, 512), (4, 512), (4, 300), (4, 512), (4, 300), (4, 512)]
    assert res["attention"][0][0][1, :2].tolist() == [1000.0, 1001.0]
    f = io.StringIO()
    tr.setAttnFile(f)
    tr.translate(src, batch_size=6, attn_debug=True)
    rows = [ln for ln in f.getvalue().split("\n") if ln.strip() and not ln.lstrip().startswith(">")]
    assert [len(r.split()) for r in rows] == [n for n in (150, 512, 77, 300, 100, 200) for _ in range(4)]
    # --fast: the 512 chunk finishes and is dropped at step 1, so at the other
    # hypotheses' last step (3) the alive sorted batch is 300 200 150 100 77:
    # 77 sits at index 4 -> cut = alive[1] = 200, the others -> alive[0] = 300
    tr, eng = make_tr(beam_size=4, fast=True, max_length=6, batch_size=6)
    orig = eng.translate_beam

    def beam_done(*a, **k):
        k["done_step"] = np.array([0, 2, 0, 0, 0, 0] + [0] * 2, np.int32)
        return orig(*a, **k)

    eng.translate_beam = beam_done
    res = tr.translate_batch(_batch_of(src), None, True, fast=True)
    assert [a[0].shape for a in res["attention"]] == [(4, 300), (2, 512), (4, 200), (4, 300), (4, 300), (4, 300)]


def test_classic_beam_reference_batches():
    """The classic onmt Beam advances a reference batch until all of its beams
    are done, so every chunk carries its reference batch id (batch_size
    consecutive chunks of one read) however the engine packs reads."""
    reads = [chunks([512, 512, 77], seed=1), chunks([512, 300], seed=2), chunks([60], seed=3)]
    tr, eng = make_tr(beam_size=4, fast=False, n_best=2, length_penalty="wu", alpha=0.6)
    tr.translate_reads(reads, batch_size=2)
    (kind, shape, L, S, groups, lp), = eng.calls
    assert kind == "classic" and lp == "wu"
    # chunks: read0 -> batches {0,1},{2}; read1 -> {0,1}; read2 -> {0}
    assert list(groups[:6]) == [0, 0, 1, 2, 2, 3]
    assert len(set(groups[6:])) == len(groups) - 6 and min(groups[6:]) > 3   # padding rows: own batches


def test_reference_errors():
    tr, _ = make_tr()
    with pytest.raises(ValueError):
        tr.translate(chunks([10]), batch_size=None)
    make_tr(beam_size=5, fast=False)  # the classic onmt Beam is on the path
    make_tr(beam_size=5, fast=False, block_ngram_repeat=2, coverage_penalty="wu", beta=0.2)
    with pytest.raises(ValueError):
        make_tr(beam_size=5, fast=False, coverage_penalty="bogus", beta=0.2)
    with pytest.raises(AssertionError):
        make_tr(beam_size=5, fast=True, block_ngram_repeat=2)
    with pytest.raises(AssertionError):
        make_tr(beam_size=5, fast=True, dump_beam="x.json")
    with pytest.raises(ValueError):
        make_tr(random_sampling_topk=9)
    with pytest.raises(AssertionError):
        make_tr(beam_size=5, fast=True, beta=0.5)
    with pytest.raises(RuntimeError):
        Translator(synth.ModelConfig(), None, types.SimpleNamespace(gpu=-1))


def test_translate_batch_reference_layout():
    tr, eng = make_tr()
    src = torch.zeros(512, 2, 1)
    src[:, 0, 0] = 1.5
    src[:300, 1, 0] = 2.0
    b = types.SimpleNamespace(src=src, src_lengths=torch.tensor([512, 300]), batch_size=2)
    res = tr.translate_batch(b, None, False)
    assert len(res["predictions"]) == 2 and res["predictions"][0][0].dtype == torch.long
    assert list(eng.calls[0][3][:2]) == [512, 512]


def test_classic_options_reach_the_engine(tmp_path):
    """Coverage / stepwise penalties, n-gram blocking with its exclusion
    tokens (ids through the vocab), the attention cut, and -dump_beam's
    accumulator file (translator.py:166-173, :365-368)."""
    dump = tmp_path / "beam.json"
    tr, eng = make_tr(beam_size=4, fast=False, coverage_penalty="summary", beta=0.3, stepwise_penalty=True,
                      block_ngram_repeat=3, ignore_when_blocking=["A", "G"], dump_beam=str(dump))
    tr.translate(chunks([512, 512, 512, 512, 77]), batch_size=5)
    o = eng.classic_opts
    assert o["coverage_penalty"] == "summary" and o["beta"] == 0.3 and o["stepwise_penalty"] is True
    assert o["block_ngram_repeat"] == 3 and sorted(o["ignore_ids"]) == [4, 6]
    assert list(o["cut"][:5]) == [512, 512, 512, 512, 512]
    import json
    assert json.loads(dump.read_text()) == {"predicted_ids": [], "beam_parent_ids": [], "scores": [],
                                            "log_probs": []}


def test_random_sampling_reaches_the_engine():
    """-random_sampling_topk / -random_sampling_temp (translator.py:371-394):
    keep_topk 1 or temp 0 stay on the argmax path; otherwise the sampling
    entry point runs with a seed that advances per call and repeats with -seed."""
    tr, eng = make_tr(random_sampling_topk=1, random_sampling_temp=0.5)
    tr.translate(chunks([100]), batch_size=1)
    assert eng.calls[-1][0] == "greedy"
    tr, eng = make_tr(random_sampling_topk=3, random_sampling_temp=0.0)
    tr.translate(chunks([100]), batch_size=1)
    assert eng.calls[-1][0] == "greedy"
    tr, eng = make_tr(random_sampling_topk=3, random_sampling_temp=0.7, seed=5)
    tr.translate(chunks([100]), batch_size=1)
    tr.translate(chunks([100]), batch_size=1)
    (k1, _, _, _, t1, top1, s1), (k2, _, _, _, _, _, s2) = eng.calls
    assert k1 == k2 == "sample" and t1 == 0.7 and top1 == 3 and s1 != s2
    tr2, eng2 = make_tr(random_sampling_topk=3, random_sampling_temp=0.7, seed=5)
    tr2.translate(chunks([100]), batch_size=1)
    assert eng2.calls[0][6] == s1
