"""Checkpoint loader (reference .pt layout, restricted unpickler) and the
signal front end / assembly host code.  CPU only."""
import argparse
import collections
import io
import os
import pickle
import sys
import types

import numpy as np
import pytest
import torch

from nanodecoder_amd import checkpoint, frontend, synth


def _fake_modules():
    """Stand-ins so a reference-style checkpoint can be WRITTEN here."""
    tt = types.ModuleType("torchtext")
    ttv = types.ModuleType("torchtext.vocab")

    class Vocab:
        pass
    Vocab.__module__, Vocab.__qualname__ = "torchtext.vocab", "Vocab"
    ttv.Vocab = Vocab
    opt_mod = types.ModuleType("onmt.utils.optimizers")

    class Optimizer:
        pass
    Optimizer.__module__, Optimizer.__qualname__ = "onmt.utils.optimizers", "Optimizer"
    opt_mod.Optimizer = Optimizer
    return {"torchtext": tt, "torchtext.vocab": ttv, "onmt": types.ModuleType("onmt"),
            "onmt.utils": types.ModuleType("onmt.utils"), "onmt.utils.optimizers": opt_mod}


def test_reference_layout_checkpoint_roundtrip(tmp_path, monkeypatch):
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=3)
    mods = _fake_modules()
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    vocab = mods["torchtext.vocab"].Vocab()
    vocab.itos = list(cfg.itos)
    vocab.stoi = collections.defaultdict(int, {s: i for i, s in enumerate(cfg.itos)})
    optim = mods["onmt.utils.optimizers"].Optimizer()
    optim.lr = 1.0
    model = collections.OrderedDict((k, torch.from_numpy(v)) for k, v in W.items() if not k.startswith("generator"))
    # a legacy custom-LayerNorm key (models/model_builder.py:345-353)
    model["decoder.layer_norm.a_2"] = model.pop("decoder.layer_norm.weight")
    model["decoder.transformer_layers.0.mask"] = torch.zeros(1, 4, 4, dtype=torch.uint8)
    gen = collections.OrderedDict((k[len("generator."):], torch.from_numpy(v)) for k, v in W.items()
                                  if k.startswith("generator"))
    opt = argparse.Namespace(encoder_type="transformer", decoder_type="transformer", enc_layers=3, dec_layers=3,
                             rnn_size=256, heads=8, transformer_ff=2048, position_encoding=False,
                             self_attn_type="scaled-dot", copy_attn=False)
    path = tmp_path / "ref.pt"
    torch.save({"model": model, "generator": gen, "vocab": [("src", None), ("tgt", vocab)], "opt": opt,
                "optim": optim}, path)
    for k in mods:
        monkeypatch.delitem(sys.modules, k)
    cfg2, W2 = checkpoint.load(str(path))
    assert cfg2.itos == cfg.itos and cfg2.d_model == 256 and cfg2.encoder_type == "transformer"
    np.testing.assert_array_equal(W2["decoder.layer_norm.weight"], W["decoder.layer_norm.weight"])
    np.testing.assert_array_equal(W2["generator.0.bias"], W["generator.0.bias"])


def test_synthetic_checkpoint_weights_only(tmp_path):
    cfg = synth.ModelConfig(encoder_type="nano")
    W = synth.make_weights(cfg, seed=4)
    p = tmp_path / "s.pt"
    checkpoint.save_synthetic(str(p), cfg, W)
    torch.load(p, weights_only=True)   # loadable with the safe loader
    cfg2, W2 = checkpoint.load(str(p))
    assert cfg2.encoder_type == "nano" and cfg2.rnn_hidden == 128
    assert set(W2) == set(W)


def test_restricted_unpickler_refuses_arbitrary_globals():
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    data = pickle.dumps(Evil())
    with pytest.raises(pickle.UnpicklingError):
        checkpoint._RestrictedUnpickler(io.BytesIO(data)).load()


def test_unsupported_model_opts_raise():
    with pytest.raises(NotImplementedError):
        checkpoint.config_from_opt({"encoder_type": "transformer", "decoder_type": "rnn"}, synth.DEFAULT_ITOS)
    with pytest.raises(NotImplementedError):
        checkpoint.config_from_opt({"encoder_type": "transformer", "decoder_type": "transformer",
                                    "self_attn_type": "relative"}, synth.DEFAULT_ITOS)


def test_average_self_attention_opt_maps_to_config():
    cfg = checkpoint.config_from_opt({"encoder_type": "transformer", "decoder_type": "transformer",
                                      "self_attn_type": "average"}, synth.DEFAULT_ITOS)
    assert cfg.self_attn_type == "average"


def test_window_matches_labelop_rules():
    sig = np.arange(1300, dtype=np.float64)
    w = frontend.window(sig, 512, 512)
    assert [len(c) for c in w] == [512, 512, 276]
    w = frontend.window(sig, 300, 60)           # overlapping production setting
    assert w[0][0] == 0 and w[1][0] == 60 and len(w[-1]) <= 300 and w[-1][-1] == 1299
    assert frontend.window(np.arange(512.0), 512, 512)[-1].size == 512
    assert len(frontend.window(np.arange(512.0), 512, 512)) == 1


def test_median_mad_normalisation():
    raw = synth.synth_raw_read(5, 4000)
    x = frontend.normalize(raw, "median")
    assert abs(np.median(x)) < 1e-12
    assert abs(np.median(np.abs(x)) - synth.MAD_SCALE) < 1e-9
    np.testing.assert_array_equal(frontend.normalize(raw, "None"), raw)


def test_simple_assembly_overlap_consensus():
    preds = [["A C G T A C"], ["G T A C G G"], ["A C G G T T"]]
    cons = frontend.simple_assembly(preds)
    assert frontend.index2base(np.argmax(cons, axis=0)) == "ACGTACGGTT"
    assert frontend.simple_assembly(preds, flag_intersection=False) == "ACGTACGTACGGACGGTT"
    assert frontend.assemble_read([["A C"], [""], ["G"]], 512, 512) == "ACG"


def test_extract_raw_signal_file(tmp_path):
    raw = synth.synth_raw_read(1, 1100)
    p = tmp_path / "r.signal"
    p.write_text(" ".join(str(int(v)) for v in raw))
    out = frontend.extract_raw(str(p), "r.txt", "median", 512, 512, "signal")
    assert out[0] == "r.txt" and [len(c) for c in out[1:]] == [512, 512, 76]
    np.testing.assert_array_equal(np.concatenate(out[1:]), frontend.normalize(raw, "median").astype(np.float32))


def test_windows_match_window():
    """frontend.windows (the GPU front end's chunk list) cuts exactly what
    window() (utils/labelop.py:225-233) cuts."""
    from nanodecoder_amd import frontend
    for n in (1, 2, 299, 300, 512, 513, 1024, 1300, 4000):
        for L, st in ((512, 512), (300, 60), (512, 256)):
            x = np.arange(n, dtype=np.float64)
            exp = frontend.window(x, L, st)
            got = frontend.windows(n, L, st)
            assert len(got) == len(exp)
            for (a, b), e in zip(got, exp):
                assert b == len(e) and (x[a: a + b].astype(np.float32) == e).all()


# ---------------------------------------------------------------- pinned to the reference's labelop.py
def _golden_frontend():
    from tests import golden_util as gu
    return gu, *gu.load_frontend()


def test_extract_raw_vs_reference_labelop(tmp_path):
    """frontend.extract_raw on .signal files against the chunks the
    reference's own extract_fast5_raw cut from the same files
    (tests/golden/frontend.npz, oracle/make_golden_frontend.py): median / mean
    / None normalisation at 512/512 and the 300/60 overlap setting; bit-exact
    float32, NaN where the reference divides by a zero MAD or std."""
    gu, z, meta = _golden_frontend()
    for i in range(meta["reads"]):
        raw = z[f"raw{i}"]
        path = tmp_path / f"read{i}.signal"
        path.write_text(" ".join(str(int(v)) if float(v).is_integer() else repr(float(v)) for v in raw))
        for si, (norm, ml, st) in enumerate(meta["settings"]):
            with np.errstate(divide="ignore", invalid="ignore"):
                got = frontend.extract_raw(str(path), f"read{i}.txt", norm, ml, st, "signal")
            exp = gu.frontend_chunks(z, i, si)
            assert got[0] == f"read{i}.txt" and len(got) - 1 == len(exp), (i, si)
            for g, e in zip(got[1:], exp):
                assert gu.same_f32(g, e), (i, si)


def test_simple_assembly_vs_reference_labelop():
    """frontend.simple_assembly / index2base against the reference's own
    simple_assembly on overlapping-window predictions with substitutions,
    indels, an empty chunk and a read that grows the consensus past 1000
    columns: identical count matrices and base strings, both branches."""
    gu, z, meta = _golden_frontend()
    for j in range(len(meta["assembly"])):
        preds = [[str(p)] for p in z[f"asm_preds{j}"]]
        cons = frontend.simple_assembly(preds)
        assert cons.shape == z[f"asm_cons{j}"].shape and (cons == z[f"asm_cons{j}"]).all(), j
        assert frontend.index2base(np.argmax(cons, axis=0)) == str(z[f"asm_seq{j}"]), j
        assert frontend.simple_assembly(preds, flag_intersection=False) == str(z[f"asm_concat{j}"]), j
        assert frontend.assemble_read(preds, 300, 60) == str(z[f"asm_seq{j}"])
