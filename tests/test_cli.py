"""translate.py drop-in end to end on CPU with the engine replaced by a
deterministic stand-in: file discovery, resume, windowing, writers."""
import os

import numpy as np
import torch

from nanodecoder_amd import checkpoint, cli, opts, synth
from tests.test_translator_host import FakeEngine


class _Eng(FakeEngine):
    def __init__(self, cfg, W, device=0, max_batch=8, max_src_len=512, max_steps=100, max_beam=1):
        super().__init__(max_batch=max_batch, max_src_len=max_src_len)


def test_cli_end_to_end(tmp_path, monkeypatch):
    import nanodecoder_amd.translator as T
    monkeypatch.setattr(T, "Engine", _Eng)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    cfg = synth.ModelConfig()
    ck = tmp_path / "m.pt"
    checkpoint.save_synthetic(str(ck), cfg, synth.make_weights(cfg, seed=1))
    src = tmp_path / "reads"
    src.mkdir()
    for i, n in enumerate((1300, 700, 400)):
        raw = synth.synth_raw_read(i, n)
        (src / f"read{i}.signal").write_text(" ".join(str(int(v)) for v in raw))
    (src / "notes.txt").write_text("ignored")
    out = tmp_path / "out"
    o = opts.parse_translate_opts(["-model", str(ck), "-src_dir", str(src), "-save_data", str(out), "-gpu", "0",
                                   "-beam_size", "1", "-batch_size", "2", "-thread", "2", "-max_length", "10",
                                   "-pack_reads", "2"])
    assert cli.main(o) == 3
    for i in range(3):
        fa = (out / "result" / f"read{i}.fasta").read_text()
        assert fa.startswith(f">read{i}\n")
        seg = (out / "segment" / f"read{i}.txt").read_text().splitlines()
        assert len(seg) == {0: 3, 1: 2, 2: 1}[i]
    speed = (out / "speed.txt").read_text().splitlines()
    assert len(speed) == 3 and all(len(l.split("\t")) == 4 for l in speed)
    # resume: nothing left to do
    assert cli.main(o) == 0


def test_cli_attn_debug_and_beam_flags(tmp_path, monkeypatch):
    """-attn_debug writes save_data/attention/<read> per read (translate.py:64-71,
    110-120); the classic Beam's flags parse and reach the translator."""
    import nanodecoder_amd.translator as T
    monkeypatch.setattr(T, "Engine", _Eng)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    cfg = synth.ModelConfig()
    ck = tmp_path / "m.pt"
    checkpoint.save_synthetic(str(ck), cfg, synth.make_weights(cfg, seed=1))
    src = tmp_path / "reads"
    src.mkdir()
    for i, n in enumerate((700, 400)):
        raw = synth.synth_raw_read(i, n)
        (src / f"read{i}.signal").write_text(" ".join(str(int(v)) for v in raw))
    out = tmp_path / "out"
    o = opts.parse_translate_opts(["-model", str(ck), "-src_dir", str(src), "-save_data", str(out), "-gpu", "0",
                                   "-beam_size", "4", "-batch_size", "2", "-thread", "1", "-max_length", "6",
                                   "-attn_debug", "-coverage_penalty", "summary", "-beta", "0.2",
                                   "-stepwise_penalty", "-block_ngram_repeat", "3", "-ignore_when_blocking", "A",
                                   "-pack_reads", "2"])
    assert cli.main(o) == 2
    for i, n_chunks in enumerate((2, 1)):
        lines = [ln for ln in (out / "attention" / f"read{i}.txt").read_text().splitlines() if ln.strip()]
        headers = [ln for ln in lines if ln.lstrip().startswith(">")]
        assert len(headers) == n_chunks


def test_cli_empty_read_and_auto_pack(tmp_path, monkeypatch):
    """An empty .signal read is skipped, not fatal (translate.py:102-103), on
    both front ends' worker paths; -pack_reads 0 (default) packs reads until
    the engine batch is full and writes every read."""
    import nanodecoder_amd.translator as T
    monkeypatch.setattr(T, "Engine", _Eng)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    cfg = synth.ModelConfig()
    ck = tmp_path / "m.pt"
    checkpoint.save_synthetic(str(ck), cfg, synth.make_weights(cfg, seed=1))
    src = tmp_path / "reads"
    src.mkdir()
    for i, n in enumerate((1300, 700, 400, 2100)):
        raw = synth.synth_raw_read(i, n)
        (src / f"read{i}.signal").write_text(" ".join(str(int(v)) for v in raw))
    (src / "empty.signal").write_text("")
    # the -frontend gpu worker: an empty read is [prefix] alone (skipped), not [prefix, empty]
    job = (str(src / "empty.signal"), "empty.txt", "signal", "median", 512, 512)
    assert cli._read_only(job) == ["empty.txt"]
    out = tmp_path / "out"
    o = opts.parse_translate_opts(["-model", str(ck), "-src_dir", str(src), "-save_data", str(out), "-gpu", "0",
                                   "-beam_size", "1", "-batch_size", "2", "-thread", "2", "-max_length", "10",
                                   "-engine_max_batch", "4"])
    assert o.pack_reads == 0
    assert cli.main(o) == 4
    for i in range(4):
        assert (out / "result" / f"read{i}.fasta").exists()
    assert not (out / "result" / "empty.fasta").exists()
