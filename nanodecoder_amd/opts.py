"""translate.py flag surface (models/opts.py:504-658 translate_opts), with the
reference's single-dash and double-dash spellings.  configargparse is not
available offline, so ``-config FILE`` (YAML, models/opts.py:8-13) is handled
here: its keys become defaults that explicit flags override."""
from __future__ import annotations

import argparse
import sys

import yaml


def _add(g, name, **kw):
    g.add_argument("--" + name, "-" + name, **kw)


def translate_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="translate.py (NanoDecoder on MI355X)",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    _add(p, "config", default=None, help="YAML config file (keys = flag names)")
    g = p.add_argument_group("Model")
    g.add_argument("--model", "-model", dest="models", metavar="MODEL", nargs="+", type=str, default=[],
                   required=True, help="Path to model .pt file(s)")
    g = p.add_argument_group("Data")
    _add(g, "thread", type=int, default=4, help="signal extraction worker processes")
    g.add_argument("--normalization_raw", default="median", help="median | mean | None")
    _add(g, "src_dir", default="", help="directory of .signal / .fast5 reads")
    _add(g, "src_seq_length", type=int, default=512)
    _add(g, "src_seq_stride", type=int, default=512)
    _add(g, "save_data", required=True, help="output folder")
    g = p.add_argument_group("Random Sampling")
    _add(g, "random_sampling_topk", default=1, type=int)
    _add(g, "random_sampling_temp", default=1.0, type=float)
    g = p.add_argument_group("Beam")
    _add(g, "fast", action="store_true")
    _add(g, "beam_size", type=int, default=5)
    _add(g, "min_length", type=int, default=0)
    _add(g, "max_length", type=int, default=100)
    _add(g, "stepwise_penalty", action="store_true")
    _add(g, "length_penalty", default="none", choices=["none", "wu", "avg"])
    _add(g, "coverage_penalty", default="none", choices=["none", "wu", "summary"])
    _add(g, "alpha", type=float, default=0.0)
    _add(g, "beta", type=float, default=-0.0)
    _add(g, "block_ngram_repeat", type=int, default=0)
    _add(g, "ignore_when_blocking", nargs="+", type=str, default=[])
    _add(g, "replace_unk", action="store_true")
    g = p.add_argument_group("Logging")
    _add(g, "verbose", action="store_true")
    _add(g, "log_file", type=str, default="")
    _add(g, "log_file_level", type=str, default="0")
    _add(g, "attn_debug", action="store_true")
    _add(g, "dump_beam", type=str, default="")
    _add(g, "n_best", type=int, default=1)
    g = p.add_argument_group("Efficiency")
    _add(g, "batch_size", type=int, default=100)
    _add(g, "gpu", type=int, default=-1)
    g = p.add_argument_group("SpeechLike")
    _add(g, "fft", type=bool, default=False)
    _add(g, "sample_rate", type=int, default=4000)
    _add(g, "window_size", type=float, default=0.075)
    _add(g, "window_stride", type=float, default=0.015)
    _add(g, "window", default="hamming")
    g = p.add_argument_group("MI355X engine (additions)")
    _add(g, "pack_reads", type=int, default=0,
         help="translate this many reads per engine pass (chunks packed across reads; same outputs); "
              "0 = as many reads as fill the engine batch")
    _add(g, "engine_max_batch", type=int, default=0,
         help="engine batch capacity in chunks (0 = max(batch_size, 256): a full MI355X batch)")
    _add(g, "engine_lanes", type=int, default=0,
         help="translate calls kept on the GPU at once (EnginePool lanes: one engine context and hardware queue "
              "each, each holding its own workspaces; the calls' kernels share the CUs); 1 = one call at a time; "
              "0 = 3 for greedy / sampling, 1 for beam search")
    _add(g, "seed", type=int, default=-1, help="random sampling seed (-1: fresh entropy per run)")
    _add(g, "frontend", default="cpu", choices=["cpu", "gpu"],
         help="gpu: normalise and window the reads on the GPU (frontend.hip) instead of in the worker pool")
    return p


def parse_translate_opts(argv=None):
    p = translate_parser()
    argv = sys.argv[1:] if argv is None else list(argv)
    cfg_path = None
    for i, a in enumerate(argv):
        if a in ("-config", "--config") and i + 1 < len(argv):
            cfg_path = argv[i + 1]
    if cfg_path:
        with open(cfg_path) as f:
            conf = yaml.safe_load(f) or {}
        conf = {("models" if k in ("model", "models") else k): v for k, v in conf.items()}
        p.set_defaults(**conf)
        for a in p._actions:
            if a.dest in conf:
                a.required = False
    opt = p.parse_args(argv)
    if isinstance(opt.models, str):
        opt.models = [opt.models]
    if opt.fft:
        raise NotImplementedError("-fft spectrogram input is not on the MI355X path")
    return opt
