"""Checkpoint loading for the drop-in (replaces models/model_builder.py:217-382).

Reference checkpoints (onmt/models/model_saver.py:105-119) are pickles of
``{'model': state_dict, 'generator': state_dict, 'vocab': [(field, Vocab)],
'opt': argparse.Namespace, 'optim': onmt Optimizer}``.  torchtext and onmt
are not importable here, so they are read with a RESTRICTED unpickler: only
torch's tensor-rebuild functions, containers and argparse.Namespace resolve to
real objects; torchtext / onmt / torch.optim classes resolve to an inert stub
that just records its state.  Nothing else can be constructed — a file asking
for any other global raises.

The engine's own synthetic checkpoints (``save_synthetic``) hold only tensors,
dicts, lists, strings and numbers and load with ``weights_only=True``.
"""
from __future__ import annotations

import argparse
import collections
import pickle
import re
import types
from typing import Dict, List, Tuple

import numpy as np
import torch

from .synth import ModelConfig

# models/opts.py model_opts defaults the loader merges under the checkpoint opt
# (models/model_builder.py:225-229) — only the ones that shape the hot path.
MODEL_OPT_DEFAULTS = dict(encoder_type="rnn", decoder_type="rnn", layers=-1, enc_layers=2, dec_layers=2,
                          rnn_size=-1, enc_rnn_size=500, dec_rnn_size=500, heads=8, transformer_ff=2048,
                          position_encoding=False, self_attn_type="scaled-dot", copy_attn=False,
                          generator_function="softmax", rnn_type="LSTM", audio_enc_pooling="1")


class _Stub:
    """Inert stand-in for torchtext / onmt / torch.optim objects."""

    def __init__(self, *a, **k):
        self.__dict__["_args"] = a

    def __setstate__(self, state):
        if isinstance(state, dict):
            self.__dict__.update(state)
        else:
            self.__dict__["_state"] = state

    def __call__(self, *a, **k):  # e.g. defaultdict default factories
        return None


def _stub_class(module, name):
    return type(name, (_Stub,), {"__module__": module})


_ALLOWED = {
    ("collections", "OrderedDict"): collections.OrderedDict,
    ("collections", "defaultdict"): collections.defaultdict,
    ("collections", "Counter"): collections.Counter,
    ("argparse", "Namespace"): argparse.Namespace,
    ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
    ("torch._utils", "_rebuild_parameter"): torch._utils._rebuild_parameter,
    ("torch", "Size"): torch.Size,
}
for _b in (set, frozenset, slice, int, float, complex, bool, str, bytes, bytearray, list, dict, tuple, range):
    _ALLOWED[("builtins", _b.__name__)] = _b
for _t in ("FloatStorage", "DoubleStorage", "HalfStorage", "LongStorage", "IntStorage", "ShortStorage",
           "CharStorage", "ByteStorage", "BoolStorage", "BFloat16Storage"):
    if hasattr(torch, _t):
        _ALLOWED[("torch", _t)] = getattr(torch, _t)
_STUB_PREFIXES = ("torchtext", "onmt", "torch.optim", "inputters", "models", "utils")


class _RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        # protocol-2 pickles carry Python 2 names (__builtin__.long, ...)
        import _compat_pickle
        if (module, name) in _compat_pickle.NAME_MAPPING:
            module, name = _compat_pickle.NAME_MAPPING[(module, name)]
        elif module in _compat_pickle.IMPORT_MAPPING:
            module = _compat_pickle.IMPORT_MAPPING[module]
        if (module, name) in _ALLOWED:
            return _ALLOWED[(module, name)]
        if module.startswith(_STUB_PREFIXES):
            return _stub_class(module, name)
        raise pickle.UnpicklingError(f"checkpoint references a disallowed global {module}.{name}")


_restricted = types.SimpleNamespace(Unpickler=_RestrictedUnpickler, load=pickle.load, __name__="restricted_pickle")


def _fix_key(s: str) -> str:
    """models/model_builder.py:345-353 (legacy custom LayerNorm a_2/b_2)."""
    s = re.sub(r"(.*)\.layer_norm((_\d+)?)\.b_2", r"\1.layer_norm\2.bias", s)
    s = re.sub(r"(.*)\.layer_norm((_\d+)?)\.a_2", r"\1.layer_norm\2.weight", s)
    return s


def _itos_from_vocab(vocab) -> List[str]:
    """checkpoint['vocab'] = [(field_name, torchtext Vocab)] (inputters/inputter.py:164-178)."""
    if isinstance(vocab, dict):
        v = vocab.get("tgt")
    else:
        v = dict(vocab).get("tgt") if vocab is not None else None
    if v is None:
        raise ValueError("checkpoint has no tgt vocabulary")
    itos = getattr(v, "itos", None) if not isinstance(v, (list, tuple)) else list(v)
    if itos is None:
        raise ValueError("tgt vocabulary has no itos")
    return list(itos)


def config_from_opt(opt: Dict, itos: List[str]) -> ModelConfig:
    o = dict(MODEL_OPT_DEFAULTS)
    o.update({k: v for k, v in opt.items() if v is not None})
    if o.get("rnn_size", -1) != -1:  # models/model_builder.py:250-252
        o["enc_rnn_size"] = o["dec_rnn_size"] = o["rnn_size"]
    if o["decoder_type"] != "transformer":
        raise NotImplementedError(f"decoder_type {o['decoder_type']!r}: only the transformer decoder is on the "
                                  "MI355X path (SURVEY.md §2)")
    if o["encoder_type"] not in ("transformer", "nano"):
        raise NotImplementedError(f"encoder_type {o['encoder_type']!r} is not on the MI355X path")
    if o["self_attn_type"] not in ("scaled-dot", "average"):
        raise NotImplementedError(f"self_attn_type {o['self_attn_type']!r} (decoder/transformer.py:33-37 "
                                  "knows scaled-dot and average)")
    if o["copy_attn"]:
        raise NotImplementedError("copy_attn models are not supported")
    if o["generator_function"] != "softmax":
        raise NotImplementedError("only the softmax generator is supported")
    if o["encoder_type"] == "nano":
        if o.get("rnn_type", "LSTM") != "LSTM":
            raise NotImplementedError("NanoEncoder supports rnn_type LSTM only")
        if str(o.get("audio_enc_pooling", "1")).replace(",", "").strip("1"):
            raise NotImplementedError("NanoEncoder supports audio_enc_pooling 1 only")
    return ModelConfig(encoder_type=o["encoder_type"], enc_layers=int(o["enc_layers"]),
                       dec_layers=int(o["dec_layers"]), d_model=int(o["dec_rnn_size"]), heads=int(o["heads"]),
                       d_ff=int(o["transformer_ff"]), rnn_hidden=int(o["enc_rnn_size"]) // 2,
                       position_encoding=bool(o["position_encoding"]), self_attn_type=o["self_attn_type"],
                       itos=itos)


def _np(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        return t.detach().to(torch.float32).cpu().numpy()
    return np.asarray(t, np.float32)


def load(path: str) -> Tuple[ModelConfig, Dict[str, np.ndarray]]:
    """Returns (ModelConfig, weights by reference state-dict name, generator
    keys prefixed 'generator.')."""
    try:
        ck = torch.load(path, map_location="cpu", weights_only=True)
    except Exception:
        ck = torch.load(path, map_location="cpu", weights_only=False, pickle_module=_restricted)
    if "vocab_itos" in ck:            # engine synthetic format
        itos = list(ck["vocab_itos"])
    else:
        itos = _itos_from_vocab(ck.get("vocab"))
    opt = ck.get("opt")
    opt = vars(opt) if isinstance(opt, argparse.Namespace) else dict(opt or {})
    cfg = config_from_opt(opt, itos)
    W = {_fix_key(k): _np(v) for k, v in ck["model"].items()}
    for k, v in ck["generator"].items():
        W["generator." + k] = _np(v)
    return cfg, W


def save_synthetic(path: str, cfg: ModelConfig, W: Dict[str, np.ndarray]):
    """Write a checkpoint in the reference's key layout that loads with
    weights_only=True (no torchtext / argparse objects)."""
    opt = dict(encoder_type=cfg.encoder_type, decoder_type="transformer", enc_layers=cfg.enc_layers,
               dec_layers=cfg.dec_layers, enc_rnn_size=(2 * cfg.rnn_hidden if cfg.encoder_type == "nano"
                                                        else cfg.d_model),
               dec_rnn_size=cfg.d_model, rnn_size=-1, heads=cfg.heads, transformer_ff=cfg.d_ff,
               position_encoding=cfg.position_encoding, self_attn_type=cfg.self_attn_type, copy_attn=False,
               generator_function="softmax", rnn_type="LSTM", audio_enc_pooling="1")
    model = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in W.items() if not k.startswith("generator.")}
    gen = {k[len("generator."):]: torch.from_numpy(np.ascontiguousarray(v)) for k, v in W.items()
           if k.startswith("generator.")}
    torch.save({"model": model, "generator": gen, "vocab_itos": list(cfg.itos), "opt": opt}, path)
