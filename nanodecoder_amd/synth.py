"""Synthetic model checkpoints and synthetic nanopore reads.

No trained NanoDecoder checkpoint ships with the reference (the
README's ``model/demo-step-10000.pt`` is absent), so every benchmark and parity
test runs on a seeded random-init model with the reference architecture.

* Weights use numpy's PCG64 ``default_rng(seed)`` (version-stable) and are laid
  out under the reference's state-dict names, so the same
  dict can be loaded into the reference modules (golden generation) and into
  the HIP engine.
* Reads follow SURVEY.md §8d: event levels ~N(90,15), dwell ~Geometric(1/9),
  N(0,2) noise, rounded to integers like a raw DAC trace, then median/MAD
  normalised exactly as ``utils/labelop.py:194-233`` does and windowed into
  ``src_seq_length`` chunks.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional

import numpy as np

# onmt/inputters/dataset_base.py:10-13 + inputters/inputter.py:151-152: specials
# first, so unk=0, pad=1, bos=2, eos=3; bases follow in training-frequency order.
DEFAULT_ITOS = ["<unk>", "<blank>", "<s>", "</s>", "A", "C", "G", "T"]
MAD_SCALE = 0.6744897501960817  # statsmodels.robust.mad normalisation constant


@dataclasses.dataclass
class ModelConfig:
    """Architecture of a NanoDecoder translate model (checkpoint ``opt``)."""
    encoder_type: str = "transformer"   # "transformer" | "nano"
    enc_layers: int = 3
    dec_layers: int = 3
    d_model: int = 256
    heads: int = 8
    d_ff: int = 2048
    rnn_hidden: int = 128               # per direction, NanoEncoder only
    position_encoding: bool = False     # models/opts.py:41-44 (off by default)
    self_attn_type: str = "scaled-dot"  # decoder self-attention: "scaled-dot" | "average" (AAN)
    itos: List[str] = dataclasses.field(default_factory=lambda: list(DEFAULT_ITOS))

    @property
    def vocab(self) -> int:
        return len(self.itos)

    @property
    def pad_idx(self) -> int:
        return self.itos.index("<blank>")

    @property
    def bos_idx(self) -> int:
        return self.itos.index("<s>")

    @property
    def eos_idx(self) -> int:
        return self.itos.index("</s>")

    @property
    def unk_idx(self) -> int:
        return self.itos.index("<unk>")


def _xavier(rng, shape):
    fan_out, fan_in = shape[0], shape[1]
    a = math.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-a, a, size=shape).astype(np.float32)


def _bias(rng, n, scale=0.05):
    return rng.uniform(-scale, scale, size=(n,)).astype(np.float32)


def _ln(rng, n):
    return (1.0 + rng.uniform(-0.1, 0.1, size=(n,))).astype(np.float32), _bias(rng, n, 0.05)


def _linear(rng, W, prefix, out_f, in_f, bias=True):
    W[prefix + ".weight"] = _xavier(rng, (out_f, in_f))
    if bias:
        W[prefix + ".bias"] = _bias(rng, out_f)


def _mha(rng, W, prefix, d):
    for name in ("linear_keys", "linear_values", "linear_query", "final_linear"):
        _linear(rng, W, f"{prefix}.{name}", d, d)


def _ffn(rng, W, prefix, d, d_ff):
    _linear(rng, W, prefix + ".w_1", d_ff, d)
    _linear(rng, W, prefix + ".w_2", d, d_ff)
    W[prefix + ".layer_norm.weight"], W[prefix + ".layer_norm.bias"] = _ln(rng, d)


def positional_table(d: int, max_len: int = 5000) -> np.ndarray:
    """onmt/modules/embeddings.py:23-31 (computed in fp32 like torch does)."""
    import torch
    pe = torch.zeros(max_len, d)
    position = torch.arange(0, max_len).unsqueeze(1)
    div_term = torch.exp((torch.arange(0, d, 2, dtype=torch.float) * -(math.log(10000.0) / d)))
    pe[:, 0::2] = torch.sin(position.float() * div_term)
    pe[:, 1::2] = torch.cos(position.float() * div_term)
    return pe.unsqueeze(1).numpy()


def make_weights(cfg: ModelConfig, seed: int = 0, eos_bias: float = 0.0) -> Dict[str, np.ndarray]:
    """Random-init weights under the reference state-dict names.

    The generator bias is -1e4 on <unk>/<blank>/<s> so that argmax emits bases
    or EOS (random weights otherwise emit only specials);
    ``eos_bias`` shifts the EOS logit to tune how early beams finish.
    """
    rng = np.random.default_rng(seed)
    d, V = cfg.d_model, cfg.vocab
    W: Dict[str, np.ndarray] = {}
    if cfg.encoder_type == "transformer":
        _linear(rng, W, "encoder.linear", d, 1)
        for i in range(cfg.enc_layers):
            p = f"encoder.transformer.{i}"
            W[p + ".layer_norm.weight"], W[p + ".layer_norm.bias"] = _ln(rng, d)
            _mha(rng, W, p + ".self_attn", d)
            _ffn(rng, W, p + ".feed_forward", d, cfg.d_ff)
        W["encoder.layer_norm.weight"], W["encoder.layer_norm.bias"] = _ln(rng, d)
    elif cfg.encoder_type == "nano":
        H = cfg.rnn_hidden
        k = 1.0 / math.sqrt(H)
        for l in range(cfg.enc_layers):
            in_f = 1 if l == 0 else 2 * H
            for sfx in ("", "_reverse"):
                p = f"encoder.rnn_{l}"
                W[f"{p}.weight_ih_l0{sfx}"] = rng.uniform(-k, k, (4 * H, in_f)).astype(np.float32)
                W[f"{p}.weight_hh_l0{sfx}"] = rng.uniform(-k, k, (4 * H, H)).astype(np.float32)
                W[f"{p}.bias_ih_l0{sfx}"] = rng.uniform(-k, k, (4 * H,)).astype(np.float32)
                W[f"{p}.bias_hh_l0{sfx}"] = rng.uniform(-k, k, (4 * H,)).astype(np.float32)
            b = f"encoder.batchnorm_{l}"
            W[b + ".weight"], W[b + ".bias"] = _ln(rng, 2 * H)
            W[b + ".running_mean"] = rng.uniform(-0.1, 0.1, (2 * H,)).astype(np.float32)
            W[b + ".running_var"] = rng.uniform(0.02, 0.08, (2 * H,)).astype(np.float32)
        W["encoder.W.weight"] = _xavier(rng, (d, 2 * H))
    else:
        raise ValueError(f"unknown encoder_type {cfg.encoder_type!r}")

    W["decoder.embeddings.make_embedding.emb_luts.0.weight"] = rng.normal(0, 1, (V, d)).astype(np.float32)
    if cfg.position_encoding:
        W["decoder.embeddings.make_embedding.pe.pe"] = positional_table(d)
    for i in range(cfg.dec_layers):
        p = f"decoder.transformer_layers.{i}"
        if cfg.self_attn_type == "average":
            # onmt/modules/average_attn.py:26-29: PositionwiseFeedForward(d, d) + Linear(2d, 2d)
            _ffn(rng, W, p + ".self_attn.average_layer", d, d)
            _linear(rng, W, p + ".self_attn.gating_layer", 2 * d, 2 * d)
        else:
            _mha(rng, W, p + ".self_attn", d)
        _mha(rng, W, p + ".context_attn", d)
        W[p + ".layer_norm_1.weight"], W[p + ".layer_norm_1.bias"] = _ln(rng, d)
        W[p + ".layer_norm_2.weight"], W[p + ".layer_norm_2.bias"] = _ln(rng, d)
        _ffn(rng, W, p + ".feed_forward", d, cfg.d_ff)
    W["decoder.layer_norm.weight"], W["decoder.layer_norm.bias"] = _ln(rng, d)

    W["generator.0.weight"] = _xavier(rng, (V, d)) * 4.0
    gb = _bias(rng, V, 0.1)
    for tok in ("<unk>", "<blank>", "<s>"):
        gb[cfg.itos.index(tok)] = -1e4
    gb[cfg.eos_idx] += eos_bias
    W["generator.0.bias"] = gb.astype(np.float32)
    return W


# ----------------------------------------------------------------------------
# synthetic reads
# ----------------------------------------------------------------------------

def synth_raw_read(read_id: int, n_samples: int) -> np.ndarray:
    """Integer-valued raw current trace, float64."""
    rng = np.random.default_rng(1234 + read_id)
    out = np.empty(n_samples, dtype=np.float64)
    pos = 0
    while pos < n_samples:
        level = rng.normal(90.0, 15.0)
        dwell = int(rng.geometric(1.0 / 9.0))
        end = min(n_samples, pos + dwell)
        out[pos:end] = level
        pos = end
    out += rng.normal(0.0, 2.0, size=n_samples)
    return np.round(out)


def normalize_median(raw: np.ndarray) -> np.ndarray:
    """(x - median) / MAD, MAD = median(|x - median|) / 0.67449 (utils/labelop.py:222-223)."""
    raw = np.asarray(raw, dtype=np.float64)
    med = np.median(raw)
    # statsmodels.robust.scale.mad: np.median(np.abs(a - center) / c)
    mad = np.median(np.abs(raw - med) / MAD_SCALE)
    return (raw - med) / mad


def window(signal: np.ndarray, length: int = 512, stride: int = 512) -> List[np.ndarray]:
    """Chunking of utils/labelop.py:225-233: windows start every `stride`,
    the last one is cut at the end of the read; stops after the window that
    reaches the end.  Returns float32 chunks (the reference's str/float round
    trip of a float64 equals a direct float32 cast)."""
    out = []
    n = len(signal)
    for i in range(0, math.ceil(n / stride)):
        s = i * stride
        e = min(s + length, n)
        out.append(np.asarray(signal[s:e], dtype=np.float32))
        if e >= n:
            break
    return out


def synth_read_chunks(read_id: int, n_samples: int, length: int = 512, stride: int = 512) -> List[np.ndarray]:
    return window(normalize_median(synth_raw_read(read_id, n_samples)), length, stride)


def synth_chunk_batch(n_chunks: int, T: int = 512, seed: int = 0, inject_masks: bool = True):
    """A [n_chunks, T] float32 batch of full-length chunks cut from synthetic
    reads; with ``inject_masks`` a few exact 0.0 / 1.0 samples are planted so
    both mask quirks (src==0 key mask, src==1 context mask) are exercised."""
    chunks = []
    rid = seed * 100003
    while len(chunks) < n_chunks:
        for c in synth_read_chunks(rid, 8 * T, T, T):
            if len(c) == T and len(chunks) < n_chunks:
                chunks.append(c)
        rid += 1
    x = np.stack(chunks).astype(np.float32)
    if inject_masks:
        rng = np.random.default_rng(seed + 7)
        idx = rng.integers(0, x.size, size=max(1, x.size // 200))
        x.reshape(-1)[idx[: len(idx) // 2]] = 0.0
        x.reshape(-1)[idx[len(idx) // 2:]] = 1.0
    return x
