"""Function-preserving "outlier dimension" transforms of a model's weights.

Trained transformers commonly carry a few activation dimensions far larger
than the rest.  The engine's three 24-bit storage forms hold a
power-of-two or per-row scale that such a dimension sets, so every other
dimension of the row keeps fewer significant bits.  These transforms put one
such dimension into exactly the tensors those forms store, while leaving the
model's function unchanged in exact arithmetic, so the engine can be held
against the oracle (the reference's fp32 algorithm) on the very same outputs:

- ``bank``: the memory bank (the encoder's final LayerNorm output,
  encoder/transformer.py:125-127) gets dimension ``d0`` ``f`` times larger
  (its LN gain and bias scaled), and every decoder layer's context K / V
  projection reads that dimension ``1/f`` as strongly.  The greedy decoder's
  24-bit digit bank holds these rows with one scale per row.
- ``ctx_k`` / ``ctx_v``: the context attention's keys (values) get output
  dimension ``j`` ``f`` times larger; the query (the output projection) takes
  ``1/f`` of it, so every score (every context vector after Wo) is unchanged.
  The beam's 24-bit context K/V holds one scale per (key, head).
- ``self_k`` / ``self_v``: the same on the decoder self-attention, whose
  24-bit history rows (beam) hold one scale per (key, head).

Reference: onmt/modules/multi_headed_attn.py:124-177 (the projections and
the score / context products these transforms commute with).
"""
from typing import Dict, Iterable

import numpy as np


def outlier_weights(cfg, W: Dict[str, np.ndarray], f: float = 1e3, forms: Iterable[str] = ("bank", "ctx_k",
                    "ctx_v", "self_k", "self_v"), d0: int = 77, j: int = 45) -> Dict[str, np.ndarray]:
    W = {k: v.copy() for k, v in W.items()}
    f = np.float32(f)
    forms = set(forms)
    if "bank" in forms:
        assert cfg.encoder_type == "transformer"
        W["encoder.layer_norm.weight"][d0] *= f
        W["encoder.layer_norm.bias"][d0] *= f
    for i in range(cfg.dec_layers):
        p = f"decoder.transformer_layers.{i}"
        if "bank" in forms:
            for n in ("linear_keys", "linear_values"):
                W[f"{p}.context_attn.{n}.weight"][:, d0] /= f
        for att, tag in (("context_attn", "ctx"), ("self_attn", "self")):
            a = f"{p}.{att}"
            if f"{tag}_k" in forms:
                W[f"{a}.linear_keys.weight"][j] *= f
                W[f"{a}.linear_keys.bias"][j] *= f
                W[f"{a}.linear_query.weight"][j] /= f
                W[f"{a}.linear_query.bias"][j] /= f
            if f"{tag}_v" in forms:
                W[f"{a}.linear_values.weight"][j] *= f
                W[f"{a}.linear_values.bias"][j] *= f
                W[f"{a}.final_linear.weight"][:, j] /= f
    return W
