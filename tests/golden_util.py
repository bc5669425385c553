"""Helpers to read the committed golden fixtures (tests/golden/*.npz)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["transformer_greedy", "transformer_pe_short", "transformer_beam", "nano_greedy", "transformer_aan",
         "transformer_classic_beam", "transformer_classic_beam_mid", "transformer_beam_attn",
         "transformer_classic_ext", "transformer_classic_cov", "transformer_cpg"]


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    return {k: z[k] for k in z.files if k != "meta"}, meta


def model_for(meta):
    from nanodecoder_amd import synth
    cfg = synth.ModelConfig(**meta["cfg"])
    W = synth.make_weights(cfg, seed=meta["seed"], eos_bias=meta["eos_bias"])
    return cfg, W


def chunks_of(z):
    return [z["src"][i, : z["lengths"][i]].copy() for i in range(len(z["lengths"]))]


def logp_close(a, b, atol=1e-3, rtol=1e-5):
    """|a-b| <= atol + rtol*|b| (rtol covers the -1e4-biased specials whose fp32
    ulp is ~1e-3)."""
    return np.abs(a - b) <= atol + rtol * np.abs(b)


def load_frontend():
    """tests/golden/frontend.npz (oracle/make_golden_frontend.py: the
    reference's own extract_fast5_raw / simple_assembly outputs)."""
    z = np.load(os.path.join(GOLDEN, "frontend.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    return z, meta


def frontend_chunks(z, i, si):
    """Reference chunks of read i under setting si, as float32 (the
    translator's FloatTensor of the parsed strings)."""
    flat, lens = z[f"chunks{i}_{si}"], z[f"clens{i}_{si}"]
    off = np.concatenate([[0], np.cumsum(lens)])
    return [flat[off[j]:off[j + 1]].astype(np.float32) for j in range(len(lens))]


def same_f32(a, b):
    """Bit-identical float32 arrays, NaN matching NaN (a constant read's MAD
    or std is 0: the reference divides by it)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    return bool((na == nb).all() and (a[~na].view(np.uint32) == b[~nb].view(np.uint32)).all())
