"""Golden vectors for the front end and the output assembly, from the
REFERENCE's own ``utils/labelop.py`` (this container only).

Test infrastructure.  Runs the reference's ``extract_fast5_raw`` (.signal
branch, utils/labelop.py:194-243) and ``simple_assembly`` / ``index2base``
(:295-352) and writes ``tests/golden/frontend.npz``: the raw reads, the
chunks the reference cuts from them (its ``str(x)`` strings parsed back to
float64, exact: Python's float repr round-trips) for each normalisation and
window setting, and the consensus matrices / base strings of overlap
assembly cases.

labelop.py imports two modules this image lacks, neither on these paths:
  * ``h5py`` -- only the fast5 branch opens files with it: a bare stub module.
  * ``statsmodels.robust`` -- only ``robust.mad`` is called (the 'median'
    normalisation, :223).  The stub restates statsmodels' published
    ``statsmodels.robust.scale.mad`` (statsmodels 0.9 - 0.14, unpinned in
    requirements.txt): ``np.median(np.abs(a - center(a)) / c)`` with
    ``c = scipy.stats.norm.ppf(0.75) = 0.6744897501960817``, ``center =
    np.median``, axis 0.
and it calls ``np.float`` (removed in numpy 1.24) and ``np.lib.pad`` (removed
in numpy 2.0): shimmed as ``float`` and ``np.pad``, the aliases they were.

Regenerate with:  ``python oracle/make_golden_frontend.py``  (needs
/root/reference).  The reference never travels to the GPU box; only the
fixture (data) does.
"""
from __future__ import annotations

import importlib.util
import json
import os
import random
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from nanodecoder_amd import synth  # noqa: E402
from oracle._refimport import REF  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "frontend.npz")
MAD_C = 0.6744897501960817

# (normalization, max_length, stride): the README/bench setting and the
# authors' production overlap setting (pipeline.evaluate.sh:83-85)
SETTINGS = [("median", 512, 512), ("mean", 512, 512), ("None", 512, 512), ("median", 300, 60)]


def load_labelop():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("h5py", types.ModuleType("h5py"))
    sm = types.ModuleType("statsmodels")
    robust = types.ModuleType("statsmodels.robust")

    def mad(a, c=MAD_C, axis=0, center=np.median):
        a = np.asarray(a)
        ctr = np.apply_over_axes(center, a, axis) if a.size else 0.0
        return np.median(np.abs(a - ctr) / c, axis=axis)

    robust.mad = mad
    sm.robust = robust
    sys.modules["statsmodels"] = sm
    sys.modules["statsmodels.robust"] = robust
    if not hasattr(np, "float"):
        np.float = float  # the alias labelop.py:221-223 was written against
    if not hasattr(np.lib, "pad"):
        np.lib.pad = np.pad  # labelop.py:341
    spec = importlib.util.spec_from_file_location("ref_labelop", os.path.join(REF, "utils", "labelop.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def reads():
    """Raw traces as the .signal files hold them: DAC-like integer reads of
    several lengths (odd / even / one chunk +- 1 / many chunks) and a few odd
    cases (1-3 samples, real-valued, heavy ties)."""
    rng = np.random.default_rng(2024)
    rs = [synth.synth_raw_read(i, n) for i, n in enumerate((1300, 700, 512, 513, 511, 4099, 2049))]
    rs += [np.array([5.0]), np.array([3.0, 9.0]), np.array([1.0, 1.0, 2.0]),
           np.round(rng.normal(size=1001) * 50 - 20, 3), rng.integers(-100, 100, size=2048).astype(np.float64)]
    return rs


def _fmt(v):
    return str(int(v)) if float(v).is_integer() else repr(float(v))


def assembly_cases():
    """Predictions of overlapping windows of one base sequence (length 300 /
    stride 60 samples is ~34 bases every ~7), with substitutions, dropped and
    inserted bases and empty predictions; one long read crosses the 1000-
    column consensus growth (:334-337)."""
    rnd = random.Random(7)
    cases = []
    for n_bases, win, step, noise in ((120, 34, 7, 0.0), (200, 34, 7, 0.05), (600, 57, 12, 0.08),
                                      (1600, 57, 40, 0.03), (60, 20, 20, 0.0), (90, 30, 5, 0.2)):
        seq = "".join(rnd.choice("ACGT") for _ in range(n_bases))
        preds = []
        for s in range(0, n_bases, step):
            w = list(seq[s:s + win])
            out = []
            for b in w:
                u = rnd.random()
                if u < noise / 3:
                    continue                      # dropped base
                if u < 2 * noise / 3:
                    out.append(rnd.choice("ACGT"))  # substitution
                    continue
                out.append(b)
                if u > 1 - noise / 3:
                    out.append(rnd.choice("ACGT"))  # inserted base
            preds.append(" ".join(out))
        if len(preds) > 3:
            preds[2] = ""                         # a chunk that decoded to nothing
        cases.append(preds)
    return cases


def main():
    lab = load_labelop()
    rs = reads()
    arrays, meta = {}, {"settings": SETTINGS, "reads": len(rs), "assembly": []}
    with tempfile.TemporaryDirectory() as d:
        for i, r in enumerate(rs):
            arrays[f"raw{i}"] = r
            path = os.path.join(d, f"read{i}.signal")
            with open(path, "w") as f:
                f.write(" ".join(_fmt(v) for v in r))
            for si, (norm, ml, st) in enumerate(SETTINGS):
                out = lab.extract_fast5_raw(path, f"read{i}.txt", norm, ml, st, "signal")
                assert out[0] == f"read{i}.txt"
                chunks = [np.array([float(x) for x in c.split()], np.float64) for c in out[1:]]
                arrays[f"chunks{i}_{si}"] = np.concatenate(chunks)
                arrays[f"clens{i}_{si}"] = np.array([len(c) for c in chunks], np.int64)
    for j, preds in enumerate(assembly_cases()):
        bp = [[p] for p in preds]
        cons = lab.simple_assembly(bp)
        arrays[f"asm_preds{j}"] = np.array(preds)
        arrays[f"asm_cons{j}"] = cons
        arrays[f"asm_seq{j}"] = np.array(lab.index2base(np.argmax(cons, axis=0)))
        arrays[f"asm_concat{j}"] = np.array(lab.simple_assembly(bp, flag_intersection=False))
        meta["assembly"].append(len(preds))
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT}: {len(rs)} reads x {len(SETTINGS)} settings, {len(meta['assembly'])} assembly cases, "
          f"{os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
