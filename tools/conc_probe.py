"""Which part of a translate call is disturbed by a concurrent call on
another engine context/stream?  Lane 0 translates a batch while lane 1 runs
something else; lane 0's outputs are compared with a serial run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import Engine  # noqa: E402

B, S = 64, 40
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
sig = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=300)).cuda()
sig2 = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=301)).cuda()
lens = torch.full((B,), 512, dtype=torch.int32).cuda()
A = Engine(cfg, W, max_batch=B, max_steps=S)
Bn = Engine(cfg, W, max_batch=B, max_steps=S)


def res(r):
    return r["logp"].cpu().numpy()


def greedy(e, x):
    return e.translate_greedy(x, lens, lens, max_len=S, min_len=5, return_logp=True)


def conc(setup, other, tag, n=4):
    setup()
    ref = res(greedy(A, sig))
    torch.cuda.synchronize()
    worst, first = 0.0, None
    for _ in range(n):
        cur = torch.cuda.current_stream()
        A.stream.wait_stream(cur)
        Bn.stream.wait_stream(cur)
        with torch.cuda.stream(A.stream):
            ra = greedy(A, sig)
        with torch.cuda.stream(Bn.stream):
            other()
        torch.cuda.synchronize()
        d = np.abs(res(ra) - ref)
        worst = max(worst, float(d.max()))
        if d.max() > 1e-5 and first is None:
            bad = np.argwhere(d > 1e-5)
            first = tuple(int(v) for v in bad[np.argmin(bad[:, 1])])
    print(f"{tag:50s} max|dlogp| {worst:.3e}  first bad (row, step, tok) {first}", flush=True)


def reset():
    for e in (A, Bn):
        e.set_exact_fp32(False)
        e.set_ctx_path(0)


tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("ND_"))
conc(reset, lambda: greedy(Bn, sig2), f"other: greedy  [{tag}]")
conc(reset, lambda: Bn.encode(sig2, lens, lens), f"other: encode  [{tag}]")
if len(sys.argv) > 1:
    sys.exit(0)
conc(lambda: (A.set_ctx_path(1), Bn.set_ctx_path(1)), lambda: greedy(Bn, sig2), "both ctx_path 1 (K/V form)")
conc(lambda: (A.set_exact_fp32(True), Bn.set_exact_fp32(True)), lambda: greedy(Bn, sig2), "both exact fp32")
conc(lambda: (reset(), Bn.set_exact_fp32(True)), lambda: greedy(Bn, sig2), "A split, other exact")
conc(lambda: (reset(), A.set_exact_fp32(True)), lambda: greedy(Bn, sig2), "A exact, other split")
