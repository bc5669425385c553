"""Is a translate call disturbed by unrelated work on another queue?  Lane B
runs LDS-canary spinners (no global writes but one error word); lane A
translates; A's outputs vs a serial run."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd import engine as E  # noqa: E402

can = ctypes.CDLL(os.path.join(ROOT, "tools", "liblds_canary.so"))
can.lds_canary.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
B, S = 64, 40
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
A = E.Engine(cfg, W, max_batch=B, max_steps=S)
Bn = E.Engine(cfg, W, max_batch=8, max_steps=8)
sig = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=300)).to(dev)
lens = torch.full((B,), 512, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
ref = A.translate_greedy(sig, lens, lens, max_len=S, min_len=5, return_logp=True)["logp"].cpu().numpy()
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("ND_"))
for wgs, lds_kb, us in ((256, 4, 50), (1024, 4, 20), (2048, 16, 20), (512, 64, 30)):
    worst = 0.0
    for it in range(4):
        cur = torch.cuda.current_stream()
        A.stream.wait_stream(cur)
        Bn.stream.wait_stream(cur)
        with torch.cuda.stream(Bn.stream):
            for _ in range(100):
                can.lds_canary(err.data_ptr(), wgs, lds_kb * 1024, us, Bn.stream.cuda_stream)
        with torch.cuda.stream(A.stream):
            r = A.translate_greedy(sig, lens, lens, max_len=S, min_len=5, return_logp=True)
        torch.cuda.synchronize()
        worst = max(worst, float(np.abs(r["logp"].cpu().numpy() - ref).max()))
    print(f"[{tag}] spinners {wgs} WG x {lds_kb} KB x {us} us: A max|dlogp| {worst:.3e}", flush=True)
