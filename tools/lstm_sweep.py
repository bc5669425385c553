"""BiLSTM layer time against the number of workgroups (diagnostic).

The recurrence's per-step work in one workgroup is a 16 x 512 x 128 product
(split-fp16: 3 x 48 MFMAs per wave) whatever the number of sequences it
holds (rows past them are padding), so if a layer's time stays flat as the
batch (and so the number of workgroups, B / 4 x 2 directions) grows, the
per-step latency of ONE workgroup is the bound and spreading 256 sequences
over more workgroups cannot shorten it.  Times one layer (layer-1 form) at
B = 32 .. 1024 (16 .. 512 workgroups); run once per ND_LSTM_SEQ value.
    python tools/lstm_sweep.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd.engine import op_lstm_layer  # noqa: E402

dev = torch.device("cuda", 0)
T = 512
g = torch.Generator(device="cpu").manual_seed(3)
whh = ((torch.rand(2, 512, 128, generator=g) - 0.5) * 0.2).to(dev)
ns = int(os.environ.get("ND_LSTM_SEQ", "4"))
for B in (32, 64, 128, 256, 512, 1024):
    xp = torch.randn(B * T, 1024, generator=g).to(dev)
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    out = torch.zeros(B * T, 256, device=dev)
    for _ in range(2):
        op_lstm_layer(whh, lens, T, xp=xp, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 5
    for _ in range(n):
        op_lstm_layer(whh, lens, T, xp=xp, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    wgs = 2 * ((B + ns - 1) // ns)
    print(f"NS={ns} B={B:5d} workgroups={wgs:4d}: {ms:.3f} ms per layer = {ms * 1e3 / T:.2f} us per step", flush=True)
    del xp, out
