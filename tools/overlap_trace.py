"""Concurrency probe: does one process overlap independent translate chains?

  python tools/overlap_trace.py --mode one    --B 256           one engine, B chunks
  python tools/overlap_trace.py --mode serial --B 256 --parts 2 parts engines of B/parts, one after another
  python tools/overlap_trace.py --mode conc   --B 256 --parts 2 parts engines of B/parts, concurrently

Every engine owns its HIP stream (nd_create); ``conc`` enqueues all parts
before waiting, so their graphs are in flight together.  Prints ms per B
chunks.  Run under ``rocprofv3 --kernel-trace`` and read the CSV with
tools/overlap_analyze.py to see which queue each kernel ran on and how much
kernel time overlapped across queues.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="conc", choices=["one", "serial", "conc", "ext"])
ap.add_argument("--B", type=int, default=256)
ap.add_argument("--parts", type=int, default=2)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--graphs", type=int, default=1)
ap.add_argument("--encoder", default="transformer")
a = ap.parse_args()

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
cfg = synth.ModelConfig(encoder_type=a.encoder)
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
parts = 1 if a.mode == "one" else a.parts
Bp = a.B // parts
engs = [Engine(cfg, W, device=0, max_batch=Bp, max_steps=100, graphs=bool(a.graphs)) for _ in range(parts)]
ins = []
for i in range(parts):
    sig = torch.from_numpy(synth.synth_chunk_batch(Bp, 512, seed=3 + i, inject_masks=False)).to(dev)
    lens = torch.full((Bp,), 512, dtype=torch.int32, device=dev)
    ins.append((sig, lens))
# one torch stream per part, so each call's input/output joins are per part
strs = [torch.cuda.Stream(dev) for _ in range(parts)]
# ext: every part enqueued on its engine's own stream (nd_stream: a dedicated
# hardware queue), so no caller stream joins the parts
ext = [torch.cuda.ExternalStream(e._L.nd_stream(e._h), device=dev) for e in engs]


def run():
    cur = torch.cuda.current_stream(dev)
    if a.mode == "ext":
        for e, s, (sig, ln) in zip(engs, ext, ins):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                e.translate_greedy(sig, ln, ln, max_len=100, min_len=57)
        for s in ext:
            cur.wait_stream(s)
        return
    if a.mode == "serial":
        for e, (sig, ln) in zip(engs, ins):
            e.translate_greedy(sig, ln, ln, max_len=100, min_len=57)
        return
    for e, s, (sig, ln) in zip(engs, strs, ins):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            e.translate_greedy(sig, ln, ln, max_len=100, min_len=57)
    for s in strs:
        cur.wait_stream(s)


for _ in range(a.warmup):
    run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.iters):
    run()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / a.iters * 1e3
print(f"mode={a.mode} parts={parts} B={a.B} graphs={a.graphs}: {ms:.2f} ms per {a.B} chunks -> "
      f"{a.B * 512 / ms / 1e3:.3f} M samples/s", flush=True)
for e in engs:
    e.close()
