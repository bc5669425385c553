"""Probe: do independent translate chains overlap on one MI355X?
(1) one engine, B=256 greedy; (2) two engines x B=128 on two streams;
(3) four engines x B=64 on four streams; (4) B=256 greedy beside an
encoder-only call of another engine (cross-call pipelining)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import Engine  # noqa: E402

dev = torch.device("cuda", 0)
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=1, eos_bias=-3.0)


def inputs(B):
    sig = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=3)).to(dev)
    lens = torch.full((B,), 512, dtype=torch.int32, device=dev)
    return sig, lens, lens.clone()


def bench(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for parts in (1, 2, 4):
    B = 256 // parts
    engs = [Engine(cfg, W, device=0, max_batch=B, max_steps=100) for _ in range(parts)]
    strs = [torch.cuda.Stream(dev) for _ in range(parts)]
    ins = [inputs(B) for _ in range(parts)]

    def run():
        cur = torch.cuda.current_stream(dev)
        for e, s, (sig, ln, sp) in zip(engs, strs, ins):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                e.translate_greedy(sig, ln, sp, max_len=100, min_len=57)
        for s in strs:
            cur.wait_stream(s)

    ms = bench(run)
    print(f"{parts} x B={B}: {ms:.2f} ms per 256 chunks -> {256 * 512 / ms / 1e3:.3f} M samples/s", flush=True)
    for e in engs:
        e.close()

# cross-call: decoder of one call beside the encoder of the next
eA = Engine(cfg, W, device=0, max_batch=256, max_steps=100)
eB = Engine(cfg, W, device=0, max_batch=256, max_steps=100)
sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
sig, ln, sp = inputs(256)
ms_dec = bench(lambda: eA.translate_greedy(sig, ln, sp, max_len=100, min_len=57))
ms_enc = bench(lambda: eB.encode(sig, ln, sp))


def both():
    cur = torch.cuda.current_stream(dev)
    sA.wait_stream(cur)
    sB.wait_stream(cur)
    with torch.cuda.stream(sA):
        eA.translate_greedy(sig, ln, sp, max_len=100, min_len=57)
    with torch.cuda.stream(sB):
        eB.encode(sig, ln, sp)
    cur.wait_stream(sA)
    cur.wait_stream(sB)


ms_both = bench(both)
print(f"translate {ms_dec:.2f} ms, encode {ms_enc:.2f} ms, both concurrently {ms_both:.2f} ms", flush=True)
