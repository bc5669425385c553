"""Where does an EnginePool teardown crash?  Step-by-step prints."""
import faulthandler
import gc
import os
import sys

import numpy as np
import torch

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import EnginePool  # noqa: E402

cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
B, S = 64, 40
lens = np.full(B, 512, np.int32)
dev_b = [torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=300 + k)).cuda() for k in range(4)]
pool = EnginePool(cfg, W, device=0, lanes=2, max_batch=B, max_steps=S)
print("pool made", flush=True)
got = [pool.translate_greedy(b, lens, lens, max_len=S, min_len=5, return_logp=True) for b in dev_b]
pool.synchronize()
torch.cuda.synchronize()
print("calls done", flush=True)
x = [g["tokens"].cpu() for g in got]
print("read", flush=True)
pool.close()
print("closed", flush=True)
del got
gc.collect()
print("results freed", flush=True)
del dev_b
gc.collect()
print("inputs freed", flush=True)
y = torch.empty(1 << 20, device="cuda")
torch.cuda.synchronize()
print("alloc after", flush=True)
del pool
gc.collect()
torch.cuda.empty_cache()
print("done", flush=True)
