"""When do the chunks of the configs[3] beam workload finish?

Runs --fast beam 5 on B chunks of synthetic signal with the bench's model
(random-init weights, min_length 57, EOS bias -3) and prints the distribution
of the decoder steps each chunk ran (done_step: the reference drops a chunk's
batch from the decode loop at that step, translate/translator.py:793-823)
and the share of chunk-steps a decoder that keeps every chunk to the last
one's finish spends on finished chunks.
Usage: python tools/beam_finish_probe.py [B] [min_length] [eos_bias]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import Engine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
min_len = int(sys.argv[2]) if len(sys.argv) > 2 else 57
eos_bias = float(sys.argv[3]) if len(sys.argv) > 3 else -3.0
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=eos_bias)
eng = Engine(cfg, W, device=0, max_batch=B, max_src_len=512, max_steps=100, max_beam=5)
sig = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=1000, inject_masks=False)).cuda()
lens = torch.full((B,), 512, dtype=torch.int32, device="cuda")
r = eng.translate_beam(sig, lens, lens, beam=5, n_best=1, max_len=100, min_len=min_len, return_attn=True)
torch.cuda.synchronize()
done = r["done_step"].cpu().numpy()
steps = int(r["steps"].cpu()[0])
q = np.percentile(done, [0, 10, 50, 90, 99, 100])
print(json.dumps({"B": B, "min_length": min_len, "eos_bias": eos_bias, "steps_executed": steps,
                  "done_step_percentiles_0_10_50_90_99_100": q.tolist(), "mean": float(done.mean()),
                  "alive_chunk_steps_share": float(done.sum() / (B * steps)),
                  "histogram_by_10": np.histogram(done, bins=range(0, 111, 10))[0].tolist()}))
