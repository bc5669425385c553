"""Search synthetic-model knobs for realistic decode lengths (first EOS near
~55 steps, diverse bases), used by bench --mode beam.  CPU only."""
import itertools
import sys

import numpy as np

sys.path.insert(0, ".")
from nanodecoder_amd import synth  # noqa: E402
from oracle import ref_cpu  # noqa: E402

sig = synth.synth_chunk_batch(8, 512, seed=77, inject_masks=False)
lens = np.full(8, 512)
res = []
for seed, pe, eb in itertools.product([11, 21, 31, 41], [False, True], [-1.0, 0.0, 1.0, 2.0]):
    cfg = synth.ModelConfig(position_encoding=pe)
    W = synth.make_weights(cfg, seed=seed, eos_bias=eb)
    r = ref_cpu.greedy(ref_cpu.RefModel(cfg, W), sig, lens, max_length=100)
    t = r["tokens"]
    first = np.where((t == 3).any(1), (t == 3).argmax(1), 100)
    nb = [len(set(row[:f].tolist())) for row, f in zip(t, first)]
    res.append((seed, pe, eb, first.tolist(), nb))
    print(seed, pe, eb, "first EOS", first.tolist(), "distinct", nb, flush=True)
