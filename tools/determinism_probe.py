"""Are translate results bit-reproducible?  Same batch through: one engine
three times; a second engine; two engines one after the other; two engines
concurrently (EnginePool lanes).  Prints the max |diff| of scores / logp
against the first call for each case."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import Engine, EnginePool  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S = 40
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
sig = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=300)).cuda()
other = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=301)).cuda()
lens = torch.full((B,), 512, dtype=torch.int32).cuda()


def run(e, x=sig):
    r = e.translate_greedy(x, lens, lens, max_len=S, min_len=5, return_logp=True)
    torch.cuda.synchronize()
    return r["scores"].cpu().numpy(), r["logp"].cpu().numpy(), r["tokens"].cpu().numpy()


def cmp(tag, a, b):
    print(f"{tag:40s} scores {np.abs(a[0] - b[0]).max():.3e} logp {np.abs(a[1] - b[1]).max():.3e} "
          f"tokens {'same' if (a[2] == b[2]).all() else 'DIFF'}", flush=True)


e1 = Engine(cfg, W, max_batch=B, max_steps=S)
ref = run(e1)
cmp("engine 1, call 2", ref, run(e1))
run(e1, other)
cmp("engine 1, after another batch", ref, run(e1))
e1.set_graphs = None
e2 = Engine(cfg, W, max_batch=B, max_steps=S)
cmp("engine 2, first call", ref, run(e2))
cmp("engine 2, call 2", ref, run(e2))
ng = Engine(cfg, W, max_batch=B, max_steps=S, graphs=False)
cmp("engine 3 (no graphs)", ref, run(ng))
pool = EnginePool(cfg, W, lanes=2, max_batch=B, max_steps=S)
for k in range(3):
    rs = [pool.translate_greedy(x, lens, lens, max_len=S, min_len=5, return_logp=True) for x in (sig, sig, sig, sig)]
    pool.synchronize()
    torch.cuda.synchronize()
    for i, r in enumerate(rs):
        cmp(f"pool round {k} call {i} (lane {r['lane']})", ref,
            (r["scores"].cpu().numpy(), r["logp"].cpu().numpy(), r["tokens"].cpu().numpy()))
for k in range(2):
    r = pool.translate_greedy(sig, lens, lens, max_len=S, min_len=5, return_logp=True)
    pool.synchronize()
    torch.cuda.synchronize()
    cmp(f"pool serial call {k} (lane {r['lane']})", ref,
        (r["scores"].cpu().numpy(), r["logp"].cpu().numpy(), r["tokens"].cpu().numpy()))

# --- isolate: graphs off in the pool; encoder alone concurrently
pool_ng = EnginePool(cfg, W, lanes=2, max_batch=B, max_steps=S, graphs=False)
for k in range(2):
    rs = [pool_ng.translate_greedy(x, lens, lens, max_len=S, min_len=5, return_logp=True) for x in (sig, sig, sig, sig)]
    pool_ng.synchronize()
    torch.cuda.synchronize()
    for i, r in enumerate(rs):
        cmp(f"pool no-graphs round {k} call {i} (lane {r['lane']})", ref,
            (r["scores"].cpu().numpy(), r["logp"].cpu().numpy(), r["tokens"].cpu().numpy()))
mem_ref = e1.encode(sig, lens, lens)
torch.cuda.synchronize()
mem_ref = mem_ref.cpu().numpy()
for k in range(3):
    outs = []
    for i, e in enumerate(pool.engines * 2):
        st = e.stream
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            outs.append(e.encode(sig, lens, lens))
    pool.synchronize()
    torch.cuda.synchronize()
    for i, m in enumerate(outs):
        print(f"encode concurrently round {k} #{i}: max|diff| {np.abs(m.cpu().numpy() - mem_ref).max():.3e}", flush=True)
