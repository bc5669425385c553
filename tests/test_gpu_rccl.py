"""The multi-GPU read-shard path on RCCL, at world 1 on the one-GPU box
(needs an MI355X).

The world-2/4/8 tests (tests/test_shard_gloo.py) run the sharding logic on
gloo with a stand-in engine.  Here the production path runs once for real:
a fresh child process (started before it touches the GPU) initialises the
process group with backend "nccl" (RCCL on ROCm) at world 1, and
shard.run_distributed runs on a 3-lane EnginePool: the weight blob broadcast
from HIP memory over RCCL, the read shard through the device front end, the
flag exchange, counter all_reduce and MAX over the CPU gloo group.  Its
outputs and counters must equal a plain ReadShard run of the same reads in
the same process without any process group.  Reference:
onmt/utils/distributed.py:20-32 (the rendezvous), pipeline.evaluate.sh:111-115
(one process per GPU).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _child_main():
    import types

    import numpy as np
    import torch
    import torch.distributed as dist

    from nanodecoder_amd import shard, synth
    from nanodecoder_amd.engine import EnginePool
    from nanodecoder_amd.translator import Translator

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = synth.ModelConfig()
    W0 = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    seen = {}

    def factory(W):
        seen["W"] = W
        opt = types.SimpleNamespace(gpu=0, n_best=1, max_length=60, min_length=10, beam_size=1, batch_size=100,
                                    engine_max_batch=64)
        pool = EnginePool(cfg, W, device=0, lanes=3, max_batch=64, max_steps=60)
        seen.setdefault("pools", []).append(pool)
        return Translator(cfg, W, opt, engine=pool)

    n = 300
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    g, preds = shard.run_distributed(n, factory, lambda: W0, dev, batch_size=100, keep_predictions=True,
                                     warmup_reads=8)
    # the blob came back through the RCCL broadcast from HIP memory: identical to rank 0's weights
    same_w = sorted(seen["W"]) == sorted(W0) and all(np.array_equal(seen["W"][k], W0[k]) for k in W0)
    dist.destroy_process_group()
    lengths = shard.read_lengths(n)
    tr = factory(W0)
    single, preds1 = shard.ReadShard(tr, batch_size=100).run(list(range(n)), lengths, keep_predictions=True)
    for p in seen["pools"]:
        p.close()
    out = dict(world=g["world"], retried=g["retried"], failed=g["failed_ranks"], same_weights=same_w,
               counts_equal=all(g[k] == single[k] for k in ("samples", "bases", "chunks")),
               preds_equal=preds == preds1, reads=len(preds), samples=g["samples"], bases=g["bases"],
               seconds=g["seconds"])
    print("RCCL_RESULT " + json.dumps(out), flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_read_shard_on_rccl_world1_matches_plain_run():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", "from tests.test_gpu_rccl import _child_main; _child_main()"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("RCCL_RESULT ")]
    assert line, r.stdout[-3000:]
    out = json.loads(line[-1][len("RCCL_RESULT "):])
    print("\n[rccl]", out)
    assert out["world"] == 1 and out["retried"] == 0 and out["failed"] == []
    assert out["same_weights"] and out["counts_equal"] and out["preds_equal"], out
    assert out["reads"] == 300 and out["bases"] > 0
