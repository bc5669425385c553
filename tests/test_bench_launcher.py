"""bench.py's multi-GPU launcher on CPU: ``--gpus 2`` outside a launcher
starts two rank processes itself (torch.distributed.run, gloo here) and
rank 0 reports the world size it joined.  No engine, no measurement."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=240, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_n_ranks():
    out = _run(["--gpus", "2", "--selftest-cpu", "--backend", "gloo"])
    assert out["n_gpus"] == 2 and out["rank_sum"] == 1.0


def test_bench_single_rank_no_launcher():
    out = _run(["--gpus", "1", "--selftest-cpu", "--backend", "gloo"])
    assert out["n_gpus"] == 1
