"""configs[3]'s context-attention HBM traffic per alive chunk, from rocprofv3
FETCH_SIZE / WRITE_SIZE passes over exactly the bench leg's workload.

The bench's configs[3] leg (bench.py config_legs) runs --fast beam 5 on 1024
chunks (synth seed 2000, weights seed 11, eos bias -3, max_length 100,
-min_length 57).  Its roofline prices a stamped dec_ctx_q24_kernel launch at
(alive chunks that launch) x 831,488 B.  A counter pass must therefore see the
same calls and nothing else (no return_attn dump, no forced-100-step calls),
and its bytes must be divided by the same alive-chunk launches.

    python tools/pmc_beam.py alive OUT.json        # unprofiled: steps each chunk ran -> alive per step
    python tools/pmc_beam.py run K                 # profiled: 1 + K plain calls of the workload
    python tools/pmc_beam.py summary ALIVE.json K FETCH.csv WRITE.csv OUT.json

Bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KiB; gfx950 FETCH_SIZE
half-count correction, MI355X_MICROARCH.md), summed over every dispatch of a
kernel in the run, divided by (1 + K) x layers x sum(alive).
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

B, BEAM, S, MINL, T, LAYERS = 1024, 5, 100, 57, 512, 3
PER_CHUNK = T * 1600 + T * 4 + 2 * BEAM * 256 * 4   # 24-bit K/V image + signal + q in / ctx out (bench.py)


def _workload():
    import numpy as np
    from nanodecoder_amd import synth
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    sig = synth.synth_chunk_batch(B, T, seed=2000, inject_masks=False)
    return cfg, W, sig, np.full(B, T, np.int32)


def alive(out):
    import torch
    from nanodecoder_amd.engine import Engine
    cfg, W, sig, lens = _workload()
    eng = Engine(cfg, W, device=0, max_batch=B, max_steps=S, max_beam=BEAM)
    r = eng.translate_beam(sig, lens, lens, beam=BEAM, max_len=S, min_len=MINL, return_attn=True)
    torch.cuda.synchronize()
    done = r["done_step"].cpu().numpy()
    steps = int(r["steps"].cpu()[0])
    al = [int((done > s).sum()) for s in range(steps)]
    json.dump({"alive": al, "steps": steps, "sum_alive": sum(al)}, open(out, "w"))
    print(json.dumps({"steps": steps, "sum_alive": sum(al)}))
    eng.close()


def run(k):
    import torch
    from nanodecoder_amd.engine import Engine
    cfg, W, sig, lens = _workload()
    eng = Engine(cfg, W, device=0, max_batch=B, max_steps=S, max_beam=BEAM)
    sd, ld = torch.from_numpy(sig).cuda(), torch.from_numpy(lens).cuda()
    for _ in range(1 + k):
        r = eng.translate_beam(sd, ld, ld, beam=BEAM, max_len=S, min_len=MINL)
    torch.cuda.synchronize()
    print("steps", int(r["steps"].cpu()[0]))
    eng.close()


def _short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("nd::", "")


def _sums(path, counter):
    tot, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name", r.get("Counter-Name")) != counter:
            continue
        k = _short(r.get("Kernel_Name", r.get("Kernel-Name", "")))
        tot[k] += float(r.get("Counter_Value", r.get("Counter-Value")))
        n[k] += 1
    return tot, n


def summary(alive_json, k, fetch_csv, write_csv, out):
    a = json.load(open(alive_json))
    calls = 1 + int(k)
    f, nf = _sums(fetch_csv, "FETCH_SIZE")
    w, _ = _sums(write_csv, "WRITE_SIZE")
    chunk_launches = calls * LAYERS * a["sum_alive"]
    rows = {}
    for name in sorted(set(f) | set(w)):
        if not (name.startswith("dec_ctx") or name.startswith("ctx_split") or name.startswith("dec_self_attention")):
            continue
        byt = 2 * f.get(name, 0.0) * 1024 + w.get(name, 0.0) * 1024
        rows[name] = {"launches": nf[name], "launches_per_call": nf[name] / calls, "hbm_bytes": int(byt),
                      "hbm_bytes_per_alive_chunk_launch": round(byt / chunk_launches, 1)}
    ctx = [v for n, v in rows.items() if n.startswith("dec_ctx") or n.startswith("ctx_split")]
    per = sum(v["hbm_bytes"] for v in ctx) / chunk_launches
    res = {"workload": "configs[3]: --fast beam 5, B 1024 (synth seed 2000), weights seed 11, eos bias -3, "
                       "max_length 100, -min_length 57 (bench.py config_legs), one engine, 1 + K plain calls",
           "calls": calls, "steps": a["steps"], "sum_alive_per_call": a["sum_alive"],
           "alive_chunk_launches": chunk_launches,
           "ctx_attention": {"traffic_per_alive_chunk_launch": round(per, 1),
                             "algorithmic_per_alive_chunk_launch": PER_CHUNK,
                             "ratio": round(per / PER_CHUNK, 4),
                             "kernels": [n for n in rows if n.startswith("dec_ctx") or n.startswith("ctx_split")]},
           "kernels": rows,
           "note": "bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB, gfx950 FETCH_SIZE half-count correction), summed "
                   "over every dispatch; per alive chunk-launch = / (calls x 3 layers x sum over steps of the "
                   "chunks alive)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["ctx_attention"]))


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "alive":
        alive(sys.argv[2])
    elif cmd == "run":
        run(int(sys.argv[2]))
    elif cmd == "summary":
        summary(*sys.argv[2:7])
    else:
        raise SystemExit(__doc__)
