"""Diagnostic (not part of the engine): --fast beam 5 at B = 1024 on the digit bank — is a call's output a
function of its inputs alone?  (1) one context, the same ragged batch before and after another batch;
(2) two contexts, one at a time; (3) two contexts at once on two streams.   python tools/bb_pool_debug.py"""
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, "tests")
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import Engine  # noqa: E402
from tests.test_gpu_configs import _ragged  # noqa: E402


def main():
    B, S, MINL = 1024, 100, 57
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    s0 = synth.synth_chunk_batch(B, 512, seed=500, inject_masks=False)
    i0 = (s0, np.full(B, 512, np.int32), np.full(B, 512, np.int32))
    i1 = _ragged(synth.synth_chunk_batch(B, 512, seed=501, inject_masks=False), 901)
    dev = [tuple(torch.from_numpy(a).cuda() for a in i) for i in (i0, i1)]

    def mk():
        return Engine(cfg, W, device=0, max_batch=B, max_steps=S, max_beam=5)

    def call(e, inp):
        r = e.translate_beam(*inp, beam=5, n_best=1, max_len=S, min_len=MINL)
        return {k: r[k].cpu() for k in ("tokens", "scores", "lens", "steps")}

    def same(a, b):
        return all(torch.equal(a[k], b[k]) for k in a)

    inputs = []
    for k in range(6):
        sg = synth.synth_chunk_batch(B, 512, seed=500 + k, inject_masks=False)
        inputs.append(_ragged(sg, 900 + k) if k % 2 else (sg, np.full(B, 512, np.int32), np.full(B, 512, np.int32)))
    dv = [tuple(torch.from_numpy(x).cuda() for x in i) for i in inputs]
    # history: batch 3 after 0,1,2 / after 0 / first
    res = {}
    for name, seq in (("0123", [0, 1, 2, 3]), ("3", [3]), ("3 3", [3, 3]), ("3 3 3", [3, 3, 3]), ("2 3", [2, 3]),
                      ("5 3", [5, 3]), ("4 3", [4, 3])):
        e = mk()
        for k in seq:
            r = call(e, dv[k])
        res[name] = r
        e.close()
        ok = same(r, res["0123"])
        ds = (r["scores"] - res["0123"]["scores"]).abs().reshape(-1)
        print(f"batch 3 after {name}: {'same' if ok else 'DIFF'} (scores differ at {torch.nonzero(ds).reshape(-1)[:8].tolist()}) "
              f"steps {int(r['steps'])}", flush=True)
    for k in range(6):
        e = mk()
        r = call(e, dv[k])
        e.close()
        print(f"batch {k} alone: steps {int(r['steps'])}", flush=True)
    # (4) the pool test's pattern: 3 lanes (bank policy / grid as EnginePool sets them), six batches
    from nanodecoder_amd.engine import EnginePool
    one = mk()
    exp = [call(one, i) for i in dv]
    one.close()
    pool = EnginePool(cfg, W, device=0, lanes=3, max_batch=B, max_steps=S, max_beam=5)
    for rnd in range(2):
        got = [None] * 6

        def plane(i):
            e = pool.engines[i]
            with torch.cuda.stream(e.stream):
                for k in range(i, 6, 3):
                    got[k] = call(e, dv[k])
        cur = torch.cuda.current_stream()
        for e in pool.engines:
            e.stream.wait_stream(cur)
        th = [threading.Thread(target=plane, args=(i,)) for i in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        for k in range(6):
            ok = same(got[k], exp[k])
            msg = ""
            if not ok:
                d = (got[k]["tokens"] != exp[k]["tokens"]).any(-1).any(-1)
                msg = f" chunks {int(d.sum())} {np.nonzero(d.numpy())[0][:12]}; " + ", ".join(
                    f"{n} {'ok' if torch.equal(got[k][n], exp[k][n]) else 'DIFF'}" for n in got[k])
                ds = (got[k]["scores"] - exp[k]["scores"]).abs().reshape(-1)
                idx = torch.nonzero(ds).reshape(-1)
                msg += f"; scores differ at {idx[:10].tolist()} max {float(ds.max()):.3e}"
                dl = torch.nonzero((got[k]["lens"] != exp[k]["lens"]).reshape(-1)).reshape(-1)
                msg += f"; lens differ at {dl[:10].tolist()}"
            print(f"pool round {rnd} batch {k} lane {k % 3}: {ok}{msg}", flush=True)
    pool.close()


if __name__ == "__main__":
    main()
