"""Which side is disturbed when one engine's encoder (layer 0 in closed form,
enc_attention_rank2_kernel) runs beside another engine's decoder on another
queue?  Engine A encodes repeatedly (its memory bank compared with a serial
run), engine B translates repeatedly (its logp compared with a serial run),
both at once; then A's encoder beside LDS-canary spinners (canary error word
and A's memory bank)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd import engine as E  # noqa: E402

dev = torch.device("cuda", 0)
B, S = 64, 40
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
A = E.Engine(cfg, W, max_batch=B, max_steps=S)
Bn = E.Engine(cfg, W, max_batch=B, max_steps=S)
sig = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=300)).to(dev)
sig2 = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=301)).to(dev)
lens = torch.full((B,), 512, dtype=torch.int32, device=dev)
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("ND_")) or "defaults"

mem_ref = A.encode(sig, lens, lens)
torch.cuda.synchronize()
mem_ref = mem_ref.cpu().numpy()
tr_ref = Bn.translate_greedy(sig2, lens, lens, max_len=S, min_len=5, return_logp=True)["logp"].cpu().numpy()
enc_only_ref = Bn.encode(sig2, lens, lens).cpu().numpy()


def both(n_enc, n_tr):
    cur = torch.cuda.current_stream()
    A.stream.wait_stream(cur)
    Bn.stream.wait_stream(cur)
    with torch.cuda.stream(Bn.stream):
        trs = [Bn.translate_greedy(sig2, lens, lens, max_len=S, min_len=5, return_logp=True) for _ in range(n_tr)]
    with torch.cuda.stream(A.stream):
        mems = [A.encode(sig, lens, lens) for _ in range(n_enc)]
    torch.cuda.synchronize()
    dm = 0.0
    for m in mems:
        d = np.abs(m.cpu().numpy() - mem_ref)
        dm = max(dm, float(d.max()))
        if d.max() > 0 and os.environ.get("PROBE_WHERE"):
            bad = d > 1e-6  # [B, T, d]
            ch = np.nonzero(bad.any(axis=(1, 2)))[0]
            c0 = ch[0]
            rows = np.nonzero(bad[c0].any(axis=1))[0]
            cols = np.nonzero(bad[c0].any(axis=0))[0]
            print(f"    bad chunks {ch.tolist()[:16]} ({ch.size}); chunk {c0}: {rows.size} rows "
                  f"[{rows.min()}..{rows.max()}], {cols.size} cols [{cols.min()}..{cols.max()}]; "
                  f"bad fraction {bad.mean():.4f}", flush=True)
    dt = max(float(np.abs(r["logp"].cpu().numpy() - tr_ref).max()) for r in trs)
    return dm, dt


ROUNDS = int(os.environ.get("PROBE_ROUNDS", "6"))
for it in range(ROUNDS):
    dm, dt = both(12, 3)
    print(f"[{tag}] round {it}: A encode (victim?) max|dmem| {dm:.3e}   B translate max|dlogp| {dt:.3e}", flush=True)

if os.environ.get("PROBE_SHORT"):
    sys.exit(0)
# B encodes only beside A encodes only (the case the determinism probe found clean)
for it in range(2):
    cur = torch.cuda.current_stream()
    A.stream.wait_stream(cur)
    Bn.stream.wait_stream(cur)
    with torch.cuda.stream(Bn.stream):
        eb = [Bn.encode(sig2, lens, lens) for _ in range(6)]
    with torch.cuda.stream(A.stream):
        ea = [A.encode(sig, lens, lens) for _ in range(6)]
    torch.cuda.synchronize()
    print(f"[{tag}] enc|enc {it}: A {max(float(np.abs(m.cpu().numpy() - mem_ref).max()) for m in ea):.3e} "
          f"B {max(float(np.abs(m.cpu().numpy() - enc_only_ref).max()) for m in eb):.3e}", flush=True)

lib = os.path.join(ROOT, "tools", "liblds_canary.so")
if os.path.exists(lib):
    can = ctypes.CDLL(lib)
    can.lds_canary.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    for wgs, lds_kb, us in ((1024, 4, 20), (2048, 16, 20), (512, 64, 30), (256, 100, 40)):
        err = torch.zeros(2, dtype=torch.int32, device=dev)
        err[1] = 0x7fffffff
        cur = torch.cuda.current_stream()
        A.stream.wait_stream(cur)
        Bn.stream.wait_stream(cur)
        with torch.cuda.stream(Bn.stream):
            for _ in range(100):
                can.lds_canary(err.data_ptr(), wgs, lds_kb * 1024, us, Bn.stream.cuda_stream)
        with torch.cuda.stream(A.stream):
            mems = [A.encode(sig, lens, lens) for _ in range(12)]
        torch.cuda.synchronize()
        dm = max(float(np.abs(m.cpu().numpy() - mem_ref).max()) for m in mems)
        e = err.cpu().numpy()
        print(f"[{tag}] spinners {wgs} WG x {lds_kb} KB: canary errors {e[0]} (first word {e[1]}), "
              f"A max|dmem| {dm:.3e}", flush=True)
