"""Localise the co-residency disturbance of tools/rank2_probe.py: engine A
encodes repeatedly (memory bank vs a serial run) while another stream runs
ONE decoder GEMM class over and over (B_MODE: p16s24 = gemm_p16s<2,4> (N =
2048, LN), p16s22 = gemm_p16s<2,2> (N = 768, LN), longk = gemm_p16<1,8,256>
(K = 2048), small = gemm_p16<1,4,64> (N = K = 256), none).  Encoder-side
switches (ND_ENC_*) pick which encoder kernels run."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd import engine as E  # noqa: E402

dev = torch.device("cuda", 0)
B = 64
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
A = E.Engine(cfg, W, max_batch=B, max_steps=8)
side = torch.cuda.Stream()
sig = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=300)).to(dev)
lens = torch.full((B,), 512, dtype=torch.int32, device=dev)
tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("ND_")) or "defaults"
g = torch.Generator(device="cpu").manual_seed(0)


def rn(*s, sc=1.0):
    return (torch.randn(*s, generator=g) * sc).to(dev)


R = 256
Ap, Ap2k, Rp = E.pack_p16(rn(R, 256)), E.pack_p16(rn(R, 2048)), E.pack_p16(rn(R, 256))
part = E.row_partials(E.unpack_p16(Ap, R))
shapes = {"p16s24": (2048, 256, True, False), "p16s22": (768, 256, True, False),
          "longk": (256, 2048, False, True), "small": (256, 256, False, True)}
ops = {}
for name, (N, K, ln, res) in shapes.items():
    Wh, ws = E.op_pack_p16h(rn(N, K, sc=K ** -0.5))
    bias = rn(N, sc=0.1)
    po = torch.zeros(R, 16, 2, device=dev) if N == 256 else None
    ops[name] = (lambda A_=(Ap2k if K == 2048 else Ap), N=N, K=K, ln=ln, res=res, Wh=Wh, ws=ws, bias=bias, po=po:
                 E.op_gemm_p16(A_, None, bias, R, N, K, Rp=Rp if res else None, part_in=part if ln else None,
                               part_out=po, Wh=Wh, wscale=ws))
mem_ref = A.encode(sig, lens, lens)
torch.cuda.synchronize()
mem_ref = mem_ref.cpu().numpy()
for mode in os.environ.get("B_MODES", "none p16s24 p16s22 longk small").split():
    worst = 0.0
    for it in range(4):
        cur = torch.cuda.current_stream()
        A.stream.wait_stream(cur)
        side.wait_stream(cur)
        if mode != "none":
            with torch.cuda.stream(side):
                for _ in range(3000):
                    ops[mode]()
        with torch.cuda.stream(A.stream):
            mems = [A.encode(sig, lens, lens) for _ in range(8)]
        torch.cuda.synchronize()
        worst = max(worst, max(float(np.abs(m.cpu().numpy() - mem_ref).max()) for m in mems))
    print(f"[{tag}] beside {mode:7s}: A max|dmem| {worst:.3e}", flush=True)
