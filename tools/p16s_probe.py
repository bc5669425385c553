"""gemm_p16s_kernel<2,2> beside LDS spinners: which variants differ, where,
and do the spinners see foreign LDS writes?"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd import engine as E  # noqa: E402
from nanodecoder_amd import _lib  # noqa: E402

can = ctypes.CDLL(os.path.join(ROOT, "tools", "liblds_canary.so"))
can.lds_canary.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
A = E.Engine(cfg, W, max_batch=8, max_steps=8)
Bn = E.Engine(cfg, W, max_batch=8, max_steps=8)
g = torch.Generator(device="cpu").manual_seed(0)
R = 256
X = torch.randn(R, 256, generator=g).to(dev)
Ap = E.pack_p16(X)
part = E.row_partials(X)
err = torch.zeros(1, dtype=torch.int32, device=dev)
for N in (768, 2048):
    Wf = (torch.randn(N, 256, generator=g) / 16).to(dev)
    Wh, ws = E.op_pack_p16h(Wf)
    for h3 in (True, False):
        for ln in (True, False):
            def f():
                C, _ = E.op_gemm_p16(Ap, Wf if not h3 else None, None, R, N, 256, part_in=part if ln else None,
                                     Wh=Wh if h3 else None, wscale=ws)
                return E.unpack_p16(C, R)
            _lib.gemm_routes(reset=True)
            ref = f().clone()
            route = [k for k, v in _lib.gemm_routes(reset=True).items() if v]
            torch.cuda.synchronize()
            for lds_kb in (16, 64):
                err.zero_()
                cur = torch.cuda.current_stream()
                A.stream.wait_stream(cur)
                Bn.stream.wait_stream(cur)
                outs = []
                with torch.cuda.stream(Bn.stream):
                    for _ in range(40):
                        can.lds_canary(err.data_ptr(), 1024, lds_kb * 1024, 20, Bn.stream.cuda_stream)
                with torch.cuda.stream(A.stream):
                    for _ in range(40):
                        outs.append(f())
                torch.cuda.synchronize()
                bad = torch.zeros(R // 16, N // 16, dtype=torch.int64, device=dev)
                worst = 0.0
                for o in outs:
                    d = (o - ref).abs()
                    worst = max(worst, float(d.max().item()))
                    bad += (d.view(R // 16, 16, N // 16, 16) > 0).any(3).any(1).long()
                nz = bad.nonzero()
                print(f"N{N} h3={int(h3)} ln={int(ln)} {route} spinners {lds_kb}KB: max|diff| {worst:.3e}, "
                      f"16x16 blocks ever wrong {nz.shape[0]} (first {nz[:6].tolist()}), canary foreign words "
                      f"{int(err.item())}", flush=True)
