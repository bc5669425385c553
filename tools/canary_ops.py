"""Which kernel returns different results when LDS-holding spinner
workgroups (tools/lds_canary.hip) run beside it on another queue?  Each op is
run alone (reference), then repeatedly beside spinners; max |diff| printed."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd import engine as E  # noqa: E402

can = ctypes.CDLL(os.path.join(ROOT, "tools", "liblds_canary.so"))
can.lds_canary.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
A = E.Engine(cfg, W, max_batch=8, max_steps=8)
Bn = E.Engine(cfg, W, max_batch=8, max_steps=8)
g = torch.Generator(device="cpu").manual_seed(0)


def rn(*s, sc=1.0):
    return (torch.randn(*s, generator=g) * sc).to(dev)


ones, zeros = torch.ones(256, device=dev), torch.zeros(256, device=dev)
R = 256
Ap = E.pack_p16(rn(R, 256))
Ap2k = E.pack_p16(rn(R, 2048))
Rp = E.pack_p16(rn(R, 256))
part = E.row_partials(E.unpack_p16(Ap, R))
ops = {}
for N, K, ln, relu, res, stats in ((256, 256, False, False, True, True), (2048, 256, True, False, False, False),
                                   (768, 256, True, False, False, False), (2048, 256, True, True, False, False),
                                   (256, 2048, False, False, True, True)):
    Wf = rn(N, K, sc=K ** -0.5)
    Wh, ws = E.op_pack_p16h(Wf)
    Wrm, wsr = E.op_split_weight(Wf)
    bias = rn(N, sc=0.1)
    A_ = Ap2k if K == 2048 else Ap
    po = torch.zeros(R, 16, 2, device=dev) if stats else None

    def f(A_=A_, N=N, K=K, ln=ln, relu=relu, res=res, Wh=Wh, ws=ws, bias=bias, po=po):
        C, _ = E.op_gemm_p16(A_, None, bias, R, N, K, Rp=Rp if res else None, part_in=part if ln else None,
                             relu=relu, part_out=po, Wh=Wh, wscale=ws)
        return C if po is None else torch.cat([C.flatten(), po.flatten()])
    ops[f"gemm_p16 N{N} K{K} ln{int(ln)} relu{int(relu)} res{int(res)} st{int(stats)}"] = f
cache = rn(R, 100, 512)
qkv_d = rn(R, 768)
for step in (5, 40, 80):
    ops[f"self_attention step {step}"] = (lambda step=step: E.op_dec_self_attention(qkv_d, cache.clone(), step))
C, T = 128, 512
x = rn(C * T, 256)
bank = E.op_bank_pack_h3(x, C, T, ones, zeros)
qp = E.pack_p16(rn(C, 2048, sc=0.05))
sig = rn(C, T)
span = torch.full((C,), T, dtype=torch.int32, device=dev)
ops["bank_pack_h3"] = lambda: E.op_bank_pack_h3(x, C, T, ones, zeros).float()
ops["dec_bank_h3"] = lambda: E.op_dec_bank_h3(qp, bank, sig, span, 1.0)
memb = E.op_memory_pack(x, C, T, ones, zeros)
ops["dec_mem_attention"] = lambda: E.op_dec_mem_attention(qp, memb, sig, span, 1.0, 1)
kv = rn(C * T, 512)
q5 = E.pack_p16(rn(C * 5, 256))
ops["dec_ctx_attention rpc5"] = lambda: E.op_dec_ctx_attention(q5, kv, 512, 0, sig, span, 1.0, 5, packed=True)
y = rn(16384, 256)
W1, b1, W2, b2 = rn(2048, 256, sc=1 / 16), rn(2048, sc=0.1), rn(256, 2048, sc=1 / 45), rn(256, sc=0.1)
ops["enc_ffn"] = lambda: E.op_enc_ffn(y, W1, b1, W2, b2, ones, zeros)[0]
Wg = rn(768, 256, sc=1 / 16)
ops["gemm_split ln"] = lambda: E.op_gemm(y, Wg, None, ln_g=ones, ln_b=zeros, split=True)
qkv = rn(32 * 512, 768)
ops["enc_attention"] = lambda: E.op_enc_attention(qkv, sig[:32], span[:32])
err = torch.zeros(1, dtype=torch.int32, device=dev)
for name, fn in ops.items():
    ref = fn()
    torch.cuda.synchronize()
    ref = ref.clone()
    worst = 0.0
    for lds_kb in (16, 64):
        cur = torch.cuda.current_stream()
        A.stream.wait_stream(cur)
        Bn.stream.wait_stream(cur)
        outs = []
        with torch.cuda.stream(Bn.stream):
            for _ in range(40):
                can.lds_canary(err.data_ptr(), 1024, lds_kb * 1024, 20, Bn.stream.cuda_stream)
        with torch.cuda.stream(A.stream):
            for _ in range(40):
                outs.append(fn())
        torch.cuda.synchronize()
        for o in outs:
            d = (o - ref).abs()
            worst = max(worst, float(torch.nan_to_num(d, nan=1e30).max().item()))
    print(f"{name:45s} max|diff| beside spinners {worst:.3e}", flush=True)
