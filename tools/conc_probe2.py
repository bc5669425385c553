"""Concurrency victim/disturber bisection with op-level kernels on two
engine streams (distinct hardware queues): lane A runs the split-fp16 bank
kernels (bank_pack_h3, dec_bank_h3) repeatedly, lane B one encoder kernel
(enc_ffn / split GEMM / encoder attention); A's outputs vs a serial run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd import engine as E  # noqa: E402

dev = torch.device("cuda", 0)
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
A = E.Engine(cfg, W, max_batch=8, max_steps=8)
Bn = E.Engine(cfg, W, max_batch=8, max_steps=8)
g = torch.Generator(device="cpu").manual_seed(0)
C, T = 64, 512
x = torch.randn(C * T, 256, generator=g).to(dev)
lng, lnb = (1 + 0.1 * torch.randn(256, generator=g)).to(dev), (0.1 * torch.randn(256, generator=g)).to(dev)
qp = E.pack_p16(torch.randn(C, 2048, generator=g).to(dev) * 0.05)
sig = torch.randn(C, T, generator=g).to(dev)
span = torch.full((C,), T, dtype=torch.int32, device=dev)


def victim_pack():
    return E.op_bank_pack_h3(x, C, T, lng, lnb)


bank_ref = victim_pack()
torch.cuda.synchronize()


def victim_bank():
    return E.op_dec_bank_h3(qp, bank_ref, sig, span, 1.0)


u_ref = victim_bank()
pk_ref = bank_ref.clone()
torch.cuda.synchronize()

M, F = 64 * 1024, 2048
y = torch.randn(M, 256, generator=g).to(dev)
W1, b1 = (torch.randn(F, 256, generator=g) / 16).to(dev), (0.1 * torch.randn(F, generator=g)).to(dev)
W2, b2 = (torch.randn(256, F, generator=g) / 45).to(dev), (0.1 * torch.randn(256, generator=g)).to(dev)
ones, zeros = torch.ones(256, device=dev), torch.zeros(256, device=dev)
Wg = (torch.randn(768, 256, generator=g) / 16).to(dev)
qkv = torch.randn(256 * 512, 768, generator=g).to(dev)
sig2 = torch.randn(256, 512, generator=g).to(dev)
span2 = torch.full((256,), 512, dtype=torch.int32, device=dev)
dist = {
    "enc_ffn": lambda: E.op_enc_ffn(y, W1, b1, W2, b2, ones, zeros),
    "gemm_split": lambda: E.op_gemm(y, Wg, None, split=True),
    "enc_attention": lambda: E.op_enc_attention(qkv, sig2, span2),
}
for vname, vfn, ref in (("bank_pack_h3", victim_pack, pk_ref), ("dec_bank_h3", victim_bank, u_ref)):
    for dname, dfn in dist.items():
        worst = 0.0
        for it in range(6):
            cur = torch.cuda.current_stream()
            A.stream.wait_stream(cur)
            Bn.stream.wait_stream(cur)
            outs = []
            with torch.cuda.stream(Bn.stream):
                dfn()
            with torch.cuda.stream(A.stream):
                for _ in range(20):
                    outs.append(vfn())
            torch.cuda.synchronize()
            for o in outs:
                if o.dtype == torch.int16:
                    worst = max(worst, float((o != ref).sum().item()))
                else:
                    worst = max(worst, float((o - ref).abs().max().item()))
        print(f"victim {vname:14s} disturber {dname:14s}: worst {'mismatched halves' if vname == 'bank_pack_h3' else 'max|diff|'} {worst:.3e}", flush=True)
