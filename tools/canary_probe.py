"""Does any engine kernel write LDS outside its own allocation?  LDS canary
workgroups (tools/lds_canary.hip) spin on one stream while the suspect runs
on another; mismatches in the canaries' LDS = foreign writes."""
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
can = ctypes.CDLL(os.path.join(ROOT, "tools", "liblds_canary.so"))
can.lds_canary.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
A = E.Engine(cfg, W, max_batch=64, max_steps=20)
Bn = E.Engine(cfg, W, max_batch=8, max_steps=8)
g = torch.Generator(device="cpu").manual_seed(0)
sig = torch.from_numpy(synth.synth_chunk_batch(64, 512, seed=3)).to(dev)
lens = torch.full((64,), 512, dtype=torch.int32, device=dev)
M, F = 32 * 1024, 2048
y = torch.randn(M, 256, generator=g).to(dev)
W1, b1 = (torch.randn(F, 256, generator=g) / 16).to(dev), (0.1 * torch.randn(F, generator=g)).to(dev)
W2, b2 = (torch.randn(256, F, generator=g) / 45).to(dev), (0.1 * torch.randn(256, generator=g)).to(dev)
ones, zeros = torch.ones(256, device=dev), torch.zeros(256, device=dev)
Wg = (torch.randn(768, 256, generator=g) / 16).to(dev)
qkv = torch.randn(64 * 512, 768, generator=g).to(dev)
sig2 = torch.randn(64, 512, generator=g).to(dev)
span2 = torch.full((64,), 512, dtype=torch.int32, device=dev)
x = torch.randn(64 * 512, 256, generator=g).to(dev)
bank = E.op_bank_pack_h3(x, 64, 512, ones, zeros)
qp = E.pack_p16(torch.randn(64, 2048, generator=g).to(dev) * 0.05)
Ap = E.pack_p16(torch.randn(256, 2048, generator=g).to(dev))
Wp = torch.randn(256, 2048, generator=g).to(dev) / 45
Wh, ws = E.op_pack_p16h(Wp)
Ap2 = E.pack_p16(torch.randn(256, 256, generator=g).to(dev))
Wq = torch.randn(2048, 256, generator=g).to(dev) / 16
Whq, wsq = E.op_pack_p16h(Wq)
Whq_rm, wsq_rm = E.op_split_weight(Wq)
part = E.row_partials(torch.randn(256, 256, generator=g).to(dev))
cache = torch.zeros(256, 100, 512, device=dev)
qkv_d = torch.randn(256, 768, generator=g).to(dev)
suspects = {
    "translate_greedy": lambda: A.translate_greedy(sig, lens, lens, max_len=20, min_len=2),
    "encode": lambda: A.encode(sig, lens, lens),
    "enc_ffn": lambda: E.op_enc_ffn(y, W1, b1, W2, b2, ones, zeros),
    "gemm_split": lambda: E.op_gemm(y, Wg, None, split=True),
    "gemm_split_ln": lambda: E.op_gemm(y, Wg, None, ln_g=ones, ln_b=zeros, split=True),
    "enc_attention": lambda: E.op_enc_attention(qkv, sig2, span2),
    "dec_bank_h3": lambda: E.op_dec_bank_h3(qp, bank, sig2, span2, 1.0),
    "p16_longk": lambda: E.op_gemm_p16(Ap, None, None, 256, 256, 2048, Wh=Wh, wscale=ws),
    "p16s_ln": lambda: E.op_gemm_p16(Ap2, None, None, 256, 2048, 256, part_in=part, Wh=Whq, wscale=wsq),
    "self_attention": lambda: E.op_dec_self_attention(qkv_d, cache, 50),
}
err = torch.zeros(1, dtype=torch.int32, device=dev)
for lds_kb in (4, 12):
    for name, fn in suspects.items():
        err.zero_()
        torch.cuda.synchronize()
        cur = torch.cuda.current_stream()
        A.stream.wait_stream(cur)
        Bn.stream.wait_stream(cur)
        with torch.cuda.stream(Bn.stream):
            for _ in range(30):
                can.lds_canary(err.data_ptr(), 2048, lds_kb * 1024, 100, Bn.stream.cuda_stream)
        with torch.cuda.stream(A.stream):
            for _ in range(30):
                fn()
        torch.cuda.synchronize()
        print(f"canary {lds_kb:2d} KB beside {name:18s}: {int(err.item())} foreign LDS words", flush=True)
