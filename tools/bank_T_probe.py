"""Timing probe (not part of the engine): the greedy context attention's two bank kernels at chunk lengths
T below 512 (256 chunks; the reference authors' production runs use T = 300): the 24-bit digit
bank (dec_bank_d8_kernel, key blocks per wave = ceil(T / 128)) against the fp32 bank (dec_mem_attention_kernel),
one workgroup per chunk, eager back-to-back launches, Infinity-Cache resident.
    python tools/bank_T_probe.py"""
import sys

import torch

sys.path.insert(0, ".")
from nanodecoder_amd import engine as E  # noqa: E402


def timeit(fn, n=60):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1000.0


def main():
    dev = torch.device("cuda", 0)
    C = 256
    qp = torch.randn(C, 2048, device=dev) * 0.05
    out = torch.empty_like(qp)
    for T in (128, 192, 256, 300, 384, 448, 449, 512):
        x = torch.randn(C * T, 256, device=dev)
        sig = torch.randn(C, T, device=dev)
        span = torch.full((C,), T, dtype=torch.int32, device=dev)
        bank = E.op_bank_pack_d8(x, C, T, span=span)
        mem = E.op_memory_pack(x, C, T, ldT=512)
        d8 = timeit(lambda: E.op_dec_bank_d8(qp, bank, sig, span, 1.0))
        f32 = timeit(lambda: E.op_dec_mem_attention(qp, mem, sig, span, 1.0, 1, out=out))
        print(f"T {T:4d}: digit bank {d8:7.2f} us   fp32 bank {f32:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
