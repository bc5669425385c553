"""Timing probe (not part of the engine): the greedy digit-bank kernel alone at the bench shape (256 chunks x
512 keys, 104 MB of bank), re-reading one bank (Infinity Cache resident) against rotating over 4 banks
(416 MB, past the 256 MB cache), and a plain device copy of one bank's bytes for scale.
    python tools/bank_mall.py"""
import sys

import torch

sys.path.insert(0, ".")
from nanodecoder_amd import engine as E  # noqa: E402


def timeit(fn, n=60):
    for _ in range(3):
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
    C, T = 256, 512
    qp = torch.randn(C, 2048, device=dev) * 0.05
    sig = torch.randn(C, T, device=dev)
    span = torch.full((C,), T, dtype=torch.int32, device=dev)
    banks = [E.op_bank_pack_d8(torch.randn(C * T, 256, device=dev), C, T, span=span) for _ in range(4)]
    nbytes = banks[0][0].numel()
    for nb in (1, 2, 4):
        it = [0]

        def launch():
            E.op_dec_bank_d8(qp, banks[it[0] % nb], sig, span, 1.0)
            it[0] += 1
        us = timeit(launch)
        print(f"bank d8 rotating over {nb} bank(s) ({nb * nbytes / 2**20:.0f} MiB): {us:7.2f} us "
              f"{nbytes / (us * 1e-6) / 1e12:5.2f} TB/s of digits", flush=True)
    dst = torch.empty_like(banks[0][0])
    for nb in (1, 4):
        it = [0]

        def cp():
            dst.copy_(banks[it[0] % nb][0])
            it[0] += 1
        us = timeit(cp)
        print(f"device copy of one bank's bytes, source rotating over {nb}: {us:7.2f} us "
              f"({nbytes / (us * 1e-6) / 1e12:5.2f} TB/s read)", flush=True)


if __name__ == "__main__":
    main()
