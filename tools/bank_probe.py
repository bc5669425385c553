"""Timing probe (not part of the engine): the greedy digit-bank kernel alone at the bench shape (256 chunks x
512 keys), Infinity-Cache resident (one bank re-read) and evicted (4 banks rotating), for the library
NANODEC_LIB names (tools/bank_probe.sh builds the B8_PROBE_* variants of bank8.hip).
    NANODEC_AB=1 NANODEC_LIB=tools/_ab/X.so python tools/bank_probe.py X"""
import sys

import torch

sys.path.insert(0, ".")
from nanodecoder_amd import engine as E  # noqa: E402


def timeit(fn, n=80):
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
    tag = sys.argv[1] if len(sys.argv) > 1 else "base"
    dev = torch.device("cuda", 0)
    C, T = 256, 512
    qp = torch.randn(C, 2048, device=dev) * 0.05
    sig = torch.randn(C, T, device=dev)
    span = torch.full((C,), T, dtype=torch.int32, device=dev)
    banks = [E.op_bank_pack_d8(torch.randn(C * T, 256, device=dev), C, T, span=span) for _ in range(4)]
    res = []
    for nb in (1, 4):
        it = [0]

        def launch():
            E.op_dec_bank_d8(qp, banks[it[0] % nb], sig, span, 1.0)
            it[0] += 1
        res.append(timeit(launch))
    # a trivial launch of the same grid for the boundary cost (eager back-to-back)
    z = torch.zeros(C * 512, device=dev)
    res.append(timeit(lambda: z.add_(1.0)))
    print(f"{tag:12s} resident {res[0]:7.2f} us  evicted {res[1]:7.2f} us  (trivial launch {res[2]:5.2f} us)",
          flush=True)


if __name__ == "__main__":
    main()
