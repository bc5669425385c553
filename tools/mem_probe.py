"""Timing probe (not part of the engine): the fp32 memory-bank kernel (exact fp32's context attention,
dec_mem_attention_kernel) alone at the bench shape (256 chunks x 512 keys), one bank re-read (Infinity-Cache
resident) and 3 banks rotating (evicted), one workgroup per chunk and the pool's 128 walking workgroups, for
the library NANODEC_LIB names (tools/mem_probe.sh builds the MB_PROBE_* variants of mem_attention.hip).
    NANODEC_AB=1 NANODEC_LIB=tools/_ab/X.so python tools/mem_probe.py X"""
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
    banks = [E.op_memory_pack(torch.randn(C * T, 256, device=dev), C, T) for _ in range(3)]
    out = torch.empty_like(qp)
    res = []
    for grid in (0, 128):
        for nb in (1, 3):
            it = [0]

            def launch():
                E.op_dec_mem_attention(qp, banks[it[0] % nb], sig, span, 1.0, 1, out=out, grid=grid)
                it[0] += 1
            res.append(timeit(launch))
    print(f"{tag:12s} per chunk: resident {res[0]:7.2f} us  evicted {res[1]:7.2f} us | "
          f"128 walking: resident {res[2]:7.2f} us  evicted {res[3]:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
