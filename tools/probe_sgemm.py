"""Probe: the library's fp32 GEMM rate (torch.mm -> hipBLASLt / rocBLAS) at the
exact-fp32 encoder's shapes (M = 256 chunks x 512 samples), beside the
engine's own fp32 GEMM (nd_op_gemm with exact fp32 forced, ND_GEMM_F32=1).

Only a yardstick for what fp32 MFMA work reaches on this chip at these
shapes; the product never calls the library GEMM (its LN prologue and
bias / ReLU / residual / row-statistics epilogues are fused).

    python tools/probe_sgemm.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

M = 256 * 512
SHAPES = (("QKV", 256, 768), ("FFN1", 256, 2048), ("FFN2", 2048, 256), ("Wo", 256, 256))


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps * 1e3  # us


def main():
    dev = torch.device("cuda:0")
    torch.backends.cuda.matmul.allow_tf32 = False
    for name, K, N in SHAPES:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        out = torch.empty(M, N, device=dev)
        us = timeit(lambda: torch.mm(a, w.t(), out=out))
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        print(f"torch.mm fp32 {name:5s} M={M} K={K} N={N}: {us:8.1f} us  {tf:6.1f} TF/s  "
              f"({tf / 157.3:.3f} of 157.3)", flush=True)
        del a, w, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
