"""Check: the DMA-ring fp32 GEMM (gemm_f32d_kernel, the in-tree library) against
the register-staged kernel it replaces (a build with -DND_F32D=0, e.g.
tools/build_variant.sh f32base gemm.hip -DND_F32D=0), bitwise, on the encoder's
shapes and ragged / LN / ReLU / residual cases; then both timed.

    python tools/f32d_check.py tools/_ab/f32base.so
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import _lib  # noqa: E402
from nanodecoder_amd import engine as E  # noqa: E402

CASES = [  # M, N, K, ln, relu, res
    (131072, 768, 256, True, False, False),
    (131072, 256, 256, False, False, True),
    (131072, 2048, 256, True, True, False),
    (131072, 256, 2048, False, False, True),
    (65529, 256, 2048, False, False, True),
    (65536, 512, 256, True, True, True),
    (70000, 256, 64, False, True, False),
]


def main():
    old = ctypes.CDLL(os.path.abspath(sys.argv[1]))
    P, I = ctypes.c_void_p, ctypes.c_int
    old.nd_op_gemm.restype = I
    old.nd_op_gemm.argtypes = [P, P, P, P, P, I, I, I, I, I, P]
    new = _lib.lib()
    dev = torch.device("cuda", 0)
    bad = 0
    for (M, N, K, ln, relu, res) in CASES:
        g = torch.Generator().manual_seed(M + N + K)
        A = torch.randn(M, K, generator=g).to(dev)
        W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
        b = torch.randn(N, generator=g).to(dev)
        R = torch.randn(M, N, generator=g).to(dev) if res else None
        if ln:
            W, b = E.op_fold_layernorm(W, b, torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev))
        outs = []
        for lib in (new, old):
            C = torch.full((M, N), float("nan"), device=dev)
            s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            args = (A.data_ptr(), W.data_ptr(), b.data_ptr(), R.data_ptr() if res else None, C.data_ptr(), M, N, K,
                    int(ln), int(relu), s)
            rc = lib.nd_op_gemm(*args)
            assert rc == 0, rc
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(10):
                lib.nd_op_gemm(*args)
            ev1.record()
            torch.cuda.synchronize()
            outs.append((C, ev0.elapsed_time(ev1) / 10 * 1e3))
        same = torch.equal(outs[0][0], outs[1][0])
        bad += not same
        tf = lambda us: 2.0 * M * N * K / (us * 1e-6) / 1e12  # noqa: E731
        print(f"M={M:6d} N={N:5d} K={K:5d} ln={int(ln)} relu={int(relu)} res={int(res)}: "
              f"{'bitwise equal' if same else 'DIFFERENT (max %.3e)' % (outs[0][0] - outs[1][0]).abs().max().item()}"
              f"  new {outs[0][1]:8.1f} us ({tf(outs[0][1]):6.1f} TF/s)  old {outs[1][1]:8.1f} us "
              f"({tf(outs[1][1]):6.1f} TF/s)", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
