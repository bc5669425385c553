"""Diagnostic (not part of the engine): the beam digit-bank kernel at many chunks per CU.  Runs the op twice
on C chunks (rpc rows each) and reports bitwise repeatability and the worst error of sampled chunks
against fp64.   python tools/bb_repeat.py [C] [rpc]"""
import sys

import numpy as np
import torch

from nanodecoder_amd.engine import op_bank_pack_d8, op_dec_bank_d8_beam, pack_p16, unpack_p16


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    rpc = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(1)
    T = 512
    x = torch.randn(C * T, 256, device=dev)
    q = torch.randn(C * rpc, 2048, device=dev) * 0.3
    spans = torch.from_numpy(rng.integers(1, T + 1, C).astype(np.int32)).to(dev)
    sig = torch.zeros(C, T, device=dev)
    bank = op_bank_pack_d8(x, C, T)
    qp = pack_p16(q)
    outs = [op_dec_bank_d8_beam(qp, bank, sig, spans, 1e9, rpc) for _ in range(3)]
    torch.cuda.synchronize()
    same = [torch.equal(outs[0], o) for o in outs[1:]]
    got = unpack_p16(outs[0], C * rpc).cpu().numpy().astype(np.float64)
    xs = x.cpu().numpy().astype(np.float64)
    qs = q.cpu().numpy().astype(np.float64)
    sp = spans.cpu().numpy()
    worst = 0.0
    bad = []
    for c in list(range(0, C, max(1, C // 24))) + [C - 1]:
        L = int(sp[c])
        M = xs[c * T: c * T + L]
        for j in range(rpc):
            r = c * rpc + j
            for h in range(8):
                s = M @ qs[r, h * 256:(h + 1) * 256]
                p = np.exp(s - s.max())
                want = (p / p.sum()) @ M
                e = np.abs(got[r, h * 256:(h + 1) * 256] - want).max() / max(1.0, np.abs(want).max())
                worst = max(worst, e)
                if e > 2e-5:
                    bad.append((c, j, h, L, e))
    print(f"C={C} rpc={rpc}: repeat bitwise {same}; worst rel err {worst:.3e}; bad {len(bad)} {bad[:6]}")


if __name__ == "__main__":
    main()
