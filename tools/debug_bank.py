"""Debug harness for the split-fp16 memory bank (bank_pack_h3 / dec_bank_h3)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd.engine import op_bank_pack_h3, op_dec_bank_h3, pack_p16, unpack_p16  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
C, T = 2, 512
x = rng.standard_normal((C * T, 256)).astype(np.float32)
bank = op_bank_pack_h3(torch.from_numpy(x).to(dev), C, T).cpu().numpy().view(np.float16)
fr = bank.reshape(C, 32, 8, 2, 64, 8).astype(np.float32)  # [c][kb][db][pl][lane][j]
rec = np.zeros((C, 512, 256), np.float32)
for ln in range(64):
    key = np.arange(32)[:, None] * 16 + (ln & 15)
    for j in range(8):
        d = np.arange(8)[None, :] * 32 + 8 * (ln >> 4) + j
        rec[:, key, d] = fr[:, :, :, 0, ln, j] + fr[:, :, :, 1, ln, j]
print("pack max|err|", np.abs(rec.reshape(C * 512, 256) - x).max())


def run(q, sig, spans):
    out = op_dec_bank_h3(torch.from_numpy(q).to(dev), torch.from_numpy(bank.view(np.int16)).to(dev),
                         torch.from_numpy(sig).to(dev), torch.from_numpy(spans).to(dev), 1.0)
    return unpack_p16(out, C).cpu().numpy()


def ref(q, sig, spans):
    o = np.zeros((C, 2048))
    for c in range(C):
        L = spans[c]
        M = x[c * T:c * T + L].astype(np.float64)
        for h in range(8):
            s = M @ q[c, h * 256:(h + 1) * 256]
            p = np.exp(s - s.max())
            o[c, h * 256:(h + 1) * 256] = (p / p.sum()) @ M
    return o


sig = np.zeros((C, T), np.float32)
for name, q, spans in [("q=0 full", np.zeros((C, 2048), np.float32), np.array([512, 512], np.int32)),
                       ("q=0 span16", np.zeros((C, 2048), np.float32), np.array([16, 16], np.int32)),
                       ("q=0 span1", np.zeros((C, 2048), np.float32), np.array([1, 1], np.int32)),
                       ("q small span16", (rng.standard_normal((C, 2048)) * 0.1).astype(np.float32),
                        np.array([16, 16], np.int32)),
                       ("q small full", (rng.standard_normal((C, 2048)) * 0.1).astype(np.float32),
                        np.array([512, 512], np.int32))]:
    got, want = run(q, sig, spans), ref(q, sig, spans)
    e = np.abs(got - want)
    print(f"{name}: max|err| {e.max():.3e}  worst (c, col) {np.unravel_index(e.argmax(), e.shape)}")
    if e.max() > 1e-4:
        print("  got ", got[0, :8])
        print("  want", want[0, :8])
        print("  per-head err", [float(e[0, h * 256:(h + 1) * 256].max()) for h in range(8)])
        print("  per-dim16 err head0", [float(e[0, k * 16:(k + 1) * 16].max()) for k in range(16)])
