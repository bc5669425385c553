"""Driver of tools/probe_i8.hip: ds_read_b64_tr_b8's lane map and the
v_mfma_i32_16x16x64_i8 operand pairing (exact integer data)."""
import ctypes
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libprobe_i8.so"))
torch.cuda.init()
dev = torch.device("cuda", 0)


def tr(addr):
    a = torch.tensor(np.asarray(addr, np.uint32).view(np.int32), device=dev)
    o = torch.zeros(64, dtype=torch.int64, device=dev)
    assert lib.probe_tr_b8(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(o.data_ptr())) == 0
    b = o.cpu().numpy().view(np.uint8).reshape(64, 8)
    return [[(int(x) >> 5, int(x) & 31) for x in row] for row in b]


lanes = np.arange(64)
i = lanes & 15
for name, addr in (("hyp: lane 2q+p -> row q, cols 8p..", (i >> 1) * 32 + 8 * (i & 1)),
                   ("linear: lane l -> byte 8l mod 256", (lanes * 8) % 256),
                   ("lane l -> row l&7, col 8*((l>>3)&3)", (lanes & 7) * 32 + 8 * ((lanes >> 3) & 3))):
    res = tr(addr)
    print("==", name)
    for l in range(0, 64, 1 if name.startswith("hyp") else 8):
        print(f"  lane {l:2d} addr {int(addr[l]):3d}: " + " ".join(f"r{r}c{c}" for r, c in res[l]))

rng = np.random.default_rng(0)
A = rng.integers(-128, 128, size=(64, 16)).astype(np.int8)
B = rng.integers(-128, 128, size=(64, 16)).astype(np.int8)
a = torch.from_numpy(A.view(np.int32).copy()).to(dev)
b = torch.from_numpy(B.view(np.int32).copy()).to(dev)
d = torch.zeros(64, 4, dtype=torch.int32, device=dev)
assert lib.probe_mfma_i8(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(d.data_ptr())) == 0
D = d.cpu().numpy()
Am = np.zeros((16, 64), np.int64)
Bm = np.zeros((64, 16), np.int64)
for l in range(64):
    for j in range(16):
        Am[l & 15, 16 * (l >> 4) + j] = A[l, j]
        Bm[16 * (l >> 4) + j, l & 15] = B[l, j]
ref = Am @ Bm
got = np.zeros((16, 16), np.int64)
for l in range(64):
    for r in range(4):
        got[4 * (l >> 4) + r, l & 15] = D[l, r]
print("mfma_i32_16x16x64_i8 symmetric pairing (lane l elem j of A with lane l' elem j of B, same l>>4):",
      "OK" if (got == ref).all() else f"MISMATCH ({int((got != ref).sum())} of 256)")
