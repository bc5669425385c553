"""Is LDS above 128 KB of a CU safe when two workgroups share the CU?

Two sets of LDS canaries (tools/lds_canary.hip: fill the allocation with a
per-workgroup pattern, spin, re-check) on two hardware queues at once, sized
so that one workgroup per CU of each set fits together: (A, B) KB.  When
A + B > 128, whichever is placed second has an allocation that crosses the
128 KB line.  Mismatches (and the lowest bad word) per set."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
can = ctypes.CDLL(os.path.join(ROOT, "tools", "liblds_canary.so"))
can.lds_canary.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
sys.path.insert(0, ROOT)
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import Engine  # noqa: E402

dev = torch.device("cuda", 0)
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=1)
# two engine contexts: their streams sit on distinct hardware queues
e1, e2 = Engine(cfg, W, max_batch=4, max_steps=4), Engine(cfg, W, max_batch=4, max_steps=4)
s1, s2 = e1.stream, e2.stream
KB = 1024
for a, b in ((64, 64), (96, 32), (64, 60), (96, 48), (80, 80), (100, 40), (120, 39), (39, 120), (137, 23)):
    err = [torch.zeros(2, dtype=torch.int32, device=dev) for _ in range(2)]
    for e in err:
        e[1] = 0x7FFFFFFF
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        for _ in range(10):
            can.lds_canary(err[0].data_ptr(), 256, a * KB, 200, s1.cuda_stream)
    with torch.cuda.stream(s2):
        for _ in range(10):
            can.lds_canary(err[1].data_ptr(), 256, b * KB, 200, s2.cuda_stream)
    torch.cuda.synchronize()
    r = [(int(e[0]), int(e[1]) * 4 if int(e[0]) else None) for e in err]
    print(f"canaries {a:3d} KB + {b:3d} KB (sum {a + b:3d}): bad words {r[0][0]} (first byte {r[0][1]}), "
          f"{r[1][0]} (first byte {r[1][1]})", flush=True)
