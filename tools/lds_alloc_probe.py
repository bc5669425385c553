"""Is a workgroup's LDS allocation as large as it asked?  Canaries of size X
(fill all X bytes, spin, re-check) beside 64 KB canaries on another stream;
mismatches in the X-byte canaries = another workgroup was placed inside the
X bytes (allocation smaller than requested)."""
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
for X in (32768, 65536, 65536 + 256, 65536 + 1024, 65536 + 4096, 98560, 131072 + 256, 139904):
    e1 = torch.zeros(2, dtype=torch.int32, device=dev)
    e2 = torch.zeros(2, dtype=torch.int32, device=dev)
    e1[1] = -1
    e2[1] = -1
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        for _ in range(20):
            rc = can.lds_canary(e1.data_ptr(), 512, X, 30, s1.cuda_stream)
            pass
    with torch.cuda.stream(s2):
        for _ in range(20):
            can.lds_canary(e2.data_ptr(), 1024, 65536, 30, s2.cuda_stream)
    torch.cuda.synchronize()
    print(f"canary {X:6d} B beside 64 KB canaries: bad words {int(e1[0])} (first byte {int(e1[1]) * 4 if int(e1[0]) else '-'}), "
          f"64 KB canaries bad {int(e2[0])} (first byte {int(e2[1]) * 4 if int(e2[0]) else '-'})", flush=True)
