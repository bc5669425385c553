"""Driver of tools/lds_forms_probe.hip: per LDS instruction form, victim
workgroups (one per CU, 96/128 KB) alone and beside LDS scribblers on a
second hardware queue; prints the mismatching dwords."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "liblds_forms.so"))
lib.lds_forms.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_void_p]
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import Engine  # noqa: E402

dev = torch.device("cuda", 0)
cfg = synth.ModelConfig()
W = synth.make_weights(cfg, seed=1)
# two engine contexts: their non-blocking streams sit on distinct hardware queues
e1, e2 = Engine(cfg, W, max_batch=4, max_steps=4), Engine(cfg, W, max_batch=4, max_steps=4)
sa, sb = e1.stream, e2.stream
NAMES = ["b32, VGPR >= 64K", "b32, VGPR < 64K + offset:32768", "read2/write2_b32, VGPR >= 64K",
         "read2st64/write2st64_b32, VGPR < 64K, 2nd addr >= 64K", "b128, VGPR >= 64K",
         "read2/write2_b32, all < 64K", "read2/write2_b64, VGPR >= 64K"]
cus = torch.cuda.get_device_properties(dev).multi_processor_count
sig = torch.from_numpy(synth.synth_chunk_batch(64, 512, seed=301)).to(dev)
lens = torch.full((64,), 512, dtype=torch.int32, device=dev)
e3 = Engine(cfg, synth.make_weights(cfg, seed=11), max_batch=64, max_steps=40)
e3.translate_greedy(sig, lens, lens, max_len=40)  # graphs captured
torch.cuda.synchronize()
for mode in range(7):
    res = []
    for side in ("alone", "scribblers", "churn", "engine"):
        bad = 0
        for rep in range(3):
            err = torch.zeros(2, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            if side == "engine":  # another engine's greedy call (its decoder GEMMs) on the victims' CUs
                e3.stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(e3.stream):
                    for _ in range(2):
                        e3.translate_greedy(sig, lens, lens, max_len=40)
                rc = lib.lds_forms(mode, err.data_ptr(), cus, 0, 4000, sa.cuda_stream, sb.cuda_stream)
            else:
                scrib = {"alone": 0, "scribblers": cus, "churn": -400}[side]
                rc = lib.lds_forms(mode, err.data_ptr(), cus, scrib, 2000, sa.cuda_stream, sb.cuda_stream)
            assert rc == 0, rc
            torch.cuda.synchronize()
            bad += int(err[0])
        res.append(f"{side} {bad}")
    print(f"mode {mode} ({NAMES[mode]}): bad dwords " + ", ".join(res), flush=True)
