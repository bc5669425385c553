"""Timing probe (not part of the engine): where a dec_bank_d8_kernel workgroup spends its time.  Built with
-DB8_PROBE_PHASES (tools/_ab/b8_phases.so), every wave stamps the wall clock (s_memrealtime, 100 MHz) at
8 points: entry, prologue done, key blocks 0..3 done, merge barrier, end.  256 chunks x 512 keys, bank
resident (re-read) or evicted (4 rotating).
    NANODEC_AB=1 NANODEC_LIB=tools/_ab/b8_phases.so python tools/bank_phases.py"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from nanodecoder_amd import engine as E  # noqa: E402

NAMES = ["prologue", "kb0", "kb1", "kb2", "kb3", "merge-a", "merge-b"]


def main():
    dev = torch.device("cuda", 0)
    C, T = 256, 512
    qp = torch.randn(C, 2048, device=dev) * 0.05
    sig = torch.randn(C, T, device=dev)
    span = torch.full((C,), T, dtype=torch.int32, device=dev)
    banks = [E.op_bank_pack_d8(torch.randn(C * T, 256, device=dev), C, T, span=span) for _ in range(4)]
    C16 = (C + 15) // 16 * 16
    out = torch.zeros(C16 * 2048 + C * 8 * 8 * 2, dtype=torch.float32, device=dev)
    for nb in (1, 4):
        acc = []
        for it in range(40):
            E.op_dec_bank_d8(qp, banks[it % nb], sig, span, 1.0, out=out)
            if it >= 8:
                torch.cuda.synchronize()
                st = out[C16 * 2048:].view(torch.int64).view(C, 8, 8).cpu().numpy().astype(np.float64) * 0.01  # us
                acc.append(st)
        st = np.stack(acc)                                  # [runs, C, waves, 8]
        t0 = st[..., 0].min(axis=(1, 2), keepdims=True)     # kernel's first wave entry
        rel = st - t0[..., None]
        d = np.diff(st, axis=-1)                             # [runs, C, waves, 7]
        print(f"bank {'resident' if nb == 1 else 'evicted '}: kernel span {rel[..., 7].max(axis=(1, 2)).mean():6.2f} us"
              f"  entry spread {rel[..., 0].max(axis=(1, 2)).mean():5.2f}  last wave end after its entry "
              f"{(st[..., 7] - st[..., 0]).max(axis=(1, 2)).mean():6.2f}", flush=True)
        print("   phase (mean / max over waves, us): " + "  ".join(
            f"{n} {d[..., i].mean():5.2f}/{d[..., i].max(axis=(1, 2)).mean():5.2f}" for i, n in enumerate(NAMES)),
            flush=True)


if __name__ == "__main__":
    main()
