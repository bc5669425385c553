"""Diagnostic for the beam digit-bank kernel (not part of the engine): one chunk, two rows, against fp64 and
against the greedy digit-bank kernel on the same q' rows.  Prints the error per head and per 16-dim block,
for a few q' patterns (both rows equal; one-hot keys; constant rows).   python tools/bb_debug.py"""
import numpy as np
import torch

from nanodecoder_amd.engine import op_bank_pack_d8, op_dec_bank_d8, op_dec_bank_d8_beam, pack_p16, unpack_p16


def ref(xm, q, L):
    out = np.zeros(2048)
    M = xm[:L]
    for h in range(8):
        s = M @ q[h * 256:(h + 1) * 256]
        p = np.exp(s - s.max())
        out[h * 256:(h + 1) * 256] = (p / p.sum()) @ M
    return out


def main():
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    T = 512
    C = 2
    x = rng.standard_normal((C * T, 256)).astype(np.float32)
    cases = {}
    q0 = (rng.standard_normal(2048) * 0.3).astype(np.float32)
    cases["random"] = q0
    cases["small"] = q0 * 0.01
    cases["zero"] = np.zeros(2048, np.float32)
    import os, sys
    quick = "--quick" in sys.argv
    print("lib:", os.environ.get("NANODEC_LIB", "in-tree"))
    for name, q in cases.items():
        if quick and name != "random":
            continue
        for L in ((1, 512) if quick else (512, 16, 1)):
            spans = np.array([L, L], np.int32)
            sig = np.zeros((C, T), np.float32)
            bank = op_bank_pack_d8(torch.from_numpy(x).to(dev), C, T)
            qq = np.stack([q, q, q, q]).astype(np.float32)   # 2 chunks x 2 rows
            outb = op_dec_bank_d8_beam(pack_p16(torch.from_numpy(qq).to(dev)), bank, torch.from_numpy(sig).to(dev),
                                       torch.from_numpy(spans).to(dev), 1e9, 2)
            outg = op_dec_bank_d8(torch.from_numpy(qq[::2].copy()).to(dev), bank, torch.from_numpy(sig).to(dev),
                                  torch.from_numpy(spans).to(dev), 1e9)
            torch.cuda.synchronize()
            gb = unpack_p16(outb, 4).cpu().numpy()
            gg = unpack_p16(outg, 2).cpu().numpy()
            want = ref(x[:T].astype(np.float64), q.astype(np.float64), L)
            eb = np.abs(gb[0] - want).reshape(8, 16, 16).max(2)
            eg = np.abs(gg[0] - want).reshape(8, 16, 16).max(2)
            print(f"== {name} L={L}: beam err {eb.max():.3e} greedy err {eg.max():.3e}; rows equal "
                  f"{np.array_equal(gb[0], gb[1])}")
            if eb.max() > 1e-4:
                np.set_printoptions(precision=1, linewidth=200)
                print("beam err per head (rows) x 16-dim block (cols), log10:")
                print(np.log10(eb + 1e-12))
                print("beam / want sample (head 0, dims 0..7):", gb[0][:8], want[:8])
                print("head 0 dims 16..23 beam-want:", (gb[0][16:24] - want[16:24]) / np.abs(want[16:24]).max())
                print("head 2 dims 16..23 beam-want:", (gb[0][528:536] - want[528:536]) / np.abs(want[528:536]).max())


if __name__ == "__main__":
    main()
