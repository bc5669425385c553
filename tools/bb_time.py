"""Timing probe (not part of the engine): dec_bank_d8_beam_kernel alone at C chunks x rpc rows, against the
greedy digit-bank kernel on the same chunks, torch events over N back-to-back launches.
   python tools/bb_time.py"""
import numpy as np
import torch

from nanodecoder_amd.engine import op_bank_pack_d8, op_dec_bank_d8, op_dec_bank_d8_beam, pack_p16


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1000.0  # us


def main():
    dev = torch.device("cuda", 0)
    T = 512
    for C, rpc in ((1024, 5), (256, 5), (64, 5), (1024, 2)):
        x = torch.randn(C * T, 256, device=dev)
        q = torch.randn(C * rpc, 2048, device=dev) * 0.3
        spans = torch.full((C,), T, dtype=torch.int32, device=dev)
        sig = torch.zeros(C, T, device=dev)
        bank = op_bank_pack_d8(x, C, T, span=spans)
        qp = pack_p16(q)
        out = torch.empty_like(qp)
        tb = timeit(lambda: op_dec_bank_d8_beam(qp, bank, sig, spans, 1e9, rpc, out=out))
        qg = q[::rpc].contiguous()
        og = torch.empty((C + 15) // 16 * 16, 2048, device=dev)
        tg = timeit(lambda: op_dec_bank_d8(qg, bank, sig, spans, 1e9, out=og))
        mb = C * (512 * 256 * 3 + 512 * 4) / 1e6
        print(f"C={C} rpc={rpc}: beam {tb:.1f} us ({mb / tb:.2f} TB/s on {mb:.0f} MB), greedy 1 row {tg:.1f} us", flush=True)


if __name__ == "__main__":
    main()
