"""Timing probe (not part of the engine): the beam context attention alone at B = 1024 chunks x 5 rows, all
alive, fp32 K/V and the 24-bit image; torch events over back-to-back launches.  Run once per library variant
(NANODEC_LIB=tools/_ab/NAME.so).   python tools/ctx_time.py [tag]"""
import sys

import torch

from nanodecoder_amd import engine as E


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1000.0


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    dev = torch.device("cuda", 0)
    C, T, rpc, Ld = 1024, 512, 5, 3
    q = E.pack_p16(torch.randn(C * rpc, 256, device=dev))
    kv = torch.randn(C * T, Ld * 512, device=dev)
    sig = torch.randn(C, T, device=dev)
    span = torch.full((C,), T, dtype=torch.int32, device=dev)
    img = E.op_ctx_pack_q24(kv, Ld * 512, Ld, span, C, T)
    t32 = timeit(lambda: E.op_dec_ctx_attention(q, kv, Ld * 512, 512, sig, span, 1.0, rpc, packed=True))
    t24 = timeit(lambda: E.op_dec_ctx_attention_q24(q, img, 1, sig, span, 1.0, rpc))
    # one layer's image alone ([C*T][1600]: every chunk's keys contiguous, the layer-major layout's stream)
    img1 = E.op_ctx_pack_q24(kv[:, 512:1024].contiguous(), 512, 1, span, C, T)
    t1 = timeit(lambda: E.op_dec_ctx_attention_q24(q, img1, 0, sig, span, 1.0, rpc))
    print(f"{tag:10s} ctx C={C} rpc={rpc}: fp32 K/V {t32:7.1f} us ({C * T * 2048 / t32 / 1e6:.2f} TB/s), "
          f"24-bit {t24:7.1f} us ({C * T * 1600 / t24 / 1e6:.2f} TB/s), "
          f"24-bit contiguous {t1:7.1f} us ({C * T * 1600 / t1 / 1e6:.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
