"""Timing probe (not part of the engine): the beam rows' self-attention on the 24-bit history at configs[3]'s
shape (1024 chunks x 5 rows), the chunk-per-workgroup kernel (nd_op_dec_self_attention_q24 with rpc 5), a
history shared by a chunk's rows up to a divergence point then split over the rows' slots; torch events over
back-to-back launches, for the library NANODEC_LIB names (SB_* variants of attention.hip).
    NANODEC_AB=1 NANODEC_LIB=tools/_ab/X.so python tools/self_q24_time.py X"""
import sys

import torch

sys.path.insert(0, ".")
import ctypes  # noqa: E402

from nanodecoder_amd import _lib  # noqa: E402
from nanodecoder_amd import engine as E  # noqa: E402


def timeit(fn, n=30):
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
    tag = sys.argv[1] if len(sys.argv) > 1 else "base"
    dev = torch.device("cuda", 0)
    C, rpc, S = 1024, 5, 100
    R = C * rpc
    qkv = torch.randn(R, 768, device=dev)
    cache = torch.randint(0, 255, (R, S, 1600), dtype=torch.uint8, device=dev)
    # valid scales (bytes 1536.. hold f32 pairs): 2^-20
    sc = torch.full((R, S, 16), 2.0 ** -20, device=dev)
    cache[..., 1536:1600] = sc.view(torch.uint8).view(R, S, 64)
    g = torch.Generator(device="cpu").manual_seed(1)
    out = []
    for step in (16, 48, 90):
        anc = torch.empty(R, S, dtype=torch.int32)
        base = (torch.arange(R) // rpc * rpc).to(torch.int32)
        div = torch.randint(0, step, (C,), generator=g).repeat_interleave(rpc)
        t = torch.arange(S)[None, :]
        # after the divergence point most keys still come from one or two of the chunk's slots
        pick = torch.randint(0, 2, (R, S), generator=g) * torch.randint(0, rpc, (R, 1), generator=g)
        anc[:] = torch.where(t < div[:, None], base[:, None], base[:, None] + pick.to(torch.int32))
        ad = anc.to(dev)
        qp = E.pack_p16(qkv)
        o = torch.empty(qp.shape[0], 256, dtype=torch.float32, device=dev)
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        L = _lib.lib()

        def run():
            _lib.check(L.nd_op_dec_self_attention_q24(qp.data_ptr(), cache.data_ptr(), ad.data_ptr(), S, step, S,
                                                      o.data_ptr(), R, rpc, None, st))
        us = timeit(run)
        out.append(f"step {step:3d} {us:7.1f} us")
    print(f"{tag:10s} " + "   ".join(out), flush=True)


if __name__ == "__main__":
    main()
