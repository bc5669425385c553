"""Timing probe (not part of the engine): beam rows' self-attention at configs[3]'s shape (1024 chunks x 5 rows,
history of `step` keys shared up to a divergence point), the per-row kernel (nd_op_dec_self_attention, rpc 1 with
the ancestry) against the chunk-per-workgroup kernel (nd_op_dec_self_attention_beam); torch events over
back-to-back launches.   python tools/self_time.py"""
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
    dev = torch.device("cuda", 0)
    C, rpc, S = 1024, 5, 100
    R = C * rpc
    qkv = torch.randn(R, 768, device=dev)
    cache = torch.randn(R, S, 512, device=dev)
    g = torch.Generator(device="cpu").manual_seed(1)
    for step in (16, 48, 90):
        anc = torch.empty(R, S, dtype=torch.int32)
        base = (torch.arange(R) // rpc * rpc).to(torch.int32)
        div = torch.randint(0, step, (C,), generator=g).repeat_interleave(rpc)
        t = torch.arange(S)[None, :]
        anc[:] = torch.where(t < div[:, None], base[:, None], base[:, None] + torch.randint(0, rpc, (R, S), generator=g))
        ad = anc.to(dev)
        old = timeit(lambda: E.op_dec_self_attention(qkv, cache, step, anc=ad, anc_ld=S))
        new = timeit(lambda: E.op_dec_self_attention_beam(qkv, cache, step, ad, rpc))
        logical = R * step * 2048
        print(f"step {step:3d}: per-row {old:7.1f} us   chunk-per-workgroup {new:7.1f} us   "
              f"({logical / 1e6:.0f} MB logical)", flush=True)


if __name__ == "__main__":
    main()
