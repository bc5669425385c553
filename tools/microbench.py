"""Time individual kernels through the op-level C-ABI entry points (HIP
events on the current torch stream).  Usage: python tools/microbench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodecoder_amd import engine as E  # noqa: E402

dev = torch.device("cuda", 0)
ONLY = sys.argv[1] if len(sys.argv) > 1 else ""


EAGER = os.environ.get("MB_EAGER") == "1"  # plain launches (for PMC counter passes)


def timeit(fn, n=50):
    """Per-launch time inside a captured graph of n back-to-back launches
    (the way the engine runs them), in microseconds."""
    if EAGER:
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return float("nan")
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / (5 * n) * 1e3  # us


def gemm_case(M, N, K, ln, relu, res, split=False):
    A = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    R = torch.randn(M, N, device=dev) if res else None
    if ln:  # the engine folds the LayerNorm affine once at load time
        W, b = E.op_fold_layernorm(W, b, torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev))
    C = torch.empty(M, N, device=dev)
    if split:
        import ctypes
        from nanodecoder_amd import _lib
        Wh, sc = E.op_split_weight(W)
        st = lambda: ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)  # noqa: E731
        fn = lambda: _lib.lib().nd_op_gemm_split(A.data_ptr(), Wh.data_ptr(), sc, b.data_ptr(),  # noqa: E731
                                                 R.data_ptr() if res else None, C.data_ptr(), M, N, K, int(ln),
                                                 int(relu), st())
    else:
        fn = lambda: E.op_gemm(A, W, b, R, relu=relu, norm=ln)  # noqa: E731
    us = timeit(fn)
    tf = 2 * M * N * K / (us * 1e-6) / 1e12
    print(f"gemm{'-split' if split else '      '} M={M:6d} N={N:5d} K={K:5d} ln={int(ln)} relu={int(relu)} "
          f"res={int(res)}: {us:9.2f} us  {tf:6.1f} TF/s")


if ONLY == "enc":
    # the encoder's GEMM shapes at B = 256 chunks x 512 samples, fp32 MFMA and split-fp16
    for sp in (False, True):
        gemm_case(131072, 768, 256, True, False, False, sp)    # QKV (LN)
        gemm_case(131072, 256, 256, False, False, True, sp)    # Wo (+res)
        gemm_case(131072, 2048, 256, True, True, False, sp)    # FFN1 (LN, relu)
        gemm_case(131072, 256, 2048, False, False, True, sp)   # FFN2 (+res)
    sys.exit(0)
if ONLY == "encffn":  # the fused FFN block against the two split GEMMs it replaces
    M = 131072
    y = torch.randn(M, 256, device=dev)
    W1 = torch.randn(2048, 256, device=dev) / 16
    W2 = torch.randn(256, 2048, device=dev) / 45
    b1, b2 = torch.randn(2048, device=dev), torch.randn(256, device=dev)
    lg, lb = torch.rand(256, device=dev) + 0.5, torch.randn(256, device=dev)
    import ctypes
    from nanodecoder_amd import _lib
    W1f, b1f = E.op_fold_layernorm(W1, b1, lg, lb)
    w1h, w1s = E.op_pack_p16h(W1f)
    w2h, w2s = E.op_pack_p16h(W2)
    x = torch.empty_like(y)
    part = torch.empty(M, 16, 2, device=dev)
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)  # noqa: E731
    us = timeit(lambda: _lib.lib().nd_op_enc_ffn(y.data_ptr(), w1h.data_ptr(), w1s, b1f.data_ptr(), w2h.data_ptr(),
                                                  w2s, b2.data_ptr(), x.data_ptr(), part.data_ptr(), M, 2048, None,
                                                  st()), n=5)
    print(f"enc-ffn fused M={M}: {us:9.2f} us  {2 * 2 * M * 2048 * 256 / (us * 1e-6) / 1e12:6.1f} TF/s (fp32-equiv)")
    Wo = torch.randn(256, 256, device=dev) / 16
    woh, wos = E.op_pack_p16h(Wo)
    att, bo = torch.randn(M, 256, device=dev), torch.randn(256, device=dev)
    us = timeit(lambda: _lib.lib().nd_op_enc_ffn_wo(att.data_ptr(), y.data_ptr(), woh.data_ptr(), wos, bo.data_ptr(),
                                                     w1h.data_ptr(), w1s, b1f.data_ptr(), w2h.data_ptr(), w2s,
                                                     b2.data_ptr(), x.data_ptr(), part.data_ptr(), None, 1.0, None,
                                                     None, M, 2048, None, st()), n=5)
    fl = 2 * M * 256 * (2 * 2048 + 256)
    print(f"enc-ffn + Wo M={M}: {us:9.2f} us  {fl / (us * 1e-6) / 1e12:6.1f} TF/s (fp32-equiv)")
    qh, qs = E.op_pack_p16h(torch.randn(768, 256, device=dev) / 16)
    qb, qkv = torch.randn(768, device=dev), torch.empty(M, 768, device=dev)
    us = timeit(lambda: _lib.lib().nd_op_enc_ffn_wo(att.data_ptr(), y.data_ptr(), woh.data_ptr(), wos, bo.data_ptr(),
                                                     w1h.data_ptr(), w1s, b1f.data_ptr(), w2h.data_ptr(), w2s,
                                                     b2.data_ptr(), x.data_ptr(), part.data_ptr(), qh.data_ptr(), qs,
                                                     qb.data_ptr(), qkv.data_ptr(), M, 2048, None, st()), n=5)
    fl = 2 * M * 256 * (2 * 2048 + 256 + 768)
    print(f"enc-ffn + Wo + QKV M={M}: {us:9.2f} us  {fl / (us * 1e-6) / 1e12:6.1f} TF/s (fp32-equiv)")
    gemm_case(M, 2048, 256, True, True, False, True)
    gemm_case(M, 256, 2048, False, False, True, True)
    sys.exit(0)
if ONLY == "ffn1s":  # one encoder GEMM in the split-fp16 form (PMC passes: MB_EAGER=1)
    gemm_case(131072, 2048, 256, True, True, False, True)
    sys.exit(0)
if ONLY == "eattn":  # encoder self-attention at B = 256 x 512
    B, T = 256, 512
    qkv = torch.randn(B * T, 768, device=dev)
    sig = torch.randn(B, T, device=dev)
    span = torch.full((B,), T, dtype=torch.int32, device=dev)
    us = timeit(lambda: E.op_enc_attention(qkv, sig, span), n=10)
    print(f"enc-attn B={B}: {us:9.2f} us  {4*B*8*T*T*32/(us*1e-6)/1e12:6.1f} TF/s")
    sys.exit(0)
if ONLY == "self":  # decoder self-attention at the greedy shape (R = 256, P16 q | k | v)
    R, S = 256, 100
    qkv = E.pack_p16(torch.randn(R, 768, device=dev))
    cache = torch.randn(R, S, 512, device=dev)
    for step in (20, 50, 90):
        us = timeit(lambda: E.op_dec_self_attention(qkv, cache, step, packed=True))
        print(f"self-attn R={R} step={step:3d}: {us:7.2f} us  {R * step * 2048 / (us * 1e-6) / 1e9:7.1f} GB/s")
    sys.exit(0)
if ONLY == "bank":  # the split-fp16 bank kernel alone at the bench shape (C = 256, T = 512)
    C, T = 256, 512
    qp = E.pack_p16(torch.randn(C, 2048, device=dev) * 0.05)
    sig = torch.randn(C, T, device=dev)
    span = torch.full((C,), T, dtype=torch.int32, device=dev)
    bank = E.op_bank_pack_h3(torch.randn(C * T, 256, device=dev), C, T)
    us = timeit(lambda: E.op_dec_bank_h3(qp, bank, sig, span, 1.0))
    print(f"bank-h3  C={C:4d} T={T}: {us:8.2f} us  {C * T * 256 * 4 / (us * 1e-6) / 1e9:7.1f} GB/s")
    sys.exit(0)
if ONLY == "bankmall":  # Infinity Cache residency: one bank re-read vs 3 banks in rotation (402 MB)
    C, T = 256, 512
    qp = E.pack_p16(torch.randn(C, 2048, device=dev) * 0.05)
    sig = torch.randn(C, T, device=dev)
    span = torch.full((C,), T, dtype=torch.int32, device=dev)
    banks = [E.op_bank_pack_h3(torch.randn(C * T, 256, device=dev), C, T) for _ in range(3)]
    for nb in (1, 2, 3):
        it = [0]

        def launch():
            E.op_dec_bank_h3(qp, banks[it[0] % nb], sig, span, 1.0)
            it[0] += 1
        us = timeit(launch, n=48)
        print(f"bank-h3 rotation over {nb} bank(s) ({nb * C * T * 1024 / 2**20:.0f} MiB): {us:8.2f} us  "
              f"{C * T * 256 * 4 / (us * 1e-6) / 1e9:7.1f} GB/s")
    sys.exit(0)
if ONLY == "mem":
    # memory-bank attention: scaling in the chunk count and the key count
    for C, T in ((64, 512), (128, 512), (256, 512), (512, 512), (256, 256), (256, 128)):
        qp = E.pack_p16(torch.randn(C, 2048, device=dev))
        memp = E.op_memory_pack(torch.randn(C * T, 256, device=dev), C, T)
        sig = torch.randn(C, T, device=dev)
        span = torch.full((C,), T, dtype=torch.int32, device=dev)
        us = timeit(lambda: E.op_dec_mem_attention(qp, memp, sig, span, 1.0, 1))
        print(f"mem-attn C={C:4d} T={T}: {us:8.2f} us  {C * T * 256 * 4 / (us * 1e-6) / 1e9:7.1f} GB/s  "
              f"{2 * 2 * 8 * C * T * 256 / (us * 1e-6) / 1e12:6.1f} TF/s (algorithmic, 8 heads)")
        if T == 512:  # the split-fp16 fragment bank (the greedy path at 512-sample chunks)
            bank = E.op_bank_pack_h3(torch.randn(C * T, 256, device=dev), C, T)
            us = timeit(lambda: E.op_dec_bank_h3(qp, bank, sig, span, 1.0))
            print(f"bank-h3  C={C:4d} T={T}: {us:8.2f} us  {C * T * 256 * 4 / (us * 1e-6) / 1e9:7.1f} GB/s")
    sys.exit(0)
if ONLY == "dec256":
    # decoder-step shapes on the engine's P16 layout (greedy R=256, beam R=1280)
    for M in (256, 1280, 5120):
        for N, K, ln, relu, res in ((768, 256, True, False, False), (256, 256, False, False, True),
                                    (256, 256, True, False, False), (2048, 256, True, True, False),
                                    (256, 2048, False, False, True)):
            Ap = E.pack_p16(torch.randn(M, K, device=dev))
            Wp = E.pack_p16(torch.randn(N, K, device=dev) / K ** 0.5)
            b = torch.randn(N, device=dev)
            Rp = E.pack_p16(torch.randn(M, N, device=dev)) if res else None
            part = E.row_partials(torch.randn(M, K, device=dev)) if ln else None
            pout = torch.empty(M, 16, 2, device=dev) if N == 256 else None
            Wr = torch.randn(N, K, device=dev) / K ** 0.5
            Wh, sc = E.op_pack_p16h(Wr)
            Wm, sm = E.op_split_weight(Wr)
            for sp in ("", "-split", "-rm"):
                kw = dict(Wh=Wh, wscale=sc) if sp else {}
                if sp == "-rm":
                    kw.update(Wh_rm=Wm, wscale_rm=sm)
                us = timeit(lambda: E.op_gemm_p16(Ap, Wp, b, M, N, K, Rp, part, relu, pout, **kw))
                tf = 2 * M * N * K / (us * 1e-6) / 1e12
                print(f"gemm_p16{sp:6s} M={M:5d} N={N:5d} K={K:5d} ln={int(ln)} "
                      f"relu={int(relu)} res={int(res)}: {us:8.2f} us  {tf:6.1f} TF/s")
    qkv = E.pack_p16(torch.randn(256, 768, device=dev))
    cache = torch.randn(256, 100, 512, device=dev)
    us = timeit(lambda: E.op_dec_self_attention(qkv, cache, 60, packed=True))
    print(f"self-attn R=256 step=60: {us:8.2f} us")
    for C, rpc in ((256, 1), (256, 5)):
        T = 512
        q = E.pack_p16(torch.randn(C * rpc, 256, device=dev))
        kv = torch.randn(C * T, 1536, device=dev)
        sig = torch.randn(C, T, device=dev)
        span = torch.full((C,), T, dtype=torch.int32, device=dev)
        us = timeit(lambda: E.op_dec_ctx_attention(q, kv, 1536, 0, sig, span, 1.0, rpc, packed=True))
        print(f"ctx-attn C={C} rpc={rpc}: {us:8.2f} us  {C * T * 512 * 4 / (us * 1e-6) / 1e9:7.1f} GB/s (K+V bytes)")
    C, T = 256, 512
    qp = E.pack_p16(torch.randn(C, 2048, device=dev))
    memp = E.op_memory_pack(torch.randn(C * T, 256, device=dev), C, T)
    sig = torch.randn(C, T, device=dev)
    span = torch.full((C,), T, dtype=torch.int32, device=dev)
    us = timeit(lambda: E.op_dec_mem_attention(qp, memp, sig, span, 1.0, 1))
    print(f"mem-attn C={C} rpc=1: {us:8.2f} us  {C * T * 256 * 4 / (us * 1e-6) / 1e9:7.1f} GB/s (bank bytes)  "
          f"{2 * 2 * 8 * C * T * 256 / (us * 1e-6) / 1e12:6.1f} TF/s (algorithmic, 8 heads)")
    sys.exit(0)
for M in (256, 1280, 5120):
    gemm_case(M, 768, 256, True, False, False)
    gemm_case(M, 256, 256, False, False, True)
    gemm_case(M, 256, 256, True, False, False)
    gemm_case(M, 2048, 256, True, True, False)
    gemm_case(M, 256, 2048, False, False, True)
gemm_case(131072, 768, 256, True, False, False)
gemm_case(131072, 256, 256, False, False, True)
gemm_case(131072, 2048, 256, True, True, False)
gemm_case(131072, 256, 2048, False, False, True)
gemm_case(131072, 1536, 256, True, False, False)

# decoder self-attention at several steps
for R in (256, 5120):
    S = 100
    qkv = torch.randn(R, 768, device=dev)
    cache = torch.randn(R, S, 512, device=dev)
    for step in (0, 50, 99):
        us = timeit(lambda: E.op_dec_self_attention(qkv, cache, step))
        print(f"self-attn R={R} step={step}: {us:8.2f} us")

# decoder context attention
for C, rpc in ((256, 1), (256, 5)):
    T = 512
    q = torch.randn(C * rpc, 256, device=dev)
    kv = torch.randn(C * T, 1536, device=dev)
    sig = torch.randn(C, T, device=dev)
    span = torch.full((C,), T, dtype=torch.int32, device=dev)
    us = timeit(lambda: E.op_dec_ctx_attention(q, kv, 1536, 0, sig, span, 1.0, rpc))
    gbs = C * T * 512 * 4 / (us * 1e-6) / 1e9
    print(f"ctx-attn C={C} rpc={rpc}: {us:8.2f} us  {gbs:7.1f} GB/s (K+V bytes)")

# encoder attention
B, T = 256, 512
qkv = torch.randn(B * T, 768, device=dev)
sig = torch.randn(B, T, device=dev)
span = torch.full((B,), T, dtype=torch.int32, device=dev)
us = timeit(lambda: E.op_enc_attention(qkv, sig, span), n=10)
print(f"enc-attn B={B}: {us:9.2f} us  {4*B*8*T*T*32/(us*1e-6)/1e12:6.1f} TF/s")
