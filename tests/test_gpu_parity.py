"""HIP engine vs the oracle and the golden vectors (needs an MI355X).

Tolerances (BASELINE.json north_star): log-probs within 1e-3 (fp32), greedy
tokens identical.  The only allowed token difference is a genuine near-tie in
the oracle (top-2 log-prob margin < 1e-4), after which that row's history
diverges and is not compared further.
"""
import os

import numpy as np
import pytest
import torch

from nanodecoder_amd import synth
from tests import golden_util as gu

pytestmark = pytest.mark.gpu

LOGP_ATOL = 1e-3
TIE_MARGIN = 1e-4


def _engine(cfg, W, **kw):
    from nanodecoder_amd.engine import Engine
    return Engine(cfg, W, device=0, **kw)


def _oracle():
    from oracle import ref_cpu
    return ref_cpu


# ----------------------------------------------------------------- kernels
@pytest.mark.parametrize("M,N,K,ln,relu,res", [(4096, 768, 256, True, False, False),
                                                (16384, 512, 256, True, True, False),
                                                (16384, 512, 2048, False, False, True),
                                                (5000, 256, 2048, False, False, True),
                                                (256, 2048, 256, True, True, False),
                                                (37, 256, 256, False, False, True),
                                                (65536, 256, 256, True, True, True),      # 256x256 tiles
                                                (65529, 256, 2048, False, False, True)])  # ragged last tile
@pytest.mark.parametrize("split", [False, True])
def test_gemm_vs_fp64(M, N, K, ln, relu, res, split):
    """fp32 MFMA kernels and the split-fp16 form (hi*hi + hi*lo + lo*hi on
    fp16 MFMAs) against fp64, both to the same 2e-4 absolute bound."""
    from nanodecoder_amd.engine import op_gemm
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g) if res else None
    lg = 1 + 0.1 * torch.randn(K, generator=g) if ln else None
    lb = 0.1 * torch.randn(K, generator=g) if ln else None
    dev = torch.device("cuda", 0)
    out = op_gemm(A.to(dev), W.to(dev), b.to(dev), R.to(dev) if res else None, lg.to(dev) if ln else None,
                  lb.to(dev) if ln else None, relu, split=split).cpu().double()
    a = A.double()
    if ln:
        a = torch.nn.functional.layer_norm(a, (K,), lg.double(), lb.double(), 1e-6)
    ref = a @ W.double().t() + b.double()
    if relu:
        ref = ref.clamp_min(0)
    if res:
        ref = ref + R.double()
    assert (out - ref).abs().max().item() < 2e-4


@pytest.mark.parametrize("M,F", [(1000, 2048), (256, 2048), (131, 64), (384, 512)])
@pytest.mark.parametrize("wo", ["none", "wo", "wo_inplace", "wo_qkv"])
def test_enc_ffn_fused_vs_fp64(M, F, wo):
    """The encoder's fused FFN block (nd_op_enc_ffn: LayerNorm, W1, ReLU, W2
    and the residual in one launch, the hidden kept on chip) against fp64,
    with a ragged last 128-row block (M = 1000, 131), d_ff 64..2048: the same
    2e-4 absolute bound as the split GEMMs, and the exact row statistics it
    hands to the next LayerNorm.  wo: the attention's output projection and
    residual folded in front (nd_op_enc_ffn_wo: y = x + att Wo^T + bo never
    leaves the chip), written over the input as the engine does (inplace);
    wo_qkv: the next layer's LN + QKV projection folded behind (its q | k | v
    from the block's registers) against LN(x) Wq^T + bq in fp64."""
    from nanodecoder_amd.engine import op_enc_ffn
    g = torch.Generator().manual_seed(M + F)
    y = torch.randn(M, 256, generator=g) * 2 + 0.5
    W1 = torch.randn(F, 256, generator=g) / 16
    b1 = torch.randn(F, generator=g) * 0.1
    W2 = torch.randn(256, F, generator=g) / F ** 0.5
    b2 = torch.randn(256, generator=g) * 0.1
    lg = 1 + 0.1 * torch.randn(256, generator=g)
    lb = 0.1 * torch.randn(256, generator=g)
    att = torch.randn(M, 256, generator=g)
    Wo = torch.randn(256, 256, generator=g) / 16
    bo = torch.randn(256, generator=g) * 0.1
    dev = torch.device("cuda", 0)
    Wq = torch.randn(768, 256, generator=g) / 16
    bq = torch.randn(768, generator=g) * 0.1
    lq = 1 + 0.1 * torch.randn(256, generator=g)
    lqb = 0.1 * torch.randn(256, generator=g)
    kw = {}
    if wo != "none":
        kw = dict(att=att.to(dev), Wo=Wo.to(dev), bo=bo.to(dev), inplace=wo != "wo")
    if wo == "wo_qkv":
        kw.update(Wq=Wq.to(dev), bq=bq.to(dev), lnq_g=lq.to(dev), lnq_b=lqb.to(dev))
        x, st, ov, qkv = op_enc_ffn(*(t.to(dev) for t in (y, W1, b1, W2, b2, lg, lb)), **kw)
    else:
        x, st, ov = op_enc_ffn(*(t.to(dev) for t in (y, W1, b1, W2, b2, lg, lb)), **kw)
    torch.cuda.synchronize()
    yd = y.double()
    if wo != "none":
        yd = yd + att.double() @ Wo.double().t() + bo.double()
    h = torch.relu(torch.nn.functional.layer_norm(yd, (256,), lg.double(), lb.double(), 1e-6) @ W1.double().t()
                   + b1.double())
    ref = yd + h @ W2.double().t() + b2.double()
    got = x.cpu().double()
    assert (got - ref).abs().max().item() < 2e-4
    st = st.cpu().double()
    assert torch.allclose(st[:, 0], got.mean(1), atol=1e-5)
    assert torch.allclose(st[:, 1], ((got - got.mean(1, keepdim=True)) ** 2).sum(1), rtol=1e-4, atol=1e-3)
    assert int(ov.cpu()[0]) == 0
    if wo == "wo_qkv":
        qref = torch.nn.functional.layer_norm(ref, (256,), lq.double(), lqb.double(), 1e-6) @ Wq.double().t() \
            + bq.double()
        assert (qkv.cpu().double() - qref).abs().max().item() < 2e-4


@pytest.mark.parametrize("M,F,ns", [(5120, 2048, 6), (1024, 2048, 8), (1040, 2048, 8), (1280, 512, 3),
                                     (256, 2048, 1)])
def test_dec_ffn_split_vs_fp64(M, F, ns):
    """The beam decoder's fused FFN block (nd_op_dec_ffn: P16 rows, d_ff split
    over ns workgroups per 128-row block, partials summed in split order by the
    block's last arriver) against fp64 within the split GEMMs' 2e-4; the exact
    row statistics; three launches on the same tickets bitwise equal and the
    tickets back at zero; a ragged last row block (M = 1040); and with a skip
    vector the row blocks whose chunks are all done left untouched (rows of a
    live block computed whole)."""
    from nanodecoder_amd.engine import op_dec_ffn, pack_p16, unpack_p16
    g = torch.Generator().manual_seed(M + F + ns)
    y = torch.randn(M, 256, generator=g) * 2 + 0.5
    W1 = torch.randn(F, 256, generator=g) / 16
    b1 = torch.randn(F, generator=g) * 0.1
    W2 = torch.randn(256, F, generator=g) / F ** 0.5
    b2 = torch.randn(256, generator=g) * 0.1
    lg = 1 + 0.1 * torch.randn(256, generator=g)
    lb = 0.1 * torch.randn(256, generator=g)
    dev = torch.device("cuda", 0)
    yp = pack_p16(y.to(dev))
    args = [t.to(dev) for t in (W1, b1, W2, b2, lg, lb)]
    outs, tk = [], None
    for _ in range(3):
        x, st, ov, tk = op_dec_ffn(yp, *args, ns, tickets=tk)
        torch.cuda.synchronize()
        assert int(tk.abs().sum().item()) == 0
        outs.append(unpack_p16(x, M).cpu())
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    yd = y.double()
    h = torch.relu(torch.nn.functional.layer_norm(yd, (256,), lg.double(), lb.double(), 1e-6) @ W1.double().t()
                   + b1.double())
    ref = yd + h @ W2.double().t() + b2.double()
    got = outs[0].double()
    assert (got - ref).abs().max().item() < 2e-4
    st = st[:M].cpu().double()
    assert torch.allclose(st[:, 0], got.mean(1), atol=1e-5)
    assert torch.allclose(st[:, 1], ((got - got.mean(1, keepdim=True)) ** 2).sum(1), rtol=1e-4, atol=1e-3)
    assert int(ov.cpu()[0]) == 0
    if M >= 1024:
        # beam rows: 5 per chunk; every chunk of row block 1 done, one chunk of row block 2 alive
        rpc = 5
        done = torch.ones((M + rpc - 1) // rpc, dtype=torch.int32)
        done[: 128 // rpc] = 0
        done[(2 * 128 + 40) // rpc] = 0
        done[(3 * 128) // rpc:] = 0
        x2, _, _, tk = op_dec_ffn(yp, *args, ns, skip=done.to(dev), skip_rpc=rpc, tickets=tk)
        torch.cuda.synchronize()
        assert int(tk.abs().sum().item()) == 0
        got2 = unpack_p16(x2, M).cpu()
        dead = torch.zeros(M, dtype=torch.bool)
        for rb in range((M + 127) // 128):
            r0, r1 = rb * 128, min(M, rb * 128 + 128)
            dead[r0:r1] = bool(done[r0 // rpc:(r1 - 1) // rpc + 1].all())
        assert dead[128:256].all() and not dead[256:384].any()
        assert torch.isnan(got2[dead]).all()  # untouched (op_dec_ffn fills x with NaN)
        assert torch.equal(got2[~dead], outs[0][~dead])


@pytest.mark.parametrize("N,K,mag", [(256, 256, 1.0), (768, 256, 3e-4), (256, 2048, 40.0)])
def test_split_weight_image(N, K, mag):
    """nd_op_split_weight: hi + lo reproduces W * 2^s to 2^-21 relative (half
    an fp16 ulp of the residual), max|W| 2^s sits in [2^13, 2^14), and the
    image layout is [N][K/8][hi 8 | lo 8]."""
    from nanodecoder_amd.engine import op_split_weight
    g = torch.Generator().manual_seed(N + K)
    W = torch.randn(N, K, generator=g) * mag
    W[0, :8] = torch.tensor([0.0, -0.0, 1e-30, -1e-12, 1e-7, mag, -2 * mag, 0.5 * mag])
    Wh, sc = op_split_weight(W.to(torch.device("cuda", 0)))
    h = Wh.cpu().view(torch.float16).float().view(N, K // 8, 2, 8)
    s = 1.0 / sc
    assert 2 ** 13 <= W.abs().max().item() * s < 2 ** 14
    rec = (h[:, :, 0] + h[:, :, 1]).reshape(N, K).double() / s
    err = (rec - W.double()).abs()
    # relative to each element, with an absolute floor for the elements whose
    # residual falls into the fp16 subnormals (2^-25 of the scaled image)
    assert (err <= W.double().abs() * 2.0 ** -21 + 2.0 ** -25 / s).all(), err.max().item()


@pytest.mark.parametrize("M,N,K,res", [(256, 256, 2048, True), (256, 256, 1024, False), (1024, 256, 2048, True),
                                         (144, 256, 2048, True), (400, 512, 2048, False)])
def test_gemm_p16_splitk_vs_fp64(M, N, K, res):
    """The split-K long-K P16 GEMM (W_vo / FFN2 route at 128 < rows <= 1024):
    against fp64 within the split-fp16 bound, row partials for the next
    LayerNorm, rows past M (M not a multiple of 32) left to the padding, the
    tickets back at zero after every launch, and three launches on the same
    tickets bitwise equal (the slices are summed in slice order whichever
    workgroup arrives last)."""
    from nanodecoder_amd.engine import op_gemm_p16_splitk, op_pack_p16h, pack_p16, row_partials, unpack_p16
    g = torch.Generator().manual_seed(3 * M + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    dev = torch.device("cuda", 0)
    Wh, sc = op_pack_p16h(W.to(dev))
    Ap = pack_p16(torch.cat([A, A.new_zeros((-M) % 16, K)]).to(dev))
    Rp = pack_p16(torch.cat([R, R.new_zeros((-M) % 16, N)]).to(dev)) if res else None
    # row partials are statistics of whole 256-wide rows (the next LayerNorm's); wider outputs have none
    part_out = torch.full(((M + 15) // 16 * 16, 16, 2), float("nan"), device=dev) if N == 256 else None
    outs, tk = [], None
    for _ in range(3):
        Cp, pn, tk = op_gemm_p16_splitk(Ap, Wh, sc, b.to(dev), M, N, K, Rp, part_out, tickets=tk)
        torch.cuda.synchronize()
        assert int(tk.abs().sum().item()) == 0  # every tile's last arriver reset its ticket
        outs.append(unpack_p16(Cp, M).cpu())
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    ref = A.double() @ W.double().t() + b.double() + (R.double() if res else 0)
    assert (outs[0].double() - ref).abs().max().item() < 2e-4
    if part_out is None:
        return
    assert pn == N // 16
    want = row_partials(outs[0], pn)[:, :pn]
    got = part_out[:M, :pn].cpu()
    assert torch.allclose(got[:, :, 0], want[:, :, 0], atol=1e-5)
    assert torch.allclose(got[:, :, 1], want[:, :, 1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K,res", [(256, 256, 2048, True), (400, 256, 1024, False)])
def test_gemm_p16_splitk_f32_vs_fp64(M, N, K, res):
    """The split-K route in exact fp32 (the pool lanes' W_vo / FFN2 under
    nd_set_exact_fp32): fp32 products against fp64 within fp32 rounding of a
    K-term sum, row partials, tickets reset, repeat launches bitwise equal."""
    from nanodecoder_amd.engine import op_gemm_p16_splitk_f32, pack_p16, row_partials, unpack_p16
    g = torch.Generator().manual_seed(5 * M + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    dev = torch.device("cuda", 0)
    Wp = pack_p16(W.to(dev))
    Ap = pack_p16(torch.cat([A, A.new_zeros((-M) % 16, K)]).to(dev))
    Rp = pack_p16(torch.cat([R, R.new_zeros((-M) % 16, N)]).to(dev)) if res else None
    part_out = torch.full(((M + 15) // 16 * 16, 16, 2), float("nan"), device=dev)
    outs, tk = [], None
    for _ in range(3):
        Cp, pn, tk = op_gemm_p16_splitk_f32(Ap, Wp, b.to(dev), M, N, K, Rp, part_out, tickets=tk)
        torch.cuda.synchronize()
        assert int(tk.abs().sum().item()) == 0
        outs.append(unpack_p16(Cp, M).cpu())
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    ref = A.double() @ W.double().t() + b.double() + (R.double() if res else 0)
    assert (outs[0].double() - ref).abs().max().item() < 2e-5
    assert pn == N // 16
    want = row_partials(outs[0], pn)[:, :pn]
    got = part_out[:M, :pn].cpu()
    assert torch.allclose(got[:, :, 0], want[:, :, 0], atol=1e-5)
    assert torch.allclose(got[:, :, 1], want[:, :, 1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K,ln,relu,res,stats", [(256, 768, 256, True, False, False, False),
                                                      (256, 256, 256, False, False, True, True),
                                                      (256, 256, 256, True, False, False, False),
                                                      (256, 2048, 256, True, True, False, False),
                                                      (256, 256, 2048, False, False, True, True),
                                                      (1280, 768, 256, True, False, False, False),
                                                      (1280, 2048, 256, True, True, False, False),
                                                      (1280, 256, 256, False, False, True, True),
                                                      (1280, 256, 256, True, False, True, True),
                                                      (112, 2048, 256, True, True, False, False),
                                                      (200, 768, 256, True, False, False, False),
                                                      (40, 256, 2048, False, False, True, True),
                                                      (5120, 2048, 256, True, True, False, False),   # beam 5 x 1024
                                                      (5120, 256, 2048, False, False, True, True),
                                                      (5120, 768, 256, True, False, False, False),
                                                      (2560, 256, 256, True, False, True, True),
                                                      (5120, 256, 256, False, False, True, True),    # beam Wo (64 x 64 tiles)
                                                      (5120, 256, 256, True, False, False, False),   # beam context query
                                                      (2048, 128, 256, True, True, False, False),
                                                      (4100, 256, 256, False, False, True, True)])   # ragged last tile
@pytest.mark.parametrize("split", [False, True, "rm"])
def test_gemm_p16_vs_fp64(M, N, K, ln, relu, res, stats, split):
    """The decoder-step GEMM on the P16 layout: LN from handed-over row
    partials (affine folded on the device), relu, residual, and the output
    row partials it hands to the next LayerNorm; fp32 MFMA and split-fp16
    kernels to the same bound."""
    from nanodecoder_amd.engine import (op_fold_layernorm, op_gemm_p16, op_pack_p16h, op_split_weight, pack_p16,
                                        row_partials, unpack_p16)
    g = torch.Generator().manual_seed(7 * M + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    lg = 1 + 0.1 * torch.randn(K, generator=g)
    lb = 0.1 * torch.randn(K, generator=g)
    dev = torch.device("cuda", 0)
    Wd, bd = W.to(dev), b.to(dev)
    part_in = None
    if ln:
        Wd, bd = op_fold_layernorm(Wd, bd, lg.to(dev), lb.to(dev))
        part_in = row_partials(torch.cat([A, A.new_zeros((-M) % 16, K)]).to(dev))  # producer's hand-off
    part_out = torch.full(((M + 15) // 16 * 16, 16, 2), float("nan"), device=dev) if stats else None
    Wh, sc = op_pack_p16h(Wd) if split else (None, 1.0)
    Wr, sr = op_split_weight(Wd) if split == "rm" else (None, 1.0)  # large M: the LDS-tiled kernel on P16 operands
    Cp, pn = op_gemm_p16(pack_p16(A.to(dev)), pack_p16(Wd), bd, M, N, K, pack_p16(R.to(dev)) if res else None,
                         part_in, relu, part_out, Wh=Wh, wscale=sc, Wh_rm=Wr, wscale_rm=sr)
    out = unpack_p16(Cp, M).cpu().double()
    a = A.double()
    if ln:
        a = torch.nn.functional.layer_norm(a, (K,), lg.double(), lb.double(), 1e-6)
    ref = a @ W.double().t() + b.double()
    if relu:
        ref = ref.clamp_min(0)
    if res:
        ref = ref + R.double()
    assert (out - ref).abs().max().item() < 2e-4
    if stats:
        assert pn in (N // 16, N // 64, N // 128, N // 256)   # one partial per column tile of the kernel taken
        want = row_partials(out.float(), pn)[:, :pn]
        got = part_out[:M, :pn].cpu()
        assert torch.allclose(got[:, :, 0], want[:, :, 0], atol=1e-5)
        assert torch.allclose(got[:, :, 1], want[:, :, 1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("lg", [0, -7, -14, -20])
@pytest.mark.parametrize("M,K", [(256, 256), (256, 2048), (1280, 256)])
def test_gemm_split_small_rows_follow_the_scheme(lg, M, K):
    """Activation rows of scale 2^lg through the split-fp16 P16 GEMM (no
    LayerNorm in front: W_o / W_2 / W_vo's operands): the kernel follows the
    numpy restatement of the split (tests/test_split_fp16_scheme.py) to fp32
    accumulation -- fp16 subnormal lo parts are kept, not flushed -- so its
    error relative to the row's own output is ~2^-24 / sigma below sigma ~
    2^-3 and, added to an O(1) residual, within twice that residual's fp32
    rounding at every scale."""
    from nanodecoder_amd.engine import op_gemm_p16, op_pack_p16h, pack_p16, unpack_p16
    from tests.test_split_fp16_scheme import split_product
    N = 256
    g = torch.Generator().manual_seed(11 * M + K - lg)
    A = torch.randn(M, K, generator=g) * 2.0 ** lg
    W = torch.randn(N, K, generator=g) / 16
    R = torch.rand(M, N, generator=g) + 1.0  # a residual in [1, 2): its fp32 rounding is 2^-24 .. 2^-23
    dev = torch.device("cuda", 0)
    zero = torch.zeros(N, device=dev)
    Wh, sc = op_pack_p16h(W.to(dev))
    Ap = pack_p16(A.to(dev))
    C0 = unpack_p16(op_gemm_p16(Ap, None, zero, M, N, K, Wh=Wh, wscale=sc)[0], M).cpu().double()
    C1 = unpack_p16(op_gemm_p16(Ap, None, zero, M, N, K, pack_p16(R.to(dev)), Wh=Wh, wscale=sc)[0], M).cpu().double()
    emu = torch.from_numpy(split_product(A.numpy(), W.numpy()))
    ref = A.double() @ W.double().t()
    rms = ref.pow(2).mean(1, keepdim=True).sqrt()
    l1 = W.abs().sum(1).max().item()
    # the kernel is the scheme, to fp32 accumulation (plus 2^-30 / sigma: at sigma 2^-20, M = 1280 differs from
    # the restatement by 3.9e-6 of the row, against the scheme's own 8e-2; a flushed lo would differ by ~1e-1)
    assert ((C0 - emu).abs() / rms).max().item() < 2.0 ** -18 * (K / 256) ** 0.5 + 2.0 ** -30 / 2.0 ** lg
    # the scheme's error: relative to the row below 4e-6 + 2^-23 / sigma ...
    assert ((C0 - ref).abs() / rms).max().item() < 4e-6 + 2.0 ** -23 / 2.0 ** lg
    # ... and scale-free in absolute terms: rows of scale <= 2^-7 added to a residual in [1, 2) stay within
    # the residual sum's own rounding (at scale 1 the output's own fp32 rounding dominates: the line above)
    if lg <= -7:
        assert (C1 - (ref + R.double())).abs().max().item() < 2.0 ** -23 + 2.0 ** -24 * l1 * (K / 256) ** 0.5


@pytest.mark.parametrize("step", [0, 1, 31, 32, 63, 64, 99, 127, 128, 200, 300, 511])
@pytest.mark.parametrize("beam", [False, True])
def test_dec_self_attention_vs_fp64(step, beam):
    """Decoder self-attention step (multi_headed_attn.py:124-141 + :167-179):
    keys 0..step-1 from the cache through the ancestry table (beam) or the
    row's own slot, key `step` from this step's k/v, which is also appended
    to the row's slot.  Steps past 256 on a 512-step cache (max_length up to
    512: three and four key passes)."""
    from nanodecoder_amd.engine import op_dec_self_attention
    R, S = 37, (256 if step < 256 else 512)
    g = torch.Generator().manual_seed(step + 1000 * beam)
    qkv = torch.randn(R, 768, generator=g)
    cache = torch.randn(R, S, 512, generator=g)
    anc = torch.randint(0, R, (R, S), generator=g, dtype=torch.int32) if beam else None
    dev = torch.device("cuda", 0)
    cd = cache.to(dev)
    out = op_dec_self_attention(qkv.to(dev), cd, step, anc=anc.to(dev) if beam else None,
                                anc_ld=S if beam else 0).cpu().double()
    q = qkv[:, :256].double().view(R, 8, 32) / np.float32(np.sqrt(32.0))
    ref = torch.empty(R, 256, dtype=torch.float64)
    for r in range(R):
        slots = anc[r, :step].long() if beam else torch.full((step,), r, dtype=torch.long)
        kv = cache[slots, torch.arange(step)].double()                       # [step, 512]
        k = torch.cat([kv[:, :256], qkv[r:r + 1, 256:512].double()]).view(-1, 8, 32)
        v = torch.cat([kv[:, 256:], qkv[r:r + 1, 512:].double()]).view(-1, 8, 32)
        p = torch.softmax(torch.einsum("hd,thd->ht", q[r], k), dim=-1)
        ref[r] = torch.einsum("ht,thd->hd", p, v).reshape(256)
    assert (out - ref).abs().max().item() < 1e-5
    appended = cd[torch.arange(R), step].cpu()
    assert torch.equal(appended, qkv[:, 256:])


@pytest.mark.parametrize("rpc,step", [(5, 0), (5, 1), (5, 47), (2, 130), (6, 63), (3, 255), (5, 256), (5, 300),
                                      (6, 511), (8, 100), (7, 300)])
def test_dec_self_attention_beam_vs_fp64(rpc, step):
    """Beam rows' self-attention on the chunk-per-workgroup kernel: the rows of
    a chunk share most of their history (slots from the chunk's rows, with
    divergent tails), keys 0..step-1 through each row's ancestry, key `step`
    from this step's k/v, appended to the row's own slot; rows of a finished
    chunk untouched (multi_headed_attn.py:124-141, translate/translator.py:
    793-823).  Tolerance as the per-row form's test (1e-5).  Steps from 256
    on a 512-step cache: the keys past 64 per wave take the second slot table."""
    from nanodecoder_amd.engine import op_dec_self_attention_beam
    C, S = 7, (256 if step < 256 else 512)
    R = C * rpc
    g = torch.Generator().manual_seed(step + 100 * rpc)
    qkv = torch.randn(R, 768, generator=g)
    cache = torch.randn(R, S, 512, generator=g)
    anc = torch.empty(R, S, dtype=torch.int32)
    for c in range(C):
        split = int(torch.randint(0, max(step, 1), (1,), generator=g))  # shared prefix, then per-row slots
        for j in range(rpc):
            r = c * rpc + j
            anc[r, :split] = c * rpc
            anc[r, split:] = torch.randint(0, rpc, (S - split,), generator=g, dtype=torch.int32) + c * rpc
    done = torch.zeros(C, dtype=torch.int32)
    done[3] = 1
    dev = torch.device("cuda", 0)
    cd = cache.to(dev)
    out = op_dec_self_attention_beam(qkv.to(dev), cd, step, anc.to(dev), rpc, done.to(dev)).cpu().double()
    q = qkv[:, :256].double().view(R, 8, 32) / np.float32(np.sqrt(32.0))
    for r in range(R):
        if done[r // rpc]:
            continue
        slots = anc[r, :step].long()
        kv = cache[slots, torch.arange(step)].double()
        k = torch.cat([kv[:, :256], qkv[r:r + 1, 256:512].double()]).view(-1, 8, 32)
        v = torch.cat([kv[:, 256:], qkv[r:r + 1, 512:].double()]).view(-1, 8, 32)
        p = torch.softmax(torch.einsum("hd,thd->ht", q[r], k), dim=-1)
        ref = torch.einsum("ht,thd->hd", p, v).reshape(256)
        assert (out[r] - ref).abs().max().item() < 1e-5, (r, step)
    live = torch.tensor([not done[r // rpc] for r in range(R)])
    appended = cd[torch.arange(R), step].cpu()
    assert torch.equal(appended[live], qkv[live, 256:])
    assert torch.equal(appended[~live], cache[~live, step])  # a finished chunk's rows are not written


@pytest.mark.parametrize("rpc,beam", [(1, False), (1, True), (5, True), (2, True)])
def test_dec_self_attention_q24_history_vs_fp64(rpc, beam):
    """The engine's default self-attention history: every step quantises its
    k|v to the 24-bit rows and appends them; 70 steps run in order (the
    per-row kernel's 4- and 8-wave forms, one and two key passes are crossed
    at 16 / 32 / 64 keys) and each step's output is held against fp64 over
    the fp32 k|v every earlier step appended (beam: through a fixed ancestry,
    a shared prefix then per-row slots of the chunk).  Tolerance 2e-5 of the
    values' magnitude (a 24-bit element carries 2^-23 of its head's largest
    value, as the context image)."""
    from nanodecoder_amd.engine import op_dec_self_attention_q24
    C, S, steps = 9, 128, 70
    R = C * rpc
    g = torch.Generator().manual_seed(17 + rpc + 10 * beam)
    qkv = [torch.randn(R, 768, generator=g) for _ in range(steps)]
    qkv[40][:, 256 + 32: 256 + 64] *= 1e3   # one head of one step's keys 1000x the rest
    anc = None
    if beam:
        anc = torch.empty(R, S, dtype=torch.int32)
        for c in range(C):
            for j in range(rpc):
                r = c * rpc + j
                anc[r, :20] = c * rpc
                anc[r, 20:] = torch.randint(0, rpc, (S - 20,), generator=g, dtype=torch.int32) + c * rpc
    dev = torch.device("cuda", 0)
    cache = torch.zeros(R, S, 1600, dtype=torch.uint8, device=dev)
    ad = anc.to(dev) if beam else None
    for step in range(steps):
        out = op_dec_self_attention_q24(qkv[step].to(dev), cache, step, anc=ad, rpc=rpc).cpu().double()
        if step not in (0, 1, 15, 16, 17, 33, 40, 41, 64, 65, 69):
            continue
        q = qkv[step][:, :256].double().view(R, 8, 32) / np.float32(np.sqrt(32.0))
        for r in range(R):
            src = [(int(anc[r, t]) if beam else r) for t in range(step)] + [r]
            kv = torch.stack([qkv[t][src[t], 256:].double() for t in range(step + 1)])   # [step + 1, 512]
            k, v = kv[:, :256].view(-1, 8, 32), kv[:, 256:].view(-1, 8, 32)
            p = torch.softmax(torch.einsum("hd,thd->ht", q[r], k), dim=-1)
            ref = torch.einsum("ht,thd->hd", p, v).reshape(256)
            err = (out[r] - ref).abs().max().item()
            assert err < 2e-5 * max(1.0, v.abs().max().item()), (r, step, err)


@pytest.mark.parametrize("scale", [1.0, 4.0, "rising"])
def test_enc_attention_vs_oracle(scale):
    """Split-fp16 encoder attention against the oracle's attend: masked keys,
    an all-masked chunk, a ragged span; ``scale`` 4 spreads the scores over
    ~±60 so the lazy running maximum rescales mid-row, ``rising`` makes every
    query's scores grow along the keys (a rescale in most tiles)."""
    from nanodecoder_amd.engine import op_enc_attention
    ref = _oracle()
    B, T = 3, 512
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(B * T, 768, generator=g)
    if scale == "rising":
        qkv[:, :256] = qkv[:, :256].abs() * 0.5 + 1.0                       # queries > 0
        ramp = torch.linspace(0.0, 3.0, T).repeat(B)[:, None]
        qkv[:, 256:512] = qkv[:, 256:512] * 0.2 + ramp                      # keys rise with t
    else:
        qkv = qkv * scale
    sig = torch.randn(B, T, generator=g)
    sig[0, ::7] = 0.0          # masked keys
    sig[2, :] = 0.0            # every key masked -> uniform attention
    span = torch.tensor([512, 300, 512], dtype=torch.int32)
    dev = torch.device("cuda", 0)
    out = op_enc_attention(qkv.to(dev), sig.to(dev), span.to(dev)).cpu()
    m = ref.RefModel.__new__(ref.RefModel)
    m.h, m.dh, m.d = 8, 32, 256
    for b in range(B):
        L = int(span[b])
        rows = qkv[b * T: b * T + L]
        q, k, v = (m._heads(rows[None, :, i * 256:(i + 1) * 256]) for i in range(3))
        mask = (sig[b, :L] == 0).view(1, 1, L)
        c, _ = m.attend(q, k, v, mask)
        exp = m._unheads(c)[0]
        tol = 1e-4 * (4.0 if scale == 4.0 else 1.0) * max(1.0, exp.abs().max().item() / 4.0)
        assert (out[b * T: b * T + L] - exp).abs().max().item() < tol, b


@pytest.mark.parametrize("T,grid", [(512, 0), (200, 0), (37, 0), (512, 5), (512, 7), (200, 1), (300, 0), (384, 6),
                                    (448, 0), (300, 4)])
def test_mem_attention_vs_fp64(T, grid):
    """Memory-bank context attention (dec_mem_attention_kernel) against an
    fp64 softmax(q' M^T) M per head, with ragged spans (tile/wave boundaries,
    single key, waves owning no key), pad-masked keys and an all-masked chunk;
    grid > 0: that many workgroups walk the 12 chunks (the pool lanes' form)."""
    from nanodecoder_amd.engine import op_dec_mem_attention, op_memory_pack, pack_p16, unpack_p16
    rng = np.random.default_rng(3)
    C, PAD = 12, 1.0
    spans = np.array([T, 1, min(T, 64), min(T, 65), min(T, 70), min(T, 8), min(T, 9), T, max(1, T - 3),
                      min(T, 130), T, T], np.int32)
    sig = rng.standard_normal((C, T)).astype(np.float32)
    sig[2, ::5] = PAD                      # pad-masked keys
    sig[7, :] = PAD                        # every key masked -> uniform over the span
    x = rng.standard_normal((C * T, 256)).astype(np.float32)
    q = (rng.standard_normal((C, 2048)) * 0.3).astype(np.float32)
    dev = torch.device("cuda", 0)
    mem = op_memory_pack(torch.from_numpy(x).to(dev), C, T)
    out = op_dec_mem_attention(pack_p16(torch.from_numpy(q).to(dev)), mem, torch.from_numpy(sig).to(dev),
                               torch.from_numpy(spans).to(dev), PAD, 1, grid=grid)
    got = unpack_p16(out, C).cpu().numpy()
    for c in range(C):
        L = int(spans[c])
        M = x[c * T: c * T + L].astype(np.float64)
        for h in range(8):
            s = M @ q[c, h * 256:(h + 1) * 256].astype(np.float64)
            s[sig[c, :L] == PAD] = -1e18
            p = np.exp(s - s.max())
            want = (p / p.sum()) @ M
            err = np.abs(got[c, h * 256:(h + 1) * 256] - want).max()
            assert err < 2e-5, (c, h, L, err)


@pytest.mark.parametrize("T,ln,grid", [(512, True, 0), (480, False, 0), (449, True, 0), (512, True, 5),
                                       (512, False, 1), (512, True, 8), (480, False, 6), (384, True, 0),
                                       (300, False, 0), (300, True, 6), (200, True, 0), (100, False, 5)])
def test_bank_d8_vs_fp64(T, ln, grid):
    """24-bit digit-bank attention (bank_pack_d8 + dec_bank_d8_kernel, the
    greedy path at 512-sample chunks) against an fp64 softmax(q' M^T) M per
    head: ragged spans (key-block / wave boundaries, single key, waves owning
    no key), pad-masked keys, an all-masked chunk, a peaked chunk whose scores
    climb past the lazy-rescale threshold, with and without the LayerNorm
    (grid > 0: that many workgroups walk the 12 chunks, nd_set_bank_grid's
    form; 5 leaves a ragged last round; 8 and 6 take the two-chunk
    straight-line form, the second chunk's head loaded during the first
    one's merge; T <= 384: the launch streams only the first ceil(T / 128)
    key blocks of each wave, the reference authors' T = 300 among them), plus rows of very
    different magnitude (per-row exponents 2^e_t far below the chunk's
    largest) and a head of q' a thousand times the others (per-head digit
    scales).  Tolerance: 2e-5 relative to the output's magnitude (digits
    carry 22-23 bits per row)."""
    from nanodecoder_amd.engine import op_bank_pack_d8, op_dec_bank_d8, unpack_p16
    rng = np.random.default_rng(7)
    C, PAD = 12, 1.0
    spans = np.array([T, 1, 64, 65, 16, 17, 8, T, T - 3, 130, 300, T], np.int32)
    sig = rng.standard_normal((C, T)).astype(np.float32)
    sig[2, ::5] = PAD                      # pad-masked keys
    sig[7, :] = PAD                        # every key masked -> uniform over the span
    x = rng.standard_normal((C * T, 256)).astype(np.float32)
    q = (rng.standard_normal((C, 2048)) * 0.3).astype(np.float32)
    q[11] *= 8.0                           # scores spread ~+-50: running-maximum rescales
    x[11 * T + min(400, T - 1)] *= 4.0     # a late key far above the first blocks' maximum
    x[3 * T: 4 * T: 3] *= 1e-3             # rows of very different magnitude in one chunk
    x[9 * T + 7] = 0.0                     # an all-zero row
    q[5, 3 * 256:4 * 256] *= 1e3           # one head's q' far above the others
    q[6, 5 * 256:6 * 256] = 0.0            # a zero head
    g = (rng.random(256) + 0.5).astype(np.float32)
    b = (rng.standard_normal(256) * 0.1).astype(np.float32)
    dev = torch.device("cuda", 0)
    xt = torch.from_numpy(x).to(dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    span_d = torch.from_numpy(spans).to(dev)
    if ln:
        bank = op_bank_pack_d8(xt, C, T, torch.from_numpy(g).to(dev), torch.from_numpy(b).to(dev), ovf=ovf,
                               span=span_d)
        mu = x.mean(1, keepdims=True)
        var = ((x - mu) ** 2).mean(1, keepdims=True)
        xm = ((x - mu) / np.sqrt(var + 1e-6) * g + b).astype(np.float64)
    else:
        bank = op_bank_pack_d8(xt, C, T, ovf=ovf, span=span_d)
        xm = x.astype(np.float64)
    out = op_dec_bank_d8(torch.from_numpy(q).to(dev), bank, torch.from_numpy(sig).to(dev),
                         torch.from_numpy(spans).to(dev), PAD, ovf=ovf, grid=grid)
    got = unpack_p16(out, C).cpu().numpy()
    assert int(ovf.item()) == 0
    for c in range(C):
        L = min(int(spans[c]), T)  # the kernel attends min(span, T) keys
        M = xm[c * T: c * T + L]
        for h in range(8):
            s = M @ q[c, h * 256:(h + 1) * 256].astype(np.float64)
            s[sig[c, :L] == PAD] = -1e18
            p = np.exp(s - s.max())
            want = (p / p.sum()) @ M
            err = np.abs(got[c, h * 256:(h + 1) * 256] - want).max()
            assert err < 2e-5 * max(1.0, np.abs(want).max()), (c, h, L, err)


def test_ctx_pack_q24_bitexact():
    """The 24-bit context K/V image (nd_op_ctx_pack_q24) equals the numpy
    restatement byte for byte (tests/test_ctx_q24_scheme.py): heads from 1e-30
    to 1e30, a zero head, values that round to the clamp, rows past a span
    left unwritten; a non-finite head gets a NaN scale."""
    from nanodecoder_amd.engine import op_ctx_pack_q24
    from tests.test_ctx_q24_scheme import pack_q24
    rng = np.random.default_rng(23)
    B, T, Ld = 6, 512, 3
    kv = rng.standard_normal((B * T, Ld * 512)).astype(np.float32)
    kv[5, :32] = 0.0
    kv[7] *= np.float32(1e-30)
    kv[8] *= np.float32(1e30)
    kv[9, 64:96] = np.float32(1.0) - np.float32(2.0 ** -24)
    kv[10, 600:632] *= 1e-3
    kv[10, 600] = 7e4
    spans = np.array([T, 1, 300, T - 1, 17, T], np.int32)
    dev = torch.device("cuda", 0)
    got = op_ctx_pack_q24(torch.from_numpy(kv).to(dev), Ld * 512, Ld, torch.from_numpy(spans).to(dev), B, T)
    torch.cuda.synchronize()
    got = got.cpu().numpy()
    want = pack_q24(kv, Ld * 512, Ld, spans, B, T)
    bad = np.argwhere(got != want)
    assert bad.size == 0, bad[:8]
    kv[3 * T + 2, 256 + 40] = np.nan  # v of head 1, layer 0
    got = op_ctx_pack_q24(torch.from_numpy(kv).to(dev), Ld * 512, Ld, torch.from_numpy(spans).to(dev), B, T)
    sc = got[0, 3 * T + 2, 1536:1600].cpu().numpy().view(np.float32).reshape(8, 2)
    assert np.isnan(sc[1, 1]) and np.isfinite(np.delete(sc.reshape(-1), 3)).all()


@pytest.mark.parametrize("norm", [False, True])
def test_gemm_q24_epilogue_equals_pack(norm):
    """The engine's K / V projection writing the 24-bit image from its epilogue
    (nd_op_gemm_split_q24) equals the fp32 GEMM's output packed by
    nd_op_ctx_pack_q24, byte for byte (same 256 x 256 tiles, same quantiser);
    M not a multiple of the tile (rows past M untouched)."""
    from nanodecoder_amd.engine import op_ctx_pack_q24, op_gemm, op_gemm_split_q24
    rng = np.random.default_rng(7 + int(norm))
    M, K, Ld = 64 * 512 + 100, 256, 3
    dev = torch.device("cuda", 0)
    A = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32)).to(dev)
    W = torch.from_numpy((rng.standard_normal((Ld * 512, K)) / 16).astype(np.float32)).to(dev)
    b = torch.from_numpy((rng.standard_normal(Ld * 512) * 0.1).astype(np.float32)).to(dev)
    C = op_gemm(A, W, b, norm=norm, split=True)
    img = op_gemm_split_q24(A, W, b, norm=norm)
    span = torch.full((1,), M, dtype=torch.int32, device=dev)
    want = op_ctx_pack_q24(C, Ld * 512, Ld, span, 1, M)
    torch.cuda.synchronize()
    bad = (img != want).nonzero()
    assert bad.numel() == 0, bad[:8].tolist()


@pytest.mark.parametrize("rpc", [1, 2, 5, 6, 7, 8])
@pytest.mark.parametrize("q24", [False, True])
def test_ctx_attention_vs_fp64(rpc, q24):
    """The beam's context attention (dec_ctx_attention_kernel, fp32 K/V or the
    24-bit image) against fp64 softmax(q k^T / sqrt(32), mask) v per row and
    head (multi_headed_attn.py:142-177): ragged spans (1, a partial block,
    512), pad-masked keys, an all-masked chunk, a late key far above the
    first keys' maximum, heads 1e3 apart, a zero q row.  Tolerance: 1e-5 of
    the output's magnitude (fp32 K/V), 2e-5 on the image (its elements carry
    2^-23 of their head's largest value)."""
    from nanodecoder_amd.engine import (op_ctx_pack_q24, op_dec_ctx_attention, op_dec_ctx_attention_q24,
                                        pack_p16, unpack_p16)
    rng = np.random.default_rng(31 + rpc)
    C, T, Ld, PAD = 7, 512, 3, 1.0
    spans = np.array([T, 1, 15, 300, T, T - 5, 77], np.int32)
    sig = rng.standard_normal((C, T)).astype(np.float32)
    sig[2, ::3] = PAD
    sig[4, :] = PAD
    kv = rng.standard_normal((C * T, Ld * 512)).astype(np.float32)
    kv[0 * T + 450, 512:1024] *= 6.0            # layer 1: a late key past the first blocks' maximum
    kv[5 * T: 6 * T, 512 + 64: 512 + 96] *= 1e3  # layer 1, head 2 of chunk 5
    R = C * rpc
    q = rng.standard_normal((R, 256)).astype(np.float32)
    q[6 * rpc] = 0.0
    dev = torch.device("cuda", 0)
    kvd = torch.from_numpy(kv).to(dev)
    sp = torch.from_numpy(spans).to(dev)
    sg = torch.from_numpy(sig).to(dev)
    qp = pack_p16(torch.from_numpy(q).to(dev))
    layer = 1
    if q24:
        img = op_ctx_pack_q24(kvd, Ld * 512, Ld, sp, C, T)
        out = op_dec_ctx_attention_q24(qp, img, layer, sg, sp, PAD, rpc)
    else:
        out = op_dec_ctx_attention(qp, kvd, Ld * 512, layer * 512, sg, sp, PAD, rpc, packed=True)
    torch.cuda.synchronize()
    got = unpack_p16(out, R).cpu().numpy()
    K = kv[:, layer * 512: layer * 512 + 256].astype(np.float64)
    V = kv[:, layer * 512 + 256: (layer + 1) * 512].astype(np.float64)
    tol = 2e-5 if q24 else 1e-5
    for c in range(C):
        L = int(spans[c])
        for j in range(rpc):
            r = c * rpc + j
            for h in range(8):
                hs = slice(h * 32, (h + 1) * 32)
                s = K[c * T: c * T + L, hs] @ q[r, hs].astype(np.float64) / np.sqrt(32)
                s[sig[c, :L] == PAD] = -1e18
                p = np.exp(s - s.max())
                want = (p / p.sum()) @ V[c * T: c * T + L, hs]
                err = np.abs(got[r, hs] - want).max()
                assert err < tol * max(1.0, np.abs(V[c * T: c * T + L, hs]).max()), (c, j, h, L, err)


def test_alive_list():
    """nd_op_alive_list: the chunks not done, ascending, then -1; more alive
    than slots raises the guard word."""
    from nanodecoder_amd.engine import op_alive_list
    dev = torch.device("cuda", 0)
    done = np.ones(200, np.int32)
    alive = [0, 5, 63, 64, 65, 127, 128, 199]
    done[alive] = 0
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    got = op_alive_list(torch.from_numpy(done).to(dev), 13, ovf).cpu().numpy()
    assert got.tolist() == alive + [-1] * 5 and int(ovf.item()) == 0
    got = op_alive_list(torch.from_numpy(done).to(dev), 5, ovf).cpu().numpy()
    assert got.tolist() == alive[:5] and int(ovf.item()) == 1


@pytest.mark.parametrize("rpc,nsplit,q24", [(5, 16, True), (5, 16, False), (2, 7, True), (6, 32, True), (5, 1, True),
                                           (8, 16, True), (7, 8, False)])
def test_ctx_attention_tail_list_split(rpc, nsplit, q24):
    """The --fast beam tail's context attention: workgroups over a chunk list
    only, each chunk's keys in nsplit workgroups combined by a second launch,
    equal to the one-workgroup form within fp32 rounding and to fp64; rows of
    unlisted and done chunks untouched.  Spans of 1 key (most splits empty),
    a partial block, 512; an all-masked chunk; a late key far above the
    first keys' maximum (the splits' maxima differ by far)."""
    from nanodecoder_amd.engine import (op_ctx_pack_q24, op_dec_ctx_attention, op_dec_ctx_attention_list,
                                        op_dec_ctx_attention_q24, pack_p16, unpack_p16)
    rng = np.random.default_rng(41 + rpc + nsplit)
    C, T, Ld, PAD = 12, 512, 3, 1.0
    spans = np.array([T, 1, 15, 300, T, T - 5, 77, T, 2, 511, 40, T], np.int32)
    sig = rng.standard_normal((C, T)).astype(np.float32)
    sig[4, :] = PAD
    sig[7, ::2] = PAD
    kv = rng.standard_normal((C * T, Ld * 512)).astype(np.float32)
    kv[0 * T + 480, 0:256] *= 8.0
    kv[11 * T + 3, 0:256] *= 8.0
    R = C * rpc
    q = rng.standard_normal((R, 256)).astype(np.float32)
    done = np.zeros(C, np.int32)
    done[5] = 1
    listed = [0, 1, 2, 3, 4, 5, 7, 8, 9, 11]   # 6 and 10 not listed
    clist = np.array(listed + [-1, -1], np.int32)
    dev = torch.device("cuda", 0)
    kvd = torch.from_numpy(kv).to(dev)
    sp = torch.from_numpy(spans).to(dev)
    sg = torch.from_numpy(sig).to(dev)
    qp = pack_p16(torch.from_numpy(q).to(dev))
    dn = torch.from_numpy(done).to(dev)
    if q24:
        img = op_ctx_pack_q24(kvd, Ld * 512, Ld, sp, C, T)
        whole = op_dec_ctx_attention_q24(qp, img, 0, sg, sp, PAD, rpc)
        got = op_dec_ctx_attention_list(qp, img, 1600, 0, sg, sp, PAD, rpc, torch.from_numpy(clist).to(dev),
                                        nsplit, q24=True, done=dn)
    else:
        whole = op_dec_ctx_attention(qp, kvd, Ld * 512, 0, sg, sp, PAD, rpc, packed=True)
        got = op_dec_ctx_attention_list(qp, kvd, Ld * 512, 0, sg, sp, PAD, rpc, torch.from_numpy(clist).to(dev),
                                        nsplit, done=dn)
    torch.cuda.synchronize()
    got = unpack_p16(got, R).cpu().numpy()
    whole = unpack_p16(whole, R).cpu().numpy()
    K = kv[:, 0:256].astype(np.float64)
    V = kv[:, 256:512].astype(np.float64)
    for c in range(C):
        rows = slice(c * rpc, (c + 1) * rpc)
        if c not in listed or done[c]:
            assert not got[rows].any(), c
            continue
        assert np.abs(got[rows] - whole[rows]).max() <= 2e-6 * max(1.0, np.abs(whole[rows]).max()), c
        L = int(spans[c])
        for j in range(rpc):
            r = c * rpc + j
            for h in range(8):
                hs = slice(h * 32, (h + 1) * 32)
                s = K[c * T: c * T + L, hs] @ q[r, hs].astype(np.float64) / np.sqrt(32)
                s[sig[c, :L] == PAD] = -1e18
                p = np.exp(s - s.max())
                want = (p / p.sum()) @ V[c * T: c * T + L, hs]
                err = np.abs(got[r, hs] - want).max()
                assert err < 2e-5 * max(1.0, np.abs(V[c * T: c * T + L, hs]).max()), (c, j, h, L, err)


def test_engine_reports_bank_form():
    """A greedy call at 512-sample chunks streams the 24-bit digit bank by
    default (nd_bank_form 2), exact fp32 the fp32 bank (0).  The digit bank's end-to-end parity is the golden
    and config tests, which run on it."""
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    sig = synth.synth_chunk_batch(8, 512, seed=5)
    lens = np.full(8, 512, np.int32)
    eng = _engine(cfg, W, max_batch=8, max_steps=20, max_beam=3)
    eng.translate_greedy(sig, lens, lens, max_len=20)
    assert eng.bank_form() == 2
    eng.set_exact_fp32(True)
    eng.translate_greedy(sig, lens, lens, max_len=20)
    assert eng.bank_form() == 0
    # beam rows: the 24-bit context K/V (3) by default, fp32 K/V in exact fp32 (0)
    eng.translate_beam(sig, lens, lens, beam=3, max_len=20)
    assert eng.bank_form() == 0
    eng.set_exact_fp32(False)
    eng.translate_beam(sig, lens, lens, beam=3, max_len=20)
    assert eng.bank_form() == 3
    eng.close()


# ----------------------------------------------------------------- golden
@pytest.mark.parametrize("name", ["transformer_greedy", "transformer_pe_short", "nano_greedy"])
def test_encoder_memory_vs_golden(name):
    z, meta = gu.load(name)
    cfg, W = gu.model_for(meta)
    eng = _engine(cfg, W, max_batch=8, max_steps=100)
    chunks = gu.chunks_of(z)
    T = int(z["T"])
    from nanodecoder_amd.engine import pad_chunks
    sig, lens = pad_chunks(chunks, T)
    spans = np.full(len(chunks), T, np.int32)
    mem = eng.encode(sig, lens, spans).cpu().numpy()            # [B, T, d]
    sub = mem.transpose(1, 0, 2)[:: meta["mem_stride"]]
    assert np.abs(sub - z["memory_sub"]).max() < 1e-4


@pytest.mark.parametrize("name", ["transformer_greedy", "transformer_pe_short", "nano_greedy", "transformer_aan",
                                  "transformer_cpg"])
@pytest.mark.parametrize("graphs,ctx_path", [(True, 0), (False, 0), (True, 1)])
def test_greedy_vs_golden(name, graphs, ctx_path):
    """ctx_path 0: memory-bank context attention, 1: per-layer K/V form."""
    z, meta = gu.load(name)
    cfg, W = gu.model_for(meta)
    g = meta["greedy"]
    eng = _engine(cfg, W, max_batch=8, max_steps=g["max_length"], graphs=graphs)
    eng.set_ctx_path(ctx_path)
    from nanodecoder_amd.engine import pad_chunks
    chunks = gu.chunks_of(z)
    T = int(z["T"])
    sig, lens = pad_chunks(chunks, T)
    spans = np.full(len(chunks), T, np.int32)
    r = eng.translate_greedy(sig, lens, spans, max_len=g["max_length"], min_len=g.get("min_length", 0),
                             return_logp=True)
    lp = r["logp"].cpu().numpy()
    assert gu.logp_close(lp, z["logp"], atol=LOGP_ATOL).all(), np.abs(lp - z["logp"]).max()
    assert (r["tokens"].cpu().numpy() == z["tokens"]).all()
    assert np.abs(r["scores"].cpu().numpy() - z["scores"]).max() < LOGP_ATOL


@pytest.mark.parametrize("graphs,ctx_path", [(True, 0), (False, 0), (True, 1)])
def test_greedy_attention_vs_golden(graphs, ctx_path):
    """-attn_debug attention (the last layer's head-0 context attention per
    step) against the reference's return_attention output, memory-bank and
    K/V forms."""
    z, meta = gu.load("transformer_pe_short")
    cfg, W = gu.model_for(meta)
    g = meta["greedy"]
    eng = _engine(cfg, W, max_batch=8, max_steps=g["max_length"], graphs=graphs)
    eng.set_ctx_path(ctx_path)
    from nanodecoder_amd.engine import pad_chunks
    chunks = gu.chunks_of(z)
    T = int(z["T"])
    sig, lens = pad_chunks(chunks, T)
    spans = np.full(len(chunks), T, np.int32)
    r = eng.translate_greedy(sig, lens, spans, max_len=g["max_length"], min_len=g.get("min_length", 0),
                             return_attn=True)
    at = r["attn"].cpu().numpy()
    assert (r["tokens"].cpu().numpy() == z["tokens"]).all()
    for i, L in enumerate(z["lengths"]):
        assert np.abs(at[i, :, :L] - z["attn"][i, :, :L]).max() < 1e-4, i


@pytest.mark.parametrize("name,which", [("transformer_beam", ""), ("transformer_beam", "2"),
                                        ("transformer_aan", ""), ("transformer_cpg", "")])
def test_beam_vs_golden(name, which):
    """--fast beam (average self-attention included: its running average
    follows the beam ancestry)."""
    z, meta = gu.load(name)
    cfg, W = gu.model_for(meta)
    kw = meta["beam" + which]
    eng = _engine(cfg, W, max_batch=8, max_steps=kw["max_length"], max_beam=kw["beam_size"])
    from nanodecoder_amd.engine import pad_chunks
    chunks = gu.chunks_of(z)
    sig, lens = pad_chunks(chunks, 512)
    spans = np.full(len(chunks), 512, np.int32)
    r = eng.translate_beam(sig, lens, spans, beam=kw["beam_size"], n_best=kw["n_best"], max_len=kw["max_length"],
                           min_len=kw.get("min_length", 0))
    tok, sc, ln = (r[k].cpu().numpy() for k in ("tokens", "scores", "lens"))
    assert (ln == z["beam_lens" + which]).all(), (ln, z["beam_lens" + which])
    for i in range(len(chunks)):
        for nb in range(kw["n_best"]):
            L = ln[i, nb]
            assert (tok[i, nb, :L] == z["beam_tokens" + which][i, nb, :L]).all()
    assert np.abs(sc - z["beam_scores" + which]).max() < 1e-3


@pytest.mark.parametrize("name,which", [("transformer_classic_beam", "classic"),
                                        ("transformer_classic_beam", "classic2"),
                                        ("transformer_classic_beam_mid", "classic")])
def test_classic_beam_vs_golden(name, which):
    """The classic onmt Beam (no --fast) against the reference's own
    _translate_batch: tokens, lengths (EOS included) and global scores."""
    z, meta = gu.load(name)
    cfg, W = gu.model_for(meta)
    kw = meta[which]
    eng = _engine(cfg, W, max_batch=8, max_steps=kw["max_length"], max_beam=kw["beam_size"])
    from nanodecoder_amd.engine import pad_chunks
    chunks = gu.chunks_of(z)
    sig, lens = pad_chunks(chunks, 512)
    spans = np.full(len(chunks), 512, np.int32)
    r = eng.translate_beam_classic(sig, lens, spans, beam=kw["beam_size"], n_best=kw["n_best"],
                                   length_penalty=kw.get("length_penalty", "none"), alpha=kw.get("alpha", 0.0),
                                   max_len=kw["max_length"], min_len=kw.get("min_length", 0))
    tok, sc, ln = (r[k].cpu().numpy() for k in ("tokens", "scores", "lens"))
    assert (ln == z[which + "_lens"]).all(), (ln, z[which + "_lens"])
    for i in range(len(chunks)):
        for nb in range(kw["n_best"]):
            L = ln[i, nb]
            assert (tok[i, nb, :L] == z[which + "_tokens"][i, nb, :L]).all()
    assert np.abs(sc - z[which + "_scores"]).max() < 1e-3


@pytest.mark.parametrize("name,which,fast", [("transformer_beam_attn", "beam", True),
                                             ("transformer_beam_attn", "classic", False),
                                             ("transformer_classic_ext", "classic", False),
                                             ("transformer_classic_ext", "classic2", False),
                                             ("transformer_classic_cov", "classic", False),
                                             ("transformer_classic_cov", "classic2", False),
                                             ("transformer_classic_cov", "classic3", False)])
def test_beam_options_vs_golden(name, which, fast):
    """Through the Translator (translate_batch on the reference batch layout):
    -attn_debug with --fast and classic beam search (each hypothesis' head-0
    attention rows, cut at memory_lengths[i] as the reference indexes it),
    the classic Beam's n-gram blocking (with exclusion tokens) and coverage
    penalties (wu / summary, stepwise or at scoring time, the scorer's
    in-place update of beam.scores) against the reference's own runs.
    Tolerances: scores 1e-3 absolute + 1e-5 relative (coverage sums run over
    512 keys in another order), attention 1e-5.  A chunk whose every beam is
    blocked (all candidates -10e20) is compared on its score only: the
    reference's choice among equal candidates is torch's CPU topk order."""
    import types
    import torch
    from nanodecoder_amd.translator import Translator
    z, meta = gu.load(name)
    cfg, W = gu.model_for(meta)
    kw = meta[which]
    eng = _engine(cfg, W, max_batch=8, max_steps=kw["max_length"], max_beam=kw["beam_size"])
    opt = types.SimpleNamespace(
        gpu=0, n_best=kw["n_best"], max_length=kw["max_length"], min_length=kw.get("min_length", 0),
        beam_size=kw["beam_size"], fast=fast, alpha=kw.get("alpha", 0.0), beta=kw.get("beta", 0.0),
        length_penalty=kw.get("length_penalty", "none"), coverage_penalty=kw.get("coverage_penalty", "none"),
        stepwise_penalty=kw.get("stepwise_penalty", False), block_ngram_repeat=kw.get("block_ngram_repeat", 0),
        ignore_when_blocking=kw.get("ignore_when_blocking", []), batch_size=8)
    tr = Translator(cfg, None, opt, engine=eng)
    chunks = gu.chunks_of(z)
    T = max(len(c) for c in chunks)
    src = torch.zeros(T, len(chunks), 1)
    for i, c in enumerate(chunks):
        src[: len(c), i, 0] = torch.from_numpy(c)
    batch = types.SimpleNamespace(src=src, src_lengths=torch.tensor([len(c) for c in chunks]),
                                  batch_size=len(chunks))
    att_on = bool(kw.get("attention", False))
    res = tr.translate_batch(batch, None, att_on, fast=fast)
    p = which + "_"
    for i in range(len(chunks)):
        for nb in range(kw["n_best"]):
            exp_s = float(z[p + "scores"][i, nb])
            got_s = float(res["scores"][i][nb])
            assert abs(got_s - exp_s) <= 1e-3 + 1e-5 * abs(exp_s), (i, nb, got_s, exp_s)
            if exp_s <= -1e20:
                continue
            L = int(z[p + "lens"][i, nb])
            got = res["predictions"][i][nb].numpy()
            assert len(got) == L and (got == z[p + "tokens"][i, nb, :L]).all(), (i, nb)
            if att_on:
                a = res["attention"][i][nb].numpy()
                cut = int(z[p + "attn_cut"][i, nb])
                assert a.shape == (L, cut), (i, nb, a.shape, (L, cut))
                np.testing.assert_allclose(a, z[p + "attn"][i, nb, :L, :cut], atol=1e-5)


@pytest.mark.parametrize("temp,topk", [(1.0, -1), (0.7, 2), (1.5, 3)])
def test_random_sampling_distribution(temp, topk):
    """-random_sampling_temp / -random_sampling_topk (translator.py:371-394).
    The draws cannot match torch's generator, so parity is distributional:
    64 copies of each golden chunk, 8 seeds, and the step-0 tokens tested
    (chi-square, p > 1e-4) against softmax of the oracle's sampling logits
    built from the reference's own step-0 log-probs; tokens outside the top-k
    never drawn; the score is the drawn token's tempered log-prob; equal seeds
    repeat."""
    from scipy import stats
    from nanodecoder_amd.engine import pad_chunks
    ref = _oracle()
    z, meta = gu.load("transformer_greedy")
    cfg, W = gu.model_for(meta)
    chunks = gu.chunks_of(z)
    rep = 64
    eng = _engine(cfg, W, max_batch=len(chunks) * rep, max_steps=2)
    sig, lens = pad_chunks([c for c in chunks for _ in range(rep)], 512)
    spans = np.full(len(chunks) * rep, 512, np.int32)
    lg = ref.sampling_logits(z["logp"][:, 0, :], temp, topk)
    p = torch.softmax(lg, -1).numpy()
    counts = np.zeros_like(p)
    for seed in range(8):
        r = eng.translate_sample(sig, lens, spans, temp=temp, keep_topk=topk, seed=1000 + seed, max_len=1,
                                 return_logp=True)
        tok = r["tokens"].cpu().numpy()[:, 0]
        lp = r["logp"].cpu().numpy()[:, 0, :]
        sc = r["scores"].cpu().numpy()
        np.testing.assert_allclose(sc, lp[np.arange(len(tok)), tok] / temp, rtol=1e-6, atol=1e-6)
        for i in range(len(chunks)):
            np.add.at(counts[i], tok[i * rep:(i + 1) * rep], 1)
        if seed == 0:
            r2 = eng.translate_sample(sig, lens, spans, temp=temp, keep_topk=topk, seed=1000, max_len=1)
            assert (r2["tokens"].cpu().numpy()[:, 0] == tok).all()
    for i in range(len(chunks)):
        assert counts[i][p[i] == 0].sum() == 0
        exp = p[i] * counts[i].sum()
        big = exp >= 5
        f_obs = np.append(counts[i][big], counts[i][~big].sum())
        f_exp = np.append(exp[big], exp[~big].sum())
        if f_exp[-1] < 1e-9:
            f_obs, f_exp = f_obs[:-1], f_exp[:-1]
        if len(f_obs) > 1:
            assert stats.chisquare(f_obs, f_exp * f_obs.sum() / f_exp.sum()).pvalue > 1e-4, (i, counts[i], exp)


def test_classic_beam_packed_batches_vs_oracle():
    """Several reference batches packed into one engine call keep their own
    stopping points: equal to the oracle run batch by batch."""
    ref = _oracle()
    z, meta = gu.load("transformer_classic_beam_mid")
    cfg, W = gu.model_for(meta)
    kw = dict(meta["classic"])
    m = ref.RefModel(cfg, W)
    chunks = gu.chunks_of(z) + [c[::-1].copy() for c in gu.chunks_of(z)[:3]]
    groups = [0, 0, 1, 1, 2, 2, 2]          # reference batches of 2 / 2 / 3 chunks
    exp = {}
    for g in sorted(set(groups)):
        idx = [i for i, gg in enumerate(groups) if gg == g]
        part = [chunks[i] for i in idx]
        src, lens, order = ref.make_batch(part)
        res = ref.classic_beam(m, src, lens, **kw)
        for j, o in enumerate(order):
            exp[idx[o]] = (res[j], src.shape[1])
    from nanodecoder_amd.engine import pad_chunks
    sig, lens = pad_chunks(chunks, 512)
    spans = np.array([exp[i][1] for i in range(len(chunks))], np.int32)
    eng = _engine(cfg, W, max_batch=8, max_steps=kw["max_length"], max_beam=kw["beam_size"])
    r = eng.translate_beam_classic(sig, lens, spans, groups=groups, beam=kw["beam_size"], n_best=kw["n_best"],
                                   length_penalty=kw["length_penalty"], max_len=kw["max_length"],
                                   min_len=kw["min_length"])
    tok, sc, ln = (r[k].cpu().numpy() for k in ("tokens", "scores", "lens"))
    for i in range(len(chunks)):
        for nb, (s, p) in enumerate(exp[i][0]):
            assert ln[i, nb] == len(p), (i, nb)
            assert (tok[i, nb, : len(p)] == p).all(), (i, nb)
            assert abs(sc[i, nb] - s) < 1e-3


# ----------------------------------------------------------------- oracle, larger
def _compare_tokens(got, exp_tokens, exp_logp):
    """Exact tokens, except after a genuine oracle near-tie."""
    B, S = exp_tokens.shape
    n_tie = 0
    for b in range(B):
        for s in range(S):
            if got[b, s] != exp_tokens[b, s]:
                top2 = np.sort(exp_logp[b, s])[-2:]
                assert top2[1] - top2[0] < TIE_MARGIN, (b, s, got[b, s], exp_tokens[b, s], top2)
                n_tie += 1
                break
    return n_tie


@pytest.mark.parametrize("itos", [None, ["<unk>", "<blank>", "<s>", "</s>", "A", "C"]])
def test_greedy_vs_oracle_batch32(itos):
    """V = 8 (the largest vocabulary whose head runs inside the next step's
    self-attention, its candidate table rows in LDS) and V = 6 (fewer table
    rows than the staging threads: clamped loads)."""
    ref = _oracle()
    cfg = synth.ModelConfig() if itos is None else synth.ModelConfig(itos=list(itos))
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    sig = synth.synth_chunk_batch(32, 512, seed=3)
    lens = np.full(32, 512, np.int32)
    lens[5] = 400
    sig[5, 400:] = 0.0
    eng = _engine(cfg, W, max_batch=32, max_steps=100)
    r = eng.translate_greedy(sig, lens, np.full(32, 512, np.int32), max_len=100, return_logp=True)
    o = ref.greedy(ref.RefModel(cfg, W), sig, lens, max_length=100)
    got_lp = r["logp"].cpu().numpy()
    got_tok = r["tokens"].cpu().numpy()
    n_tie = _compare_tokens(got_tok, o["tokens"], o["logp"])
    same = (got_tok == o["tokens"]).all(axis=1)
    assert n_tie <= 1
    assert gu.logp_close(got_lp[same], o["logp"][same], atol=LOGP_ATOL).all()


def test_greedy_short_max_len_vs_oracle():
    """A call with max_len below the context's max_steps: the head-fused
    self-attention's token history has the call's max_len as its stride, the
    layer-0 cache the context's max_steps."""
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    sig = synth.synth_chunk_batch(32, 512, seed=5)
    lens = np.full(32, 512, np.int32)
    eng = _engine(cfg, W, max_batch=32, max_steps=100)
    r = eng.translate_greedy(sig, lens, lens, max_len=37, return_logp=True)
    o = ref.greedy(ref.RefModel(cfg, W), sig, lens, max_length=37)
    got_tok = r["tokens"].cpu().numpy()
    assert got_tok.shape == (32, 37)
    assert _compare_tokens(got_tok, o["tokens"], o["logp"]) <= 1
    same = (got_tok == o["tokens"]).all(axis=1)
    assert gu.logp_close(r["logp"].cpu().numpy()[same], o["logp"][same], atol=LOGP_ATOL).all()


def _reads_for_packing():
    """Median/MAD-normalised synthetic reads windowed at 512: short last
    chunks, one-chunk reads, a read shorter than a chunk."""
    from nanodecoder_amd import frontend
    reads = []
    for i, n in enumerate((1300, 700, 512, 2049, 300, 1100, 1536, 90)):
        reads.append(frontend.window(frontend.normalize(synth.synth_raw_read(50 + i, n), "median"), 512, 512))
    return reads


@pytest.mark.parametrize("beam", [1, 5])
def test_translate_reads_packed_vs_oracle(beam):
    """Translator.translate_reads, the CLI / read-shard production path: the
    chunks of many reads packed into engine batches of 8 (so one call mixes
    reads and reference batches, and a reference batch of 3 can straddle two
    calls), each chunk keeping its reference batch's padded length as its
    span.  Against the oracle run read by read in the reference's own
    batching (ref_cpu.translate, translate/translator.py:181-369): identical
    strings, scores within 1e-3."""
    import types
    from nanodecoder_amd.translator import Translator
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-1.0 if beam == 1 else 1.0)
    S, bs = 40, 3
    eng = _engine(cfg, W, max_batch=8, max_steps=S, max_beam=beam)
    opt = types.SimpleNamespace(gpu=0, n_best=1, max_length=S, min_length=4, beam_size=beam, fast=True,
                                batch_size=bs, engine_max_batch=8)
    tr = Translator(cfg, None, opt, engine=eng)
    reads = _reads_for_packing()
    got = tr.translate_reads(reads, batch_size=bs)
    m = ref.RefModel(cfg, W)
    n_chunks = 0
    for ri, chunks in enumerate(reads):
        es, ep = ref.translate(m, chunks, bs, beam_size=beam, n_best=1, max_length=S, min_length=4)
        gs, gp = got[ri]
        assert len(gp) == len(ep) == len(chunks)
        for ci in range(len(chunks)):
            assert gp[ci] == ep[ci], (ri, ci, gp[ci], ep[ci])
            assert abs(gs[ci][0] - es[ci][0]) < 1e-3, (ri, ci)
            n_chunks += 1
    assert n_chunks > 16


@pytest.mark.parametrize("where", ["ffn", "attn"])
def test_split_fp16_range_guard(where):
    """Activations beyond fp16's range (|x| >= 65504) in a split-fp16
    product.  ffn: the FFN hiddens of encoder layer 0 and decoder layer 1
    scaled up 1e5x (their W_2 down 1e5x, so the model's function is
    unchanged).  attn: encoder layer 1's queries scaled up 1e6x and its keys
    down 1e6x (the scores are unchanged; the split Q * log2(e) / sqrt(32)
    leaves fp16's range).  The engine's split path flags the call
    (nd_take_overflow) instead of returning infs, the Translator reruns it on
    exact fp32, and the strings and scores equal the fp32 oracle's.  The
    unscaled model never trips it."""
    import types
    from nanodecoder_amd.translator import Translator
    ref = _oracle()
    cfg = synth.ModelConfig()
    W0 = synth.make_weights(cfg, seed=11, eos_bias=-1.0)
    W = dict(W0)
    if where == "attn":
        p = "encoder.transformer.1.self_attn."
        for k, f in (("linear_query", 1e6), ("linear_keys", 1e-6)):
            W[p + k + ".weight"] = W0[p + k + ".weight"] * np.float32(f)
            W[p + k + ".bias"] = W0[p + k + ".bias"] * np.float32(f)
    for p in ("encoder.transformer.0.feed_forward", "decoder.transformer_layers.1.feed_forward"):
        if where != "ffn":
            break
        W[p + ".w_1.weight"] = W0[p + ".w_1.weight"] * np.float32(1e5)
        W[p + ".w_1.bias"] = W0[p + ".w_1.bias"] * np.float32(1e5)
        W[p + ".w_2.weight"] = W0[p + ".w_2.weight"] * np.float32(1e-5)
    S = 30
    reads = _reads_for_packing()[:4]
    chunks = [c for r in reads for c in r]
    from nanodecoder_amd.engine import pad_chunks
    sig, lens = pad_chunks(chunks, 512)
    for w, expect in ((W0, 0), (W, 1)):
        eng = _engine(cfg, w, max_batch=16, max_steps=S)
        r = eng.translate_greedy(sig, lens, np.full(len(chunks), 512, np.int32), max_len=S)
        assert int(r["overflow"].cpu()[0]) == expect
    opt = types.SimpleNamespace(gpu=0, n_best=1, max_length=S, min_length=4, beam_size=1, batch_size=3,
                                engine_max_batch=16)
    got = Translator(cfg, None, opt, engine=eng).translate_reads(reads, batch_size=3)
    m = ref.RefModel(cfg, W)
    for ri, chunks in enumerate(reads):
        es, ep = ref.translate(m, chunks, 3, max_length=S, min_length=4)
        assert got[ri][1] == ep, ri
        assert np.abs(np.array(got[ri][0]) - np.array(es)).max() < 1e-3


def test_beam_large_batch_vs_oracle():
    """--fast beam 5 on 416 chunks (2080 decoder rows: the LDS-tiled
    split-fp16 GEMMs of the large-M path (from 2048 rows), as configs[3]'s
    B = 1024 runs) against the oracle on a sample of the chunks.  Every
    chunk is a full 512-sample window, so its padded length (and result) does
    not depend on the rest of its batch: the sample runs as its own batch."""
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=13, eos_bias=1.0)
    B, S = 416, 30
    sig = synth.synth_chunk_batch(B, 512, seed=77, inject_masks=False)
    lens = np.full(B, 512, np.int32)
    eng = _engine(cfg, W, max_batch=B, max_steps=S, max_beam=5)
    r = eng.translate_beam(sig, lens, lens, beam=5, n_best=2, max_len=S, min_len=3)
    tok, sc, ln = (r[k].cpu().numpy() for k in ("tokens", "scores", "lens"))
    pick = [0, 1, 97, 203, 204, 333, 414, 415]
    exp = ref.fast_beam(ref.RefModel(cfg, W), sig[pick], lens[pick], beam_size=5, n_best=2, max_length=S,
                        min_length=3)
    for j, i in enumerate(pick):
        for nb, (s, p) in enumerate(exp[j]):
            assert ln[i, nb] == len(p), (i, nb)
            assert (tok[i, nb, : len(p)] == p).all(), (i, nb)
            assert abs(sc[i, nb] - s) < 1e-3, (i, nb)


def test_transformer_encoder_vs_oracle_masks():
    """The transformer encoder (layer 0's QKV in closed form from the
    embedding; every layer through the folded FFN launches) against the oracle's
    encoder: masked keys (signal 0), an all-zero chunk (uniform attention), a
    ragged span, a large-amplitude chunk; rows past a chunk's span are not
    compared (no query there)."""
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=21)
    B = 6
    sig = synth.synth_chunk_batch(B, 512, seed=21)
    lens = np.full(B, 512, np.int32)
    spans = np.full(B, 512, np.int32)
    sig[1, ::7] = 0.0
    sig[2, :] = 0.0
    lens[3], spans[3] = 300, 300
    sig[3, 300:] = 0.0
    lens[4] = 200
    sig[4, 200:] = 0.0          # zero padding inside the span: masked keys
    sig[5] *= 5.0
    eng = _engine(cfg, W, max_batch=B, max_steps=10)
    mem = eng.encode(sig, lens, spans).cpu().numpy()
    exp_mem = ref.RefModel(cfg, W).encode(torch.from_numpy(sig), lens).numpy()
    for i in range(B):
        L = spans[i]
        assert np.abs(mem[i, :L] - exp_mem[i, :L]).max() < 1e-4, i


def test_nano_greedy_vs_oracle_ragged():
    """NanoEncoder packing: ragged lengths inside one batch (reverse LSTM
    starts at len-1), B not a multiple of the 16-sequence LSTM group."""
    ref = _oracle()
    cfg = synth.ModelConfig(encoder_type="nano")
    W = synth.make_weights(cfg, seed=14, eos_bias=-2.0)
    B = 19
    sig = synth.synth_chunk_batch(B, 512, seed=9)
    lens = np.full(B, 512, np.int32)
    for i, L in ((3, 77), (7, 300), (18, 1)):
        lens[i] = L
        sig[i, L:] = 0.0
    eng = _engine(cfg, W, max_batch=B, max_steps=30)
    mem = eng.encode(sig, lens, np.full(B, 512, np.int32)).cpu().numpy()
    m = ref.RefModel(cfg, W)
    exp_mem = m.encode(torch.from_numpy(sig), lens).numpy()
    for i in range(B):
        assert np.abs(mem[i] - exp_mem[i]).max() < 2e-4, i
    r = eng.translate_greedy(sig, lens, np.full(B, 512, np.int32), max_len=30, return_logp=True)
    o = ref.greedy(m, sig, lens, max_length=30)
    n_tie = _compare_tokens(r["tokens"].cpu().numpy(), o["tokens"], o["logp"])
    assert n_tie == 0
    assert gu.logp_close(r["logp"].cpu().numpy(), o["logp"], atol=LOGP_ATOL).all()


def test_memory_bank_path_matches_kv_path_ragged_spans():
    """Greedy with cross-read packing (per-chunk spans < T, T not a multiple
    of 16): the memory-bank context attention and the per-layer K/V form give
    the same log-probs (fp32 rounding) and tokens."""
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=5, eos_bias=-3.0)
    B, T = 24, 200
    rng = np.random.default_rng(17)
    sig = synth.synth_chunk_batch(B, T, seed=21)
    spans = rng.integers(1, T + 1, B).astype(np.int32)
    spans[0], spans[1] = T, 1
    lens = np.minimum(spans, rng.integers(1, T + 1, B)).astype(np.int32)
    for i in range(B):
        sig[i, lens[i]:] = 0.0
    eng = _engine(cfg, W, max_batch=B, max_src_len=T, max_steps=40)
    out = []
    for path in (0, 1):
        eng.set_ctx_path(path)
        r = eng.translate_greedy(sig, lens, spans, max_len=40, return_logp=True)
        out.append((r["tokens"].cpu().numpy(), r["logp"].cpu().numpy()))
    assert (out[0][0] == out[1][0]).all()
    # generator biases put some log-probs near -1e4, where one fp32 ulp is 1e-3
    assert np.allclose(out[0][1], out[1][1], rtol=2e-6, atol=1e-4)


# ----------------------------------------------------------------- front end
@pytest.mark.parametrize("method", ["median", "mean", "None"])
def test_frontend_normalize_window_vs_host(method):
    """nd_normalize_reads + nd_window_reads against the host restatement of
    extract_fast5_raw (frontend.normalize + window, numpy float64): DAC-like
    integer reads (ties everywhere), float reads, odd / even / tiny / long
    lengths.  Bit-exact float32 chunks for median and None; mean within 1
    ulp (its std is a reduction in another order)."""
    from nanodecoder_amd import frontend, synth
    rng = np.random.default_rng(7)
    raws = [synth.synth_raw_read(i, n) for i, n in enumerate((1300, 700, 512, 513, 511, 100_003))]
    raws += [np.array([5.0]), np.array([3.0, 9.0]), np.array([1.0, 1.0, 2.0]),
             rng.normal(size=1001) * 50 - 20, rng.integers(-100, 100, size=2048).astype(np.float64)]
    sig, lens, rd = frontend.normalize_window_gpu(raws, method, 512, 512)
    got = sig.cpu().numpy()
    c = 0
    for r, raw in enumerate(raws):
        exp = frontend.window(frontend.normalize(raw, method), 512, 512)
        for e in exp:
            assert rd[c] == r and lens[c] == len(e)
            g = got[c, : len(e)]
            if method == "mean":
                np.testing.assert_array_max_ulp(g, e, maxulp=1)
            else:
                assert (g.view(np.uint32) == e.view(np.uint32)).all(), (r, c)
            assert (got[c, len(e):] == 0).all()
            c += 1
    assert c == len(rd)


def test_frontend_gpu_vs_reference_labelop():
    """nd_normalize_reads + nd_window_reads against the chunks the
    reference's own extract_fast5_raw cut (tests/golden/frontend.npz): every
    normalisation at 512/512 and the 300/60 overlap windows.  Bit-exact
    float32 for median and None (NaN where the reference divides by a zero
    MAD); mean within 1 ulp (its std is a reduction in another order)."""
    from nanodecoder_amd import frontend
    z, meta = gu.load_frontend()
    raws = [z[f"raw{i}"] for i in range(meta["reads"])]
    for si, (norm, ml, st) in enumerate(meta["settings"]):
        sig, lens, rd = frontend.normalize_window_gpu(raws, norm, ml, st)
        got = sig.cpu().numpy()
        c = 0
        for i in range(len(raws)):
            for e in gu.frontend_chunks(z, i, si):
                assert rd[c] == i and lens[c] == len(e), (si, i, c)
                g = got[c, : len(e)]
                if norm == "mean" and not np.isnan(e).any():
                    np.testing.assert_array_max_ulp(g, e, maxulp=1)
                else:
                    assert gu.same_f32(g, e), (si, i, c)
                c += 1
        assert c == len(rd)


def test_cli_gpu_frontend_matches_host(tmp_path):
    """translate.py end to end on the drop-in default (build_translator ->
    EnginePool, -engine_lanes 3) with both front ends: -frontend cpu (the
    worker pool normalises and windows, translate_reads) and -frontend gpu
    (raw reads to the translator, every engine batch normalised and windowed
    on the device on its call's stream, translate_raw_reads).  The segment
    files (one line per chunk) and the assembled reads are identical, and
    every chunk's string equals the oracle's per-read translate on the
    reference front end's chunks (translate.py:76-129, translator.py:181-369,
    utils/labelop.py:194-243)."""
    from nanodecoder_amd import checkpoint, cli, frontend, opts, synth
    from nanodecoder_amd.engine import EnginePool
    import nanodecoder_amd.translator as T
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-1.0)
    ck = tmp_path / "m.pt"
    checkpoint.save_synthetic(str(ck), cfg, W)
    src = tmp_path / "reads"
    src.mkdir()
    raws = {}
    for i, n in enumerate((1300, 700, 400, 2049, 90, 1024, 3000)):
        raw = synth.synth_raw_read(i, n)
        raws[f"read{i}"] = raw
        (src / f"read{i}.signal").write_text(" ".join(str(int(v)) for v in raw))
    built = []
    orig = T.Translator.__init__

    def spy(self, *a, **k):
        orig(self, *a, **k)
        built.append(self.engine)
    S, bs = 30, 2
    outs = {}
    try:
        T.Translator.__init__ = spy
        for m in ("cpu", "gpu"):
            out = tmp_path / ("out_" + m)
            o = opts.parse_translate_opts(["-model", str(ck), "-src_dir", str(src), "-save_data", str(out), "-gpu",
                                           "0", "-beam_size", "1", "-batch_size", str(bs), "-thread", "2",
                                           "-max_length", str(S), "-min_length", "4", "-engine_max_batch", "8",
                                           "-frontend", m])
            assert o.engine_lanes == 0  # auto: 3 lanes for a greedy translator (the spy below checks)
            assert cli.main(o) == len(raws)
            outs[m] = {name: ((out / "segment" / f"{name}.txt").read_text(),
                              (out / "result" / f"{name}.fasta").read_text()) for name in raws}
    finally:
        T.Translator.__init__ = orig
    assert len(built) == 2 and all(isinstance(e, EnginePool) and e.lanes == 3 for e in built)
    for e in built:
        e.close()
    assert outs["cpu"] == outs["gpu"]
    rm = ref.RefModel(cfg, W)
    for name, raw in raws.items():
        chunks = frontend.window(frontend.normalize(raw, "median"), 512, 512)
        _, ep = ref.translate(rm, chunks, bs, max_length=S, min_length=4)
        assert outs["gpu"][name][0].splitlines() == [p[0] for p in ep], name


@pytest.mark.parametrize("layer0,bn", [(True, False), (False, False), (False, True), (True, True)])
def test_nano_lstm_layer_vs_torch_lstm(layer0, bn):
    """One BiLSTM layer through nd_op_lstm_layer against torch.nn.LSTM (CPU,
    fp32) over packed ragged sequences (encoder/nano_encoder.py:92-111: pack,
    bidirectional LSTM, unpack with zeros past each length, eval BatchNorm).
    B = 6 leaves a partly filled last workgroup (4 sequences per workgroup
    on the split-fp16 path, 16 on the fp32 one).  Tolerance 1e-4 absolute:
    split-fp16 recurrent products (22-bit operands) and the hardware exp /
    reciprocal in the cell, over 48 steps."""
    from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence

    from nanodecoder_amd.engine import op_lstm_layer
    g = torch.Generator().manual_seed(7 + 2 * layer0 + bn)
    B, T, H = 6, 48, 128
    insz = 1 if layer0 else 256
    lstm = torch.nn.LSTM(insz, H, bidirectional=True)
    with torch.no_grad():
        for p in lstm.parameters():
            p.uniform_(-0.15, 0.15, generator=g)
        lens = torch.tensor([48, 48, 40, 33, 17, 5])
        x = torch.randn(T, B, insz, generator=g)
        y, _ = lstm(pack_padded_sequence(x, lens))
        y, _ = pad_packed_sequence(y, total_length=T)
    ref = y.transpose(0, 1).reshape(B * T, 2 * H)
    whh = torch.stack([lstm.weight_hh_l0, lstm.weight_hh_l0_reverse]).detach()
    bsum = torch.stack([lstm.bias_ih_l0 + lstm.bias_hh_l0,
                        lstm.bias_ih_l0_reverse + lstm.bias_hh_l0_reverse]).detach()
    wih = [lstm.weight_ih_l0.detach(), lstm.weight_ih_l0_reverse.detach()]
    dev = torch.device("cuda", 0)
    kw = {}
    if bn:
        scale = torch.rand(2, H, generator=g) + 0.5
        shift = torch.randn(2, H, generator=g) * 0.1
        kw = {"bn_scale": scale.to(dev), "bn_shift": shift.to(dev)}
        valid = (torch.arange(T)[None, :] < lens[:, None]).reshape(B * T, 1)
        ref = torch.where(valid, ref * scale.reshape(1, -1) + shift.reshape(1, -1), ref)
    if layer0:
        signal = x[:, :, 0].T.contiguous()
        wih0 = torch.stack([w[:, 0] for w in wih])
        out = op_lstm_layer(whh.to(dev), lens.int().to(dev), T, signal=signal.to(dev), wih0=wih0.to(dev),
                            bsum=bsum.to(dev), **kw)
    else:
        xb = x.transpose(0, 1).reshape(B * T, insz)
        xp = torch.cat([xb @ wih[0].T + bsum[0], xb @ wih[1].T + bsum[1]], dim=1).contiguous()
        out = op_lstm_layer(whh.to(dev), lens.int().to(dev), T, xp=xp.to(dev), **kw)
    torch.cuda.synchronize()
    got = out.cpu()
    pad = ~(torch.arange(T)[None, :] < lens[:, None]).reshape(B * T)
    assert (got[pad] == 0).all(), "rows past a sequence's length must stay zero"
    err = float((got - ref).abs().max())
    assert err < 1e-4, err
    # step 0 of each direction (forward pos 0, reverse pos len - 1): the rows
    # written before the first in-loop barrier, BatchNorm table included
    for b in range(B):
        for row, cols in ((b * T, slice(0, H)), (b * T + int(lens[b]) - 1, slice(H, 2 * H))):
            assert float((got[row, cols] - ref[row, cols]).abs().max()) < 1e-4, (b, row)
