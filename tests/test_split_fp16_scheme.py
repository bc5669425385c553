"""The split-fp16 product (gemm.hip H3 / P16H, ffn.hip) restated in numpy, CPU
only: where its fp32-class accuracy holds and what it becomes for activation
rows of small magnitude (the verdict's "underflow of the lo parts").

A weight matrix is scaled by 2^s (max |W| 2^s in [2^13, 2^14)) and split
once, W' = wh + wl; an activation x is split unscaled as the kernels stage it,
x = hi + lo with hi = fp16(x), lo = fp16(x - hi); the product is
hi wh + hi wl + lo wh accumulated in fp32 (every fp16 x fp16 product is exact
in fp32).  lo keeps 11 more bits while it is a normal fp16 (elements above
~2^-3); below that it is a subnormal with an absolute spacing of 2^-24.  So:
- relative to its own output, a row whose elements are all of scale sigma
  carries an error of about 2^-24 / sigma (fp32 class down to sigma ~ 2^-3);
- in absolute terms the error is scale-free: at most ~2^-25 sum_k |w_k| per
  output, whatever sigma is.
In the network the operands split without a LayerNorm in front (the attention
context into W_o, the FFN hidden into W_2, the bank context U into W_vo) all
feed a residual add x + f(.), whose own fp32 rounding is 2^-24 |x|; the split
error sits below that for |x| ~ 1 (the LayerNorm'd operands are split after
the normalisation, before the affine folded into W: rows of scale ~1 whatever
gamma is).  tests/test_gpu_parity.py::test_gemm_split_small_rows_follow_the_scheme
holds the GPU kernel to this restatement (fp16 subnormals preserved, not flushed).
"""
import numpy as np

K, N = 256, 256


def weight_split(W):
    """W f32 [N, K] -> (wh, wl) f16 and the power-of-two scale s (launch_pack_p16h)."""
    mx = float(np.abs(W).max())
    s = 2.0 ** (14 - np.frexp(mx)[1]) if mx > 0 else 1.0
    Ws = (W * np.float32(s)).astype(np.float32)
    wh = Ws.astype(np.float16)
    wl = (Ws - wh.astype(np.float32)).astype(np.float16)
    return wh, wl, s


def split_product(A, W):
    """A [M, K] f32 times W^T in the split form, accumulated in fp64 (the
    kernels accumulate in fp32: their rounding is added on top)."""
    wh, wl, s = weight_split(W)
    ah = A.astype(np.float16)
    al = (A - ah.astype(np.float32)).astype(np.float16)

    def f(a, b):
        return a.astype(np.float64) @ b.astype(np.float64).T
    return (f(ah, wh) + f(ah, wl) + f(al, wh)) / s


def rel_err(got, ref):
    rms = np.sqrt((ref ** 2).mean(axis=1, keepdims=True))
    return float((np.abs(got - ref) / rms).max())


def bound(sigma):
    """The error bound the GPU test asserts, relative to each output row's rms."""
    return 4e-6 + 2.0 * 2.0 ** -24 / sigma


def test_fp32_class_while_lo_stays_normal():
    """Rows of scale 1 and 2^-3: below a plain fp32 dot product's rounding."""
    rng = np.random.default_rng(0)
    W = (rng.standard_normal((N, K)) / 16).astype(np.float32)
    for sigma in (1.0, 2.0 ** -3):
        A = (rng.standard_normal((64, K)) * sigma).astype(np.float32)
        ref = A.astype(np.float64) @ W.astype(np.float64).T
        fp32 = rel_err((A @ W.T).astype(np.float64), ref)
        assert rel_err(split_product(A, W), ref) < fp32


def test_error_grows_as_the_lo_part_turns_subnormal():
    """Below 2^-3 the error follows 2^-24 / sigma (within 2x) and stays under
    bound(sigma); at 2^-14 it is ~1e-3 of the row, 500x a plain fp32 dot."""
    rng = np.random.default_rng(1)
    W = (rng.standard_normal((N, K)) / 16).astype(np.float32)
    errs = {}
    for lg in (-7, -10, -14, -18):
        sigma = 2.0 ** lg
        A = (rng.standard_normal((64, K)) * sigma).astype(np.float32)
        ref = A.astype(np.float64) @ W.astype(np.float64).T
        e = rel_err(split_product(A, W), ref)
        assert 2.0 ** -24 / sigma / 2 < e < bound(sigma), (lg, e)
        errs[lg] = e
    assert errs[-14] > 1e-4


def test_absolute_error_is_scale_free():
    """max |split - exact| stays below 2^-24 max_n sum_k |W_nk| for row
    scales 1 .. 2^-24, and within twice a residual's own fp32 rounding
    (2^-24 at |x| ~ 1) for this W (sum_k |w_k| ~ 14; measured 6.5e-8 .. 7.9e-8
    over 16384 outputs): a sublayer's output added to an O(1) residual is fp32
    class however small the sublayer's input rows are."""
    rng = np.random.default_rng(3)
    W = (rng.standard_normal((N, K)) / 16).astype(np.float32)
    l1 = float(np.abs(W).sum(axis=1).max())
    for lg in range(0, -25, -4):
        A = (rng.standard_normal((64, K)) * 2.0 ** lg).astype(np.float32)
        ref = A.astype(np.float64) @ W.astype(np.float64).T
        err = float(np.abs(split_product(A, W) - ref).max())
        assert err < 2.0 ** -24 * l1, (lg, err)
        if lg <= -4:
            assert err < 2.0 ** -23, (lg, err)


def test_scale_invariance_of_the_weight_side():
    """The weight's 2^s scale makes its split independent of |W|: W and
    2^-20 W give the same relative error (only the activation side is unscaled)."""
    rng = np.random.default_rng(2)
    W = (rng.standard_normal((N, K)) / 16).astype(np.float32)
    A = rng.standard_normal((32, K)).astype(np.float32)
    ref = A.astype(np.float64) @ W.astype(np.float64).T
    e1 = rel_err(split_product(A, W), ref)
    Wt = (W * np.float32(2.0 ** -20)).astype(np.float32)
    e2 = rel_err(split_product(A, Wt), ref * 2.0 ** -20)
    assert abs(e1 - e2) <= 1e-12
