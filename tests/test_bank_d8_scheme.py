"""The 24-bit digit memory bank's arithmetic (nanodecoder_amd/csrc/bank8.hip),
restated in numpy on the CPU: row exponents, balanced digits, the retained
digit products of the scores, the exact f16 digit conversion and the P scale
of the context product.  The GPU kernels are tested against fp64 in
tests/test_gpu_parity.py::test_bank_d8_vs_fp64; this pins the scheme itself
(every bound DESIGN.md states for it) without a GPU."""
import numpy as np


AMAX = np.float32(126 * 65536)


def sext8(x):
    return ((np.asarray(x, np.int64) + 128) % 256) - 128


def digits(A):
    """bank8.hip digits: balanced base-256 digits of |A| <= 126 * 2^16."""
    d0 = sext8(A)
    A1 = (A - d0) >> 8
    d1 = sext8(A1)
    d2 = (A1 - d1) >> 8
    return d2, d1, d0


def quantise_rows(m):
    """bank8.hip fix_q / bank_pack_d8_kernel: [rows, 256] float32 -> (A int64, s float32 per row), m ~ s A,
    s = fp32(max|row| * (1 / (126 * 2^16))), A = rint(fp32(m / s))."""
    mx = np.abs(m).max(1).astype(np.float32)
    s = (mx * np.float32(1 / AMAX)).astype(np.float32)
    safe = np.where(s > 0, s, np.float32(1))
    A = np.where(s[:, None] > 0, np.rint((m.astype(np.float32) / safe[:, None]).astype(np.float32)), 0)
    return A.astype(np.int64), s


def test_digits_range_and_reconstruction():
    rng = np.random.default_rng(0)
    m = (rng.standard_normal((512, 256)) * rng.choice([1e-3, 1.0, 30.0], size=(512, 1))).astype(np.float32)
    m[7] = 0.0
    A, s = quantise_rows(m)
    assert np.abs(A).max() <= 126 * 65536 + 1
    d2, d1, d0 = digits(A)
    for d in (d2, d1, d0):
        assert d.min() >= -128 and d.max() <= 127
    assert np.abs(d2).max() <= 126
    assert ((d2 << 16) + (d1 << 8) + d0 == A).all()
    assert (A[7] == 0).all() and s[7] == 0
    # per element: |m - s A| <= 0.75 s (the quotient's fp32 rounding + rint) ~ 2^-23.3 max|m_row|
    err = np.abs(m.astype(np.float64) - A * s.astype(np.float64)[:, None])
    assert (err <= 0.75 * s[:, None].astype(np.float64) + 1e-45).all()
    assert (err.max(1) <= 2.0 ** -23.3 * np.abs(m).max(1)).all()


def test_scores_from_retained_digit_products():
    """The kernel's five i8 products per 64 dims (a2 x [q2|q1], a2 x [0|q0], a1 x [q2|q1], and
    a0 x [q2|q1] + a1 x [0|q0] in one accumulator) keep every digit product of weight >= 2^8; combined in
    fp32 with the kernel's per-column weights the scores err less than a plain fp32 dot product does."""
    rng = np.random.default_rng(1)
    m = rng.standard_normal((512, 256)).astype(np.float32)
    q = (rng.standard_normal((8, 256)) * 0.3).astype(np.float32)
    A, s = quantise_rows(m)
    Q, sq = quantise_rows(q)
    a2, a1, a0 = digits(A)
    q2, q1, q0 = digits(Q)
    X1a, X1b = a2 @ q2.T, a2 @ q1.T        # a2 x B1: columns q2 | q1
    X2b = a2 @ q0.T                        # a2 x B2: 0 | q0
    X3a, X3b = a1 @ q2.T, a1 @ q1.T        # a1 x B1
    X4a, X4b = a0 @ q2.T, a0 @ q1.T + a1 @ q0.T  # a0 x B1 + a1 x B2
    for X in (X1a, X2b, X3a, X4a, X4b):    # exact int32 sums (256 products of |digit| <= 128)
        assert np.abs(X).max() < 2 ** 31
    f = np.float32
    lo = X1a.astype(f) * f(65536) + X3a.astype(f) * f(256) + X4a.astype(f)            # columns h: weights x 2^-16
    hi = X1b.astype(f) * f(256) + X2b.astype(f) + X3b.astype(f) + X4b.astype(f) * f(1 / 256)  # columns h + 8
    sig = (sq * f(65536 / AMAX) * AMAX / f(65536)).astype(f)  # the kernel keeps sigma_h * 2^16
    sc = (s[:, None] * (sig * f(65536))[None, :]).astype(f)
    got = ((lo + hi) * sc).astype(np.float64)
    exact = m.astype(np.float64) @ q.astype(np.float64).T
    plain = (m @ q.T).astype(np.float64)   # the reference's fp32 matmul
    assert np.abs(got - exact).max() < np.abs(plain - exact).max(), (np.abs(got - exact).max(),
                                                                      np.abs(plain - exact).max())
    assert np.abs(got - exact).max() < 2e-7 * np.abs(m).max() * np.abs(q).max() * 16


def cvt(bytes4, plane):
    """bank8.hip d8_cvt: 4 signed bytes -> f16 via bits 0x64uu (u = b ^ 0x80) = 1024 + u, then exact ops."""
    b = np.asarray(bytes4, np.int64)
    u = (b & 255) ^ 0x80
    bits = (0x64 << 8) | u
    x = bits.astype(np.uint16).view(np.float16)
    if plane == 2:
        return ((x - np.float16(1152)) * np.float16(256)).astype(np.float16)
    if plane == 1:
        return (x - np.float16(1152)).astype(np.float16)
    return (x * np.float16(1 / 256) - np.float16(4.5)).astype(np.float16)


def test_f16_digit_conversion_is_exact():
    b = np.arange(-128, 128)
    assert (cvt(b, 2).astype(np.float64) == b * 256.0).all()
    assert (cvt(b, 1).astype(np.float64) == b * 1.0).all()
    assert (cvt(b, 0).astype(np.float64) == b / 256.0).all()


def test_context_product_scale():
    """U = sum_t p_t m_t from P'' = p s_t 2^7 / s_max split hi | lo in f16 and M' = a2 2^8 + a1 + a0 2^-8
    (exact f16 values = A / 2^8), scaled back by 2 s_max: within 2^-21 of max|m| per unit of sum(p)."""
    rng = np.random.default_rng(2)
    m = (rng.standard_normal((512, 256)) * rng.uniform(0.3, 3.0, size=(512, 1))).astype(np.float32)
    s = rng.standard_normal(512) * 3
    p = np.exp(s - s.max() + rng.uniform(0, 6))  # lazy maximum: p <= e^6
    A, st = quantise_rows(m)
    smax = st.max()
    a2, a1, a0 = digits(A)
    Mp = cvt(a2, 2).astype(np.float64) + cvt(a1, 1).astype(np.float64) + cvt(a0, 0).astype(np.float64)
    assert (Mp == A / 256.0).all()
    x = (p.astype(np.float32) * (st * np.float32(128 / smax))).astype(np.float32)
    assert x.max() < 65504
    hi = x.astype(np.float16)
    lo = (x - hi.astype(np.float32)).astype(np.float16)
    U = (hi.astype(np.float64) + lo.astype(np.float64)) @ Mp * (2.0 * smax)
    exact = p @ m.astype(np.float64)
    assert np.abs(U - exact).max() <= 2.0 ** -21 * np.abs(m).max() * p.sum()


def bank_dim_scales(g, b):
    """engine.hip derive_bank_dim_scales: per-dimension powers of two c_i =
    2^clamp(floor(log2(a_i / median a)), 0, 12), a_i = 3 |g_i| + |b_i|, of the
    encoder's final LayerNorm affine; the bank holds m_i / c_i."""
    a = 3.0 * np.abs(np.asarray(g, np.float64)) + np.abs(np.asarray(b, np.float64))
    med = np.partition(a, a.size // 2)[a.size // 2]
    with np.errstate(divide="ignore"):
        k = np.where((a > 0) & (med > 0), np.floor(np.log2(np.where(a > 0, a, 1.0) / med)), 0.0)
    return np.ldexp(np.float32(1), np.clip(k, 0, 12).astype(np.int32)).astype(np.float32)


def test_bank_dim_scales_remove_an_outlier_dimension():
    """An LN gain 10^3 x the rest: its dimension is divided by 2^9 (2^10 > the
    ratio of 10^3 x 1.5 / median), every other stays 1; the rows of m / c then
    lose at most ~2 bits to it instead of ~10 (the 24-bit per-row scale, above)."""
    rng = np.random.default_rng(4)
    g = (rng.random(256) + 0.5).astype(np.float32)
    b = (rng.standard_normal(256) * 0.1).astype(np.float32)
    assert (bank_dim_scales(g, b) == 1).all()
    g[77] *= 1e3
    b[77] *= 1e3
    c = bank_dim_scales(g, b)
    assert c[77] in (512.0, 1024.0) and (np.delete(c, 77) == 1).all()
    n = rng.standard_normal((512, 256))
    m = (n * g + b) / c
    ratio = np.abs(m).max(1) / np.abs(np.delete(m, 77, axis=1)).max(1)
    assert ratio.max() < 4.0
