"""The beam's 24-bit context K/V image (attention.hip ctx_pack_q24_kernel,
include/nanodec.h nd_op_ctx_pack_q24) restated in numpy, CPU only.

The reference keeps the context keys / values in fp32
(onmt/modules/multi_headed_attn.py:142-150, the memory's linear_keys /
linear_values outputs that translate/translator.py:667-676 tiles per beam).
The image stores every (key, head) as 24-bit integers times a power-of-two
scale 2^(e-23), max|x| < 2^e.  These tests pin the byte layout the GPU kernel
must reproduce bit for bit (tests/test_gpu_parity.py compares the two) and
the error bound: |x - x'| <= 2^(e-24) <= 2^-23 max|x| per element, and the
attention on the image within fp32 rounding of the fp64 attention.
"""
import numpy as np

D, H, DH = 256, 8, 32
ROW = 1600  # bytes per (key, layer): k 768 | v 768 | 8 x {k scale, v scale}


def _quant(x):
    """x [..., 8, 32] f32 -> (int32 [..., 8, 32], f32 scale [..., 8])."""
    x = x.astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        finite = np.isfinite(x).all(-1)
        mx = np.where(finite, np.abs(x).max(-1), np.float32(np.inf))
        _, e = np.frexp(np.where(finite, mx, np.float32(1)))
        e = np.maximum(e, -100).astype(np.int32)
        up = np.ldexp(np.float32(1), 23 - e).astype(np.float32)
        v = np.rint(x * up[..., None]).astype(np.float32)
        v = np.nan_to_num(np.clip(v, -8388607, 8388607), nan=0.0).astype(np.int32)
    scale = np.where(finite, np.ldexp(np.float32(1), e - 23), np.float32(np.nan)).astype(np.float32)
    return v, scale


def pack_q24(kv, ld, layers, span, B, T):
    """numpy image of nd_op_ctx_pack_q24: kv [B*T, ld] f32 -> uint8 [layers, B*T,
    1600] (layer-major); rows t >= span[c] stay zero (the kernel does not write them)."""
    out = np.zeros((layers, B * T, ROW), np.uint8)
    for layer in range(layers):
        k = kv[:, layer * 2 * D: layer * 2 * D + D].reshape(-1, H, DH)
        v = kv[:, layer * 2 * D + D: (layer + 1) * 2 * D].reshape(-1, H, DH)
        for off, x in ((0, k), (768, v)):
            q, _ = _quant(x)
            b = q.reshape(-1, D).astype("<i4").view(np.uint8).reshape(-1, D, 4)[:, :, :3]
            out[layer, :, off:off + 768] = b.reshape(-1, 768)
        sk, sv = _quant(k)[1], _quant(v)[1]
        out[layer, :, 1536:1600] = np.stack([sk, sv], -1).astype("<f4").view(np.uint8).reshape(-1, 64)
    t = np.arange(B * T) % T
    live = t < np.minimum(np.repeat(np.asarray(span), T), T)
    out[:, ~live] = 0
    return out


def unpack_q24(img, layer):
    """image -> (k, v) f32 [rows, 256], decoded as the kernel does (q24_unpack)."""
    r = img[layer]

    def ints(b):
        b = b.reshape(-1, D, 3).astype(np.int32)
        v = b[..., 0] | (b[..., 1] << 8) | (b[..., 2] << 16)
        return np.where(v >= 1 << 23, v - (1 << 24), v)

    sc = r[:, 1536:1600].copy().view("<f4").reshape(-1, H, 2)
    k = ints(r[:, :768]).reshape(-1, H, DH) * sc[..., 0:1]
    v = ints(r[:, 768:1536]).reshape(-1, H, DH) * sc[..., 1:2]
    return k.reshape(-1, D).astype(np.float32), v.reshape(-1, D).astype(np.float32)


def test_bit_layout_matches_the_kernels_word_form():
    """The kernel packs lane i's four integers into three words (b.x = v0 |
    v1 << 24, ...); the image must be plain little-endian 3-byte integers in
    dim order, which is what a lane's dwordx3 load at byte 12 i sees."""
    rng = np.random.default_rng(0)
    v = rng.integers(-(1 << 23) + 1, 1 << 23, size=(64, 4)).astype(np.int64)
    m = 0xFFFFFFFF
    bx = ((v[:, 0] & 0xFFFFFF) | (v[:, 1] << 24)) & m
    by = (((v[:, 1] >> 8) & 0xFFFF) | (v[:, 2] << 16)) & m
    bz = (((v[:, 2] >> 16) & 0xFF) | (v[:, 3] << 8)) & m
    words = np.stack([bx, by, bz], 1).astype("<u4").view(np.uint8).reshape(-1)
    plain = v.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :3].reshape(-1)
    assert np.array_equal(words, plain)
    # and the kernel's decode (alignbit + arithmetic shifts) inverts it
    w = np.stack([bx, by, bz], 1).astype(np.uint64)

    def sx(u):  # (int)(u << 8) >> 8 on 32 bits
        u = (u << 8) & m
        return np.where(u >= 1 << 31, u.astype(np.int64) - (1 << 32), u.astype(np.int64)) >> 8

    i0 = sx(w[:, 0])
    i1 = sx(((w[:, 1] << 32 | w[:, 0]) >> 24) & m)
    i2 = sx(((w[:, 2] << 32 | w[:, 1]) >> 16) & m)
    i3 = np.where(w[:, 2] >= 1 << 31, w[:, 2].astype(np.int64) - (1 << 32), w[:, 2].astype(np.int64)) >> 8
    assert np.array_equal(np.stack([i0, i1, i2, i3], 1), v)


def test_error_bound_per_head():
    """|x - x'| <= 2^(e-24) <= 2^-23 max|x| per element, on heads spanning
    1e-30 .. 1e30, a zero head, a head of one large value among tiny ones,
    and values that round up to the clamp."""
    rng = np.random.default_rng(1)
    B, T, layers = 2, 16, 3
    kv = rng.standard_normal((B * T, layers * 2 * D)).astype(np.float32)
    kv[0, :DH] = 0.0
    kv[1, DH:2 * DH] = rng.standard_normal(DH) * 1e-3
    kv[1, DH] = 1e3
    kv[2] *= np.float32(1e-30)
    kv[3] *= np.float32(1e30)
    kv[4, :DH] = np.float32(1.0) - np.float32(2.0 ** -24)  # |x| 2^23 / 2^e rounds to 2^23: clamped
    kv[4, 0] = -kv[4, 0]
    span = np.array([T, T], np.int32)
    img = pack_q24(kv, layers * 2 * D, layers, span, B, T)
    for layer in range(layers):
        k, v = unpack_q24(img, layer)
        for x, y in ((kv[:, layer * 512: layer * 512 + 256], k), (kv[:, layer * 512 + 256:(layer + 1) * 512], v)):
            xh, yh = x.reshape(-1, H, DH).astype(np.float64), y.reshape(-1, H, DH).astype(np.float64)
            mx = np.abs(xh).max(-1, keepdims=True)
            err = np.abs(xh - yh)
            assert (err <= mx * 2.0 ** -23 + 1e-300).all(), err.max()
    assert not unpack_q24(img, 0)[0][0, :DH].any()


def test_rows_past_span_untouched_and_nonfinite_heads_stay_nonfinite():
    B, T, layers = 2, 8, 1
    kv = np.ones((B * T, 512), np.float32)
    kv[3, 5] = np.nan
    kv[4, 300] = np.inf
    img = pack_q24(kv, 512, layers, np.array([6, 2], np.int32), B, T)
    assert not img[:, 6:8].any() and not img[:, T + 2:].any() and img[:, :6].any()
    k, v = unpack_q24(img, 0)
    assert np.isnan(k[3, :DH]).all() and np.isfinite(k[3, DH:]).all()
    assert np.isnan(v[4, DH:2 * DH]).all() and np.isfinite(v[4, :DH]).all()


def test_attention_on_the_image_within_fp32_rounding():
    """softmax(q k'^T / sqrt(32)) v' per head against fp64 on the exact K / V:
    the image's error is below what fp32 accumulation adds."""
    rng = np.random.default_rng(2)
    T = 512
    kv = rng.standard_normal((T, 512)).astype(np.float32)
    q = rng.standard_normal(256).astype(np.float32)
    img = pack_q24(kv, 512, 1, np.array([T], np.int32), 1, T)
    k, v = unpack_q24(img, 0)
    for h in range(H):
        sl = slice(h * DH, (h + 1) * DH)
        s64 = kv[:, sl].astype(np.float64) @ q[sl] / np.sqrt(32)
        p64 = np.exp(s64 - s64.max())
        want = p64 @ kv[:, 256 + h * DH: 256 + (h + 1) * DH] / p64.sum()
        s = k[:, sl].astype(np.float64) @ q[sl] / np.sqrt(32)
        p = np.exp(s - s.max())
        got = p @ v[:, sl].astype(np.float64) / p.sum()
        assert np.abs(got - want).max() < 2e-6, np.abs(got - want).max()
