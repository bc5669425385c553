"""CPU emulation of dec_bank_d8_beam_kernel's data movement (nanodecoder_amd/csrc/bank8.hip): the LDS
ring image of a key block, the per-lane addresses of the score fragments, the transposed (tr_b8) reads of
the context operand, the P hand-off and the MFMA lane maps, restated lane by lane in numpy and checked
against fp64 attention.  Pins the kernel's index arithmetic without a GPU (the GPU kernel itself:
tests/test_gpu_parity.py::test_bank_d8_beam_vs_fp64)."""
import numpy as np

from tests.test_bank_d8_scheme import AMAX, digits, quantise_rows

FR, BLK = 1152, 12 * 1152


def pack_bank(m):
    """bank_pack_d8_kernel without LN: [512, 256] -> per key block 12 fragments of 64 lanes x 16 B (db * 3 + pl),
    lane l: key l & 15, dims 64 db + 16 (l >> 4) .. +15."""
    A, s = quantise_rows(m)
    d2, d1, d0 = digits(A)
    planes = [d0, d1, d2]
    blocks = []
    for kb in range(32):
        blk = np.zeros((12, 64, 16), np.uint8)
        for db in range(4):
            for pl in range(3):
                for ln in range(64):
                    key, gq = 16 * kb + (ln & 15), ln >> 4
                    blk[db * 3 + pl, ln] = (planes[pl][key, 64 * db + 16 * gq: 64 * db + 16 * gq + 16] & 255)
        blocks.append(blk)
    return blocks, s


def lds_image(blk):
    """ring slot: fragment f at f * FR, lane-linear 16 B (what buffer_load ... lds writes)."""
    img = np.zeros(BLK, np.uint8)
    for f in range(12):
        img[f * FR: f * FR + 1024] = blk[f].reshape(-1)
    return img


def sx(b):
    return ((b.astype(np.int64) + 128) % 256) - 128


def mfma_i8(A, B):
    """v_mfma_i32_16x16x64_i8 on per-lane 16-byte fragments: A lane l row l & 15, k 16 (l >> 4) ..;
    B lane l col l & 15, same k; returns D [16 rows, 16 cols]."""
    Am = np.zeros((16, 64), np.int64)
    Bm = np.zeros((64, 16), np.int64)
    for l in range(64):
        Am[l & 15, 16 * (l >> 4): 16 * (l >> 4) + 16] = sx(A[l])
        Bm[16 * (l >> 4): 16 * (l >> 4) + 16, l & 15] = sx(B[l])
    return Am @ Bm


def mfma_f16(A, B, kper):
    """16x16x(4 kper) f16: A[l] / B[l] hold kper values each (A row l & 15, B col l & 15, k kper (l >> 4) ..)."""
    Am = np.zeros((16, 4 * kper))
    Bm = np.zeros((4 * kper, 16))
    for l in range(64):
        Am[l & 15, kper * (l >> 4): kper * (l >> 4) + kper] = A[l]
        Bm[kper * (l >> 4): kper * (l >> 4) + kper, l & 15] = B[l]
    return Am @ Bm


def tr_b8(img, addr):
    """ds_read_b64_tr_b8: per 16-lane group, lane 2q + p supplies the address of row q bytes 8p..8p+7; lane i
    receives byte i of rows 0..7."""
    out = np.zeros((64, 8), np.int64)
    for grp in range(4):
        rows = np.zeros((8, 16), np.uint8)
        for q in range(8):
            for p in range(2):
                a = addr[16 * grp + 2 * q + p]
                rows[q, 8 * p: 8 * p + 8] = img[a: a + 8]
        for i in range(16):
            out[16 * grp + i] = sx(rows[:, i])
    return out


def emulate(m, q_rows, L):
    """One chunk, RPC = len(q_rows) rows (no masks): the kernel's arithmetic in float64 where it is exact,
    float32 / float16 where the kernel rounds."""
    RPC = len(q_rows)
    blocks, s = pack_bank(m)
    smax = np.float32(s.max())
    kp = np.float32(128.0) / smax
    lanes = np.arange(64)
    col, g = lanes & 15, lanes >> 4
    # q digits, B operands per row (qb1, qb2 [db][lane] 16 bytes)
    qb = []
    sgm = []
    for q in q_rows:
        Q = np.zeros((8, 256), np.int64)
        sg = np.zeros(8, np.float32)
        for h in range(8):
            qh = q[h * 256:(h + 1) * 256].astype(np.float32)
            qs = np.float32(np.abs(qh).max() * np.float32(1 / AMAX))
            Q[h] = np.rint(qh / (qs if qs > 0 else np.float32(1))).astype(np.int64)
            sg[h] = qs * np.float32(65536)
        q2, q1, q0 = digits(Q)
        b1 = np.zeros((4, 64, 16), np.int64)
        b2 = np.zeros((4, 64, 16), np.int64)
        for db in range(4):
            for l in range(64):
                h, gq = l & 7, l >> 4
                sl = slice(64 * db + 16 * gq, 64 * db + 16 * gq + 16)
                b1[db, l] = (q2 if (l & 15) < 8 else q1)[h, sl] & 255
                b2[db, l] = 0 if (l & 15) < 8 else (q0[h, sl] & 255)
        qb.append((b1, b2))
        sgm.append(sg[col & 7])
    w1 = np.where(col < 8, 65536.0, 256.0)
    w3 = np.where(col < 8, 256.0, 1.0)
    w4 = np.where(col < 8, 1.0, 1 / 256)
    NB = (RPC + 1) // 2
    U = np.zeros((NB, 16, 16, 16))  # [row block][16-dim block] D[row][col]
    mrow = [np.full(64, -np.inf) for _ in range(RPC)]
    lrow = [np.zeros(64) for _ in range(RPC)]
    nkb = (L + 15) // 16
    for kb in range(nkb):
        img = lds_image(blocks[kb])
        P = np.zeros((6, 4, 8, 8))  # [row][g][head][hi x4 | lo x4]
        SC = np.ones((6, 8))
        FL = np.zeros(6, bool)
        for j in range(RPC):
            fb = lambda f: np.stack([img[f * FR + 16 * l: f * FR + 16 * l + 16] for l in range(64)])
            X1 = sum(mfma_i8(fb(db * 3 + 2), qb[j][0][db]) for db in range(4))
            X3 = sum(mfma_i8(fb(db * 3 + 2), qb[j][1][db]) + mfma_i8(fb(db * 3 + 1), qb[j][0][db]) for db in range(4))
            X4 = sum(mfma_i8(fb(db * 3), qb[j][0][db]) + mfma_i8(fb(db * 3 + 1), qb[j][1][db]) for db in range(4))
            sv = np.zeros((64, 4))
            for l in range(64):
                for i in range(4):
                    r = 4 * (l >> 4) + i
                    sv[l, i] = X1[r, l & 15] * w1[l] + X3[r, l & 15] * w3[l] + X4[r, l & 15] * w4[l]
            ks4 = np.stack([s[16 * kb + 4 * (l >> 4): 16 * kb + 4 * (l >> 4) + 4] for l in range(64)])
            sv = (sv + sv[(lanes & 48) | ((lanes + 8) & 15)]) * (ks4 * sgm[j][:, None])
            keys = 16 * kb + 4 * g[:, None] + np.arange(4)[None, :]
            sv = np.where(keys < L, sv, -np.inf)
            gm = sv.max(1)
            gm = np.array([gm[(lanes & 15) == (l & 15)].max() for l in range(64)])
            if np.any(gm > mrow[j] + 6):
                nm = np.maximum(mrow[j], gm)
                sc = np.where(nm == mrow[j], 1.0, np.exp(mrow[j] - nm))
                mrow[j], lrow[j] = nm, lrow[j] * sc
                SC[j] = sc[:8]
                FL[j] = True
            p = np.where(sv == -np.inf, 0.0, np.exp(sv - mrow[j][:, None]))
            lrow[j] += p.sum(1)
            x = (p * (ks4 * kp)).astype(np.float32)
            hi = x.astype(np.float16)
            lo = (x - hi.astype(np.float32)).astype(np.float16)
            for l in range(64):
                if (l & 15) < 8:
                    P[j, l >> 4, l & 15, :4] = hi[l]
                    P[j, l >> 4, l & 15, 4:] = lo[l]
        for b in range(NB):  # rescale each row block once (every wave does its own dim blocks)
            j0, j1 = 2 * b, 2 * b + 1 if 2 * b + 1 < RPC else 2 * b
            if FL[j0] or FL[j1]:
                for r in range(16):
                    jj = 2 * b + (r >> 3)
                    U[b, :, r, :] *= SC[jj, r & 7] if jj < RPC else 1.0
        for w in range(8):
            db_u, G0 = w >> 1, 2 * (w & 1)
            q8, p8 = (lanes & 15) >> 1, lanes & 1
            o1 = (db_u * 3 + np.where(q8 < 4, 2, 1)) * FR + (4 * g + (q8 & 3) + 16 * G0) * 16 + 8 * p8
            o3 = db_u * 3 * FR + (4 * g + (q8 & 3) + 16 * (G0 + np.where(q8 < 4, 0, 1))) * 16 + 8 * p8
            r1, r2, r3 = tr_b8(img, o1), tr_b8(img, o1 + 256), tr_b8(img, o3)
            ops = ((r1[:, :4] * 256.0, r1[:, 4:] * 1.0, r3[:, :4] / 256.0),
                   (r2[:, :4] * 256.0, r2[:, 4:] * 1.0, r3[:, 4:] / 256.0))
            for b in range(NB):
                pa = np.stack([P[2 * b + ((l & 15) >> 3), l >> 4, l & 7] for l in range(64)])
                for kk, (c2, c1, b0) in enumerate(ops):
                    U[b, 2 * w + kk] += (mfma_f16(pa, np.concatenate([c2, c2], 1), 8)
                                         + mfma_f16(pa, np.concatenate([c1, c1], 1), 8)
                                         + mfma_f16(pa[:, :4], b0, 4))
    out = np.zeros((RPC, 2048))
    for j in range(RPC):
        lt = np.array([lrow[j][(lanes & 15) == h].sum() for h in range(8)])  # the four lanes of column h
        for h in range(8):
            fs = 2 * smax / lt[h]
            for blkk in range(16):
                r = 8 * (j & 1) + h
                out[j, h * 256 + 16 * blkk: h * 256 + 16 * blkk + 16] = U[j // 2, blkk, r] * fs
    return out


import pytest


@pytest.mark.parametrize("RPC,L,qscale", [(3, 40, 0.3), (2, 72, 2.4)])
def test_beam_bank_index_math_matches_fp64(RPC, L, qscale):
    """Odd rows (the padded second row of the last block), a partial last key block, and (qscale 2.4) scores
    spread enough for running-maximum rescales inside the chunk."""
    rng = np.random.default_rng(5)
    m = rng.standard_normal((512, 256)).astype(np.float32)
    q_rows = (rng.standard_normal((RPC, 2048)) * qscale).astype(np.float32)
    got = emulate(m, q_rows, L)
    M = m[:L].astype(np.float64)
    for j in range(RPC):
        for h in range(8):
            sc = M @ q_rows[j, h * 256:(h + 1) * 256].astype(np.float64)
            p = np.exp(sc - sc.max())
            want = (p / p.sum()) @ M
            err = np.abs(got[j, h * 256:(h + 1) * 256] - want).max()
            assert err < 2e-5 * max(1.0, np.abs(want).max()), (j, h, err)
