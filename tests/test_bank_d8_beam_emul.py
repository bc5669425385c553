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


def emulate(m, q_rows, L, pipe=True):
    """One chunk, RPC = len(q_rows) rows (no masks): the kernel's arithmetic in float64 where it is exact,
    float32 / float16 where the kernel rounds.  Score wave p owns rows (2p, 2p + 1): column col = (row
    2p + (col >> 3), head col & 7)."""
    RPC = len(q_rows)
    NP = (RPC + 1) // 2
    blocks, s = pack_bank(m)
    smax = np.float32(s.max())
    kp = np.float32(128.0) / smax
    lanes = np.arange(64)
    col, g = lanes & 15, lanes >> 4
    qd, sgm = [], []  # per pair: [plane][db][lane] 16 digit bytes; sigma per lane
    for pr in range(NP):
        Qd = np.zeros((3, 4, 64, 16), np.int64)
        sg = np.zeros(64, np.float32)
        for l in range(64):
            j, h, gq = 2 * pr + ((l & 15) >> 3), l & 7, l >> 4
            if j >= RPC:
                continue
            qh = q_rows[j, h * 256:(h + 1) * 256].astype(np.float32)
            qs = np.float32(np.abs(qh).max() * np.float32(1 / AMAX))
            Q = np.rint(qh / (qs if qs > 0 else np.float32(1))).astype(np.int64)
            q2, q1, q0 = digits(Q)
            for db in range(4):
                sl = slice(64 * db + 16 * gq, 64 * db + 16 * gq + 16)
                Qd[2, db, l], Qd[1, db, l], Qd[0, db, l] = q2[sl] & 255, q1[sl] & 255, q0[sl] & 255
            sg[l] = qs * np.float32(65536)
        qd.append(Qd)
        sgm.append(sg)
    U = np.zeros((NP, 16, 16, 16))  # [pair][16-dim block] D[row][col]
    mrow = [np.full(64, -np.inf) for _ in range(NP)]
    lrow = [np.zeros(64) for _ in range(NP)]
    nkb = (L + 15) // 16
    for kb in range(nkb):
        img = lds_image(blocks[kb])
        P = np.zeros((NP, 4, 16, 8))  # [pair][g][col][hi x4 | lo x4]
        SC = np.ones((NP, 16))
        fb = lambda f: np.stack([img[f * FR + 16 * l: f * FR + 16 * l + 16] for l in range(64)])
        for pr in range(NP):
            X = np.zeros((4, 16, 16), np.int64)
            for db in range(4):
                a2, a1, a0 = fb(db * 3 + 2), fb(db * 3 + 1), fb(db * 3)
                Q2, Q1, Q0 = qd[pr][2, db], qd[pr][1, db], qd[pr][0, db]
                X[0] += mfma_i8(a2, Q2)
                X[1] += mfma_i8(a2, Q1) + mfma_i8(a1, Q2)
                X[2] += mfma_i8(a2, Q0) + mfma_i8(a1, Q1) + mfma_i8(a0, Q2)
                X[3] += mfma_i8(a1, Q0) + mfma_i8(a0, Q1)
            sv = np.zeros((64, 4))
            for l in range(64):
                for i in range(4):
                    r = 4 * (l >> 4) + i
                    sv[l, i] = X[0, r, l & 15] * 65536.0 + X[1, r, l & 15] * 256.0 + X[2, r, l & 15] \
                        + X[3, r, l & 15] / 256.0
            ks4 = np.stack([s[16 * kb + 4 * (l >> 4): 16 * kb + 4 * (l >> 4) + 4] for l in range(64)])
            sv = sv * (ks4 * sgm[pr][:, None])
            keys = 16 * kb + 4 * g[:, None] + np.arange(4)[None, :]
            sv = np.where(keys < L, sv, -np.inf)
            gm = sv.max(1)
            gm = np.array([gm[(lanes & 15) == (l & 15)].max() for l in range(64)])
            if np.any(gm > mrow[pr] + 6):
                nm = np.maximum(mrow[pr], gm)
                sc = np.where(nm == mrow[pr], 1.0, np.exp(mrow[pr] - nm))
                mrow[pr], lrow[pr] = nm, lrow[pr] * sc
                SC[pr] = sc[:16]
            p = np.where(sv == -np.inf, 0.0, np.exp(sv - mrow[pr][:, None]))
            lrow[pr] += p.sum(1)
            x = (p * (ks4 * kp)).astype(np.float32)
            hi = x.astype(np.float16)
            lo = (x - hi.astype(np.float32)).astype(np.float16)
            for l in range(64):
                P[pr, l >> 4, l & 15, :4] = hi[l]
                P[pr, l >> 4, l & 15, 4:] = lo[l]
        for b in range(NP):  # accumulator rows 4 g + i = columns 4 g + i of the pair
            for r in range(16):
                U[b, :, r, :] *= SC[b, r]
        # (dim-block pair, offsets): the two-phase kernel's wave w owns 16-dim blocks 2w, 2w + 1; the pipelined
        # kernel's context wave u owns 64-dim block u as the pairs gp = 0, 1 (offsets + 512 gp)
        q8, p8 = (lanes & 15) >> 1, lanes & 1
        units = []
        if pipe:
            for uu in range(4):
                o1 = (uu * 3 + np.where(q8 < 4, 2, 1)) * FR + (4 * g + (q8 & 3)) * 16 + 8 * p8
                o3 = uu * 3 * FR + (4 * g + (q8 & 3) + 16 * np.where(q8 < 4, 0, 1)) * 16 + 8 * p8
                units += [(4 * uu + 2 * gp, o1 + 512 * gp, o3 + 512 * gp) for gp in range(2)]
        else:
            for w in range(8):
                db_u, G0 = w >> 1, 2 * (w & 1)
                o1 = (db_u * 3 + np.where(q8 < 4, 2, 1)) * FR + (4 * g + (q8 & 3) + 16 * G0) * 16 + 8 * p8
                o3 = db_u * 3 * FR + (4 * g + (q8 & 3) + 16 * (G0 + np.where(q8 < 4, 0, 1))) * 16 + 8 * p8
                units.append((2 * w, o1, o3))
        for k0, o1, o3 in units:
            r1, r2, r3 = tr_b8(img, o1), tr_b8(img, o1 + 256), tr_b8(img, o3)
            ops = ((r1[:, :4] * 256.0, r1[:, 4:] * 1.0, r3[:, :4] / 256.0),
                   (r2[:, :4] * 256.0, r2[:, 4:] * 1.0, r3[:, 4:] / 256.0))
            for b in range(NP):
                pa = np.stack([P[b, l >> 4, l & 15] for l in range(64)])
                for kk, (c2, c1, b0) in enumerate(ops):
                    U[b, k0 + kk] += (mfma_f16(pa, np.concatenate([c2, c2], 1), 8)
                                         + mfma_f16(pa, np.concatenate([c1, c1], 1), 8)
                                         + mfma_f16(pa[:, :4], b0, 4))
    out = np.zeros((RPC, 2048))
    for b in range(NP):
        lt = np.array([lrow[b][(lanes & 15) == cc].sum() for cc in range(16)])  # the four lanes of a column
        for r in range(16):
            j, h = 2 * b + (r >> 3), r & 7
            if j >= RPC:
                continue
            fs = 2 * smax / lt[r]
            for blkk in range(16):
                out[j, h * 256 + 16 * blkk: h * 256 + 16 * blkk + 16] = U[b, blkk, r] * fs
    return out


import pytest


@pytest.mark.parametrize("RPC,L,qscale,pipe", [(3, 40, 0.3, True), (2, 72, 2.4, True), (3, 40, 0.3, False)])
def test_beam_bank_index_math_matches_fp64(RPC, L, qscale, pipe):
    """Odd rows (the padded second row of the last block), a partial last key block, and (qscale 2.4) scores
    spread enough for running-maximum rescales inside the chunk."""
    rng = np.random.default_rng(5)
    m = rng.standard_normal((512, 256)).astype(np.float32)
    q_rows = (rng.standard_normal((RPC, 2048)) * qscale).astype(np.float32)
    got = emulate(m, q_rows, L, pipe)
    M = m[:L].astype(np.float64)
    for j in range(RPC):
        for h in range(8):
            sc = M @ q_rows[j, h * 256:(h + 1) * 256].astype(np.float64)
            p = np.exp(sc - sc.max())
            want = (p / p.sum()) @ M
            err = np.abs(got[j, h * 256:(h + 1) * 256] - want).max()
            assert err < 2e-5 * max(1.0, np.abs(want).max()), (j, h, err)
