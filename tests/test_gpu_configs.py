"""BASELINE.json configs at their real sizes, end to end, against the oracle
(needs an MI355X).

Which kernels a call runs depends on the batch: at 256 chunks the decoder
GEMMs take the LDS-staged ``gemm_p16s_kernel`` and the K = 2048 products the
long-K P16 kernel; at 1024 chunks x beam 5 the LDS-tiled large-M route, and
the --fast beam's tail segments (few chunks alive) the small-M kernels again.
The smaller parity tests in test_gpu_parity.py run none of the first.  Each
test here asserts the route it covers (nd_gemm_routes) and compares with
oracle/ref_cpu.py (the reference's algorithm, pinned to its own outputs):
log-probs within 1e-3, identical tokens except after a genuine oracle
near-tie (top-2 margin < 1e-4).  Reference: translate/translator.py:396-503
(greedy), :619-825 (--fast beam).

Also here: the EnginePool (several calls in flight on one GPU) against the
single engine, and a graph-cache regression (the decoder's memory view after
an exact-fp32 call).
"""
import types

import numpy as np
import pytest

from nanodecoder_amd import synth
from tests import golden_util as gu

pytestmark = pytest.mark.gpu

LOGP_ATOL = 1e-3
TIE_MARGIN = 1e-4


def _oracle():
    from oracle import ref_cpu
    return ref_cpu


def _engine(cfg, W, **kw):
    from nanodecoder_amd.engine import Engine
    return Engine(cfg, W, device=0, **kw)


def _routes(reset=True):
    from nanodecoder_amd import _lib
    return _lib.gemm_routes(reset=reset)


def _tie_rows(got, exp_tokens, exp_logp):
    """Rows whose tokens differ from the oracle's; each first difference must
    be a genuine oracle near-tie.  Returns the set of such rows."""
    rows = set()
    for b in range(exp_tokens.shape[0]):
        d = np.nonzero(got[b] != exp_tokens[b])[0]
        if d.size:
            s = int(d[0])
            top2 = np.sort(exp_logp[b, s])[-2:]
            assert top2[1] - top2[0] < TIE_MARGIN, (b, s, got[b, s], exp_tokens[b, s], top2)
            rows.add(b)
    return rows


@pytest.mark.parametrize("encoder,splitk", [("transformer", True), ("transformer", False), ("nano", True)])
def test_greedy_config_batch256_vs_oracle(encoder, splitk):
    """configs[1] (3+3 transformer) and configs[2] (NanoEncoder + transformer
    decoder): 256 chunks x 512 samples, greedy, max_length 100, -min_length 57
    (the bench's workload, mask samples injected), every chunk against the
    oracle.  Asserts the M = 256 GEMM kernels ran (gemm_p16s, and the K = 2048
    products split over workgroups as EnginePool lanes run them, or on the
    long-K P16 kernel as a lone engine does: nd_set_gemm_splitk)."""
    ref = _oracle()
    cfg = synth.ModelConfig(encoder_type=encoder)
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    B, S, MINL = 256, 100, 57
    sig = synth.synth_chunk_batch(B, 512, seed=1000)
    lens = np.full(B, 512, np.int32)
    eng = _engine(cfg, W, max_batch=B, max_steps=S)
    eng.set_gemm_splitk(splitk)
    _routes()
    r = eng.translate_greedy(sig, lens, lens, max_len=S, min_len=MINL)  # the bench's graph (no log-prob dump)
    routes = _routes()
    # 256 rows: the N = 2048 products (query projection, FFN1) on gemm_p16s<2,4>, the QKV products on
    # gemm_p16s<2,2>, the K = 2048 products (W_vo, FFN2) split over K (gemm_p16k_kernel) or on the long-K P16
    # kernel (Wo, N = K = 256, stays on gemm_p16<1,4,64>)
    assert routes["p16s_2x4"] > 0 and routes["p16s_2x2"] > 0, routes
    if splitk:
        assert routes["p16_splitk"] > 0 and routes["p16_longk"] == 0, routes
    else:
        assert routes["p16_splitk"] == 0 and routes["p16_longk"] > 0, routes
    rl = eng.translate_greedy(sig, lens, lens, max_len=S, min_len=MINL, return_logp=True)
    tok = r["tokens"].cpu().numpy()
    assert (tok == rl["tokens"].cpu().numpy()).all()
    assert (r["scores"].cpu().numpy() == rl["scores"].cpu().numpy()).all()
    o = ref.greedy(ref.RefModel(cfg, W), sig, lens, max_length=S, min_length=MINL)
    ties = _tie_rows(tok, o["tokens"], o["logp"])
    assert len(ties) <= 3, ties
    keep = np.array([b not in ties for b in range(B)])
    lp = rl["logp"].cpu().numpy()
    assert gu.logp_close(lp[keep], o["logp"][keep], atol=LOGP_ATOL).all()
    assert np.abs(r["scores"].cpu().numpy()[keep] - o["scores"][keep]).max() < LOGP_ATOL
    assert int(r["overflow"].cpu()[0]) == 0


def test_beam_config3_batch1024_sampled_vs_oracle():
    """configs[3]: --fast beam 5 on 1024 chunks, max_length 100, -min_length
    57, mask samples injected (src==0 encoder keys, src==1 context keys: the
    24-bit context K/V image and the tail's list-split kernels meet masked
    keys at size).  Most chunks finish at step ~58; the few that run on are
    decoded by the tail segments (GraphKey.tail: <= 1/16 of the chunks alive,
    small-M GEMM kernels).  64 chunks are compared with the oracle: every
    chunk that ran into the tail (up to 32) plus random others."""
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    B, S, MINL, NPICK = 1024, 100, 57, 64
    sig = synth.synth_chunk_batch(B, 512, seed=2000, inject_masks=True)
    lens = np.full(B, 512, np.int32)
    eng = _engine(cfg, W, max_batch=B, max_steps=S, max_beam=5)
    _routes()
    r = eng.translate_beam(sig, lens, lens, beam=5, n_best=1, max_len=S, min_len=MINL)  # the bench's graphs
    routes = _routes()
    assert eng.bank_form() == 3
    ra = eng.translate_beam(sig, lens, lens, beam=5, n_best=1, max_len=S, min_len=MINL, return_attn=True)
    tok, sc, ln = (r[k].cpu().numpy() for k in ("tokens", "scores", "lens"))
    assert (tok == ra["tokens"].cpu().numpy()).all() and (ln == ra["lens"].cpu().numpy()).all()
    assert int(r["overflow"].cpu()[0]) == 0
    done = ra["done_step"].cpu().numpy()
    steps = int(r["steps"].cpu()[0])
    # the segment polls see at most B / 16 chunks alive from some step on: the tail ran
    alive_at = [int((done > s0).sum()) for s0 in range(10, steps, 10)]
    assert any(16 * a <= B for a in alive_at), alive_at
    assert routes["p16_big"] > 0 and routes["p16_longk"] > 0, routes  # large-M route and the tail's small-M kernels
    tail = [int(i) for i in np.nonzero(done > 60)[0]][: NPICK // 2]
    assert tail, "no chunk ran into the tail"
    rng = np.random.default_rng(5)
    rest = [int(i) for i in rng.choice(np.setdiff1d(np.arange(B), tail), NPICK - len(tail), replace=False)]
    pick = sorted(tail + rest)
    exp = ref.fast_beam(ref.RefModel(cfg, W), sig[pick], lens[pick], beam_size=5, n_best=1, max_length=S,
                        min_length=MINL)
    for j, i in enumerate(pick):
        s, p = exp[j][0]
        assert ln[i, 0] == len(p), (i, ln[i, 0], len(p))
        assert (tok[i, 0, : len(p)] == p).all(), i
        assert abs(sc[i, 0] - s) < LOGP_ATOL, (i, sc[i, 0], s)


@pytest.mark.parametrize("B,T,encoder", [(256, 300, "transformer"), (64, 200, "transformer"), (64, 300, "nano")])
def test_greedy_short_chunks_vs_oracle(B, T, encoder):
    """Chunks shorter than 512 samples: the reference authors' production
    runs use -src_seq_length 300 (pipeline.evaluate.sh:83-89),
    the 24-bit digit bank streams ceil(T / 128) key blocks per wave there
    (bank8.hip bank8_kpw).  Greedy, max_length 100, -min_length 57, mask
    samples injected, every chunk against the oracle."""
    ref = _oracle()
    cfg = synth.ModelConfig(encoder_type=encoder)
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    S, MINL = 100, 57
    sig = synth.synth_chunk_batch(B, T, seed=4000 + T, inject_masks=True)
    lens = np.full(B, T, np.int32)
    eng = _engine(cfg, W, max_batch=B, max_steps=S)
    r = eng.translate_greedy(sig, lens, lens, max_len=S, min_len=MINL, return_logp=True)
    assert eng.bank_form() == 2
    assert int(r["overflow"].cpu()[0]) == 0
    eng.close()
    tok, lp = r["tokens"].cpu().numpy(), r["logp"].cpu().numpy()
    o = ref.greedy(ref.RefModel(cfg, W), sig, lens, max_length=S, min_length=MINL)
    ties = _tie_rows(tok, o["tokens"], o["logp"])
    assert len(ties) <= 3, ties
    keep = np.array([b not in ties for b in range(B)])
    assert gu.logp_close(lp[keep], o["logp"][keep], atol=LOGP_ATOL).all()
    assert np.abs(r["scores"].cpu().numpy()[keep] - o["scores"][keep]).max() < LOGP_ATOL


@pytest.mark.parametrize("beam,fast", [(7, True), (8, True), (8, False)])
def test_beam_up_to_8_vs_oracle(beam, fast):
    """beam_size 7 and 8 (the reference takes any, models/opts.py:581; the
    engine's bound is 8): --fast beam (and the classic Beam at 8) on 16
    chunks, n_best 2, max_length 100, -min_length 57, masks injected, every
    chunk's two best hypotheses against the oracle."""
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    B, S, MINL, NB = 16, 100, 57, 2
    sig = synth.synth_chunk_batch(B, 512, seed=4200 + beam, inject_masks=True)
    lens = np.full(B, 512, np.int32)
    eng = _engine(cfg, W, max_batch=B, max_steps=S, max_beam=beam)
    if fast:
        r = eng.translate_beam(sig, lens, lens, beam=beam, n_best=NB, max_len=S, min_len=MINL)
    else:
        r = eng.translate_beam_classic(sig, lens, lens, beam=beam, n_best=NB, max_len=S, min_len=MINL)
    assert int(r["overflow"].cpu()[0]) == 0
    eng.close()
    tok, sc, ln = (r[k].cpu().numpy() for k in ("tokens", "scores", "lens"))
    run = ref.fast_beam if fast else ref.classic_beam
    exp = run(ref.RefModel(cfg, W), sig, lens, beam_size=beam, n_best=NB, max_length=S, min_length=MINL)
    for i in range(B):
        for n in range(NB):
            s, p = exp[i][n]
            assert ln[i, n] == len(p), (i, n, ln[i, n], len(p))
            assert (tok[i, n, : len(p)] == p).all(), (i, n)
            assert abs(sc[i, n] - s) < LOGP_ATOL, (i, n, sc[i, n], s)


def test_beam_short_chunks_vs_oracle():
    """The production beam flags' chunk length (-src_seq_length 300, beam 5,
    pipeline.evaluate.sh:100-106): --fast beam 5 on 64 chunks of 300 samples
    (the 24-bit context K/V image and the tail's list kernels at T = 300),
    max_length 100, -min_length 57, masks injected, every chunk against the
    oracle."""
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    B, T, S, MINL = 64, 300, 100, 57
    sig = synth.synth_chunk_batch(B, T, seed=4100, inject_masks=True)
    lens = np.full(B, T, np.int32)
    eng = _engine(cfg, W, max_batch=B, max_steps=S, max_beam=5)
    r = eng.translate_beam(sig, lens, lens, beam=5, n_best=1, max_len=S, min_len=MINL)
    assert eng.bank_form() == 3
    assert int(r["overflow"].cpu()[0]) == 0
    eng.close()
    tok, sc, ln = (r[k].cpu().numpy() for k in ("tokens", "scores", "lens"))
    exp = ref.fast_beam(ref.RefModel(cfg, W), sig, lens, beam_size=5, n_best=1, max_length=S, min_length=MINL)
    for i in range(B):
        s, p = exp[i][0]
        assert ln[i, 0] == len(p), (i, ln[i, 0], len(p))
        assert (tok[i, 0, : len(p)] == p).all(), i
        assert abs(sc[i, 0] - s) < LOGP_ATOL, (i, sc[i, 0], s)


@pytest.mark.parametrize("mode", ["greedy", "beam"])
def test_long_max_length_vs_oracle(mode):
    """max_length 400 (up to 512 supported; the reference takes any,
    models/opts.py:577): -min_length 380 keeps every hypothesis decoding past
    step 256, so the self-attention histories run three and four key passes
    and the beam rows' chunk kernel its second slot table.  Greedy: 16 chunks,
    every one against the oracle; --fast beam 5: 4 chunks (20 rows, the
    chunk-per-workgroup self-attention over the 24-bit history)."""
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    S, MINL = 400, 380
    B = 16 if mode == "greedy" else 4
    sig = synth.synth_chunk_batch(B, 512, seed=3000, inject_masks=True)
    lens = np.full(B, 512, np.int32)
    if mode == "greedy":
        eng = _engine(cfg, W, max_batch=B, max_steps=S)
        r = eng.translate_greedy(sig, lens, lens, max_len=S, min_len=MINL, return_logp=True)
        assert int(r["overflow"].cpu()[0]) == 0
        tok, lp = r["tokens"].cpu().numpy(), r["logp"].cpu().numpy()
        o = ref.greedy(ref.RefModel(cfg, W), sig, lens, max_length=S, min_length=MINL)
        ties = _tie_rows(tok, o["tokens"], o["logp"])
        assert len(ties) <= 1, ties
        keep = np.array([b not in ties for b in range(B)])
        assert gu.logp_close(lp[keep], o["logp"][keep], atol=LOGP_ATOL).all()
        assert np.abs(r["scores"].cpu().numpy()[keep] - o["scores"][keep]).max() < LOGP_ATOL
    else:
        eng = _engine(cfg, W, max_batch=B, max_steps=S, max_beam=5)
        r = eng.translate_beam(sig, lens, lens, beam=5, n_best=1, max_len=S, min_len=MINL)
        assert int(r["overflow"].cpu()[0]) == 0
        assert int(r["steps"].cpu()[0]) > 300
        tok, sc, ln = (r[k].cpu().numpy() for k in ("tokens", "scores", "lens"))
        exp = ref.fast_beam(ref.RefModel(cfg, W), sig, lens, beam_size=5, n_best=1, max_length=S, min_length=MINL)
        for i in range(B):
            s, p = exp[i][0]
            assert ln[i, 0] == len(p), (i, ln[i, 0], len(p))
            assert (tok[i, 0, : len(p)] == p).all(), i
            assert abs(sc[i, 0] - s) < LOGP_ATOL, (i, sc[i, 0], s)
    eng.close()


@pytest.mark.parametrize("encoder,mode", [("transformer", "greedy"), ("nano", "greedy"), ("transformer", "beam")])
def test_pool_matches_single_engine(encoder, mode):
    """EnginePool (two calls in flight, one engine context and hardware
    queue each, their kernels sharing the CUs) returns bit-for-bit what one
    engine returns for the same batches.  Greedy calls are issued from one
    host thread; --fast beam calls (host-synchronous segment polls) from one
    thread per lane, as bench.py runs them."""
    import threading
    import torch
    from nanodecoder_amd.engine import EnginePool
    cfg = synth.ModelConfig(encoder_type=encoder)
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0 if mode == "greedy" else 1.0)
    B, S = 64, 40
    beam = 5 if mode == "beam" else 1
    batches = [synth.synth_chunk_batch(B, 512, seed=300 + k) for k in range(6)]
    lens = np.full(B, 512, np.int32)
    keys = ("tokens", "scores", "logp") if mode == "greedy" else ("tokens", "scores", "lens")

    def call(e, b):
        if mode == "greedy":
            return e.translate_greedy(b, lens, lens, max_len=S, min_len=5, return_logp=True)
        return e.translate_beam(b, lens, lens, beam=beam, n_best=2, max_len=S, min_len=3)
    one = _engine(cfg, W, max_batch=B, max_steps=S, max_beam=beam)
    one.set_gemm_splitk(True)  # the pool lanes' form
    exp = [{k: v.cpu() for k, v in call(one, b).items() if k in keys} for b in batches]
    one.close()
    # bank_grid 16: each lane's memory-bank workgroups walk 4 of the 64 chunks (nd_set_bank_grid)
    pool = EnginePool(cfg, W, device=0, lanes=2, max_batch=B, max_steps=S, max_beam=beam, bank_grid=16)
    dev_b = [torch.from_numpy(b).cuda() for b in batches]
    for rnd in range(2):
        if mode == "greedy":
            got = [call(pool, b) for b in dev_b]
            assert [g["lane"] for g in got] == [0, 1] * 3
            pool.synchronize()
        else:
            got = [None] * len(dev_b)
            cur = torch.cuda.current_stream()

            def lane(i):
                e = pool.engines[i]
                with torch.cuda.stream(e.stream):
                    for k in range(i, len(dev_b), 2):
                        got[k] = call(e, dev_b[k])
            for e in pool.engines:
                e.stream.wait_stream(cur)
            th = [threading.Thread(target=lane, args=(i,)) for i in range(2)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            pool.synchronize()
        torch.cuda.synchronize()
        for k, (g, e) in enumerate(zip(got, exp)):
            for key in keys:
                assert torch.equal(g[key].cpu(), e[key]), (rnd, k, key)
    pool.close()


def _ragged(sig, seed):
    """Half the chunks cut to 300..511 samples (zero padded, span = the
    reference batch of 4 consecutive chunks' longest): pad-masked keys and
    spans < T beside full chunks."""
    rng = np.random.default_rng(seed)
    B = sig.shape[0]
    lens = np.full(B, 512, np.int32)
    cut = rng.random(B) < 0.5
    lens[cut] = rng.integers(300, 512, size=int(cut.sum()))
    sig = sig.copy()
    for b in np.nonzero(cut)[0]:
        sig[b, lens[b]:] = 0.0
    spans = lens.reshape(-1, 4).max(axis=1).repeat(4).astype(np.int32)
    return sig, lens, spans


@pytest.mark.parametrize("key", ["configs[1]", "configs[2]", "configs[3]", "configs[1] exact"])
def test_pool_at_bench_config_matches_single_engine(key):
    """The bench's headline mode exactly (bench.py run_batch / config_legs):
    EnginePool with 3 lanes, the memory-bank kernel on half the CUs (the
    pool's default bank grid, 128 workgroups walking the chunks), every
    lane's bank non-temporal, 256 chunks (1024 for --fast beam 5),
    max_length 100, -min_length 57, the graphs the bench replays (no log-prob
    dump).  Six distinct batches (every other one ragged: pad-masked chunks,
    spans < T) go through the pool twice, three calls in flight (greedy:
    one host thread; beam: one thread per lane, as the bench); every pooled
    call equals a single engine's bitwise.  The single engine is pinned to
    the oracle at these sizes by the two tests above.  "configs[1] exact":
    the bench's exact_fp32 leg (nd_set_exact_fp32 on every lane: the fp32
    bank kernel walking two chunks per workgroup with the second chunk's
    head prefetched, the fp32 split-K products), against a single exact
    engine (tests/test_gpu_precision.py pins that one to the oracle)."""
    import threading
    import torch
    from nanodecoder_amd.engine import EnginePool
    enc, mode, B = {"configs[1]": ("transformer", "greedy", 256), "configs[2]": ("nano", "greedy", 256),
                    "configs[3]": ("transformer", "beam", 1024),
                    "configs[1] exact": ("transformer", "greedy", 256)}[key]
    exact = key.endswith("exact")
    cfg = synth.ModelConfig(encoder_type=enc)
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    S, MINL, beam, lanes = 100, 57, (5 if mode == "beam" else 1), 3
    inputs = []
    for k in range(6):
        sig = synth.synth_chunk_batch(B, 512, seed=500 + k, inject_masks=(mode == "greedy"))
        if k % 2:
            inputs.append(_ragged(sig, 900 + k))
        else:
            inputs.append((sig, np.full(B, 512, np.int32), np.full(B, 512, np.int32)))
    keys = ("tokens", "scores") if mode == "greedy" else ("tokens", "scores", "lens", "steps")

    def call(e, inp):
        sig, ln, sp = inp
        if mode == "greedy":
            return e.translate_greedy(sig, ln, sp, max_len=S, min_len=MINL)
        return e.translate_beam(sig, ln, sp, beam=beam, n_best=1, max_len=S, min_len=MINL)
    one = _engine(cfg, W, max_batch=B, max_steps=S, max_beam=beam)
    one.set_gemm_splitk(True)  # the pool lanes' K = 2048 product form (its own test: the config tests above)
    one.set_exact_fp32(exact)
    exp = [{k: v.cpu() for k, v in call(one, i).items() if k in keys} for i in inputs]
    one.close()
    pool = EnginePool(cfg, W, device=0, lanes=lanes, max_batch=B, max_steps=S, max_beam=beam)
    pool.set_exact_fp32(exact)
    assert pool.splitk
    assert pool.bank_nt_lanes == (0, 1, 2)
    assert pool.bank_grid == torch.cuda.get_device_properties(0).multi_processor_count // 2
    dev_in = [tuple(torch.from_numpy(a).cuda() for a in i) for i in inputs]
    for rnd in range(2):
        if mode == "greedy":
            got = [call(pool, i) for i in dev_in]
            assert [g["lane"] for g in got] == [0, 1, 2] * 2
            pool.synchronize()
        else:
            got = [None] * len(dev_in)
            cur = torch.cuda.current_stream()

            def lane(i):
                e = pool.engines[i]
                with torch.cuda.stream(e.stream):
                    for k in range(i, len(dev_in), lanes):
                        got[k] = call(e, dev_in[k])
            for e in pool.engines:
                e.stream.wait_stream(cur)
            th = [threading.Thread(target=lane, args=(i,)) for i in range(lanes)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            pool.synchronize()
        torch.cuda.synchronize()
        for k, (g, e) in enumerate(zip(got, exp)):
            for name in keys:
                assert torch.equal(g[name].cpu(), e[name]), (key, rnd, k, name)
            assert int(g["overflow"].cpu()[0]) == 0
    pool.close()


def test_pooled_encoder_memory_matches_serial():
    """The encoder's output (the memory bank, before its pack) when another
    lane's decoders share the CUs equals the serial encoder's bitwise (ADVICE
    r04: the layer-0 closed-form attention, whose round-3 layout returned
    wrong chunks only beside another engine's kernels, DESIGN.md section 5, is
    guarded here on its own output, not only through the tokens it changes).
    Three lanes at the bench's sizes: lanes 0 and 1 run greedy calls
    (max_length 100) while lane 2 encodes on its own stream, three rounds."""
    import torch
    from nanodecoder_amd.engine import EnginePool
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    B, S = 256, 100
    inputs = []
    for k in range(3):
        sig = synth.synth_chunk_batch(B, 512, seed=700 + k, inject_masks=True)
        inputs.append(_ragged(sig, 950 + k) if k % 2 else (sig, np.full(B, 512, np.int32),
                                                            np.full(B, 512, np.int32)))
    one = _engine(cfg, W, max_batch=B, max_steps=S)
    exp = []
    for sig, ln, sp in inputs:
        m = one.encode(sig, ln, sp).cpu().numpy()
        exp.append([m[b, : sp[b]] for b in range(B)])  # rows >= span are unspecified
    one.close()
    pool = EnginePool(cfg, W, device=0, lanes=3, max_batch=B, max_steps=S)
    dev_in = [tuple(torch.from_numpy(a).cuda() for a in i) for i in inputs]
    enc = pool.engines[2]
    for rnd in range(3):
        got = []
        for k, inp in enumerate(dev_in):
            pool._next = 0  # lanes 0 and 1 decode
            r0 = pool.translate_greedy(*inp, max_len=S, min_len=57)
            r1 = pool.translate_greedy(*dev_in[(k + 1) % len(dev_in)], max_len=S, min_len=57)
            enc.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(enc.stream):
                mem = enc.encode(*inp)
            torch.cuda.current_stream().wait_stream(enc.stream)
            got.append(mem)
            del r0, r1
        pool.synchronize()
        torch.cuda.synchronize()
        for k, mem in enumerate(got):
            m = mem.cpu().numpy()
            sp = inputs[k][2]
            bad = [b for b in range(B) if not np.array_equal(m[b, : sp[b]], exp[k][b])]
            assert not bad, (rnd, k, bad[:8])
    pool.close()


def test_translator_reads_with_pool_vs_oracle():
    """Translator.translate_reads on an EnginePool (two engine batches in
    flight while the next is packed): identical strings and scores to the
    oracle run read by read (translate/translator.py:181-369)."""
    from nanodecoder_amd import frontend
    from nanodecoder_amd.engine import EnginePool
    from nanodecoder_amd.translator import Translator
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-1.0)
    S, bs = 40, 3
    reads = [frontend.window(frontend.normalize(synth.synth_raw_read(80 + i, n), "median"), 512, 512)
             for i, n in enumerate((1300, 700, 512, 2049, 300, 1100, 1536, 90, 3000, 800))]
    pool = EnginePool(cfg, W, device=0, lanes=2, max_batch=4, max_steps=S)
    opt = types.SimpleNamespace(gpu=0, n_best=1, max_length=S, min_length=4, beam_size=1, batch_size=bs,
                                engine_max_batch=4)
    got = Translator(cfg, None, opt, engine=pool).translate_reads(reads, batch_size=bs)
    m = ref.RefModel(cfg, W)
    n = 0
    for ri, chunks in enumerate(reads):
        es, ep = ref.translate(m, chunks, bs, max_length=S, min_length=4)
        assert got[ri][1] == ep, ri
        assert np.abs(np.array(got[ri][0]) - np.array(es)).max() < 1e-3, ri
        n += len(chunks)
    assert n > 20
    pool.close()


def test_read_shard_device_frontend_vs_oracle():
    """configs[4]'s per-rank path (shard.ReadShard, the default device front
    end): raw synthetic reads -> Translator.stream_raw_reads on a 3-lane
    EnginePool (every engine batch normalised and windowed on the device, on
    its call's stream; reads split across engine batches) -> token arrays.
    Every read's strings equal the oracle's per-read translate on the host
    front end's chunks, and the sample / chunk / base counts equal the host
    front-end path's (utils/labelop.py:194-233, translator.py:181-369)."""
    from nanodecoder_amd import frontend, shard
    from nanodecoder_amd.engine import EnginePool
    from nanodecoder_amd.translator import Translator
    ref = _oracle()
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-1.0)
    S, bs = 30, 100
    pool = EnginePool(cfg, W, device=0, lanes=3, max_batch=8, max_steps=S)
    opt = types.SimpleNamespace(gpu=0, n_best=1, max_length=S, min_length=4, beam_size=1, batch_size=bs,
                                engine_max_batch=8)
    tr = Translator(cfg, None, opt, engine=pool)
    n = 24
    lengths = shard.read_lengths(n, seed=9, lo=100, hi=1700)
    ids = list(range(n))
    a, pa = shard.ReadShard(tr, batch_size=bs).run(ids, lengths, keep_predictions=True)
    b, pb = shard.ReadShard(tr, batch_size=bs, frontend="cpu").run(ids, lengths, keep_predictions=True)
    assert a["frontend"] == "gpu" and b["frontend"] == "cpu"
    for k in ("samples", "chunks", "bases"):
        assert a[k] == b[k], k
    assert pa == pb
    m = ref.RefModel(cfg, W)
    for rid in ids:
        chunks = frontend.window(frontend.normalize(shard.synth_raw(rid, int(lengths[rid])), "median"), 512, 512)
        _, ep = ref.translate(m, chunks, bs, max_length=S, min_length=4)
        assert pa[rid] == ep, rid
    pool.close()


def _eos_steps(cfg, W, sig, lens, S):
    """First EOS step of every chunk under greedy (S if none)."""
    eng = _engine(cfg, W, max_batch=sig.shape[0], max_steps=S)
    tok = eng.translate_greedy(sig, lens, lens, max_len=S)["tokens"].cpu().numpy()
    eng.close()
    hit = tok == cfg.eos_idx
    return np.where(hit.any(1), hit.argmax(1), S)


def test_beam1_segments_captured_after_exact_call():
    """the decoder's memory view (split-fp16 fragment bank or fp32
    bank) must follow the call, not the last captured encoder graph.  A
    beam-1 --fast call that stops early captures only its first 10-step
    segment; an exact-fp32 call follows; the next split-fp16 beam-1 call
    replays the cached encoder graph and captures its later segments for the
    first time.  Its results must equal a fresh engine's."""
    cfg = synth.ModelConfig()
    S = 40
    pool_sig = synth.synth_chunk_batch(96, 512, seed=41, inject_masks=False)
    lens = np.full(4, 512, np.int32)
    for eb in (2.0, 3.0, 4.0, 5.0, 6.0, 8.0, 10.0):
        W = synth.make_weights(cfg, seed=12, eos_bias=eb)
        st = _eos_steps(cfg, W, pool_sig, np.full(96, 512, np.int32), S)
        order = np.argsort(st, kind="stable")
        early, late = order[:4], order[-4:]
        if st[early].max() < 9 and st[late].min() >= 12:
            break
    else:
        pytest.fail(f"no early/late chunk split found: {np.sort(st)}")
    eng = _engine(cfg, W, max_batch=4, max_steps=S, max_beam=1)
    a = eng.translate_beam(pool_sig[early], lens, lens, beam=1, max_len=S)
    assert int(a["steps"].cpu()[0]) <= 10
    eng.set_exact_fp32(True)
    eng.translate_beam(pool_sig[late], lens, lens, beam=1, max_len=S)
    eng.set_exact_fp32(False)
    c = eng.translate_beam(pool_sig[late], lens, lens, beam=1, max_len=S)
    fresh = _engine(cfg, W, max_batch=4, max_steps=S, max_beam=1)
    f = fresh.translate_beam(pool_sig[late], lens, lens, beam=1, max_len=S)
    assert int(f["steps"].cpu()[0]) > 10
    for k in ("tokens", "scores", "lens"):
        assert (c[k].cpu().numpy() == f[k].cpu().numpy()).all(), k


def test_shared_weights_outlive_an_early_close():
    """closing the engine whose weights other lanes read (lane 0,
    or a pool made by subset) must not free them under the readers: the
    source refuses calls from then on and is freed with its last reader;
    the reader's results are unchanged.  A weight load into a sharing context
    is refused (nd_share_weights' contract)."""
    import ctypes
    from nanodecoder_amd import _lib
    from nanodecoder_amd.engine import Engine
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    sig = synth.synth_chunk_batch(8, 512, seed=3)
    lens = np.full(8, 512, np.int32)
    src = Engine(cfg, W, device=0, max_batch=8, max_steps=30)
    want = src.translate_greedy(sig, lens, lens, max_len=30)["tokens"].cpu()
    lane = Engine(cfg, W, device=0, max_batch=8, max_steps=30, share_from=src)
    a = np.zeros(4, np.float32)
    shape = (ctypes.c_int64 * 1)(4)
    rc = lane._L.nd_load_weight(lane._h, b"encoder.layer_norm.bias", a.ctypes.data_as(ctypes.c_void_p), shape, 1)
    assert rc == _lib.ND_ERR_STATE
    src.close()
    assert src._h is not None and src._close_pending          # still alive: lane reads its weights
    with pytest.raises(_lib.NanodecError):
        src.translate_greedy(sig, lens, lens, max_len=30)
    got = lane.translate_greedy(sig, lens, lens, max_len=30)["tokens"].cpu()
    assert (got == want).all()
    lane.close()
    assert lane._h is None and src._h is None                  # the source went with its last reader
