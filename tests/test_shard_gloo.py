"""Multi-process read sharding on CPU (gloo, world_size 2, 4 and 8):
partition, weight broadcast, stats reduction and the rank-failure retry, with
the engine replaced by a deterministic stand-in (no GPU here)."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nanodecoder_amd import shard


def test_lpt_assign_partitions_and_balances():
    w = shard.read_lengths(1000, seed=3).tolist()
    parts = shard.lpt_assign(w, 8)
    flat = sorted(i for p in parts for i in p)
    assert flat == list(range(1000))
    loads = [sum(w[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(w)


def test_pack_unpack_roundtrip():
    W = {"b": np.arange(6, dtype=np.float32).reshape(2, 3), "a": np.ones(4, np.float32)}
    meta, blob = shard.pack_weights(W)
    out = shard.unpack_weights(meta, blob)
    for k in W:
        np.testing.assert_array_equal(out[k], W[k])


class FakeTranslator:
    """Per chunk: 'A' * (len % 7) then EOS — depends only on the chunk."""

    beam_size = 1

    def __init__(self, W, fail_sizes=()):
        self.W = W
        self.fail_sizes = set(fail_sizes)
        from nanodecoder_amd import synth
        self.cfg = synth.ModelConfig()

    def _tokens_to_sent(self, toks):
        out = []
        for t in toks:
            if t == self.cfg.eos_idx:
                break
            out.append(self.cfg.itos[t])
        return out

    def stream_reads(self, reads, batch_size):
        for ri, r in enumerate(reads):
            yield ri, [([0.0], [[4] * (len(c) % 7) + [3, 5]]) for c in r]

    def stream_raw_reads(self, raws, batch_size, normalization, L, stride, arrays=False):
        """The device front end's contract: raw reads in, windowed here;
        token arrays out (rows padded with EOS past the hypothesis)."""
        from nanodecoder_amd import frontend
        assert arrays and normalization == "median"
        for ri, raw in enumerate(raws):
            if raw.size in self.fail_sizes:
                raise RuntimeError(f"engine fault on a read of {raw.size} samples")
            w = frontend.windows(int(raw.size), L, stride)
            tok = np.full((len(w), 10), 3, np.int32)
            for j, (_, ln) in enumerate(w):
                tok[j, : ln % 7] = 4
                tok[j, ln % 7 + 1] = 5
            yield ri, tok, np.zeros(len(w), np.float32)


def test_read_shard_frontends_agree():
    """ReadShard's device front-end path (raw reads -> stream_raw_reads) and
    host path (normalise + window in the producer thread -> stream_reads)
    count the same samples, chunks and bases and give the same strings."""
    n = 30
    lengths = shard.read_lengths(n, seed=4)
    a, pa = shard.ReadShard(FakeTranslator(None)).run(list(range(n)), lengths, True)
    b, pb = shard.ReadShard(FakeTranslator(None), frontend="cpu").run(list(range(n)), lengths, True)
    assert a["frontend"] == "gpu" and b["frontend"] == "cpu"
    for k in ("samples", "chunks", "bases"):
        assert a[k] == b[k], k
    assert pa == pb


class FakeBeamTranslator(FakeTranslator):
    """A beam translator's device front end returns per-chunk (scores, n_best
    token lists), never token arrays (Translator.stream_raw_reads refuses
    arrays=True for beam_size > 1)."""
    beam_size = 5

    def stream_raw_reads(self, raws, batch_size, normalization, L, stride, arrays=False):
        from nanodecoder_amd import frontend
        if arrays:
            raise ValueError("arrays=True is for greedy / sampling decoding")
        for ri, raw in enumerate(raws):
            w = frontend.windows(int(raw.size), L, stride)
            yield ri, [([0.0, -1.0], [[4] * (ln % 7) + [3], [4]]) for _, ln in w]


def test_read_shard_beam_translator_on_device_frontend():
    """ReadShard's "auto" front end picks the device path for a
    beam translator too; it must read per-chunk results there (first
    hypothesis) and count what the host path counts."""
    n = 30
    lengths = shard.read_lengths(n, seed=5)
    a, pa = shard.ReadShard(FakeBeamTranslator(None)).run(list(range(n)), lengths, True)
    b, pb = shard.ReadShard(FakeTranslator(None), frontend="cpu").run(list(range(n)), lengths, True)
    assert a["frontend"] == "gpu"
    for k in ("samples", "chunks", "bases"):
        assert a[k] == b[k], k
    assert all(len(c) == 2 for r in pa.values() for c in r)  # n_best strings per chunk


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_reads, q, fail):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    W0 = {"w": np.arange(10, dtype=np.float32)}
    seen = {}
    lengths = shard.read_lengths(n_reads)

    def tf(W):
        seen["W"] = W
        if fail.get("rank") == rank:  # this rank's engine fails on its first read
            return FakeTranslator(W, fail_sizes={int(x) for x in lengths})
        return FakeTranslator(W, fail_sizes=fail.get("sizes", ()))

    if fail.get("sticky") and fail.get("rank") == rank:
        # a sticky device fault: once the engine has raised, every later device call on this rank raises too --
        # the rank's syncs and any collective on the default (device, RCCL in production) group
        state = {"broken": False}
        orig_run = shard.ReadShard.run

        def run(self, *a, **k):
            try:
                return orig_run(self, *a, **k)
            except Exception:
                state["broken"] = True
                raise

        def guard(fn):
            def wrapped(*a, **k):
                if state["broken"] and k.get("group") is None:
                    raise RuntimeError(f"{fn.__name__} on the device group after a sticky fault")
                return fn(*a, **k)
            return wrapped

        def sync(_dev):
            if state["broken"]:
                raise RuntimeError("device call after a sticky fault")
        shard.ReadShard.run = run
        shard._device_sync = sync
        for name in ("all_reduce", "barrier", "broadcast", "all_gather"):
            setattr(dist, name, guard(getattr(dist, name)))

    try:
        g, preds = shard.run_distributed(n_reads, tf, lambda: W0, dev, batch_size=100, keep_predictions=True)
        q.put((rank, g, preds, seen["W"]["w"].tolist(), None))
    except shard.ShardFailure as e:
        q.put((rank, None, None, None, e.read_ids))
    dist.destroy_process_group()


def _run_world(world, n, fail):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q, fail)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def _check_complete(res, n):
    # every rank received rank 0's weights through the broadcast
    assert all(r[3] == list(range(10)) for r in res)
    # all reads translated exactly once across ranks
    got = {}
    for r in res:
        assert not (set(got) & set(r[2]))
        got.update(r[2])
    assert sorted(got) == list(range(n))
    # the reduced stats equal a single-process run
    lengths = shard.read_lengths(n)
    single, preds1 = shard.ReadShard(FakeTranslator(None)).run(list(range(n)), lengths, True)
    g = res[0][1]
    assert g["samples"] == single["samples"] and g["bases"] == single["bases"] and g["chunks"] == single["chunks"]
    assert got == preds1
    return g


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_run_matches_single_process(world):
    n = 40 * world
    res = _run_world(world, n, {})
    g = _check_complete(res, n)
    assert g["world"] == world and g["retried"] == 0
    # LPT balance: no rank carries more than the mean plus one read's samples
    lengths = shard.read_lengths(n)
    assert max(g["samples_per_rank"]) - min(g["samples_per_rank"]) <= int(lengths.max())


def test_failed_rank_reads_are_reassigned():
    """World 4, rank 2's translator fails on its first read: its reads go to
    ranks 0, 1, 3 (LPT) and the job's output equals a failure-free run."""
    n, world = 120, 4
    res = _run_world(world, n, {"rank": 2})
    g = _check_complete(res, n)
    lengths = shard.read_lengths(n)
    assert g["retried"] == len(shard.lpt_assign(lengths.tolist(), world)[2])
    assert res[2][2] == {}  # the failed rank kept none of the results


def test_reads_failing_everywhere_are_named():
    """A read no rank can translate: every rank raises ShardFailure naming the
    reads left untranslated (the failing read among them)."""
    n, world = 40, 2
    lengths = shard.read_lengths(n)
    bad = int(lengths[7])
    res = _run_world(world, n, {"sizes": [bad]})
    named = [r[4] for r in res]
    assert all(x is not None for x in named) and named[0] == named[1]
    assert 7 in named[0]


def test_sticky_device_fault_keeps_rank_in_the_job():
    """world 3, rank 1's engine raises and from then on every
    device call on that rank raises too (a sticky HIP error: syncs and
    collectives on the device group).  The flag exchanges, the counters and
    the closing barrier run on the CPU gloo group, so the faulted rank still
    takes part: its reads are re-assigned, nobody blocks, every rank returns
    the job's stats (failed_ranks [1]) and the output equals a failure-free
    run."""
    n, world = 90, 3
    res = _run_world(world, n, {"rank": 1, "sticky": True})
    g = _check_complete(res, n)
    assert g["failed_ranks"] == [1]
    assert res[1][1]["device_ok"] is False and res[0][1]["device_ok"] is True
