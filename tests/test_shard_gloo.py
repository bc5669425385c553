"""Multi-process read sharding on CPU (gloo, world_size 2): partition,
weight broadcast and stats reduction, with the engine replaced by a
deterministic stand-in (no GPU here)."""
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

    def __init__(self, W):
        self.W = W
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_reads, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    W0 = {"w": np.arange(10, dtype=np.float32)}
    seen = {}

    def tf(W):
        seen["W"] = W
        return FakeTranslator(W)

    g, preds = shard.run_distributed(n_reads, tf, lambda: W0, dev, batch_size=100, keep_predictions=True)
    q.put((rank, g, preds, seen["W"]["w"].tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_run_matches_single_process(world):
    n = 40
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
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
