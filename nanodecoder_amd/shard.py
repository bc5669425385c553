"""Multi-GPU read sharding (BASELINE config 5).

Reads are independent, so the path shards with NO collective in the hot
loop: one process per GPU (torch.distributed.run), reads assigned to ranks by
a longest-processing-time balance on sample count, rank 0's weights sent once
as one packed fp32 blob (``broadcast`` — RCCL over xGMI with backend "nccl"),
and after the loop the failure flags and one ``all_reduce`` of [samples,
bases, chunks] (+ MAX of seconds) for reporting, on a CPU gloo group.  Each rank packs chunks of many reads into full engine
batches; every chunk keeps the span of its reference batch (consecutive
``batch_size`` chunks of its own read), so outputs equal the reference's
per-read translate.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m nanodecoder_amd.shard --reads 1048576
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import time
from typing import Callable, Dict, List, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import synth


def lpt_assign(weights: Sequence[int], world: int) -> List[List[int]]:
    """Longest-processing-time-first: heaviest item to the least loaded rank
    (ties: lower item index first, lower rank first).  Deterministic."""
    order = sorted(range(len(weights)), key=lambda i: (-weights[i], i))
    heap = [(0, r) for r in range(world)]
    out = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + int(weights[i]), r))
    return [sorted(x) for x in out]


def read_lengths(n_reads: int, seed: int = 0, lo: int = 256, hi: int = 1024) -> np.ndarray:
    """The synthetic 1M-read set's lengths ~ U[lo, hi] samples (§8d config 5)."""
    return np.random.default_rng(seed).integers(lo, hi + 1, size=n_reads)


def synth_raw(read_id: int, n: int) -> np.ndarray:
    """Vectorised synthetic raw DAC trace (same model as synth.synth_raw_read)."""
    rng = np.random.default_rng(1234 + read_id)
    dw = rng.geometric(1.0 / 9.0, size=n // 2 + 16)
    lv = rng.normal(90.0, 15.0, size=dw.size)
    return np.round(np.repeat(lv, dw)[:n] + rng.normal(0.0, 2.0, size=n))


def pack_weights(W: Dict[str, np.ndarray]):
    names = sorted(W)
    meta = [(n, tuple(W[n].shape)) for n in names]
    blob = np.concatenate([np.ascontiguousarray(W[n], np.float32).ravel() for n in names]) if names else \
        np.zeros(0, np.float32)
    return meta, blob


def unpack_weights(meta, blob: np.ndarray) -> Dict[str, np.ndarray]:
    out, off = {}, 0
    for n, shp in meta:
        size = int(np.prod(shp)) if shp else 1
        out[n] = blob[off: off + size].reshape(shp)
        off += size
    return out


def broadcast_weights(W, device) -> Dict[str, np.ndarray]:
    """ONE collective for the weights: rank 0's packed blob to every rank."""
    rank = dist.get_rank()
    obj = [pack_weights(W)[0] if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    meta = obj[0]
    total = sum(int(np.prod(s)) if s else 1 for _, s in meta)
    t = torch.empty(total, dtype=torch.float32, device=device)
    if rank == 0:
        t.copy_(torch.from_numpy(pack_weights(W)[1]))
    dist.broadcast(t, src=0)
    return unpack_weights(meta, t.cpu().numpy())


def count_bases(tok: np.ndarray, eos: int, specials) -> int:
    """Base tokens of [n, S] token rows: before each row's first EOS, not a
    special (<unk>, <blank>, <s>)."""
    if tok.size == 0:
        return 0
    is_eos = tok == eos
    first = np.where(is_eos.any(1), is_eos.argmax(1), tok.shape[1])
    keep = (np.arange(tok.shape[1])[None, :] < first[:, None]) & ~np.isin(tok, list(specials))
    return int(keep.sum())


class ReadShard:
    """Translates one rank's reads with a Translator-like object.

    ``frontend="gpu"`` (default when the translator has ``stream_raw_reads``):
    a producer thread hands RAW reads over and the translator normalises and
    windows each engine batch on the device (nd_normalize_reads /
    nd_window_reads, utils/labelop.py:194-233) right before the engine call,
    on the call's stream; tokens come back as arrays.  ``frontend="cpu"``:
    the host front end (median/MAD + windowing in numpy) runs in the producer
    thread and chunks go through ``stream_reads``.  Either way the translator
    keeps one engine batch per pool lane in flight while it packs the next,
    and the producer stays up to ``prefetch`` reads ahead."""

    def __init__(self, translator, batch_size: int = 100, src_seq_length: int = 512, src_seq_stride: int = 512,
                 prefetch: int = 2048, frontend: str = "auto", normalization: str = "median"):
        self.tr = translator
        self.batch_size = batch_size
        self.L, self.stride = src_seq_length, src_seq_stride
        self.prefetch = prefetch
        if frontend == "auto":
            frontend = "gpu" if hasattr(translator, "stream_raw_reads") else "cpu"
        self.frontend = frontend
        self.normalization = normalization

    def _produce(self, read_ids, lengths, raws, q, stop):
        try:
            for k, rid in enumerate(read_ids):
                if stop.is_set():
                    return
                raw = raws[k] if raws is not None else synth_raw(int(rid), int(lengths[rid]))
                if self.frontend == "gpu":
                    q.put(raw)
                else:
                    q.put(synth.window(synth.normalize_median(raw), self.L, self.stride))
            q.put(None)
        except BaseException as e:  # surfaced in the consumer
            q.put(e)

    def run(self, read_ids: Sequence[int], lengths: Sequence[int], keep_predictions: bool = False, raws=None):
        """Translate the reads ``read_ids`` (lengths indexed by read id).  With
        ``raws`` (raw DAC traces, one per read id in order) only the front end
        is timed; otherwise the synthetic reads are generated on the fly."""
        import queue
        import threading
        from . import frontend
        q: "queue.Queue" = queue.Queue(maxsize=max(1, self.prefetch))
        stop = threading.Event()
        th = threading.Thread(target=self._produce, args=(list(read_ids), lengths, raws, q, stop), daemon=True)
        samples = bases = chunks = 0
        preds = {}
        specials = {self.tr.cfg.unk_idx, self.tr.cfg.pad_idx, self.tr.cfg.bos_idx}
        eos = self.tr.cfg.eos_idx
        n_samples = {}
        gpu = self.frontend == "gpu"

        def reads():
            k = 0
            while True:
                item = q.get()
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                if gpu:
                    w = frontend.windows(int(item.size), self.L, self.stride)
                    n_samples[k] = (sum(ln for _, ln in w), len(w))
                else:
                    n_samples[k] = (sum(len(c) for c in item), len(item))
                k += 1
                yield item

        t0 = time.perf_counter()
        th.start()
        try:
            if gpu and getattr(self.tr, "beam_size", 1) == 1:
                # greedy / sampling: tokens come back as one array per read
                it = self.tr.stream_raw_reads(reads(), self.batch_size, self.normalization, self.L, self.stride,
                                              arrays=True)
                for k, tok, _ in it:
                    ns, nc = n_samples.pop(k)
                    samples += ns
                    chunks += nc
                    bases += count_bases(tok, eos, specials)
                    if keep_predictions:
                        preds[int(read_ids[k])] = [[" ".join(self.tr._tokens_to_sent(t))] for t in tok.tolist()]
            elif gpu:
                # beam: per-chunk (scores, n_best token lists), the first hypothesis counted
                it = self.tr.stream_raw_reads(reads(), self.batch_size, self.normalization, self.L, self.stride)
                for k, res in it:
                    ns, nc = n_samples.pop(k)
                    samples += ns
                    chunks += nc
                    for r in res:
                        bases += count_bases(np.asarray([r[1][0]], np.int64), eos, specials)
                    if keep_predictions:
                        preds[int(read_ids[k])] = [[" ".join(self.tr._tokens_to_sent(t)) for t in r[1]]
                                                   for r in res]
            else:
                for k, res in self.tr.stream_reads(reads(), self.batch_size):
                    ns, nc = n_samples.pop(k)
                    samples += ns
                    chunks += nc
                    for r in res:
                        bases += count_bases(np.asarray([r[1][0]], np.int64), eos, specials)
                    if keep_predictions:
                        preds[int(read_ids[k])] = [[" ".join(self.tr._tokens_to_sent(t)) for t in r[1]]
                                                   for r in res]
        finally:
            stop.set()
            while th.is_alive():  # unblock a producer waiting on a full queue
                try:
                    q.get_nowait()
                except Exception:
                    pass
                th.join(timeout=0.01)
        return dict(samples=samples, bases=bases, chunks=chunks, seconds=time.perf_counter() - t0,
                    reads=len(read_ids), frontend=self.frontend), preds


class ShardFailure(RuntimeError):
    """Reads no rank could translate (their rank failed, and so did the retry)."""

    def __init__(self, read_ids, causes):
        self.read_ids = sorted(int(i) for i in read_ids)
        head = ", ".join(str(i) for i in self.read_ids[:20]) + (" ..." if len(self.read_ids) > 20 else "")
        super().__init__(f"{len(self.read_ids)} reads not translated (read ids {head}): {causes}")


def _empty_stats(frontend):
    return dict(samples=0, bases=0, chunks=0, seconds=0.0, reads=0, frontend=frontend)


def _merge(a, b):
    for k in ("samples", "bases", "chunks", "reads"):
        a[k] += b[k]
    return a


def _device_sync(device):
    """Wait for the rank's device work (a HIP call: never made on a rank whose
    engine has failed, whose device error may be sticky)."""
    if device.type == "cuda" and torch.cuda.is_available():
        torch.cuda.synchronize(device)


def run_distributed(n_reads: int, translator_factory: Callable, weights_factory: Callable, device,
                    batch_size: int = 100, seed: int = 0, keep_predictions: bool = False, pregenerate: bool = False,
                    warmup_reads: int = 0, frontend: str = "auto", retry: bool = True):
    """Rank-local part of the sharded job; returns (global stats, local preds).
    The timed region (max over ranks) covers the front end, packing, the
    engine and the token copies of the rank's reads.

    Collectives: the weight blob goes out in ONE broadcast on the default
    group (RCCL over xGMI with backend "nccl", from HIP memory), before the
    timed region; the translate loop runs none.  Everything after the loop
    -- the failure flags, the counters, the MAX of the seconds and the closing
    barrier -- runs on a CPU gloo group (``ctl``) with host tensors: a few
    numbers, and a rank whose device has faulted can still take part.  With
    an initialised process group the collectives run at every world size,
    one included (the RCCL path is exercised by a one-GPU run).

    Rank failure (reads are independent, so a failed shard is
    rerun): a rank whose translator raises keeps its process and its place in
    the (gloo) collectives and makes NO further device call -- an engine fault
    is usually a sticky HIP error, after which any HIP call, an RCCL
    collective included, raises or hangs.  One all_reduce of per-rank failure
    flags tells every rank which shards failed; their reads are re-assigned by
    LPT to the ranks that did not fail and translated there (``retried`` and
    ``failed_ranks`` in the stats).  Reads that still fail, or a job where
    every rank failed, raise ``ShardFailure`` naming them on every rank (the
    launcher exits non-zero).  A rank PROCESS that dies is the launcher's to
    report: torch.distributed.run stops the other workers and exits non-zero;
    a rerun of the CLI skips the reads already written (translate.py's
    resume)."""
    multi = dist.is_available() and dist.is_initialized()
    rank, world = (dist.get_rank(), dist.get_world_size()) if multi else (0, 1)
    ctl = dist.new_group(backend="gloo") if multi else None
    lengths = read_lengths(n_reads, seed)
    parts = lpt_assign(lengths.tolist(), world)
    mine = parts[rank]
    W = weights_factory() if rank == 0 else None
    if multi:
        W = broadcast_weights(W, device)
    tr = translator_factory(W)
    raws = None
    if pregenerate:  # the raw traces stand in for files already read (untimed); the front end is timed
        raws = [synth_raw(int(i), int(lengths[i])) for i in mine]
    if warmup_reads:  # graphs captured and pinned buffers made outside the timed region
        ReadShard(tr, batch_size=batch_size, frontend=frontend).run(mine[:warmup_reads], lengths)
    if multi:
        dist.barrier()
    _device_sync(device)
    shard = ReadShard(tr, batch_size=batch_size, frontend=frontend)
    t0 = time.perf_counter()
    device_ok = True

    def attempt(ids, raw_list):
        nonlocal device_ok
        try:
            st, pr = shard.run(ids, lengths, keep_predictions, raws=raw_list)
            _device_sync(device)
            return st, pr, None
        except Exception as e:  # this rank's shard failed; the others take its reads
            device_ok = False
            return _empty_stats(shard.frontend), {}, f"rank {rank}: {type(e).__name__}: {e}"

    def exchange(flag):
        flags = torch.zeros(world, dtype=torch.float64)
        flags[rank] = flag
        dist.all_reduce(flags, group=ctl)
        return [r for r in range(world) if flags[r] > 0]

    stats, preds, err = attempt(mine, raws)
    retried = 0
    failed = []
    if multi:
        failed = exchange(1.0 if err is not None else 0.0)
        if failed:
            ok = [r for r in range(world) if r not in failed]
            todo = sorted(i for r in failed for i in parts[r])
            if not ok or not retry:
                raise ShardFailure(todo, f"failed ranks {failed}" + (f": {err}" if err else ""))
            share = lpt_assign([int(lengths[i]) for i in todo], len(ok))
            extra = [todo[j] for j in share[ok.index(rank)]] if rank in ok else []
            retried = len(todo)
            err2 = None
            if extra:
                xraws = [synth_raw(int(i), int(lengths[i])) for i in extra] if pregenerate else None
                st2, pr2, err2 = attempt(extra, xraws)
                stats = _merge(stats, st2)
                preds.update(pr2)
            failed2 = exchange(1.0 if err2 is not None else 0.0)
            if failed2:
                lost = sorted(i for r in failed2 for i in
                              ([todo[j] for j in share[ok.index(r)]] if r in ok else []))
                raise ShardFailure(lost, f"failed ranks {failed} then {failed2} on retry")
    elif err is not None:
        raise ShardFailure(mine, err)
    stats["seconds"] = time.perf_counter() - t0
    red = torch.tensor([stats["samples"], stats["bases"], stats["chunks"]], dtype=torch.float64)
    secs = torch.tensor([stats["seconds"]], dtype=torch.float64)
    per_rank = torch.zeros(world, dtype=torch.float64)
    per_rank[rank] = stats["samples"]
    if multi:
        dist.barrier(group=ctl)
        dist.all_reduce(red, group=ctl)
        dist.all_reduce(per_rank, group=ctl)
        dist.all_reduce(secs, op=dist.ReduceOp.MAX, group=ctl)
    loads = per_rank.numpy()
    g = dict(samples=int(red[0]), bases=int(red[1]), chunks=int(red[2]), seconds=float(secs[0]), world=world,
             reads=int(n_reads), samples_per_rank=[int(x) for x in loads], frontend=shard.frontend,
             load_imbalance=float(loads.max() / max(loads.mean(), 1.0)), retried=retried, failed_ranks=failed,
             device_ok=device_ok)
    return g, preds


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=4096)
    ap.add_argument("--batch-size", type=int, default=100, help="reference batch_size (chunks per read batch)")
    ap.add_argument("--engine-batch", type=int, default=512)
    ap.add_argument("--max-length", type=int, default=100)
    ap.add_argument("--min-length", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--inflight", type=int, default=3, help="translate calls on the device at once (EnginePool lanes)")
    ap.add_argument("--frontend", default="gpu", choices=["gpu", "cpu"],
                    help="normalise and window the reads on the device (gpu) or in a host thread (cpu)")
    args = ap.parse_args(argv)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    from .engine import EnginePool
    from .translator import Translator
    cfg = synth.ModelConfig()

    def weights_factory():
        return synth.make_weights(cfg, seed=11, eos_bias=-3.0)

    def translator_factory(W):
        opt = argparse.Namespace(gpu=local, n_best=1, max_length=args.max_length, min_length=args.min_length,
                                 beam_size=1, batch_size=args.batch_size, engine_max_batch=args.engine_batch)
        eng = EnginePool(cfg, W, device=local, lanes=args.inflight, max_batch=args.engine_batch,
                         max_steps=args.max_length)
        return Translator(cfg, W, opt, engine=eng)

    g, _ = run_distributed(args.reads, translator_factory, weights_factory, dev, batch_size=args.batch_size,
                           seed=args.seed, frontend=args.frontend)
    if dist.get_rank() == 0:
        g["samples_per_sec"] = g["samples"] / g["seconds"]
        g["bases_per_sec"] = g["bases"] / g["seconds"]
        print(json.dumps(g), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
