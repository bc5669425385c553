"""Drop-in for translate/translator.py on MI355X.

``build_translator(opt, report_score, logger, out_file)`` and
``Translator.translate(src, tgt, src_dir, batch_size, attn_debug)`` keep the
reference's names, arguments, return values and error behaviour
(translate/translator.py:65-90,181-369), so translate.py's call
(translate.py:76,113-120) works unchanged.  The model runs in
libnanodec_hip.so (``Engine``); there is no CPU path — ``-gpu -1`` raises.

Reference semantics reproduced:
* batches are ``batch_size`` consecutive chunks of ONE read, each zero padded
  to its own longest chunk (inputters/inputter.py:86-95); that padded length is
  passed to the engine as the chunk's ``span`` so results are identical to the
  reference however the engine packs chunks;
* greedy (beam_size == 1) runs all max_length steps and scores with the last
  step's top log-prob (:396-503); --fast beam for beam_size > 1 (:619-825);
* predictions are cut at the first EOS and joined with spaces
  (translate/translation.py:31-47, translate/translator.py:271-273).

Additions: chunks may be given as float32 arrays instead of strings, and
``translate_reads`` packs chunks of many reads into full engine batches (same
per-chunk results, far higher throughput than one read at a time).
"""
from __future__ import annotations

import json
import os
from typing import Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import checkpoint
from .engine import Engine
from .engine import Engine as _HipEngine  # the real engine class (tests substitute Engine)
from .engine import EnginePool


class GNMTGlobalScorer:
    """onmt/translate/beam.py:181-199: alpha/beta, and the length / coverage
    penalty kinds (onmt/translate/penalties.py) the classic Beam applies."""

    def __init__(self, opt):
        self.alpha = float(getattr(opt, "alpha", 0.0))
        self.beta = float(getattr(opt, "beta", 0.0))
        self.length_penalty = str(getattr(opt, "length_penalty", "none") or "none")
        self.coverage_penalty = str(getattr(opt, "coverage_penalty", "none") or "none")


def parse_chunk(c) -> np.ndarray:
    """NanoDataset.extract_features (inputters/nano_dataset.py:43-83) for
    corpus_type 'translate': a chunk is a whitespace-separated string of
    floats, or the path of a file holding one; returns float32."""
    if isinstance(c, np.ndarray):
        return np.ascontiguousarray(c, dtype=np.float32)
    if isinstance(c, torch.Tensor):
        return c.detach().to(torch.float32).cpu().numpy().reshape(-1)
    if isinstance(c, (list, tuple)):
        return np.asarray(c, dtype=np.float64).astype(np.float32)
    if isinstance(c, str) and os.path.exists(c):
        with open(c) as f:
            c = f.read()
    return np.asarray(str(c).split(), dtype=np.float64).astype(np.float32)


def _bucket(n: int, cap: int) -> int:
    b = 8
    while b < n:
        b *= 2
    return min(max(b, n), cap)


def build_translator(opt, report_score=False, logger=None, out_file=None):
    """translate/translator.py:65-90."""
    models = getattr(opt, "models", None) or []
    if len(models) != 1:
        raise NotImplementedError("exactly one -model is supported (ensembles are not on the MI355X path)")
    if logger:
        logger.info("Loading model...")
    cfg, W = checkpoint.load(models[0])
    scorer = GNMTGlobalScorer(opt)
    return Translator(cfg, W, opt, global_scorer=scorer, report_score=report_score, logger=logger)


class Translator(object):
    """translate/translator.py:93-173, engine-backed."""

    def __init__(self, cfg, weights, opt, global_scorer=None, report_score=False, logger=None, engine=None):
        self.cfg = cfg
        self.opt = opt
        self.gpu = getattr(opt, "gpu", -1)
        if self.gpu < 0 and engine is None:
            raise RuntimeError("nanodecoder_amd runs on MI355X only: pass -gpu N (there is no CPU path)")
        self.n_best = int(getattr(opt, "n_best", 1))
        self.max_length = int(getattr(opt, "max_length", 100))
        self.min_length = int(getattr(opt, "min_length", 0))
        self.beam_size = int(getattr(opt, "beam_size", 5))
        self.random_sampling_temp = float(getattr(opt, "random_sampling_temp", 1.0))
        self.sample_from_topk = int(getattr(opt, "random_sampling_topk", 1))
        self.block_ngram_repeat = int(getattr(opt, "block_ngram_repeat", 0))
        self.ignore_when_blocking = set(getattr(opt, "ignore_when_blocking", None) or [])
        self.dump_beam = getattr(opt, "dump_beam", "")
        # translator.py:166-173: the beam trace accumulator -dump_beam writes
        self.beam_trace = self.dump_beam != ""
        self.beam_accum = ({"predicted_ids": [], "beam_parent_ids": [], "scores": [], "log_probs": []}
                           if self.beam_trace else None)
        self.replace_unk = bool(getattr(opt, "replace_unk", False))
        self.verbose = bool(getattr(opt, "verbose", False))
        self.fast = bool(getattr(opt, "fast", False))
        self.stepwise_penalty = bool(getattr(opt, "stepwise_penalty", False))
        # random sampling draws: keyed by -seed when given (>= 0), else by fresh entropy;
        # successive calls advance like a generator
        seed = getattr(opt, "seed", -1)
        self._seed = int(seed) if seed is not None and int(seed) >= 0 else int.from_bytes(os.urandom(8), "little")
        self._draws = 0
        self.global_scorer = global_scorer or GNMTGlobalScorer(opt)
        self.report_score = report_score
        self.logger = logger
        self.out_file_attn = None
        self._check_supported()
        batch_cap = max(1, int(getattr(opt, "batch_size", 100)))
        self.max_batch = int(getattr(opt, "engine_max_batch", 0) or 0) or max(batch_cap, 256)
        if engine is None:
            dev = torch.cuda.current_device()  # the reference moves tensors to the default "cuda" device
            kw = dict(device=dev, max_batch=self.max_batch, max_steps=self.max_length,
                      max_src_len=min(512, int(getattr(opt, "src_seq_length", 512))),
                      max_beam=max(1, self.beam_size))
            # -engine_lanes: that many calls in flight on the GPU (EnginePool),
            # stream_reads keeping every lane busy.  Default 3 for greedy /
            # sampling; 1 for beam search, whose calls poll the host between
            # graph segments (stream_reads' one host thread would serialise
            # them) and whose lanes each hold the context K/V (~2.4 GB at
            # B = 1024, beam 5)
            lanes = int(getattr(opt, "engine_lanes", 0) or 0) or (3 if self.beam_size == 1 else 1)
            if lanes > 1 and Engine is _HipEngine:
                engine = EnginePool(cfg, weights, lanes=lanes, **kw)
            else:
                engine = Engine(cfg, weights, **kw)
        self.engine = engine
        self._pinned, self._pin_i = None, 0

    def _check_supported(self):
        if self.beam_size == 1:
            # translator.py:371-394: keep_topk == 1 (or temp == 0) is argmax, anything else samples
            if self.sample_from_topk > self.cfg.vocab:
                raise ValueError("random_sampling_topk larger than the vocabulary")
            if self.block_ngram_repeat != 0:
                raise AssertionError("block_ngram_repeat is not supported (translator.py:430)")
        elif not self.fast:
            # the classic onmt Beam (translator.py:827-926, onmt/translate/beam.py): length and
            # coverage penalties (stepwise or at scoring time), n-gram blocking, -dump_beam
            if self.global_scorer.length_penalty not in ("none", "wu", "avg"):
                raise ValueError(f"unknown length_penalty {self.global_scorer.length_penalty!r}")
            if self.global_scorer.coverage_penalty not in ("none", "wu", "summary"):
                raise ValueError(f"unknown coverage_penalty {self.global_scorer.coverage_penalty!r}")
            if self.block_ngram_repeat < 0 or self.block_ngram_repeat > self.max_length:
                raise ValueError("block_ngram_repeat must be in [0, max_length]")
            if self.n_best > self.beam_size:
                raise ValueError("n_best must be <= beam_size")
        else:
            if self.dump_beam:
                raise AssertionError("dump_beam is not supported with --fast (translator.py:631)")
            if self.block_ngram_repeat != 0:
                raise AssertionError("block_ngram_repeat is not supported with --fast (translator.py:633)")
            if self.global_scorer.beta != 0:
                raise AssertionError("beta must be 0 with --fast (translator.py:634)")
            if self.n_best > self.beam_size:
                raise ValueError("n_best must be <= beam_size")
        # -replace_unk is accepted: TranslationBuilder only replaces when the
        # batch carries text src (translation.py:42-47), which nano data never
        # does (src is None, :73-81), so predictions are unchanged

    def setAttnFile(self, out_file_attn):
        self.out_file_attn = out_file_attn

    # ------------------------------------------------------------------ core
    def _stage(self, B: int, T: int):
        """Host staging of one engine batch: views into a ring of pinned
        buffers (real engine; the host-to-device copies then run async, so the
        next batch is packed while the device works on this one), or plain
        numpy arrays (stand-in engines)."""
        if not self._real_engine():
            return np.zeros((B, T), np.float32), np.ones(B, np.int32), np.ones(B, np.int32), None
        if self._pinned is None:
            # one buffer per call in flight, one being packed, one spare
            cap, tl = self.engine.max_batch, self.engine.max_src_len
            self._pinned = [(torch.empty(cap * tl, dtype=torch.float32).pin_memory(),
                             torch.empty(2 * cap, dtype=torch.int32).pin_memory()) for _ in range(self._depth() + 2)]
        fbuf, ibuf = self._pinned[self._pin_i % len(self._pinned)]
        self._pin_i += 1
        sig_t = fbuf[: B * T].view(B, T)
        sig_t.zero_()
        L_t, S_t = ibuf[:B], ibuf[B: 2 * B]
        L_t.fill_(1)
        S_t.fill_(1)
        return sig_t.numpy(), L_t.numpy(), S_t.numpy(), (sig_t, L_t, S_t)

    def _real_engine(self) -> bool:
        return isinstance(self.engine, (_HipEngine, EnginePool))

    def _depth(self) -> int:
        """Engine calls kept in flight by stream_reads: one per EnginePool lane."""
        return max(1, int(getattr(self.engine, "lanes", 1)))

    def _submit(self, chunks: List[np.ndarray], spans: Sequence[int], groups: Optional[Sequence[int]] = None,
                attn: bool = False):
        """Stage up to max_batch chunks with their reference spans (and, for
        the classic Beam, their reference batch ids) and enqueue the engine
        call.  Greedy and sampling calls return before the device finishes;
        ``_finish`` collects the results."""
        n = len(chunks)
        lens = np.array([len(c) for c in chunks], np.int32)
        if (lens < 1).any():
            raise ValueError("empty signal chunk")
        spans = np.asarray(spans, np.int32)
        if spans.max() > self.engine.max_src_len:
            raise ValueError(f"chunk longer than {self.engine.max_src_len} samples (src_seq_length) is not supported")
        T = min(self.engine.max_src_len, ((int(spans.max()) + 63) // 64) * 64)
        B = _bucket(n, self.engine.max_batch)
        sig, L, S, dev_in = self._stage(B, T)
        for i, c in enumerate(chunks):
            sig[i, : len(c)] = c
        L[:n], S[:n] = lens, spans
        if dev_in is not None:
            sig, L, S = dev_in
        job = self._enqueue(sig, L, S, B, n, lens, groups, attn, dev_in)
        job["again"] = lambda: self._submit(chunks, spans, groups, attn)
        return job

    def _enqueue(self, sig, L, S, B: int, n: int, lens: np.ndarray, groups, attn: bool, inputs):
        """The engine call for one staged batch (signal [B, T], chunk lengths
        and spans [B]; the first n rows are chunks), its results copied to
        pinned host buffers on the call's own stream."""
        job = dict(n=n, lens=lens, attn=attn, B=B, inputs=inputs)
        if self.beam_size == 1:
            if not (self.random_sampling_temp == 0.0 or self.sample_from_topk == 1):
                # sample_with_temperature's random branch (translator.py:376-393)
                self._draws += 1
                seed = (self._seed * 0x9E3779B97F4A7C15 + self._draws) & (2 ** 64 - 1)
                r = self.engine.translate_sample(sig, L, S, temp=self.random_sampling_temp,
                                                 keep_topk=self.sample_from_topk, seed=seed, max_len=self.max_length,
                                                 min_len=self.min_length, return_attn=attn)
            else:
                r = self.engine.translate_greedy(sig, L, S, max_len=self.max_length, min_len=self.min_length,
                                                 return_attn=attn)
            job.update(kind="greedy", r=r)
        else:
            # reference batches: the chunks of one group, sorted by length
            # descending (stable) as the reference's batch rows are
            grp = np.zeros(n, np.int64) if groups is None else np.asarray(groups)
            members = {}
            for i in range(n):
                members.setdefault(int(grp[i]), []).append(i)
            sorted_rows = {gid: sorted(m, key=lambda i: -int(lens[i])) for gid, m in members.items()}
            beam = self.beam_size
            cut = None
            if self.fast:
                r = self.engine.translate_beam(sig, L, S, beam=beam, n_best=self.n_best,
                                               alpha=self.global_scorer.alpha, max_len=self.max_length,
                                               min_len=self.min_length, return_attn=attn)
            else:
                # dense reference-batch ids; the engine's padding rows are batches of their own
                g = np.zeros(B, np.int32)
                g[:n] = np.unique(grp, return_inverse=True)[1]
                base = int(g[:n].max()) + 1
                g[n:] = np.arange(base, base + B - n)
                # beam j of a batch reads memory_lengths[j] of the beam-tiled lengths
                # (translator.py:902-907): the length of the batch's row j // beam
                cut = np.ones(B, np.int32)
                for rows in sorted_rows.values():
                    for pos, i in enumerate(rows):
                        cut[i] = lens[rows[pos // beam]]
                gs = self.global_scorer
                exclusion = [self.cfg.itos.index(t) if t in self.cfg.itos else 0 for t in self.ignore_when_blocking]
                r = self.engine.translate_beam_classic(
                    sig, L, S, groups=g, beam=beam, n_best=self.n_best, length_penalty=gs.length_penalty,
                    alpha=gs.alpha, max_len=self.max_length, min_len=self.min_length,
                    coverage_penalty=gs.coverage_penalty, beta=gs.beta, stepwise_penalty=self.stepwise_penalty,
                    block_ngram_repeat=self.block_ngram_repeat, ignore_ids=exclusion, cut=cut, return_attn=attn)
            job.update(kind="beam", r=r, grp=grp, sorted_rows=sorted_rows, cut=cut)
        if self._real_engine():
            self._copy_out(job)
        return job

    _HOST_KEYS = ("tokens", "scores", "lens", "attn", "done_step", "overflow")

    def _copy_out(self, job):
        """Enqueue the call's device-to-host copies (into pinned buffers) on
        the stream the call ran on (its EnginePool lane, or the current
        stream the single Engine joined), then an event: ``_host`` waits on
        that event alone, never on calls submitted after this one."""
        r = job["r"]
        st = self.engine.engines[r["lane"]].stream if "lane" in r else \
            torch.cuda.current_stream(self.engine.device)
        host = {}
        with torch.cuda.stream(st):
            for k in self._HOST_KEYS:
                t = r.get(k)
                if isinstance(t, torch.Tensor):
                    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                    h.copy_(t, non_blocking=True)
                    host[k] = h
            ev = torch.cuda.Event()
            ev.record(st)
        job["host"], job["event"] = host, ev

    def _host(self, job, *names):
        """Results of a submitted call on the host (numpy; None where the
        call has no such output)."""
        if "host" in job:
            job["event"].synchronize()
            h = job["host"]
            return [h[k].numpy() if k in h else None for k in names]
        r = job["r"]  # stand-in engines: host tensors
        return [None if r.get(k) is None else r[k].cpu().numpy() for k in names]

    def _rerun_exact(self, job, finish=None):
        """Split-fp16 range guard (nd_take_overflow): a call in which some
        split activation reached |x| >= 65504 (fp16's range; the reference's
        fp32 is still finite there) runs again with every product in exact
        fp32, and its results replace the flagged ones."""
        self.engine.set_exact_fp32(True)
        try:
            again = job["again"]()
            again["exact"] = True
            return (finish or self._finish)(again)
        finally:
            self.engine.set_exact_fp32(False)

    def _overflowed(self, job, ov):
        return ov is not None and int(ov.reshape(-1)[0]) != 0 and not job.get("exact")

    def _finish(self, job):
        """Per chunk (scores[n_best], token lists[n_best]) and, with ``attn``,
        the attention rows of each hypothesis ([steps, cut] arrays, cut as the
        reference's results["attention"] has it)."""
        n, lens, attn = job["n"], job["lens"], job["attn"]
        out = []
        if job["kind"] == "greedy":
            tok, sc, at, ov = self._host(job, "tokens", "scores", "attn", "overflow")
            if self._overflowed(job, ov):
                return self._rerun_exact(job)
            for i in range(n):
                if attn:  # results["attention"]: rows cut at the chunk's length (translator.py:491-501)
                    out.append(([float(sc[i])], [tok[i].tolist()], [at[i, :, : lens[i]]]))
                else:
                    out.append(([float(sc[i])], [tok[i].tolist()]))
            return out
        grp, sorted_rows, cut, beam = job["grp"], job["sorted_rows"], job["cut"], self.beam_size
        tok, sc, ln, at, done, ov = self._host(job, "tokens", "scores", "lens", "attn", "done_step", "overflow")
        if self._overflowed(job, ov):
            return self._rerun_exact(job)
        for i in range(n):
            o = ([float(sc[i, k]) for k in range(self.n_best)],
                 [tok[i, k, : ln[i, k]].tolist() for k in range(self.n_best)])
            if attn:
                atts = []
                for k in range(self.n_best):
                    if self.fast:
                        # translator.py:780-790: attention[:, i, j, :memory_lengths[i]] with i the
                        # chunk's index among the batches alive at the hypothesis' last step
                        step = int(ln[i, k]) - 1
                        alive = [q for q in sorted_rows[int(grp[i])] if done[q] == 0 or done[q] > step]
                        c = int(lens[alive[alive.index(i) // beam]])
                    else:
                        c = int(cut[i])
                    atts.append(at[i, k, : ln[i, k], :c])
                o = o + (atts,)
            out.append(o)
        return out

    def _run(self, chunks: List[np.ndarray], spans: Sequence[int], groups: Optional[Sequence[int]] = None,
             attn: bool = False):
        """One engine batch, synchronously (see _submit / _finish)."""
        return self._finish(self._submit(chunks, spans, groups, attn))

    def _tokens_to_sent(self, toks) -> List[str]:
        """translate/translation.py:31-47."""
        words = []
        for t in toks:
            w = self.cfg.itos[t]
            if t == self.cfg.eos_idx:
                break
            words.append(w)
        return words

    def translate(self, src, tgt=None, src_dir=None, batch_size=None, attn_debug=False):
        """translate/translator.py:181-369.  Returns (all_scores,
        all_predictions): per chunk, n_best scores and n_best strings."""
        assert src is not None
        if batch_size is None:
            raise ValueError("batch_size must be set")
        chunks = [parse_chunk(c) for c in src]
        res = self.translate_reads([chunks], batch_size=batch_size, attn_debug=attn_debug)[0]
        return res

    def _write_attn(self, chunk: np.ndarray, sent: List[str], attn: np.ndarray):
        """translate/translator.py:285-336: the source samples and the
        prediction (+ </s>) as headers, then one row of attention weights per
        decoder step, into the file set by setAttnFile."""
        preds = list(sent) + ["</s>"]
        srcs = [str(x) for x in np.asarray(chunk, np.float32).reshape(-1)]
        header_format = "{:>8.7} " + "{:>8.7} " * len(srcs)
        row_format = "{:>8.5f} " * len(srcs)
        output = header_format.format(">", *srcs)
        header_format = "{:>8.7} " + "{:>8.7} " * len(preds)
        output += header_format.format("|", *preds) + "\n"
        for row in attn.tolist():
            output += row_format.format(*row) + "\n"
        self.out_file_attn.write(output)

    def stream_reads(self, reads: Iterable[Sequence], batch_size: int, attn_debug: bool = False):
        """Generator over many reads (any iterable of chunk lists): chunks are
        packed across reads into engine batches of max_batch, one batch (one
        per EnginePool lane) stays in flight on the device while the next is
        packed on the host, and
        (read index, per-chunk results) is yielded as each read completes.
        Each chunk keeps the span of the reference batch it would belong to
        (consecutive ``batch_size`` chunks of its own read), so results equal
        per-read translate()."""
        import collections
        cap = self.engine.max_batch
        depth = self._depth()
        pending, inflight = [], collections.deque()
        results, remaining = {}, {}
        nb = 0

        def collect(jb):
            job, items = jb
            done = []
            for (ri, ci, c, _, _), o in zip(items, self._finish(job)):
                results[ri][ci] = o + (c,) if attn_debug else o
                remaining[ri] -= 1
                if remaining[ri] == 0:
                    done.append(ri)
            return done

        def submit(items):
            return self._submit([g[2] for g in items], [g[3] for g in items], [g[4] for g in items],
                                attn=attn_debug), items

        for ri, read in enumerate(reads):
            chunks = [parse_chunk(c) for c in read]
            if not chunks:
                yield ri, []
                continue
            results[ri], remaining[ri] = [None] * len(chunks), len(chunks)
            for b0 in range(0, len(chunks), batch_size):
                part = chunks[b0: b0 + batch_size]
                span = max(len(c) for c in part)
                for k, c in enumerate(part):
                    pending.append((ri, b0 + k, c, span, nb))
                    if len(pending) == cap:
                        inflight.append(submit(pending))
                        pending = []
                        # `depth` calls stay on the device while the next batch is packed
                        while len(inflight) > depth:
                            for r in collect(inflight.popleft()):
                                yield r, results.pop(r)
                nb += 1
        if pending:
            inflight.append(submit(pending))
        while inflight:
            for r in collect(inflight.popleft()):
                yield r, results.pop(r)

    def translate_reads(self, reads: Sequence[Sequence], batch_size: int, attn_debug: bool = False):
        """Translate many reads (stream_reads); returns per read
        (all_scores, all_predictions) as translate() does."""
        results = [None] * len(reads)
        for ri, res in self.stream_reads(reads, batch_size, attn_debug):
            results[ri] = res
        return self._report(results, attn_debug)

    def translate_raw_reads(self, raws: Sequence[np.ndarray], batch_size: int, normalization: str = "median",
                            src_seq_length: int = 512, src_seq_stride: int = 512):
        """translate_reads on raw reads with the signal front end on the
        device (stream_raw_reads); returns per read (all_scores,
        all_predictions)."""
        results = [None] * len(raws)
        for ri, res in self.stream_raw_reads(raws, batch_size, normalization, src_seq_length, src_seq_stride):
            results[ri] = res
        return self._report(results, False)

    def _report(self, results, attn_debug: bool):
        """Per read (all_scores, all_predictions) from per-chunk results, with
        the reference's verbose / -dump_beam / report_score side outputs
        (translate/translator.py:255-369)."""
        ret = []
        counter = 0
        pred_score_total, pred_words_total = 0.0, 0
        for r in results:
            all_scores, all_predictions = [], []
            for res in r:
                scores, toks = res[0], res[1]
                sents = [self._tokens_to_sent(t) for t in toks]
                if attn_debug:
                    self._write_attn(res[3], sents[0], res[2][0])
                all_scores.append(scores[: self.n_best])
                all_predictions.append([" ".join(s) for s in sents[: self.n_best]])
                pred_score_total += scores[0]
                pred_words_total += len(sents[0])
                if self.verbose:
                    counter += 1
                    msg = "\nSENT {}: {}\n".format(counter, None) + \
                          "PRED {}: {}\n".format(counter, " ".join(sents[0])) + \
                          "PRED SCORE: {:.4f}\n".format(scores[0])
                    if len(sents) > 1:
                        msg += "\nBEST HYP:\n" + "".join("[{:.4f}] {}\n".format(sc, s)
                                                         for sc, s in zip(scores, sents))
                    if self.logger:
                        self.logger.info(msg)
                    else:
                        os.write(1, msg.encode("utf-8"))
            ret.append((all_scores, all_predictions))
        if self.dump_beam:
            # translator.py:365-368 dumps the beam trace accumulator.  (The
            # reference reads it through a `self.translator` attribute the
            # Translator does not have, and nothing in it appends to the
            # lists: the intended file is these four empty lists.)
            with open(self.dump_beam, "w", encoding="utf-8") as f:
                json.dump(self.beam_accum, f)
        if self.report_score and pred_words_total:
            msg = "PRED AVG SCORE: %.4f, PRED PPL: %.4f" % (pred_score_total / pred_words_total,
                                                           np.exp(-pred_score_total / pred_words_total))
            (self.logger.info if self.logger else print)(msg)
        return ret

    # ------------------------------------------------------ device front end
    def _next_stream(self):
        """The stream the engine's next call will run on (its EnginePool
        lane, or the current stream for a single Engine)."""
        if isinstance(self.engine, EnginePool):
            return self.engine.engines[self.engine._next].stream
        return torch.cuda.current_stream(self.engine.device)

    def _submit_raw(self, items, batch_reads, normalization: str):
        """One engine batch from raw reads: chunk descriptors ``items`` =
        (read, chunk, start, length, span, reference batch) and the reads
        they cut (``batch_reads``: read -> float64 samples).  The front end
        (frontend.device_batch) runs on the call's own stream, so the
        normalised chunks go from HBM to the engine with no host pass."""
        from . import frontend
        n = len(items)
        uniq = list(batch_reads)
        local = {ri: j for j, ri in enumerate(uniq)}
        lens = np.fromiter((it[3] for it in items), np.int32, n)
        spans = np.fromiter((it[4] for it in items), np.int32, n)
        if spans.max() > self.engine.max_src_len:
            raise ValueError(f"chunk longer than {self.engine.max_src_len} samples (src_seq_length) is not supported")
        T = min(self.engine.max_src_len, ((int(spans.max()) + 63) // 64) * 64)
        B = _bucket(n, self.engine.max_batch)
        ls = np.ones(2 * B, np.int32)
        ls[:n], ls[B: B + n] = lens, spans
        st = self._next_stream()
        with torch.cuda.stream(st):
            sig, keep = frontend.device_batch([batch_reads[r] for r in uniq],
                                              np.fromiter((local[it[0]] for it in items), np.int32, n),
                                              np.fromiter((it[2] for it in items), np.int32, n), lens,
                                              normalization, B, T, self.engine.device)
            ls_d = torch.from_numpy(ls).pin_memory().to(self.engine.device, non_blocking=True)
            job = self._enqueue(sig, ls_d[:B], ls_d[B:], B, n, lens, [it[5] for it in items], False,
                                (sig, ls_d, keep))
        job["again"] = lambda: self._submit_raw(items, batch_reads, normalization)
        return job

    def stream_raw_reads(self, raws: Iterable, batch_size: int, normalization: str = "median",
                         src_seq_length: int = 512, src_seq_stride: int = 512, arrays: bool = False):
        """stream_reads on RAW reads (float64 sample arrays, as
        frontend.read_raw returns them) with extract_fast5_raw's
        normalisation and windowing (utils/labelop.py:194-243) on the device:
        the reads of each engine batch go to HBM once and are cut into its
        [B, T] signal batch there (nd_normalize_reads / nd_window_reads),
        bit-identical to the host front end.  Chunks keep the span of their
        reference batch (``batch_size`` consecutive chunks of one read), so
        results equal per-read translate() on the host front end's chunks.
        Yields (read index, per-chunk results) as stream_reads does; with
        ``arrays`` (greedy and sampling only) (read index, tokens [n_chunks,
        max_length] int32, scores [n_chunks] float32) instead."""
        import collections

        from . import frontend
        if arrays and self.beam_size != 1:
            raise ValueError("arrays=True is for greedy / sampling decoding")
        cap = self.engine.max_batch
        depth = self._depth()
        pending, batch_reads, inflight = [], {}, collections.deque()
        results, remaining = {}, {}
        nb = 0

        def collect(jb):
            job, items = jb
            if arrays:
                tok, sc = self._finish_arrays(job)
                outs = ((tok[i], sc[i]) for i in range(len(items)))
            else:
                outs = self._finish(job)
            done = []
            for (ri, ci, _, _, _, _), o in zip(items, outs):
                if arrays:
                    results[ri][0][ci] = o[0]
                    results[ri][1][ci] = o[1]
                else:
                    results[ri][ci] = o
                remaining[ri] -= 1
                if remaining[ri] == 0:
                    done.append(ri)
            return done

        def flush():
            nonlocal pending, batch_reads
            inflight.append((self._submit_raw(pending, batch_reads, normalization), pending))
            pending, batch_reads = [], {}

        for ri, raw in enumerate(raws):
            raw = np.asarray(raw, dtype=np.float64).reshape(-1)
            if raw.size == 0:
                yield (ri, np.zeros((0, self.max_length), np.int32), np.zeros(0, np.float32)) if arrays else (ri, [])
                continue
            wins = frontend.windows(int(raw.size), src_seq_length, src_seq_stride)
            if arrays:
                results[ri] = (np.empty((len(wins), self.max_length), np.int32), np.empty(len(wins), np.float32))
            else:
                results[ri] = [None] * len(wins)
            remaining[ri] = len(wins)
            for b0 in range(0, len(wins), batch_size):
                part = wins[b0: b0 + batch_size]
                span = max(ln for _, ln in part)
                for k, (st, ln) in enumerate(part):
                    pending.append((ri, b0 + k, st, ln, span, nb))
                    batch_reads[ri] = raw
                    if len(pending) == cap:
                        flush()
                        while len(inflight) > depth:
                            for r in collect(inflight.popleft()):
                                yield (r,) + results.pop(r) if arrays else (r, results.pop(r))
                nb += 1
        if pending:
            flush()
        while inflight:
            for r in collect(inflight.popleft()):
                yield (r,) + results.pop(r) if arrays else (r, results.pop(r))

    def _finish_arrays(self, job):
        """(tokens [n, S], scores [n]) numpy of a greedy / sampling call."""
        tok, sc, ov = self._host(job, "tokens", "scores", "overflow")
        if self._overflowed(job, ov):
            return self._rerun_exact(job, self._finish_arrays)
        return tok[: job["n"]], sc[: job["n"]]

    def translate_batch(self, batch, data=None, attn_debug=False, fast=False):
        """translate/translator.py:505-540 on a batch object with
        src [T, B, 1], src_lengths [B] (reference batch layout).  Returns the
        reference's results dict; predictions are token-id tensors (greedy:
        all max_length tokens; beam: through EOS), scores floats."""
        src = batch.src[0] if isinstance(batch.src, tuple) else batch.src
        src = src.detach().to(torch.float32).cpu()
        T, B = src.shape[0], src.shape[1]
        lens = batch.src_lengths.detach().cpu().numpy().astype(np.int32)
        chunks = [src[: lens[i], i, 0].numpy() for i in range(B)]
        saved, self.fast = self.fast, bool(fast)  # translator.py:523-540 dispatches on the argument
        try:
            if self.beam_size > 1:
                self._check_supported()
            # return_attention (:521-529); the classic Beam always keeps its attention (:902-924)
            want = bool(attn_debug or self.replace_unk) or (self.beam_size > 1 and not self.fast)
            outs = self._run(chunks, [T] * B, attn=want)
        finally:
            self.fast = saved
        att = [[torch.from_numpy(np.ascontiguousarray(a)) for a in o[2]] if want else [[]] * len(o[0])
               for o in outs]
        return {"predictions": [[torch.tensor(t, dtype=torch.long) for t in o[1]] for o in outs],
                "scores": [list(o[0]) for o in outs], "attention": att,
                "gold_score": [0] * B, "batch": batch}
