"""Python face of the HIP engine: one ``Engine`` per GPU.

PyTorch-ROCm is used as plumbing only — device memory for inputs/outputs and
the current HIP stream; all compute runs in libnanodec_hip.so.

The Engine takes weights by reference state-dict name (see ``checkpoint.py``
for loading .pt files) and translates batches of signal chunks already
resident on the device.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .synth import ModelConfig


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Engine:
    """MI355X translate engine for one device (C-ABI context owner)."""

    def __init__(self, cfg: ModelConfig, weights: Dict[str, np.ndarray], device: int = 0, max_batch: int = 256,
                 max_src_len: int = 512, max_steps: int = 100, max_beam: int = 1, graphs: bool = True,
                 share_from: Optional["Engine"] = None):
        """share_from: an Engine of the same model on the same device whose weights (and the images derived
        from them) this one reads instead of loading its own (nd_share_weights; ``weights`` is then unused).
        It is kept referenced so it outlives this engine."""
        self.cfg = cfg
        self._sharers = set()        # ids of open engines that read this one's weights (share_from)
        self._close_pending = False  # close() called while sharers were open: destroyed with the last of them
        self.device = torch.device("cuda", device)
        self.max_batch, self.max_src_len, self.max_steps, self.max_beam = max_batch, max_src_len, max_steps, max_beam
        self.bank_grid = 0  # nd_set_bank_grid
        self.bank_nt = False  # nd_set_bank_policy
        self.splitk = False   # nd_set_gemm_splitk
        L = _lib.lib()
        c = _lib.NdConfig()
        c.encoder_type = _lib.ND_ENC_TRANSFORMER if cfg.encoder_type == "transformer" else _lib.ND_ENC_NANO
        c.self_attn_type = _lib.ND_SELF_AVERAGE if cfg.self_attn_type == "average" else _lib.ND_SELF_SCALED_DOT
        c.enc_layers, c.dec_layers = cfg.enc_layers, cfg.dec_layers
        c.d_model, c.heads, c.d_ff, c.vocab = cfg.d_model, cfg.heads, cfg.d_ff, cfg.vocab
        c.rnn_hidden = cfg.rnn_hidden
        c.position_encoding = int(bool(cfg.position_encoding))
        c.pad_idx, c.bos_idx, c.eos_idx = cfg.pad_idx, cfg.bos_idx, cfg.eos_idx
        c.max_batch, c.max_src_len, c.max_steps, c.max_beam = max_batch, max_src_len, max_steps, max_beam
        c.device = device
        h = ctypes.c_void_p()
        torch.cuda.set_device(self.device)
        _lib.check(L.nd_create(ctypes.byref(c), ctypes.byref(h)), "nd_create")
        self._h = h
        self._L = L
        self._src = share_from
        try:
            if share_from is not None:
                if not getattr(share_from, "_h", None) or share_from._close_pending:
                    raise _lib.NanodecError("share_from: the source engine is closed")
                _lib.check(L.nd_share_weights(h, share_from._h), "nd_share_weights")
                share_from._sharers.add(id(self))
                weights = {}
            for name, arr in weights.items():
                a = np.ascontiguousarray(arr, dtype=np.float32)
                shape = (ctypes.c_int64 * a.ndim)(*a.shape)
                _lib.check(L.nd_load_weight(h, name.encode(), a.ctypes.data_as(ctypes.c_void_p), shape, a.ndim),
                           f"nd_load_weight({name})")
            if share_from is None:
                _lib.check(L.nd_finalize(h), "nd_finalize")
            _lib.check(L.nd_set_graphs(h, int(graphs)), "nd_set_graphs")
        except Exception:
            self.close()
            raise

    # ------------------------------------------------------------------
    def close(self):
        """Free the context.  A context whose weights other engines still read
        (share_from) is freed when the last of them closes; until then it
        refuses calls."""
        if not getattr(self, "_h", None):
            return
        if self._sharers:
            self._close_pending = True
            return
        self._L.nd_destroy(self._h)
        self._h = None
        src = self._src
        self._src = None
        if src is not None:
            src._sharers.discard(id(self))
            if src._close_pending and not src._sharers:
                src.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @property
    def stream(self) -> torch.cuda.ExternalStream:
        """The context's own HIP stream (nd_stream), as a torch stream.  Work
        enqueued with it current needs no cross-stream join per call."""
        if getattr(self, "_ext", None) is None:
            self._ext = torch.cuda.ExternalStream(self._L.nd_stream(self._h), device=self.device)
        return self._ext

    def set_ctx_path(self, path: int):
        """0: memory-bank context attention for greedy (default), 1: per-layer K/V always."""
        _lib.check(self._L.nd_set_ctx_path(self._h, int(path)), "nd_set_ctx_path")

    def set_exact_fp32(self, on: bool):
        """Exact fp32 (fp32-MFMA kernels for every product) instead of the
        default split-fp16 products (22-bit operands, fp32 accumulation)."""
        _lib.check(self._L.nd_set_exact_fp32(self._h, int(on)), "nd_set_exact_fp32")

    def set_bank_policy(self, nontemporal: bool):
        """Stream the greedy memory bank with non-temporal loads (nd_set_bank_policy)."""
        _lib.check(self._L.nd_set_bank_policy(self._h, int(nontemporal)), "nd_set_bank_policy")
        self.bank_nt = bool(nontemporal)

    def set_bank_grid(self, workgroups: int):
        """Workgroups of the memory-bank kernel at most, 0 = one per chunk (nd_set_bank_grid)."""
        _lib.check(self._L.nd_set_bank_grid(self._h, int(workgroups)), "nd_set_bank_grid")
        self.bank_grid = int(workgroups)

    def set_gemm_splitk(self, on: bool):
        """Split the decoder's K = 2048 step products over workgroups (nd_set_gemm_splitk; EnginePool lanes)."""
        _lib.check(self._L.nd_set_gemm_splitk(self._h, int(on)), "nd_set_gemm_splitk")
        self.splitk = bool(on)

    def bank_form(self) -> int:
        """The memory bank the last call streamed (nd_bank_form): 0 fp32 (greedy in exact fp32, or a
        beam call on fp32 K/V), 2 24-bit digits (greedy), 3 the 24-bit context K/V (beam)."""
        return int(self._L.nd_bank_form(self._h))

    def set_timing(self, on: bool):
        _lib.check(self._L.nd_set_timing(self._h, int(on)), "nd_set_timing")

    def last_timing(self):
        e, d = ctypes.c_float(), ctypes.c_float()
        _lib.check(self._L.nd_last_timing(self._h, ctypes.byref(e), ctypes.byref(d)), "nd_last_timing")
        return e.value, d.value

    def set_kernel_stamps(self, on: bool):
        """Stamp every decoder context-attention launch (in-kernel wall clock,
        part of the graphs) — the bench's live roofline timing."""
        _lib.check(self._L.nd_set_kernel_stamps(self._h, int(on)), "nd_set_kernel_stamps")

    def kernel_stamps(self):
        """(mean launch duration in us, launches) of the last call's context attention."""
        a, n = ctypes.c_float(), ctypes.c_int32()
        _lib.check(self._L.nd_kernel_stamps(self._h, ctypes.byref(a), ctypes.byref(n)), "nd_kernel_stamps")
        return a.value, n.value

    def _take_overflow(self):
        """The split-fp16 range guard word of the calls enqueued so far
        (nd_take_overflow): a [1] int32 device tensor, nonzero when some split
        activation reached |x| >= 65504 (rerun the call with set_exact_fp32)."""
        ov = torch.empty(1, dtype=torch.int32, device=self.device)
        _lib.check(self._L.nd_take_overflow(self._h, _ptr(ov), self._stream()), "nd_take_overflow")
        return ov

    def _inputs(self, signal, lengths, spans):
        if not getattr(self, "_h", None) or self._close_pending:
            raise _lib.NanodecError("the engine is closed")
        dev = self.device
        # pinned host inputs (the Translator's staging ring) copy asynchronously
        signal = torch.as_tensor(signal, dtype=torch.float32).to(dev, non_blocking=True).contiguous()
        B, T = signal.shape
        lengths = torch.as_tensor(lengths).to(dev, torch.int32, non_blocking=True).contiguous()
        spans = lengths.clone() if spans is None else \
            torch.as_tensor(spans).to(dev, torch.int32, non_blocking=True).contiguous()
        assert lengths.shape == (B,) and spans.shape == (B,)
        return signal, lengths, spans, B, T

    def translate_greedy(self, signal, lengths, spans=None, max_len: Optional[int] = None, min_len: int = 0,
                         return_logp: bool = False, return_attn: bool = False):
        """Greedy decode.  signal [B,T] f32 (zero padded), lengths/spans [B].
        Returns dict(tokens [B,S] i32, scores [B] f32, logp [B,S,V] or None,
        attn [B,S,T] or None: the last layer's head-0 context attention)."""
        signal, lengths, spans, B, T = self._inputs(signal, lengths, spans)
        S = self.max_steps if max_len is None else max_len
        tok = torch.empty(B, S, dtype=torch.int32, device=self.device)
        sc = torch.empty(B, dtype=torch.float32, device=self.device)
        lp = torch.empty(B, S, self.cfg.vocab, dtype=torch.float32, device=self.device) if return_logp else None
        if return_attn:
            at = torch.empty(B, S, T, dtype=torch.float32, device=self.device)
            _lib.check(self._L.nd_translate_greedy_attn(self._h, _ptr(signal), _ptr(lengths), _ptr(spans), B, T, S,
                                                        min_len, _ptr(tok), _ptr(sc), _ptr(lp), _ptr(at),
                                                        self._stream()), "nd_translate_greedy_attn")
            return dict(tokens=tok, scores=sc, logp=lp, attn=at, overflow=self._take_overflow())
        _lib.check(self._L.nd_translate_greedy(self._h, _ptr(signal), _ptr(lengths), _ptr(spans), B, T, S, min_len,
                                               _ptr(tok), _ptr(sc), _ptr(lp), self._stream()), "nd_translate_greedy")
        return dict(tokens=tok, scores=sc, logp=lp, attn=None, overflow=self._take_overflow())

    def translate_sample(self, signal, lengths, spans=None, temp: float = 1.0, keep_topk: int = -1, seed: int = 0,
                         max_len: Optional[int] = None, min_len: int = 0, return_logp: bool = False,
                         return_attn: bool = False):
        """Random sampling (translator.py:371-503): as translate_greedy, the
        token of every step drawn from softmax(logp / temp) over the
        keep_topk most likely tokens (-1: all); draws keyed by ``seed``."""
        signal, lengths, spans, B, T = self._inputs(signal, lengths, spans)
        S = self.max_steps if max_len is None else max_len
        tok = torch.empty(B, S, dtype=torch.int32, device=self.device)
        sc = torch.empty(B, dtype=torch.float32, device=self.device)
        lp = torch.empty(B, S, self.cfg.vocab, dtype=torch.float32, device=self.device) if return_logp else None
        at = torch.empty(B, S, T, dtype=torch.float32, device=self.device) if return_attn else None
        _lib.check(self._L.nd_translate_sample(self._h, _ptr(signal), _ptr(lengths), _ptr(spans), B, T, S, min_len,
                                               float(temp), int(keep_topk), int(seed) & (2 ** 64 - 1), _ptr(tok),
                                               _ptr(sc), _ptr(lp), _ptr(at), self._stream()), "nd_translate_sample")
        return dict(tokens=tok, scores=sc, logp=lp, attn=at, overflow=self._take_overflow())

    def translate_beam(self, signal, lengths, spans=None, beam: int = 5, n_best: int = 1, alpha: float = 0.0,
                       max_len: Optional[int] = None, min_len: int = 0, return_attn: bool = False):
        """--fast beam search.  Returns dict(tokens [B,n_best,S] i32 (-1 pad),
        scores [B,n_best] f32, lens [B,n_best] i32, steps [1] i32); with
        ``return_attn`` also attn [B,n_best,S,T] f32 (the hypotheses'
        attention rows) and done_step [B] i32 (steps each chunk ran)."""
        signal, lengths, spans, B, T = self._inputs(signal, lengths, spans)
        S = self.max_steps if max_len is None else max_len
        tok = torch.empty(B, n_best, S, dtype=torch.int32, device=self.device)
        sc = torch.empty(B, n_best, dtype=torch.float32, device=self.device)
        ln = torch.empty(B, n_best, dtype=torch.int32, device=self.device)
        st = torch.empty(1, dtype=torch.int32, device=self.device)
        if not return_attn:
            _lib.check(self._L.nd_translate_beam(self._h, _ptr(signal), _ptr(lengths), _ptr(spans), B, T, beam,
                                                 n_best, float(alpha), S, min_len, _ptr(tok), _ptr(sc), _ptr(ln),
                                                 _ptr(st), self._stream()), "nd_translate_beam")
            return dict(tokens=tok, scores=sc, lens=ln, steps=st, overflow=self._take_overflow())
        att = torch.empty(B, n_best, S, T, dtype=torch.float32, device=self.device)
        done = torch.empty(B, dtype=torch.int32, device=self.device)
        _lib.check(self._L.nd_translate_beam_attn(self._h, _ptr(signal), _ptr(lengths), _ptr(spans), B, T, beam,
                                                  n_best, float(alpha), S, min_len, _ptr(tok), _ptr(sc), _ptr(ln),
                                                  _ptr(st), _ptr(att), _ptr(done), self._stream()),
                   "nd_translate_beam_attn")
        return dict(tokens=tok, scores=sc, lens=ln, steps=st, attn=att, done_step=done,
                    overflow=self._take_overflow())

    def translate_beam_classic(self, signal, lengths, spans=None, groups=None, beam: int = 5, n_best: int = 1,
                               length_penalty: str = "none", alpha: float = 0.0, max_len: Optional[int] = None,
                               min_len: int = 0, coverage_penalty: str = "none", beta: float = 0.0,
                               stepwise_penalty: bool = False, block_ngram_repeat: int = 0,
                               ignore_ids: Sequence[int] = (), cut=None, return_attn: bool = False):
        """Classic onmt Beam search (no --fast).  groups [B]: the reference
        batch of every chunk (default: one batch).  cut [B]: each chunk's
        attention length (memory_lengths[j] as the reference indexes it;
        needed with a coverage penalty).  Returns dict like translate_beam,
        with attn [B,n_best,S,T] when ``return_attn``."""
        signal, lengths, spans, B, T = self._inputs(signal, lengths, spans)
        S = self.max_steps if max_len is None else max_len
        g = torch.zeros(B, dtype=torch.int32) if groups is None else torch.as_tensor(groups)
        g = g.to(self.device, torch.int32).contiguous()
        opts = _lib.NdClassicOpts(
            length_penalty={"none": 0, "wu": 1, "avg": 2}[length_penalty], alpha=float(alpha), beta=float(beta),
            coverage_penalty={"none": 0, "wu": 1, "summary": 2}[coverage_penalty],
            stepwise_penalty=int(bool(stepwise_penalty)), block_ngram_repeat=int(block_ngram_repeat),
            ignore_mask=sum(1 << int(t) for t in set(ignore_ids)))
        cu = None
        if cut is not None:
            cu = torch.as_tensor(np.asarray(cut, np.int32)).to(self.device).contiguous()
        tok = torch.empty(B, n_best, S, dtype=torch.int32, device=self.device)
        sc = torch.empty(B, n_best, dtype=torch.float32, device=self.device)
        ln = torch.empty(B, n_best, dtype=torch.int32, device=self.device)
        st = torch.empty(1, dtype=torch.int32, device=self.device)
        att = torch.empty(B, n_best, S, T, dtype=torch.float32, device=self.device) if return_attn else None
        _lib.check(self._L.nd_translate_beam_classic_ex(self._h, _ptr(signal), _ptr(lengths), _ptr(spans), _ptr(g),
                                                        _ptr(cu) if cu is not None else None, B, T, beam, n_best,
                                                        ctypes.byref(opts), S, min_len, _ptr(tok), _ptr(sc), _ptr(ln),
                                                        _ptr(st), _ptr(att) if att is not None else None,
                                                        self._stream()), "nd_translate_beam_classic_ex")
        out = dict(tokens=tok, scores=sc, lens=ln, steps=st, overflow=self._take_overflow())
        if return_attn:
            out["attn"] = att
        return out

    def encode(self, signal, lengths, spans=None):
        """Memory bank [B, T, d] of the encoder (rows >= span unspecified)."""
        signal, lengths, spans, B, T = self._inputs(signal, lengths, spans)
        mem = torch.empty(B, T, self.cfg.d_model, dtype=torch.float32, device=self.device)
        _lib.check(self._L.nd_encode(self._h, _ptr(signal), _ptr(lengths), _ptr(spans), B, T, _ptr(mem),
                                     self._stream()), "nd_encode")
        return mem


class EnginePool:
    """Several translate calls in flight on one GPU: ``lanes`` engine contexts
    of the same model, each on its own HIP stream (its own hardware queue),
    used round robin.

    One call is a chain of ~2,300 dependent launches, most of them latency
    bound (decoder steps at 256 rows); a second call's chain on another
    hardware queue fills the gaps (measured on MI355X, greedy configs[1]:
    26.8 ms per 256-chunk call alone, 42.1 ms per two calls in flight).

    Interface as Engine's translate_* / encode, with one difference: a
    translate call returns before its outputs exist and does NOT join the
    caller's stream (that join would order the next call behind this one).
    The result dict carries ``event`` (recorded on the lane's stream when the
    outputs are written); wait on it (``wait``) before using the outputs on
    another stream, and keep them referenced until that use has completed
    (they are allocated on the lane's stream).
    A lane waits for the caller's current stream at submission, so inputs
    produced there are safe; the lane reuses its workspaces in call order, so
    call k + lanes waits for call k on the same lane."""

    def __init__(self, cfg: ModelConfig, weights: Dict[str, np.ndarray], device: int = 0, lanes: int = 2,
                 bank_nt_lanes: Optional[Sequence[int]] = None, bank_grid: Optional[int] = None, **kw):
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        # one copy of the weights: lanes 1.. read lane 0's (nd_share_weights), so the lanes' decoder GEMMs
        # share their weights' lines in every XCD's L2 and in the Infinity Cache
        # (configs[1] pooled, same box: 15.80 / 15.82 ms per call with a copy per lane, 15.73 / 15.84 shared;
        # one copy also spares every lane's finalize and its weight images' HBM)
        self.engines = [Engine(cfg, weights, device=device, **kw)]
        for _ in range(1, lanes):
            self.engines.append(Engine(cfg, weights, device=device, share_from=self.engines[0], **kw))
        # lanes whose memory bank streams non-temporally (nd_set_bank_policy).
        # Default: every lane when there are several (two 134 MB banks exceed
        # the 256 MB Infinity Cache; streaming both past it leaves the cache to
        # the rest: 20.6 -> 19.9 ms per call at two lanes, same box)
        if bank_nt_lanes is None:
            bank_nt_lanes = range(lanes) if lanes > 1 else ()
        self.bank_nt_lanes = tuple(sorted(set(int(i) for i in bank_nt_lanes)))
        for i in self.bank_nt_lanes:
            self.engines[i].set_bank_policy(True)
        # the memory-bank kernel's workgroup cap (nd_set_bank_grid).  Default
        # with several lanes: half the CUs, so the other lanes' kernels keep
        # the rest while one lane streams its bank (3 lanes, 256 chunks per
        # call: 18.3 -> 17.6 ms per call; 64, 96, 160 workgroups measured worse)
        if bank_grid is None:
            bank_grid = torch.cuda.get_device_properties(self.engines[0].device).multi_processor_count // 2 \
                if lanes > 1 else 0
        self.bank_grid = int(bank_grid)
        for e in self.engines:
            e.set_bank_grid(self.bank_grid)
        # several calls in flight: the K = 2048 step products split over workgroups (nd_set_gemm_splitk;
        # pooled configs[1] -2.4 %, a lone call +0.3 ms, round 5)
        self.splitk = lanes > 1
        for e in self.engines:
            e.set_gemm_splitk(self.splitk)
        e0 = self.engines[0]
        self.cfg, self.device = cfg, e0.device
        self.max_batch, self.max_src_len, self.max_steps, self.max_beam = (e0.max_batch, e0.max_src_len,
                                                                           e0.max_steps, e0.max_beam)
        self._next = 0
        self._held = [None] * lanes

    @property
    def lanes(self) -> int:
        return len(self.engines)

    def subset(self, n: int) -> "EnginePool":
        """A pool over the first n lanes (same contexts; e.g. n = 1: one call at a time)."""
        p = EnginePool.__new__(EnginePool)
        p.__dict__.update(self.__dict__)
        p.engines = self.engines[:n]
        p._next = 0
        return p

    def _call(self, name, signal, lengths, spans=None, **kw):
        i = self._next
        self._next = (i + 1) % len(self.engines)
        eng = self.engines[i]
        st = eng.stream
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            r = getattr(eng, name)(signal, lengths, spans, **kw)
            ev = torch.cuda.Event()
            ev.record(st)
        # the caller's input tensors stay referenced until the lane's next call
        # and by the result (the call copies them into its own workspace first
        # thing).  Not Tensor.record_stream: the caching allocator would record
        # an event on the lane's stream whenever such a tensor is freed, also
        # after the pool is closed and the stream destroyed.
        self._held[i] = (signal, lengths, spans)
        r["event"], r["lane"], r["inputs"] = ev, i, self._held[i]
        return r

    @staticmethod
    def wait(result, stream=None):
        """Order ``stream`` (default: the current stream) after ``result``'s call."""
        (stream or torch.cuda.current_stream()).wait_event(result["event"])
        return result

    def translate_greedy(self, signal, lengths, spans=None, **kw):
        return self._call("translate_greedy", signal, lengths, spans, **kw)

    def translate_sample(self, signal, lengths, spans=None, **kw):
        return self._call("translate_sample", signal, lengths, spans, **kw)

    def translate_beam(self, signal, lengths, spans=None, **kw):
        return self._call("translate_beam", signal, lengths, spans, **kw)

    def translate_beam_classic(self, signal, lengths, spans=None, **kw):
        return self._call("translate_beam_classic", signal, lengths, spans, **kw)

    def encode(self, signal, lengths, spans=None):
        """Engine.encode on the next lane's context, joined to the current
        stream as Engine.encode is (the memory bank is a tensor of the caller's stream)."""
        eng = self.engines[self._next]
        self._next = (self._next + 1) % len(self.engines)
        return eng.encode(signal, lengths, spans)

    def synchronize(self):
        """Order the current stream after every lane's calls so far."""
        cur = torch.cuda.current_stream(self.device)
        for e in self.engines:
            cur.wait_stream(e.stream)

    def _each(self, name, *a):
        for e in self.engines:
            getattr(e, name)(*a)

    def set_ctx_path(self, path: int):
        self._each("set_ctx_path", path)

    def set_exact_fp32(self, on: bool):
        self._each("set_exact_fp32", on)

    def set_kernel_stamps(self, on: bool):
        self._each("set_kernel_stamps", on)

    def kernel_stamps(self):
        """Launch durations of the last call's roofline kernel, averaged over the lanes."""
        st = [e.kernel_stamps() for e in self.engines]
        n = sum(k for _, k in st)
        return (sum(u * k for u, k in st) / n if n else 0.0), n

    def close(self):
        for e in reversed(self.engines):  # the lanes that read lane 0's weights first
            if getattr(e, "_h", None):
                e.stream.synchronize()
            e.close()
        self._held = [None] * len(self.engines)


# ---------------------------------------------------------------------------
# op-level entry points (kernel unit tests)
# ---------------------------------------------------------------------------

def op_fold_layernorm(W: torch.Tensor, bias, ln_g: torch.Tensor, ln_b: torch.Tensor):
    """(W diag(ln_g), bias + W ln_b): the LayerNorm affine folded into the Linear."""
    N, K = W.shape
    Wo = torch.empty_like(W)
    bo = torch.empty(N, dtype=torch.float32, device=W.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(W.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_fold_layernorm(_ptr(W), _ptr(bias), _ptr(ln_g), _ptr(ln_b), _ptr(Wo), _ptr(bo), N, K,
                                               s), "nd_op_fold_layernorm")
    return Wo, bo


def op_split_weight(W: torch.Tensor):
    """(Wh, wscale): the split-fp16 image of W [N, K] (nd_op_split_weight)."""
    N, K = W.shape
    Wh = torch.empty(N, 2 * K, dtype=torch.int16, device=W.device)
    sc = ctypes.c_float(0.0)
    s = ctypes.c_void_p(torch.cuda.current_stream(W.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_split_weight(_ptr(W), N, K, _ptr(Wh), ctypes.byref(sc), s), "nd_op_split_weight")
    return Wh, sc.value


def op_gemm(A: torch.Tensor, W: torch.Tensor, bias=None, R=None, ln_g=None, ln_b=None, relu=False, norm=False,
            split=False):
    """C = relu?(LN?(A) W^T + bias) (+ R).  With ln_g/ln_b the affine is folded
    first (nd_op_fold_layernorm) and the GEMM runs with norm=1, as the engine
    does; norm=True alone means W/bias are already folded.  split=True runs
    the engine's split-fp16 form (nd_op_split_weight + nd_op_gemm_split)."""
    M, K = A.shape
    N = W.shape[0]
    if ln_g is not None:
        W, bias = op_fold_layernorm(W, bias, ln_g, ln_b)
        norm = True
    C = torch.empty(M, N, dtype=torch.float32, device=A.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(A.device).cuda_stream)
    if split:
        Wh, sc = op_split_weight(W)
        _lib.check(_lib.lib().nd_op_gemm_split(_ptr(A), _ptr(Wh), sc, _ptr(bias), _ptr(R), _ptr(C), M, N, K,
                                               int(norm), int(relu), s), "nd_op_gemm_split")
        return C
    _lib.check(_lib.lib().nd_op_gemm(_ptr(A), _ptr(W), _ptr(bias), _ptr(R), _ptr(C), M, N, K, int(norm), int(relu),
                                     s), "nd_op_gemm")
    return C


def op_gemm_split_q24(A: torch.Tensor, W: torch.Tensor, bias=None, norm=False):
    """The beam's K / V projection writing the 24-bit image (nd_op_gemm_split_q24): A [M, K], W [layers*512, K]
    (split-fp16 as op_gemm(split=True)) -> uint8 [layers, M, 1600] (layer-major)."""
    M, K = A.shape
    N = W.shape[0]
    layers = N // 512
    img = torch.zeros(layers, M, 1600, dtype=torch.uint8, device=A.device)
    Wh, sc = op_split_weight(W)
    s = ctypes.c_void_p(torch.cuda.current_stream(A.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_gemm_split_q24(_ptr(A), _ptr(Wh), sc, _ptr(bias), _ptr(img), M, M, N, K,
                                               int(norm), s), "nd_op_gemm_split_q24")
    return img


def op_enc_attention(qkv: torch.Tensor, signal: torch.Tensor, span: torch.Tensor):
    B, T = signal.shape
    out = torch.zeros(B * T, qkv.shape[1] // 3, dtype=torch.float32, device=qkv.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_enc_attention(_ptr(qkv), _ptr(signal), _ptr(span.to(torch.int32)), _ptr(out), B, T, s),
               "nd_op_enc_attention")
    return out


def pack_p16(x: torch.Tensor) -> torch.Tensor:
    """Row-major [M, N] -> the engine's P16 layout (include/nanodec.h,
    nd_op_gemm_p16), rows zero-padded to a multiple of 16.  Returned flat
    with shape [M16, N] for bookkeeping (the memory order is P16)."""
    M, N = x.shape
    M16 = (M + 15) // 16 * 16
    if M16 != M:
        x = torch.cat([x, x.new_zeros(M16 - M, N)])
    return x.reshape(M16 // 16, 16, N // 16, 4, 4).permute(0, 2, 3, 1, 4).contiguous().view(M16, N)


def unpack_p16(p: torch.Tensor, M: Optional[int] = None) -> torch.Tensor:
    """Inverse of pack_p16 (first M rows)."""
    M16, N = p.shape
    x = p.reshape(M16 // 16, N // 16, 4, 16, 4).permute(0, 3, 1, 2, 4).reshape(M16, N)
    return x[: (M16 if M is None else M)]


def row_partials(x: torch.Tensor, n: int = 16) -> torch.Tensor:
    """Per-row {mean, M2} of the n equal column tiles of a [M, 256] matrix in
    the engine's part layout [M, 16, 2] (what a producing GEMM hands over;
    slots >= n zero)."""
    t = x.view(x.shape[0], n, 256 // n)
    mu = t.mean(dim=2)
    m2 = ((t - mu[:, :, None]) ** 2).sum(dim=2)
    out = torch.zeros(x.shape[0], 16, 2, dtype=x.dtype, device=x.device)
    out[:, :n] = torch.stack([mu, m2], dim=2)
    return out


def op_pack_p16h(W: torch.Tensor):
    """(Wh, wscale): the split-fp16 P16H image of a row-major W [N, K]."""
    N, K = W.shape
    Wh = torch.empty(N, 2 * K, dtype=torch.int16, device=W.device)
    sc = ctypes.c_float(0.0)
    s = ctypes.c_void_p(torch.cuda.current_stream(W.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_pack_p16h(_ptr(W), N, K, _ptr(Wh), ctypes.byref(sc), s), "nd_op_pack_p16h")
    return Wh, sc.value


def op_enc_ffn(y, W1, b1, W2, b2, ln_g, ln_b, att=None, Wo=None, bo=None, inplace=False, Wq=None, bq=None,
               lnq_g=None, lnq_b=None):
    """The encoder's fused FFN block (nd_op_enc_ffn): x = y + W2 relu(W1
    LN(y) + b1) + b2 for row-major y [M, 256], the LN affine folded and both
    weights packed to P16H images here as the engine does at load time.
    With att, Wo, bo (nd_op_enc_ffn_wo) y is first replaced by
    y + att Wo^T + bo (the attention block's output projection and residual);
    inplace: x is written over y, as the engine does.  With Wq, bq, lnq_g,
    lnq_b too the next layer's projection LN(x) Wq^T + bq is computed in the
    same launch and returned as a fourth value.
    Returns (x, row stats [M, 2] = {mean, M2}, overflow flag[, qkv])."""
    M, F = y.shape[0], W1.shape[0]
    W1f, b1f = op_fold_layernorm(W1, b1, ln_g, ln_b)
    w1h, w1s = op_pack_p16h(W1f)
    w2h, w2s = op_pack_p16h(W2)
    x = y if inplace else torch.empty_like(y)
    part = torch.zeros(M, 16, 2, dtype=torch.float32, device=y.device)
    ov = torch.zeros(1, dtype=torch.int32, device=y.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(y.device).cuda_stream)
    if Wo is not None:
        woh, wos = op_pack_p16h(Wo)
        qh, qs, qb, qkv = None, 1.0, None, None
        if Wq is not None:
            Wqf, qb = op_fold_layernorm(Wq, bq, lnq_g, lnq_b)
            qh, qs = op_pack_p16h(Wqf)
            qkv = torch.empty(M, Wq.shape[0], dtype=torch.float32, device=y.device)
        _lib.check(_lib.lib().nd_op_enc_ffn_wo(_ptr(att), _ptr(y), _ptr(woh), wos, _ptr(bo), _ptr(w1h), w1s,
                                               _ptr(b1f), _ptr(w2h), w2s, _ptr(b2), _ptr(x), _ptr(part),
                                               _ptr(qh) if qh is not None else None, qs,
                                               _ptr(qb) if qb is not None else None,
                                               _ptr(qkv) if qkv is not None else None, M, F, _ptr(ov), s),
                   "nd_op_enc_ffn_wo")
        if qkv is not None:
            return x, part[:, 0, :], ov, qkv
    else:
        _lib.check(_lib.lib().nd_op_enc_ffn(_ptr(y), _ptr(w1h), w1s, _ptr(b1f), _ptr(w2h), w2s, _ptr(b2), _ptr(x),
                                            _ptr(part), M, F, _ptr(ov), s), "nd_op_enc_ffn")
    return x, part[:, 0, :], ov


def op_dec_ffn(yp, W1, b1, W2, b2, ln_g, ln_b, nsplit, skip=None, skip_rpc=1, tickets=None, slab=None):
    """The beam decoder's fused FFN block (nd_op_dec_ffn) on P16-packed rows
    yp [M16, 256] (M16 % 16 == 0): x = y + W2 relu(W1 LN(y) + b1) + b2 with d_ff
    split over nsplit workgroups per 128-row block.  Weights folded / packed
    here as the engine does at load time.  Returns (x packed, row stats
    [M16, 2] = {mean, M2}, overflow flag, tickets) -- pass the tickets back
    to reuse them (zero between launches)."""
    M, F = yp.shape[0], W1.shape[0]
    W1f, b1f = op_fold_layernorm(W1, b1, ln_g, ln_b)
    w1h, w1s = op_pack_p16h(W1f)
    w2h, w2s = op_pack_p16h(W2)
    x = torch.full_like(yp, float("nan"))
    part = torch.zeros(M, 16, 2, dtype=torch.float32, device=yp.device)
    ov = torch.zeros(1, dtype=torch.int32, device=yp.device)
    if tickets is None:
        tickets = torch.zeros((M + 127) // 128, dtype=torch.int32, device=yp.device)
    if slab is None:
        n = int(_lib.lib().nd_op_dec_ffn_slab_floats(M, nsplit))
        slab = torch.empty(max(n, 1), dtype=torch.float32, device=yp.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(yp.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_ffn(_ptr(yp), _ptr(w1h), w1s, _ptr(b1f), _ptr(w2h), w2s, _ptr(b2), _ptr(x),
                                        _ptr(part), M, F, nsplit, _ptr(slab), _ptr(tickets), _ptr(skip), skip_rpc,
                                        _ptr(ov), s), "nd_op_dec_ffn")
    return x, part[:, 0, :], ov, tickets


def op_gemm_p16(Ap, Wp, bias, M, N, K, Rp=None, part_in=None, relu=False, part_out=None, Wh=None, wscale=1.0,
                Wh_rm=None, wscale_rm=1.0):
    """The decoder-step GEMM on packed operands (see pack_p16).  Returns the
    packed C [M16, N] and the number of output row partials.  With Wh (an
    op_pack_p16h image) the split-fp16 kernels run instead of the fp32 ones;
    with Wh_rm too (op_split_weight of the row-major W) large M takes the
    LDS-tiled kernel as in the engine."""
    Cp = torch.empty(Ap.shape[0], N, dtype=torch.float32, device=Ap.device)
    pn = ctypes.c_int32(0)
    pn_in = 16 if part_in is not None else 0
    s = ctypes.c_void_p(torch.cuda.current_stream(Ap.device).cuda_stream)
    if Wh_rm is not None:
        _lib.check(_lib.lib().nd_op_gemm_p16_split_rm(_ptr(Ap), _ptr(Wh), wscale, _ptr(Wh_rm), wscale_rm, _ptr(bias),
                                                      _ptr(Rp), _ptr(Cp), M, N, K, _ptr(part_in), pn_in,
                                                      _ptr(part_out), int(relu), ctypes.byref(pn), s),
                   "nd_op_gemm_p16_split_rm")
        return Cp, pn.value
    if Wh is not None:
        _lib.check(_lib.lib().nd_op_gemm_p16_split(_ptr(Ap), _ptr(Wh), wscale, _ptr(bias), _ptr(Rp), _ptr(Cp), M, N, K,
                                                   _ptr(part_in), pn_in, _ptr(part_out), int(relu), ctypes.byref(pn),
                                                   s), "nd_op_gemm_p16_split")
        return Cp, pn.value
    _lib.check(_lib.lib().nd_op_gemm_p16(_ptr(Ap), _ptr(Wp), _ptr(bias), _ptr(Rp), _ptr(Cp), M, N, K, _ptr(part_in),
                                         pn_in, _ptr(part_out), int(relu), ctypes.byref(pn), s), "nd_op_gemm_p16")
    return Cp, pn.value


def op_gemm_p16_splitk(Ap, Wh, wscale, bias, M, N, K, Rp=None, part_out=None, tickets=None, slab=None):
    """The split-K long-K P16 GEMM (nd_op_gemm_p16_splitk) on packed operands; returns (C packed [M16, N],
    output row partials per row, tickets) -- pass the tickets back to reuse them (zero between calls)."""
    tiles = ((M + 31) // 32) * (N // 32)
    Cp = torch.empty((M + 15) // 16 * 16, N, dtype=torch.float32, device=Ap.device)
    if tickets is None:
        tickets = torch.zeros(tiles, dtype=torch.int32, device=Ap.device)
    if slab is None:
        slab = torch.empty(tiles * 4096, dtype=torch.float32, device=Ap.device)
    pn = ctypes.c_int32(0)
    s = ctypes.c_void_p(torch.cuda.current_stream(Ap.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_gemm_p16_splitk(_ptr(Ap), _ptr(Wh), float(wscale), _ptr(bias), _ptr(Rp), _ptr(Cp), M, N,
                                                K, _ptr(part_out), _ptr(slab), _ptr(tickets), tiles, ctypes.byref(pn),
                                                s), "nd_op_gemm_p16_splitk")
    return Cp, pn.value, tickets


def op_gemm_p16_splitk_f32(Ap, Wp, bias, M, N, K, Rp=None, part_out=None, tickets=None, slab=None):
    """The same split-K route in exact fp32 (nd_op_gemm_p16_splitk_f32): Wp the fp32 weight [N, K] P16-packed
    (pack_p16); returns (C packed [M16, N], output row partials per row, tickets)."""
    tiles = ((M + 31) // 32) * (N // 32)
    Cp = torch.empty((M + 15) // 16 * 16, N, dtype=torch.float32, device=Ap.device)
    if tickets is None:
        tickets = torch.zeros(tiles, dtype=torch.int32, device=Ap.device)
    if slab is None:
        slab = torch.empty(tiles * 4096, dtype=torch.float32, device=Ap.device)
    pn = ctypes.c_int32(0)
    s = ctypes.c_void_p(torch.cuda.current_stream(Ap.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_gemm_p16_splitk_f32(_ptr(Ap), _ptr(Wp), _ptr(bias), _ptr(Rp), _ptr(Cp), M, N, K,
                                                    _ptr(part_out), _ptr(slab), _ptr(tickets), tiles,
                                                    ctypes.byref(pn), s), "nd_op_gemm_p16_splitk_f32")
    return Cp, pn.value, tickets


def op_dec_self_attention(qkv, cache, step, anc=None, anc_ld=0, packed=False):
    """qkv [R, 768] row-major (or P16-packed with packed=True); returns out
    [R, 256] in the same convention."""
    R = qkv.shape[0]
    S = cache.shape[1]
    qp = qkv if packed else pack_p16(qkv)
    out = torch.empty(qp.shape[0], qkv.shape[1] // 3, dtype=torch.float32, device=qkv.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_self_attention(_ptr(qp), _ptr(cache), _ptr(anc), anc_ld, step, S, _ptr(out), R, s),
               "nd_op_dec_self_attention")
    return out if packed else unpack_p16(out, R)


def op_dec_self_attention_beam(qkv, cache, step, anc, rpc, done=None):
    """Beam rows' self-attention (nd_op_dec_self_attention_beam): qkv [R, 768] row-major, R = chunks * rpc,
    anc [R, S] each row's slots; returns out [R, 256] row-major."""
    R = qkv.shape[0]
    S = cache.shape[1]
    qp = pack_p16(qkv)
    out = torch.empty(qp.shape[0], 256, dtype=torch.float32, device=qkv.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_self_attention_beam(_ptr(qp), _ptr(cache), _ptr(anc), anc.shape[1], step, S,
                                                        _ptr(out), R, rpc, _ptr(done), s),
               "nd_op_dec_self_attention_beam")
    return unpack_p16(out, R)


def op_dec_self_attention_q24(qkv, cache, step, anc=None, rpc=1, done=None):
    """The 24-bit-history self-attention (nd_op_dec_self_attention_q24): qkv [R, 768] row-major, cache uint8
    [R, S, 1600] (appended in place), anc [R, S] or None (rpc 1); returns out [R, 256] row-major."""
    R = qkv.shape[0]
    S = cache.shape[1]
    qp = pack_p16(qkv)
    out = torch.empty(qp.shape[0], 256, dtype=torch.float32, device=qkv.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_self_attention_q24(_ptr(qp), _ptr(cache), _ptr(anc), S if anc is not None else 0,
                                                       step, S, _ptr(out), R, rpc, _ptr(done), s),
               "nd_op_dec_self_attention_q24")
    return unpack_p16(out, R)


def op_dec_ctx_attention(q, kv, ld, koff, signal, span, pad_val, rpc, packed=False):
    """q [C*rpc, 256] row-major (or P16-packed with packed=True); returns out
    in the same convention."""
    C, T = signal.shape
    R = C * rpc
    qp = q if packed else pack_p16(q)
    out = torch.empty(qp.shape[0], qp.shape[1], dtype=torch.float32, device=q.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(q.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_ctx_attention(_ptr(qp), _ptr(kv), ld, koff, _ptr(signal), _ptr(span), float(pad_val),
                                                  _ptr(out), C, rpc, T, s), "nd_op_dec_ctx_attention")
    return out if packed else unpack_p16(out, R)


CTXQ_ROW = 1600  # bytes per (key row, layer) of the 24-bit context K/V image (kernels.hpp)


def op_ctx_pack_q24(kv, ld, layers, span, B, T):
    """24-bit context K/V image (nd_op_ctx_pack_q24): kv [B*T, ld] f32 (layer l's
    k | v at columns l*512 .. l*512+511) -> uint8 [layers, B*T, 1600] (layer-major);
    rows t >= span[c] of chunk c are not written (left zero here)."""
    out = torch.zeros(layers, B * T, CTXQ_ROW, dtype=torch.uint8, device=kv.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(kv.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_ctx_pack_q24(_ptr(kv), ld, layers, _ptr(out), _ptr(span), B, T, s),
               "nd_op_ctx_pack_q24")
    return out


def op_dec_ctx_attention_q24(qp, kvq, layer, signal, span, pad_val, rpc):
    """Context attention on the 24-bit image (nd_op_dec_ctx_attention_q24): qp
    [R16, 256] P16-packed, kvq = op_ctx_pack_q24's image; returns out packed."""
    C, T = signal.shape
    out = torch.empty(qp.shape[0], qp.shape[1], dtype=torch.float32, device=qp.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(qp.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_ctx_attention_q24(_ptr(qp), _ptr(kvq), kvq.shape[0], layer, _ptr(signal),
                                                      _ptr(span), float(pad_val), _ptr(out), C, rpc, T, s),
               "nd_op_dec_ctx_attention_q24")
    return out


def op_alive_list(done, cap, ovf=None):
    """nd_op_alive_list: the chunks with done == 0 (ascending) in cap int32 slots, -1 after."""
    out = torch.empty(cap, dtype=torch.int32, device=done.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(done.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_alive_list(_ptr(done), done.numel(), _ptr(out), cap, _ptr(ovf), s), "nd_op_alive_list")
    return out


def op_dec_ctx_attention_list(qp, kv, ld, koff, signal, span, pad_val, rpc, clist, nsplit, q24=False, done=None,
                              out=None):
    """nd_op_dec_ctx_attention_list (the --fast beam tail's form): qp P16-packed; kv fp32 [C*T, ld] (or the
    24-bit image, ld / koff in bytes, q24=True); only the chunks listed in clist are written into out."""
    C, T = signal.shape
    ccap = clist.numel()
    if out is None:
        out = torch.zeros(qp.shape[0], qp.shape[1], dtype=torch.float32, device=qp.device)
    part = torch.empty(ccap * nsplit * rpc * 272, dtype=torch.float32, device=qp.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(qp.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_ctx_attention_list(_ptr(qp), _ptr(kv), ld, koff, int(q24), _ptr(signal),
                                                       _ptr(span), float(pad_val), _ptr(out), C, rpc, T, _ptr(clist),
                                                       ccap, nsplit, _ptr(part), _ptr(done), s),
               "nd_op_dec_ctx_attention_list")
    return out


def op_memory_pack(x, B, T, ln_g=None, ln_b=None, ldT=None):
    """Encoder output x [B*T, 256] -> row-major memory bank [B*ldT, 256]
    (LayerNorm'd when ln_g is given; rows t >= T of each chunk zero)."""
    ldT = ldT or T
    out = torch.empty(B * ldT, x.shape[1], dtype=torch.float32, device=x.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_memory_pack(_ptr(x), _ptr(ln_g), _ptr(ln_b), _ptr(out), B, T, ldT, s),
               "nd_op_memory_pack")
    return out


def op_dec_mem_attention(qp, mem_p, signal, span, pad_val, rpc, out=None, grid=0):
    """Memory-bank context attention: qp [R16, 2048] packed, mem_p the
    row-major bank [C*ldT, 256] (op_memory_pack); returns U [R16, 2048] packed
    (rows of chunks c < C written).  rpc must be 1; grid > 0: that many
    workgroups walk the chunks (nd_set_bank_grid's form)."""
    C, T = signal.shape
    ldT = mem_p.shape[0] // C
    if out is None:
        out = torch.empty(qp.shape[0], qp.shape[1], dtype=torch.float32, device=qp.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(qp.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_mem_attention(_ptr(qp), _ptr(mem_p), _ptr(signal), _ptr(span), float(pad_val),
                                                  _ptr(out), C, rpc, T, ldT, int(grid), s), "nd_op_dec_mem_attention")
    return out


def op_bank_pack_d8(x, B, T, ln_g=None, ln_b=None, ovf=None, span=None):
    """24-bit digit bank (nd_op_bank_pack_d8): x [B*T, 256] -> (digits uint8
    [B * 512 * 256 * 3], row scales [B * 512], each chunk's largest row scale
    [B] as float bits in int32).  span [B] int32 (optional): rows at or past a
    chunk's span are zero."""
    dev = x.device
    bank = torch.empty(B * 512 * 256 * 3, dtype=torch.uint8, device=dev)
    ks = torch.empty(B * 512, dtype=torch.float32, device=dev)
    em = torch.empty(B, dtype=torch.int32, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(_lib.lib().nd_op_bank_pack_d8(_ptr(x), _ptr(ln_g), _ptr(ln_b), _ptr(bank), _ptr(ks), _ptr(em),
                                             _ptr(span), B, T, _ptr(ovf), s), "nd_op_bank_pack_d8")
    return bank, ks, em


def op_dec_bank_d8(qp, bank, signal, span, pad_val, out=None, ovf=None, grid=0):
    """Memory-bank context attention on the 24-bit digit bank (nd_op_dec_bank_d8):
    qp [C, 2048] row-major, bank = op_bank_pack_d8's triple, T in [1, 512] (ceil(T / 128) key blocks per
    wave streamed);
    returns U [C16, 2048] packed."""
    C, T = signal.shape
    digits, ks, em = bank
    if out is None:
        out = torch.empty((C + 15) // 16 * 16, qp.shape[1], dtype=torch.float32, device=qp.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(qp.device).cuda_stream)
    _lib.check(_lib.lib().nd_op_dec_bank_d8(_ptr(qp), _ptr(digits), _ptr(ks), _ptr(em), _ptr(signal), _ptr(span),
                                            float(pad_val), _ptr(out), C, T, _ptr(ovf), int(grid), s),
               "nd_op_dec_bank_d8")
    return out


def op_lstm_layer(whh, lens, T, xp=None, signal=None, wih0=None, bsum=None, bn_scale=None, bn_shift=None,
                  out=None):
    """One BiLSTM layer (both directions) through nd_op_lstm_layer:
    whh [2, 512, 128], lens [B] int32 on the device.  Layer 0: signal [B, T],
    wih0 / bsum [2, 512]; otherwise xp [B*T, 1024] = x W_ih^T + b_ih + b_hh
    (fwd | bwd).  Returns out [B*T, 256] (zeros at t >= len)."""
    B = lens.shape[0]
    dev = whh.device
    if out is None:
        out = torch.zeros(B * T, 256, dtype=torch.float32, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(_lib.lib().nd_op_lstm_layer(_ptr(xp), _ptr(signal), _ptr(wih0), _ptr(bsum), _ptr(whh), _ptr(lens), B,
                                           T, _ptr(out), _ptr(bn_scale), _ptr(bn_shift), int(xp is None), s),
               "nd_op_lstm_layer")
    return out


def pad_chunks(chunks: Sequence[np.ndarray], T: Optional[int] = None):
    """make_nano (inputters/inputter.py:86-95): zero pad to [B, T]."""
    lens = np.array([len(c) for c in chunks], np.int32)
    T = int(lens.max()) if T is None else T
    out = np.zeros((len(chunks), T), np.float32)
    for i, c in enumerate(chunks):
        out[i, : len(c)] = c
    return out, lens
