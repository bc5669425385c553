#!/usr/bin/env python
"""Benchmark of the MI355X translate path (BASELINE.json metric).

A "step" = one full translate call (encoder + all decoder steps + search) on
one batch of synthetic 512-sample chunks already resident in HBM.  Default
workload = BASELINE.json configs[1]: 3+3 transformer, d_model 256, T 512,
batch 256 chunks per GPU, greedy, max_length 100, random-init weights of the
reference architecture (no trained checkpoint exists offline).

Multi-GPU: ``--gpus N`` starts N rank processes itself (torch.distributed.run,
spawned before this process touches the GPU) unless it already runs under a
launcher (WORLD_SIZE set).  Reads shard across ranks with no collective in the
hot loop ("scaling": "weak"); rank 0 creates the weights and broadcasts them
once over RCCL.

Beside the headline ``value`` the line carries, on every run:
  roofline      the dominant kernel against its HBM roofline (live in-kernel
                timing) + the fused encoder FFN block against the MFMA peak;
  mfma          algorithmic MFMA utilisation, path-level and encoder-only,
                against the fp32 peak and the split-fp16 fp32-equivalent peak
                (and the committed rocprof counter pass, profiles/);
  exact_fp32    the same workload with every product in exact fp32;
  host_inclusive the same batches through Translator (host packing, H2D,
                token D2H) — PCIe-inclusive, never ``value``;
  read_shard    BASELINE configs[4]: the synthetic read set sharded over the
                ranks (front end + packing + engine), samples/s, bases/s,
                per-rank load, world size;
  cpu_baseline  the CPU oracle at configs[0]'s batch 50 (rank 0, N=1).
``--workload reads`` makes configs[4] the headline.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "signal-samples/sec/GPU (512-sample chunks) + bases/sec at 1/2/4/8 MI355X"
FP32_PEAK = 157.3            # TFLOP/s, dense fp32 MFMA (MI355X_MICROARCH.md)
SPLIT_PEAK = 2516.6 / 3      # TFLOP/s fp32-equivalent: dense fp16 MFMA peak / 3 split products
HBM_PEAK = 8000.0            # GB/s
HBM_MEASURED = 6290.0        # GB/s: MI355X_MICROARCH.md's measured float4 copy (79 % of the spec peak)
FLOP_PER_CHUNK = 6_273_038_336          # SURVEY.md §8d, greedy, 100 steps (12.25 MFLOP/sample)
ENC_FLOP_PER_CHUNK = 4_832_100_352      # transformer encoder term
NANO_ENC_FLOP_PER_CHUNK = 1_007_681_536  # NanoEncoder term
DEC_FLOP_PER_CHUNK = 1_440_937_984      # decoder term (greedy, 100 steps)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed steps (200 x ~29 ms: a timed region of ~6 s)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="chunks per GPU per step")
    ap.add_argument("--mode", default="greedy", choices=["greedy", "beam"])
    ap.add_argument("--beam", type=int, default=5)
    ap.add_argument("--bank-nt-lanes", default="auto",
                    help="comma list of EnginePool lanes whose memory bank streams with non-temporal loads "
                         "(auto: every lane when --inflight > 1; none: no lane)")
    ap.add_argument("--bank-grid", default="auto",
                    help="memory-bank kernel workgroups at most per pool lane (auto: half the CUs with several "
                         "lanes; 0: one per chunk)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="translate calls on the device at once (EnginePool lanes: one engine context and HIP "
                         "stream each); 1 = one call at a time")
    ap.add_argument("--encoder", default="transformer", choices=["transformer", "nano"])
    ap.add_argument("--max-length", type=int, default=100)
    ap.add_argument("--min-length", type=int, default=57,
                    help="-min_length: EOS masked before this step.  The random-init model is EOS-prone, so this "
                         "sets its decode length to a trained basecaller's ~57 bases per 512 samples (greedy cost "
                         "is unaffected: all max_length steps always run)")
    ap.add_argument("--eos-bias", type=float, default=-3.0, help="generator EOS logit shift of the random-init model")
    ap.add_argument("--workload", default="batch", choices=["batch", "reads"],
                    help="batch: configs[1..3] fixed batches resident in HBM; reads: configs[4] read sharding")
    ap.add_argument("--reads", type=int, default=16384, help="synthetic reads PER GPU for the read-shard workload")
    ap.add_argument("--read-shard", type=int, default=1, help="append the configs[4] read-shard measurement")
    ap.add_argument("--config-legs", type=int, default=1,
                    help="append configs[2] (NanoEncoder greedy) and configs[3] (--fast beam, batch 1024) measured "
                         "in the same run")
    ap.add_argument("--exact", type=int, default=1, help="append the exact-fp32 throughput")
    ap.add_argument("--host-inclusive", type=int, default=1, help="append the Translator (host-inclusive) rate")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 (0 = skip)")
    ap.add_argument("--cpu-chunks", type=int, default=50, help="CPU baseline batch (configs[0]: 50)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline: repeat batches for at least this")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--allow-switches", action="store_true",
                    help="run even when an ND_* A/B switch of the library is set to a non-default value (the line "
                         "then carries headline: false)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--selftest-cpu", action="store_true",
                    help="launcher/rank plumbing self-test on CPU (gloo, no engine, no measurement)")
    return ap.parse_args()


# ----------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args) -> int:
    """--gpus N outside a launcher: N rank processes under torch.distributed.run,
    started as CHILDREN of this process before it has made any GPU call
    (pipeline.evaluate.sh:114-115 runs one process per GPU the same way)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        if args.backend == "nccl" and not args.selftest_cpu:  # the CPU self-test is gloo whatever --backend says
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group("gloo")
    elif args.backend == "nccl" and args.read_shard and not args.selftest_cpu and torch.cuda.is_available():
        # N = 1 without a launcher: a one-rank RCCL group, so the read-shard leg's weight broadcast (from HIP
        # memory) and its gloo control exchanges run as at N > 1 (shard.run_distributed)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
    return world, rank, local


def workload(args):
    if args.workload == "reads":
        return (f"configs[4]: 3+3 transformer, d_model 256, src_seq_length 512, synthetic read set "
                f"({args.reads} reads/GPU, lengths U[256,1024]) sharded by LPT over the ranks, greedy, "
                f"engine batch {args.batch}, max_length {args.max_length}")
    idx = 3 if args.mode == "beam" else (2 if args.encoder == "nano" else 1)
    enc = "3-layer transformer encoder" if args.encoder == "transformer" else "NanoEncoder (3x BiLSTM)"
    dec = "greedy" if args.mode == "greedy" else f"--fast beam {args.beam}"
    return (f"configs[{idx}]: {enc} + 3-layer transformer decoder, d_model 256, src_seq_length 512, "
            f"batch {args.batch}, {dec}, max_length {args.max_length}")


# ----------------------------------------------------------------- CPU baseline
def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """Threads the CPU baseline may use: the cores this process is given
    (OMP_NUM_THREADS where the box sets it, else the affinity mask)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(cfg, W, sig, lens, args):
    from oracle import ref_cpu
    n = min(args.cpu_chunks, sig.shape[0])
    threads = cpu_threads()
    torch.set_num_threads(threads)
    m = ref_cpu.RefModel(cfg, W)
    done, dt, batches = 0, 0.0, 0
    t0 = time.perf_counter()
    while dt < args.cpu_seconds or batches == 0:
        s, l = sig[done % sig.shape[0]:][:n], lens[done % sig.shape[0]:][:n]
        if s.shape[0] < n:
            s, l = sig[:n], lens[:n]
        if args.mode == "greedy":
            ref_cpu.greedy(m, s, l, max_length=args.max_length, min_length=args.min_length)
        else:
            ref_cpu.fast_beam(m, s, l, beam_size=args.beam, max_length=args.max_length, min_length=args.min_length)
        done += n
        batches += 1
        dt = time.perf_counter() - t0
        if args.mode == "beam":
            break
    return {"value": round(float(done * 512 / dt), 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "machine_cpus": os.cpu_count(),
            "sample": f"oracle/ref_cpu.py {args.mode} (the reference's algorithm in torch CPU fp32, pinned to the "
                      f"reference's own outputs by tests/golden) on {batches} batch(es) of {n} chunks x 512 "
                      f"samples (configs[0] batch), max_length {args.max_length}, {threads} threads, {dt:.1f} s"}


# ----------------------------------------------------------------- helpers
class _StreamTimer:
    """HIP events on the stream the engine's kernels run on (the engine's own
    stream is joined to the current stream by events, so bracketing the
    current stream covers the whole call)."""

    def __init__(self, dev):
        self.dev = dev

    def time(self, fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream(self.dev))
        for i in range(n):
            fn(i)
        e1.record(torch.cuda.current_stream(self.dev))
        e1.synchronize()
        return e0.elapsed_time(e1) / n


def _pmc(name, key="kernels"):
    """(HBM bytes per launch, the table entry used) for kernel `name` from the
    committed PMC summary (profiles/pmc_summary.json, tools/pmc_summary.py:
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes with the gfx950 x2
    FETCH_SIZE correction), or (None, None).  The table keys kernels by their
    full template name ('dec_bank_d8_kernel<false, false, 4>'): an exact name is
    looked up as given; a bare name takes its only instantiation in the table,
    or the plain '<false, false, ...>' one among several."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            table = json.load(f)[key]
    except Exception:
        return None, None
    if name in table:
        return table[name]["hbm_bytes_per_launch"], name
    forms = sorted(k for k in table if k.split("<")[0] == name.split("<")[0])
    if len(forms) > 1:
        forms = [k for k in forms if k.split("<", 1)[-1].startswith("false, false")] or forms
    if len(forms) == 1:
        return table[forms[0]]["hbm_bytes_per_launch"], forms[0]
    return None, None


def _pmc_beam():
    """configs[3]'s context-attention counter traffic per alive chunk-launch
    from the newest committed profiles/rNN_pmc_beam.json (tools/pmc_beam.py:
    FETCH_SIZE / WRITE_SIZE passes over exactly the config_legs workload), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_beam.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        c = d["ctx_attention"]
        return {"per_alive_chunk": c["traffic_per_alive_chunk_launch"], "ratio": c["ratio"],
                "source": "profiles/" + os.path.basename(files[-1]), "workload": d["workload"]}
    except Exception:
        return None


def _mfma_counters(which):
    """The newest committed rocprof MFMA counter pass of this workload
    (profiles/rNN_mfma_summary.json, the highest round: tools/gpu.sh mfma ->
    tools/mfma_summary.py; which = greedy | beam | nano), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_mfma_summary.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)[which]
    except Exception:
        return None
    k = d["kernels"]
    top = sorted(k.items(), key=lambda kv: -kv[1]["launches"] * kv[1]["avg_us"])[:6]
    return {"source": "profiles/" + os.path.basename(files[-1]) + " (" + d["tag"] + ")", "path": d["path"],
            "top_kernels": {n: {x: v[x] for x in ("avg_us", "f16_tflops", "f32_tflops", "mfma_util")} for n, v in top}}


def dtype_of(form: int) -> str:
    """The arithmetic a call ran in, from the engine's nd_bank_form (each leg states its own)."""
    base = "f32 (fp32 values; products as split-fp16 x3 on fp16 MFMA: 22-bit operands, fp32 accumulate"
    if form == 2:
        return base + "; the greedy memory bank as 24-bit fixed point per key row: int8 digit MFMAs summed exactly in int32)"
    if form == 3:
        return base + "; the beam's context K/V as 24-bit integers with a power-of-two scale per (key, head))"
    return base + ")"


def count_bases(tok: np.ndarray, eos: int) -> int:
    """Base tokens (ids >= 4: not <unk>/<blank>/<s>/</s>) before the first EOS."""
    is_eos = tok == eos
    first = np.where(is_eos.any(1), is_eos.argmax(1), tok.shape[1])
    return int(((np.arange(tok.shape[1])[None, :] < first[:, None]) & (tok >= 4)).sum())


# ----------------------------------------------------------------- roofline
def kernel_roofline(eng, B, mode, beam, encoder="transformer", alive=None, secondary=True):
    """Dominant kernel of the translate step, timed LIVE: every launch of it
    inside the timed graph replays carries in-kernel wall-clock stamps
    (first workgroup start, last workgroup end; Engine.set_kernel_stamps), and
    the mean over the last timed call's launches is the launch duration.

    greedy: the memory-bank context attention (dec_bank_d8_kernel at
      512-sample chunks), bounded by HBM: per launch it streams the B x 512 x
      256 memory bank once (24-bit digits: 3 bytes per element + one float
      scale per key row; + q' in, U out, the signal for the key mask).  Its MFMA view (2
      products x 2 x 8 heads x 512 keys x 256 dims per chunk, split-fp16 on
      fp16 MFMAs) is reported beside it.
    beam: the per-layer K/V context attention (dec_ctx_attention_kernel),
      HBM-bound: K+V 2 x 512 keys x 256 f32 per chunk + q, signal, out, for
      the chunks still in the decode loop (finished chunks' workgroups exit
      at once; launches with none alive carry no stamp): achieved = the
      alive chunks' bytes over all stamped launches / their summed time."""
    us, n = eng.kernel_stamps()
    T, D = 512, 256
    ms = us * 1e-3
    if mode == "greedy":
        # 512-sample chunks stream the 24-bit digit bank (dec_bank_d8_kernel: 3 bytes per element + a
        # float scale per key row); exact fp32 runs the fp32 bank kernel
        form = eng.engines[0].bank_form() if hasattr(eng, "engines") else eng.bank_form()
        if form == 2:
            e0 = eng.engines[0] if hasattr(eng, "engines") else eng
            # the instantiation this call launched (bank8.hip: <non-temporal, grid walk>), as the PMC table keys it
            # <non-temporal, walking, key blocks per wave> (4 at T = 512: bank8.hip bank8_kpw)
            name = (f"dec_bank_d8_kernel<{'true' if e0.bank_nt else 'false'}, {'true' if e0.bank_grid else 'false'}, "
                    f"{min(4, (512 + 127) // 128)}>")
            nbytes = B * T * D * 3 + B * T * 4 + B * 4 + B * T * 4 + 2 * B * 8 * D * 4
        else:
            name = "dec_mem_attention_kernel<8>"
            nbytes = B * T * D * 4 + B * T * 4 + 2 * B * 8 * D * 4
        flops = 2 * 2 * 8 * T * D * B
        tf = flops / (ms * 1e-3) / 1e12
        extra = {"mfma_view": {"algorithmic_flops_per_launch": flops, "achieved": round(tf, 2), "peak": round(SPLIT_PEAK, 1),
                               "unit": "TFLOP/s fp32-equivalent (split-fp16 on fp16 MFMA)", "frac": round(tf / SPLIT_PEAK, 4)}}
    else:
        form = eng.engines[0].bank_form() if hasattr(eng, "engines") else eng.bank_form()
        if form == 3:  # the 24-bit context K/V image (1600 B per key: 3-byte k, v + 8 head scales each)
            name = f"dec_ctx_q24_kernel<{beam}>"
            per_chunk = T * 1600 + T * 4 + 2 * beam * D * 4
        else:
            name = f"dec_ctx_attention_kernel<{beam}>"
            per_chunk = T * 2 * D * 4 + T * 4 + 2 * beam * D * 4
        nbytes = B * per_chunk
        extra = {}
        if alive is not None and n > 0:
            # mean bytes of a stamped launch (3 layers per step with >= 1 alive chunk); a pool's stamps are
            # every lane's last call, each the same workload
            lanes = len(eng.engines) if hasattr(eng, "engines") else 1
            nbytes = int(3 * sum(alive) * per_chunk * lanes / n)
            extra = {"alive_chunks_per_launch": round(3 * sum(alive) * lanes / n, 1)}
    ach = nbytes / (ms * 1e-3) / 1e9
    if mode == "greedy" and form == 2:
        # SURVEY.md §8(d) prices the context attention as fp32 K and V per layer (1,048,576 B per chunk per
        # layer-step); this kernel moves neither: the K / V projections are folded into the query and output
        # sides (all three layers read the one LN'd encoder output: x 0.5) and that bank is 24-bit (x 0.75)
        s8d = B * 2 * T * D * 4
        extra["survey_8d_byte_model"] = {
            "bytes_per_launch": s8d, "equivalent_rate_gbs": round(s8d / (ms * 1e-3) / 1e9, 1),
            "note": ("fp32 K+V per chunk per layer-step (SURVEY §8d); the kernel streams a folded bank (x 0.5: "
                     "W_k folded into q', W_v into the output projection) in 24 bits (x 0.75) = 0.375 of these "
                     "bytes, so this equivalent rate is not a fraction of the HBM peak")}
        # the bound the probe found: a lone call's 104 MB bank stays in the 256 MB Infinity Cache across the
        # step's launches; resident vs evicted measured 22.5 vs 25.8 us (tools/bank_mall.py)
        extra["residency"] = {"infinity_cache_resident_us": 22.54, "evicted_us": 25.79,
                              "source": "profiles/r05_bank_mall.txt",
                              "note": ("HBM bytes set ~13% of this kernel's time; the rest is its per-key-block "
                                       "issue work (LDS image writes and transposed reads, digit -> f16 "
                                       "conversions, MFMAs at two waves per SIMD), DESIGN.md §8")}
    traffic, tsrc = _pmc(name, "kernels" if mode == "greedy" else "kernels_beam")
    if mode == "greedy":
        tnote = (f"profiles/pmc_summary.json kernels['{tsrc}'] (one configs[1] call, rocprofv3 FETCH_SIZE / "
                 f"WRITE_SIZE passes: L2 <-> fabric bytes, HBM or Infinity Cache; the non-temporal form moves "
                 f"the same lines)" if tsrc else None)
    else:
        pb = _pmc_beam() if "alive_chunks_per_launch" in extra else None
        traffic, tnote = None, None
        if pb is not None:
            # the counter pass's bytes per alive chunk-launch x this leg's alive chunks per launch (same workload)
            traffic = int(pb["per_alive_chunk"] * extra["alive_chunks_per_launch"])
            tnote = (f"{pb['source']}: {pb['per_alive_chunk']:.0f} B per alive chunk-launch, {pb['ratio']}x the "
                     f"algorithmic {nbytes / max(extra['alive_chunks_per_launch'], 1e-9):.0f}; {pb['workload']}")
    out = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1), "peak": HBM_PEAK, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK, 4), "traffic": traffic, "traffic_source": tnote,
           "algorithmic_bytes_per_launch": nbytes,
           "avg_launch_ms": round(ms, 5), "timed_launches": n,
           "timing": "in-kernel wall-clock stamps, launches of the last timed call",
           "frac_of_measured_copy": round(ach / HBM_MEASURED, 4),
           "measured_copy_gbs": HBM_MEASURED}
    out.update(extra)
    dev = eng.device
    if not secondary:
        return out
    if encoder == "nano":
        out["lstm_kernel"] = lstm_view(dev, B, T)
        return out
    import ctypes
    from nanodecoder_amd import _lib
    from nanodecoder_amd.engine import op_fold_layernorm, op_pack_p16h
    # secondary: the dominant encoder MFMA kernel in the form the engine launches for layers 0-1
    # (enc_ffn_kernel<1, true, true>: the attention's output projection Wo + residual, LN + W1 + bias +
    # ReLU + W2 + bias + residual with the hidden kept on chip, and the next layer's LN + QKV projection),
    # split-fp16: 3 fp16 MFMA products per fp32 multiply-add, so its fp32-equivalent peak is the dense fp16
    # peak / 3.  Algorithmic work: Wo 2 M D^2 + FFN 4 M F D + QKV 6 M D^2.
    M, D, F = B * T, 256, 2048
    Y = torch.randn(M, D, device=dev)
    att = torch.randn(M, D, device=dev)
    W1, b1 = op_fold_layernorm(torch.randn(F, D, device=dev) / 16, torch.randn(F, device=dev) * 0.1,
                               torch.ones(D, device=dev), torch.zeros(D, device=dev))  # as at load time
    w1h, w1s = op_pack_p16h(W1)
    w2h, w2s = op_pack_p16h(torch.randn(D, F, device=dev) / F ** 0.5)
    woh, wos = op_pack_p16h(torch.randn(D, D, device=dev) / 16)
    Wq, bq = op_fold_layernorm(torch.randn(3 * D, D, device=dev) / 16, torch.randn(3 * D, device=dev) * 0.1,
                               torch.ones(D, device=dev), torch.zeros(D, device=dev))
    qh, qs = op_pack_p16h(Wq)
    b2, bo = torch.randn(D, device=dev) * 0.1, torch.randn(D, device=dev) * 0.1
    X = torch.empty_like(Y)
    qkv = torch.empty(M, 3 * D, device=dev)
    part = torch.empty(M, 16, 2, device=dev)
    ov = torch.zeros(1, dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def ffn(i):
        _lib.check(_lib.lib().nd_op_enc_ffn_wo(att.data_ptr(), Y.data_ptr(), woh.data_ptr(), wos, bo.data_ptr(),
                                               w1h.data_ptr(), w1s, b1.data_ptr(), w2h.data_ptr(), w2s,
                                               b2.data_ptr(), X.data_ptr(), part.data_ptr(), qh.data_ptr(), qs,
                                               bq.data_ptr(), qkv.data_ptr(), M, F, ov.data_ptr(), st),
                   "nd_op_enc_ffn_wo")
    for i in range(3):
        ffn(i)
    gms = _StreamTimer(dev).time(ffn, 10)
    flops = 2 * M * D * D + 4 * M * F * D + 6 * M * D * D
    tf = flops / (gms * 1e-3) / 1e12
    out["mfma_kernel"] = {"kernel": "enc_ffn_kernel<1, true, true, false> (the engine's form for encoder layers 0-1: "
                                    "Wo + residual, LN + W1 + ReLU + W2 + residual, next layer's LN + QKV; split-fp16)",
                          "achieved": round(tf, 2), "peak": round(SPLIT_PEAK, 1),
                          "unit": "TFLOP/s fp32-equivalent (fp16 MFMA peak / 3 products)",
                          "frac": round(tf / SPLIT_PEAK, 4), "avg_launch_ms": round(gms, 4),
                          "algorithmic_flops_per_launch": int(flops), "rows": M,
                          "timing": ("10 back-to-back launches on random operands (HIP events): the sustained "
                                     "rate, at the lower clock the chip holds under this kernel alone; inside "
                                     "a translate call it runs between the decoder's short kernels and the "
                                     "kernel trace times it ~10-15% faster (profiles/r06f_one_call_kernel_"
                                     "stats.txt, DESIGN.md section 5)")}
    del Y, X, W1, w1h, w2h
    return out


def lstm_view(dev, B, T):
    """The NanoEncoder's recurrence (lstm_dir_kernel, one BiLSTM layer in
    its layer-1 form) timed alone: latency-bound (T sequential steps, one
    workgroup barrier each), so the figure of merit is the time per step; the
    MFMA rate counts the algorithmic recurrent product 2 x 2 directions x B x
    512 gates x 128 per step against the dense fp16 peak / 3 (split-fp16)."""
    from nanodecoder_amd.engine import op_lstm_layer
    g = torch.Generator(device="cpu").manual_seed(3)
    whh = ((torch.rand(2, 512, 128, generator=g) - 0.5) * 0.2).to(dev)
    xp = torch.randn(B * T, 1024, generator=g).to(dev)
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    out = torch.zeros(B * T, 256, device=dev)

    def layer(i):
        op_lstm_layer(whh, lens, T, xp=xp, out=out)
    for i in range(2):
        layer(i)
    ms = _StreamTimer(dev).time(layer, 5)
    flops = 2.0 * 2 * B * 512 * 128 * T
    tf = flops / (ms * 1e-3) / 1e12
    return {"kernel": "lstm_dir_kernel (BiLSTM layer, split-fp16)", "bound": "latency",
            "avg_launch_ms": round(ms, 4), "us_per_step": round(ms * 1e3 / T, 3),
            "achieved": round(tf, 2), "peak": round(SPLIT_PEAK, 1),
            "unit": "TFLOP/s fp32-equivalent (fp16 MFMA peak / 3 products)", "frac": round(tf / SPLIT_PEAK, 4)}


def mfma_view(args, eng, sig, lens, ms_per_step):
    """Algorithmic MFMA utilisation (SURVEY §8d FLOP counts) of the whole
    path and of the encoder alone (nd_encode timed by itself), against the
    peak of the pipe the products run on: the fp16 matrix pipe, three fp16
    products per fp32 multiply-add (split-fp16), i.e. dense fp16 peak / 3.
    The exact-fp32 leg carries its own roofline against the fp32 MFMA peak."""
    B = args.batch
    enc_flop = ENC_FLOP_PER_CHUNK if args.encoder == "transformer" else NANO_ENC_FLOP_PER_CHUNK
    path_flop = (enc_flop + DEC_FLOP_PER_CHUNK) * B
    if args.mode != "greedy":
        return None
    timer = _StreamTimer(eng.device)
    for _ in range(2):
        eng.encode(sig, lens, lens)
    enc_ms = timer.time(lambda i: eng.encode(sig, lens, lens), 10)
    path_tf = path_flop / (ms_per_step * 1e-3) / 1e12
    enc_tf = enc_flop * B / (enc_ms * 1e-3) / 1e12
    out = {"algorithmic_flop_per_chunk": enc_flop + DEC_FLOP_PER_CHUNK,
           "path": {"tflops": round(path_tf, 2), "frac_split_peak": round(path_tf / SPLIT_PEAK, 4)},
           "encoder_only": {"ms": round(enc_ms, 4), "tflops": round(enc_tf, 2),
                            "frac_split_peak": round(enc_tf / SPLIT_PEAK, 4),
                            "note": "nd_encode incl. its memory-bank pack"},
           "peak": {"split_fp16_fp32_equiv": round(SPLIT_PEAK, 1), "unit": "TFLOP/s",
                    "note": "fp32-equivalent work on the fp16 matrix pipe: dense fp16 peak 2516.6 / 3 products"}}
    cnt = _mfma_counters("nano" if args.encoder == "nano" else "greedy")
    if cnt is not None:
        out["rocprof_counters"] = cnt
    return out


# ----------------------------------------------------------------- workloads
def run_calls(pool, n, call, every_lane=False):
    """n translate calls, `pool.lanes` of them on the device at once; returns
    the last call's outputs (complete: every lane is joined to the current
    stream), or with ``every_lane`` the last outputs of each lane.
    ``call(engine_or_pool)`` issues one call.  Greedy calls are
    asynchronous, so one host thread keeps every lane busy; a beam call polls
    its alive count between 10-step graph segments (host-synchronous), so each
    lane gets a host thread of its own there."""
    import threading
    outs = [None] * pool.lanes
    if not getattr(call, "blocking", False) or pool.lanes == 1:
        for k in range(n):
            outs[k % pool.lanes] = call(pool)
        pool.synchronize()
        return outs if every_lane else outs[(n - 1) % pool.lanes]
    cur = torch.cuda.current_stream(pool.device)
    errs = []

    def lane(i):
        try:
            e = pool.engines[i]
            with torch.cuda.stream(e.stream):
                for _ in range(i, n, pool.lanes):
                    outs[i] = call(e)
        except BaseException as ex:  # surfaced below
            errs.append(ex)
    for e in pool.engines:
        e.stream.wait_stream(cur)
    th = [threading.Thread(target=lane, args=(i,)) for i in range(min(pool.lanes, n))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    pool.synchronize()
    return outs if every_lane else outs[(n - 1) % pool.lanes]


def pool_check(cfg, W, args, mode, B, beam, call, outs):
    """The timed pooled calls' outputs against one fresh single engine on the
    same inputs (tokens and scores, + lengths for beam), bitwise: "identical"
    or what differed.  The single engine is oracle-pinned at these sizes
    (tests/test_gpu_configs.py)."""
    from nanodecoder_amd.engine import Engine
    one = Engine(cfg, W, device=torch.cuda.current_device(), max_batch=B, max_src_len=512,
                 max_steps=args.max_length, max_beam=beam)
    one.set_gemm_splitk(args.inflight > 1)  # the lanes' K = 2048 product form (nd_set_gemm_splitk)
    try:
        ref = call(one)
        keys = ("tokens", "scores") + (("lens",) if mode == "beam" else ())
        bad = []
        for lane, o in enumerate(outs):
            if o is None:
                continue
            for k in keys:
                if not torch.equal(o[k].cpu(), ref[k].cpu()):
                    bad.append(f"lane {lane} {k}")
        return {"result": "identical" if not bad else "DIFFERENT: " + ", ".join(bad),
                "lanes_compared": sum(o is not None for o in outs),
                "against": "a fresh single Engine (one call in flight, bank kernel one workgroup per chunk, the "
                           "lanes' split-K form)"}
    finally:
        one.close()


def bank_grid(args):
    return None if args.bank_grid == "auto" else int(args.bank_grid)


def nt_lanes(args):
    if args.bank_nt_lanes == "auto":
        return None
    if args.bank_nt_lanes == "none":
        return []
    return [int(x) for x in args.bank_nt_lanes.split(",") if x.strip()]


def make_call(args, mode, sig, lens, min_len=None):
    ml = args.min_length if min_len is None else min_len
    if mode == "greedy":
        def call(e):
            return e.translate_greedy(sig, lens, lens, max_len=args.max_length, min_len=ml)
        return call

    def call(e):
        return e.translate_beam(sig, lens, lens, beam=args.beam, max_len=args.max_length, min_len=ml)
    call.blocking = True
    return call


def timed(pool, n, call, world, every_lane=False):
    """Seconds for n calls between a barrier + device sync on both sides, max over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = run_calls(pool, n, call, every_lane)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=pool.device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    return dt, out


def beam_steps_and_worst_case(args, pool, sig, lens, call, out, world, res):
    """--fast beam legs: the decoder steps executed, the steps each chunk ran
    (the reference drops a finished chunk's batch at that step,
    translate/translator.py:793-823), and the forced-100-step worst case (EOS
    masked at every step: -min_length = max_length), into ``res``; returns
    the alive-chunk count per step for the roofline's byte count.  Leaves the
    timed workload's graphs replayed last (the kernel stamps read after come
    from those)."""
    e0 = pool.engines[0]
    res["decoder_steps_executed"] = int(out["steps"].cpu().item())
    rr = e0.translate_beam(sig, lens, lens, beam=args.beam, max_len=args.max_length, min_len=args.min_length,
                           return_attn=True)
    done = rr["done_step"].cpu().numpy()
    alive = [int((done > s_).sum()) for s_ in range(res["decoder_steps_executed"])]
    B = int(sig.shape[0])
    res["chunk_steps"] = {"executed_share": round(sum(alive) / (B * len(alive)), 4),
                          "done_step_percentiles_0_50_99_100": np.percentile(done, [0, 50, 99, 100]).tolist(),
                          "note": "finished chunks' attention workgroups and GEMM row tiles exit at once"}
    del rr
    n_wc = max(3, min(10, args.steps // 10))
    wcall = make_call(args, "beam", sig, lens, min_len=args.max_length)
    run_calls(pool, pool.lanes, wcall)
    wc, _ = timed(pool, n_wc, wcall, world)
    wc /= n_wc
    res["worst_case_all_steps"] = {"ms_per_step": round(wc * 1e3, 3),
                                   "samples_per_sec_per_gpu": round(float(B * 512) / wc, 1),
                                   "note": f"min_length {args.max_length}: no chunk finishes before step "
                                           f"{args.max_length}, {n_wc} calls, {pool.lanes} in flight"}
    run_calls(pool, pool.lanes, call)
    torch.cuda.synchronize()
    return alive


def run_batch(args, world, rank, dev, cfg, W):
    from nanodecoder_amd import synth
    from nanodecoder_amd.engine import EnginePool

    beam = args.beam if args.mode == "beam" else 1
    eng = EnginePool(cfg, W, device=dev.index, lanes=args.inflight, max_batch=args.batch, max_src_len=512,
                     max_steps=args.max_length, max_beam=beam, bank_nt_lanes=nt_lanes(args),
                     bank_grid=bank_grid(args))
    # each rank gets its own shard of synthetic reads
    sig_np = synth.synth_chunk_batch(args.batch, 512, seed=1000 + rank, inject_masks=False)
    lens_np = np.full(args.batch, 512, np.int32)
    sig = torch.from_numpy(sig_np).to(dev)
    lens = torch.from_numpy(lens_np).to(dev)
    call = make_call(args, args.mode, sig, lens)

    eng.set_kernel_stamps(not args.no_roofline)  # live launch timing of the roofline kernel (in the graphs)
    run_calls(eng, max(args.warmup, eng.lanes), call)  # every lane captures its graphs
    dt, outs = timed(eng, args.steps, call, world, every_lane=True)
    out = outs[(args.steps - 1) % eng.lanes]
    # bases = base tokens before the first EOS (outside the timed region)
    tok = out["tokens"].cpu().numpy()
    if args.mode == "beam":
        tok = tok[:, 0]
    bases_per_step = count_bases(tok, cfg.eos_idx)
    samples = float(lens_np.sum()) * args.steps * world
    value = samples / dt
    res = {
        "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": dtype_of(eng.engines[0].bank_form()),
        "data": "synthetic reads, random-init weights",
        "config": {"workload": workload(args), "chunks_per_gpu_per_step": args.batch,
                   "global_batch": args.batch * world, "seq_len": 512, "parallelism": f"read-shard x{world}",
                   "calls_in_flight_per_gpu": eng.lanes, "bank_nontemporal_lanes": list(eng.bank_nt_lanes),
                   "bank_kernel_workgroups": eng.bank_grid or "one per chunk"},
        "samples_per_sec_per_gpu": round(value / world, 1),
        "bases_per_sec": round(bases_per_step * args.steps * world / dt, 1),
        "timed_seconds": round(dt, 3),
        "min_length": args.min_length,
        "pool_check": pool_check(cfg, W, args, args.mode, args.batch, beam, call, outs),
    }
    roof_iso = None
    greedy_roof = rank == 0 and not args.no_roofline and args.mode == "greedy"
    if eng.lanes > 1:
        if greedy_roof:
            # the roofline kernel's launches inside the timed region, sharing the GPU with the other lanes
            res["roofline_pooled"] = kernel_roofline(eng, args.batch, args.mode, beam, args.encoder, secondary=False)
            res["roofline_pooled"]["timing"] = ("in-kernel wall-clock stamps, launches of the last timed call of "
                                                "every lane (the other lanes' kernels run beside them)")
        # the same calls one at a time (lane 0 only, each joined before the next): per-call latency
        one = eng.subset(1)
        # a lone call has every CU: the bank kernel at one workgroup per chunk (nd_set_bank_grid)
        eng.engines[0].set_bank_grid(0)
        eng.engines[0].set_gemm_splitk(False)  # and the long-K products one workgroup per tile
        n1 = max(3, min(40, args.steps // 4))
        run_calls(one, 2, call)
        dt1, _ = timed(one, n1, call, world)
        res["one_call_in_flight"] = {"value": round(float(lens_np.sum()) * n1 * world / dt1, 1),
                                     "ms_per_step": round(dt1 / n1 * 1e3, 3), "steps": n1,
                                     "note": "the same calls with one call on the device at a time: the latency "
                                             "of one 256-chunk call"}
        if greedy_roof:
            # the kernel with the GPU to itself (as rocprof's serialised kernel trace times it)
            roof_iso = kernel_roofline(one, args.batch, args.mode, beam, args.encoder)
            roof_iso["timing"] = ("in-kernel wall-clock stamps, launches of the last call of the timed "
                                  "one-call-in-flight leg (the kernel alone on the GPU, one workgroup per chunk)")
        eng.engines[0].set_bank_grid(eng.bank_grid)
        eng.engines[0].set_gemm_splitk(eng.splitk)
    alive = None
    if args.mode == "beam":
        alive = beam_steps_and_worst_case(args, eng, sig, lens, call, out, world, res)
    extras = {}
    if rank == 0:
        if roof_iso is not None:
            extras["roofline"] = roof_iso
        elif not args.no_roofline:
            extras["roofline"] = kernel_roofline(eng, args.batch, args.mode, beam, args.encoder, alive)
        eng.set_kernel_stamps(False)
        mv = None if args.no_roofline else mfma_view(args, eng, sig, lens, dt / args.steps * 1e3)
        if mv is not None:
            extras["mfma"] = mv
    if args.exact:
        # the same workload with exact fp32 products (nd_set_exact_fp32)
        eng.set_exact_fp32(True)
        n_ex = max(5, min(40, args.steps // 4))
        run_calls(eng, max(2, eng.lanes), call)
        dte, _ = timed(eng, n_ex, call, world)
        eng.set_exact_fp32(False)
        extras["exact_fp32"] = {"value_per_gpu": round(float(lens_np.sum()) * n_ex / dte, 1), "unit": "samples/s",
                                "ms_per_step": round(dte / n_ex * 1e3, 3), "steps": n_ex,
                                "note": "every GEMM, the encoder attention and the BiLSTM on fp32 MFMAs"}
        if args.mode == "greedy":
            enc_flop = ENC_FLOP_PER_CHUNK if args.encoder == "transformer" else NANO_ENC_FLOP_PER_CHUNK
            etf = (enc_flop + DEC_FLOP_PER_CHUNK) * args.batch / (dte / n_ex) / 1e12
            extras["exact_fp32"]["roofline"] = {
                "bound": "mfma", "achieved": round(etf, 2), "peak": FP32_PEAK, "unit": "TFLOP/s",
                "frac": round(etf / FP32_PEAK, 4),
                "note": "path-level algorithmic FLOPs (SURVEY §8d) per call over the call time, against the dense "
                        "fp32 MFMA peak (the pipe this leg runs on)"}
    if args.host_inclusive and args.mode == "greedy":
        extras["host_inclusive"] = host_inclusive(args, cfg, eng, sig_np, lens_np)
        extras["host_inclusive"]["ratio_to_value"] = round(extras["host_inclusive"]["value_per_gpu"] /
                                                           (value / world), 4)
    res.update(extras)
    return res, eng, sig_np, lens_np


def config_legs(args, world, rank, dev):
    """BASELINE configs[2] and configs[3] in the same run as the headline
    (fewer calls each): the NanoEncoder model greedy at batch 256, and --fast
    beam 5 at batch 1024 (random-init weights, -min_length as the headline)."""
    from nanodecoder_amd import synth
    from nanodecoder_amd.engine import EnginePool
    legs = {}
    n = max(3, args.steps // 4)
    for key, enc, mode, B in (("configs[2]", "nano", "greedy", 256), ("configs[3]", "transformer", "beam", 1024)):
        cfg = synth.ModelConfig(encoder_type=enc)
        W = synth.make_weights(cfg, seed=11, eos_bias=args.eos_bias)
        beam = args.beam if mode == "beam" else 1
        pool = EnginePool(cfg, W, device=dev.index, lanes=args.inflight, max_batch=B, max_src_len=512,
                          max_steps=args.max_length, max_beam=beam, bank_nt_lanes=nt_lanes(args))
        sig = torch.from_numpy(synth.synth_chunk_batch(B, 512, seed=2000 + rank, inject_masks=False)).to(dev)
        lens = torch.full((B,), 512, dtype=torch.int32, device=dev)
        call = make_call(args, mode, sig, lens)
        pool.set_kernel_stamps(mode == "beam" and not args.no_roofline)
        run_calls(pool, max(2, pool.lanes), call)
        dt, outs = timed(pool, n, call, world, every_lane=True)
        out = outs[(n - 1) % pool.lanes]
        tok = out["tokens"].cpu().numpy()
        tok = tok[:, 0] if mode == "beam" else tok
        legs[key] = {"workload": f"{'NanoEncoder (3x BiLSTM)' if enc == 'nano' else '3-layer transformer'} encoder "
                                 f"+ 3-layer transformer decoder, d_model 256, src_seq_length 512, batch {B}, "
                                 f"{'greedy' if mode == 'greedy' else f'--fast beam {beam}'}, max_length "
                                 f"{args.max_length}",
                     "value": round(B * 512 * n * world / dt, 1), "unit": "samples/s", "n_gpus": world,
                     "samples_per_sec_per_gpu": round(B * 512 * n / dt, 1),
                     "bases_per_sec": round(count_bases(tok, cfg.eos_idx) * n * world / dt, 1),
                     "ms_per_step": round(dt / n * 1e3, 3), "steps": n, "calls_in_flight_per_gpu": pool.lanes,
                     "dtype": dtype_of(pool.engines[0].bank_form())}
        legs[key]["pool_check"] = pool_check(cfg, W, args, mode, B, beam, call, outs)
        if mode == "beam":
            bargs = argparse.Namespace(**vars(args))
            bargs.steps = n
            alive = beam_steps_and_worst_case(bargs, pool, sig, lens, call, out, world, legs[key])
            if rank == 0 and not args.no_roofline:
                legs[key]["roofline"] = kernel_roofline(pool, B, "beam", beam, "transformer", alive)
                legs[key]["roofline"]["timing"] = ("in-kernel wall-clock stamps, launches of the last call of "
                                                   "the leg's workload (other lanes' calls beside it)")
            pool.set_kernel_stamps(False)
        pool.close()
        del pool, sig, lens
        torch.cuda.empty_cache()
    return legs


def host_inclusive(args, cfg, eng, sig_np, lens_np):
    """The same batches through the Translator drop-in: float32 chunks on the
    host -> pinned staging -> H2D -> engine -> tokens D2H -> strings, with one
    batch in flight while the next is packed (Translator.stream_reads)."""
    import types
    from nanodecoder_amd.translator import Translator
    opt = types.SimpleNamespace(gpu=eng.device.index, n_best=1, max_length=args.max_length,
                                min_length=args.min_length, beam_size=1, batch_size=args.batch,
                                engine_max_batch=args.batch)
    tr = Translator(cfg, None, opt, engine=eng)
    # 40 batches whatever --steps is: with 3 calls in flight the first call's latency is paid once, and
    # at 5 batches (the driver's --steps 20 / 4) that fill alone is ~7 % of the leg
    n = 40
    # each "read" is one chunk here: batches are exactly the timed batch
    reads = [[sig_np[i % args.batch]] for i in range(args.batch * n)]
    list(tr.stream_reads(reads[: 2 * args.batch], batch_size=1))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = sum(1 for _ in tr.stream_reads(reads, batch_size=1))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value_per_gpu": round(done * 512 / dt, 1), "unit": "samples/s", "batches": n,
            "ms_per_batch": round(dt / n * 1e3, 3),
            "path": "Translator.stream_reads: host packing + pinned H2D + engine + token D2H + EOS cut"}


def run_reads(args, world, rank, dev, cfg, W, n_reads_per_gpu):
    """configs[4]: the synthetic read set (lengths U[256,1024], 1-2 chunks per
    read) sharded over the ranks by LPT on sample count; every rank packs its
    reads into full engine batches; the front end (median/MAD + windowing)
    runs on the device on each call's lane stream (ReadShard's default,
    Translator.stream_raw_reads); timed region = max over ranks
    (shard.run_distributed)."""
    import types
    from nanodecoder_amd import shard
    from nanodecoder_amd.engine import EnginePool
    from nanodecoder_amd.translator import Translator

    def translator_factory(Wr):
        opt = types.SimpleNamespace(gpu=dev.index, n_best=1, max_length=args.max_length, min_length=args.min_length,
                                    beam_size=1, batch_size=100, engine_max_batch=args.batch)
        eng = EnginePool(cfg, Wr, device=dev.index, lanes=args.inflight, max_batch=args.batch, max_src_len=512,
                         max_steps=args.max_length)
        return Translator(cfg, Wr, opt, engine=eng)

    g, _ = shard.run_distributed(n_reads_per_gpu * world, translator_factory, lambda: W, dev, batch_size=100,
                                 pregenerate=True, warmup_reads=min(2048, n_reads_per_gpu))
    return {"value": round(g["samples"] / g["seconds"], 1), "unit": "samples/s", "n_gpus": world,
            "chunk_slots_per_sec": round(g["chunks"] * 512 / g["seconds"], 1),
            "chunk_fill": round(g["samples"] / max(1, g["chunks"] * 512), 4),
            "note": ("value counts the reads' samples; a read's last chunk is partial (lengths U[256,1024]) and the "
                     "reference pads it to its batch's longest chunk, so the engine computes chunk_slots_per_sec "
                     "512-sample slots per second (the headline's unit)"),
            "samples_per_sec_per_gpu": round(g["samples"] / g["seconds"] / world, 1),
            "bases_per_sec": round(g["bases"] / g["seconds"], 1), "reads": g["reads"], "chunks": g["chunks"],
            "seconds": round(g["seconds"], 3), "samples_per_rank": g["samples_per_rank"],
            "load_imbalance_max_over_mean": round(g["load_imbalance"], 4),
            "scaling": "weak" if args.workload == "batch" else "weak (reads per GPU fixed)",
            "frontend": g.get("frontend"),
            "process_group": (f"{torch.distributed.get_backend()} x{torch.distributed.get_world_size()}: weights "
                              f"broadcast from HIP memory, flags / counters on a gloo group"
                              if torch.distributed.is_initialized() else None),
            "workload": (f"configs[4]: {n_reads_per_gpu} synthetic reads per GPU, lengths U[256,1024], LPT shard, "
                         f"engine batch {args.batch}, reference batch_size 100, greedy, max_length "
                         f"{args.max_length}; raw reads handed to the translator, median/MAD + windowing on the "
                         f"device per engine batch (nd_normalize_reads / nd_window_reads on the call's lane "
                         f"stream), raw traces pre-generated (stand-in for the files read)")}


def selftest_cpu(args):
    """Launcher plumbing on CPU: every rank joins a gloo group, rank 0 prints
    the line with the world size it saw (no engine, no measurement)."""
    world, rank, _ = dist_setup(args)
    t = torch.tensor([float(rank)])
    if world > 1:
        torch.distributed.all_reduce(t)
    if rank == 0:
        print(json.dumps({"selftest": True, "n_gpus": world, "rank_sum": float(t.item())}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    if args.selftest_cpu:
        return selftest_cpu(args)
    world, rank, local = dist_setup(args)
    # the library's A/B switches (ND_* environment variables) change the kernel
    # mix; a headline is only printed with all of them at their defaults
    from nanodecoder_amd import _lib
    switches = _lib.switches()
    if switches and not args.allow_switches:
        raise SystemExit(f"non-default ND_* switches set: {switches} (unset them, or pass --allow-switches for a "
                         f"non-headline line)")
    # rehearsal of the multi-rank flow on a one-GPU box: every rank on GPU 0
    # over gloo (RCCL refuses two ranks on one device); the line says so
    share = os.environ.get("ND_BENCH_SHARE_GPU") == "1"
    if share and args.backend != "gloo":
        raise SystemExit("ND_BENCH_SHARE_GPU=1 needs --backend gloo")
    dev = torch.device("cuda", 0 if share else local)
    torch.cuda.set_device(dev)
    from nanodecoder_amd import synth

    cfg = synth.ModelConfig(encoder_type=args.encoder)
    # rank 0 owns the weights; one RCCL broadcast of the packed blob reaches the others
    W = synth.make_weights(cfg, seed=11, eos_bias=args.eos_bias) if rank == 0 else None
    if world > 1:
        from nanodecoder_amd.shard import broadcast_weights
        W = broadcast_weights(W, dev)

    if args.workload == "reads":
        rs = run_reads(args, world, rank, dev, cfg, W, args.reads)
        res = {"metric": METRIC, "value": rs["value"], "unit": "samples/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": dtype_of(2),
               "data": "synthetic reads, random-init weights",
               "config": {"workload": workload(args), "seq_len": 512, "parallelism": f"read-shard x{world}"},
               "read_shard": rs}
        if share:
            res["rehearsal"] = f"{world} ranks sharing GPU 0 over gloo (plumbing check, not a measurement)"
        if rank == 0:
            print(json.dumps(res), flush=True)
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()
        return

    res, eng, sig_np, lens_np = run_batch(args, world, rank, dev, cfg, W)
    if args.config_legs and args.mode == "greedy" and args.encoder == "transformer" and args.batch == 256:
        res["config_legs"] = config_legs(args, world, rank, dev)
    if args.read_shard and args.mode == "greedy" and args.encoder == "transformer":
        eng.close()  # the read-shard engine replaces it
        res["read_shard"] = run_reads(args, world, rank, dev, cfg, W, max(1024, args.reads // 4))
    if share:
        res["rehearsal"] = f"{world} ranks sharing GPU 0 over gloo (plumbing check, not a measurement)"
    res["switches"] = switches
    if switches:
        res["headline"] = False
    if rank == 0:
        if args.cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(cfg, W, sig_np, lens_np, args)
        print(json.dumps(res), flush=True)
    eng.close()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
