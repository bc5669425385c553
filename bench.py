#!/usr/bin/env python
"""Benchmark of the MI355X translate path (BASELINE.json metric).

A "step" = one full translate call (encoder + all decoder steps + search) on
one batch of synthetic 512-sample chunks already resident in HBM.  Default
workload = BASELINE.json configs[1]: 3+3 transformer, d_model 256, T 512,
batch 256 chunks per GPU, greedy, max_length 100, random-init weights of the
reference architecture (no trained checkpoint exists offline).

Multi-GPU (``torch.distributed.run``): reads shard across ranks with no
collective in the hot loop ("scaling": "weak" — every rank translates its own
batch); rank 0 loads/creates the weights and broadcasts them once over RCCL.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "signal-samples/sec/GPU (512-sample chunks) + bases/sec at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256, help="chunks per GPU per step")
    ap.add_argument("--mode", default="greedy", choices=["greedy", "beam"])
    ap.add_argument("--beam", type=int, default=5)
    ap.add_argument("--encoder", default="transformer", choices=["transformer", "nano"])
    ap.add_argument("--max-length", type=int, default=100)
    ap.add_argument("--min-length", type=int, default=57,
                    help="-min_length: EOS masked before this step.  The random-init model is EOS-prone, so this "
                         "sets its decode length to a trained basecaller's ~57 bases per 512 samples (greedy cost "
                         "is unaffected: all max_length steps always run)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 (0 = skip)")
    ap.add_argument("--cpu-chunks", type=int, default=0, help="CPU baseline sample size (0: 128 greedy / 24 beam)")
    ap.add_argument("--no-roofline", action="store_true")
    return ap.parse_args()


def workload(args):
    idx = 3 if args.mode == "beam" else (2 if args.encoder == "nano" else 1)
    enc = "3-layer transformer encoder" if args.encoder == "transformer" else "NanoEncoder (3x BiLSTM)"
    dec = "greedy" if args.mode == "greedy" else f"--fast beam {args.beam}"
    return (f"configs[{idx}]: {enc} + 3-layer transformer decoder, d_model 256, src_seq_length 512, "
            f"batch {args.batch}, {dec}, max_length {args.max_length}")


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def cpu_baseline(cfg, W, sig, lens, args):
    from oracle import ref_cpu
    n = min(args.cpu_chunks or (128 if args.mode == "greedy" else 24), sig.shape[0])
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    m = ref_cpu.RefModel(cfg, W)
    t0 = time.perf_counter()
    if args.mode == "greedy":
        ref_cpu.greedy(m, sig[:n], lens[:n], max_length=args.max_length, min_length=args.min_length)
    else:
        ref_cpu.fast_beam(m, sig[:n], lens[:n], beam_size=args.beam, max_length=args.max_length,
                          min_length=args.min_length)
    dt = time.perf_counter() - t0
    return {"value": float(lens[:n].sum() / dt), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ref_cpu.py {args.mode} on {n} chunks x 512 samples, max_length {args.max_length}, "
                      f"torch CPU fp32, {threads} threads, {dt:.1f} s"}


def _time(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def _pmc_traffic(name):
    """HBM bytes per launch for `name` from the committed PMC summary
    (profiles/pmc_summary.json, written by tools/pmc_summary.py from
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes with the gfx950 x2
    FETCH_SIZE correction), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            return json.load(f)["kernels"][name]["hbm_bytes_per_launch"]
    except Exception:
        return None


def kernel_roofline(eng, B, mode, beam, encoder="transformer"):
    """Dominant kernel of the translate step, timed LIVE: every launch of it
    inside the timed graph replays carries in-kernel wall-clock stamps
    (first workgroup start, last workgroup end; Engine.set_kernel_stamps), and
    the mean over the last timed call's launches is the launch duration.

    greedy: the memory-bank context attention (dec_mem_attention_kernel),
      bounded by HBM: per launch it streams the B x 512 x 256 f32 memory bank
      once (+ q' in, U out, the signal for the key mask).  Its MFMA view
      (2 products x 2 x 8 heads x 512 keys x 256 dims per chunk, on
      v_mfma_f32_4x4x1_16b) is reported beside it.
    beam: the per-layer K/V context attention (dec_ctx_attention_kernel),
      HBM-bound: K+V 2 x 512 keys x 256 f32 per chunk + q, signal, out."""
    us, n = eng.kernel_stamps()
    T, D = 512, 256
    ms = us * 1e-3
    if mode == "greedy":
        name = "dec_mem_attention_kernel<0, 8>"
        nbytes = B * T * D * 4 + B * T * 4 + 2 * B * 8 * D * 4
        flops = 2 * 2 * 8 * T * D * B
        tf = flops / (ms * 1e-3) / 1e12
        extra = {"mfma_view": {"algorithmic_flops_per_launch": flops, "achieved": round(tf, 2), "peak": 157.3,
                               "unit": "TFLOP/s", "frac": round(tf / 157.3, 4)}}
    else:
        name = f"dec_ctx_attention_kernel<{beam}>"
        nbytes = B * T * 2 * D * 4 + B * T * 4 + 2 * B * beam * D * 4
        extra = {}
    ach = nbytes / (ms * 1e-3) / 1e9
    out = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1), "peak": 8000.0, "unit": "GB/s",
           "frac": round(ach / 8000.0, 4), "traffic": _pmc_traffic(name), "algorithmic_bytes_per_launch": nbytes,
           "avg_launch_ms": round(ms, 5), "timed_launches": n,
           "timing": "in-kernel wall-clock stamps, launches of the last timed call"}
    out.update(extra)
    dev = eng.device
    if encoder == "nano":
        out["lstm_kernel"] = lstm_view(dev, B, T)
        return out
    import ctypes
    from nanodecoder_amd import _lib
    from nanodecoder_amd.engine import op_fold_layernorm, op_split_weight
    # secondary: the dominant encoder MFMA kernel (FFN1 GEMM, LN prologue + bias
    # + ReLU) in the split-fp16 form the engine runs: 3 fp16 MFMA products per
    # fp32 multiply-add, so its fp32-equivalent peak is the dense fp16 peak / 3
    M, K, N = B * T, 256, 2048
    A = torch.randn(M, K, device=dev)
    Wt = torch.randn(N, K, device=dev) / 16
    b = torch.randn(N, device=dev)
    Wf, bf = op_fold_layernorm(Wt, b, torch.ones(K, device=dev), torch.zeros(K, device=dev))  # as at load time
    Wh, sc = op_split_weight(Wf)
    C = torch.empty(M, N, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def ffn1(i):
        _lib.check(_lib.lib().nd_op_gemm_split(A.data_ptr(), Wh.data_ptr(), sc, bf.data_ptr(), None, C.data_ptr(),
                                               M, N, K, 1, 1, st), "nd_op_gemm_split")
    for i in range(3):
        ffn1(i)
    gms = _time(ffn1, 10)
    tf = 2.0 * M * N * K / (gms * 1e-3) / 1e12
    peak = 2516.6 / 3
    out["mfma_kernel"] = {"kernel": "gemm_f32_kernel<256,256,2,4,H3,LN,RELU> (encoder FFN1, split-fp16)",
                          "achieved": round(tf, 2), "peak": round(peak, 1),
                          "unit": "TFLOP/s fp32-equivalent (fp16 MFMA peak / 3 products)",
                          "frac": round(tf / peak, 4), "avg_launch_ms": round(gms, 4)}
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
    ms = _time(layer, 5)
    flops = 2.0 * 2 * B * 512 * 128 * T
    tf = flops / (ms * 1e-3) / 1e12
    return {"kernel": "lstm_dir_kernel (BiLSTM layer, split-fp16)", "bound": "latency",
            "avg_launch_ms": round(ms, 4), "us_per_step": round(ms * 1e3 / T, 3),
            "achieved": round(tf, 2), "peak": round(2516.6 / 3, 1),
            "unit": "TFLOP/s fp32-equivalent (fp16 MFMA peak / 3 products)", "frac": round(tf / (2516.6 / 3), 4)}


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from nanodecoder_amd import synth
    from nanodecoder_amd.engine import Engine

    cfg = synth.ModelConfig(encoder_type=args.encoder)
    # rank 0 owns the weights; one RCCL broadcast of the packed blob reaches the others
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0) if rank == 0 else None
    if world > 1:
        from nanodecoder_amd.shard import broadcast_weights
        W = broadcast_weights(W, dev)
    beam = args.beam if args.mode == "beam" else 1
    eng = Engine(cfg, W, device=local, max_batch=args.batch, max_src_len=512, max_steps=args.max_length,
                 max_beam=beam)
    # each rank gets its own shard of synthetic reads
    sig_np = synth.synth_chunk_batch(args.batch, 512, seed=1000 + rank, inject_masks=False)
    lens_np = np.full(args.batch, 512, np.int32)
    sig = torch.from_numpy(sig_np).to(dev)
    lens = torch.from_numpy(lens_np).to(dev)

    def step():
        if args.mode == "greedy":
            return eng.translate_greedy(sig, lens, lens, max_len=args.max_length, min_len=args.min_length)
        return eng.translate_beam(sig, lens, lens, beam=args.beam, max_len=args.max_length,
                                  min_len=args.min_length)

    eng.set_kernel_stamps(not args.no_roofline)  # live launch timing of the roofline kernel (in the graphs)
    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bases = 0
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # bases = base tokens before the first EOS (outside the timed region)
    tok = out["tokens"].cpu().numpy()
    if args.mode == "beam":
        tok = tok[:, 0]
    eos = cfg.eos_idx
    is_eos = tok == eos
    first = np.where(is_eos.any(1), is_eos.argmax(1), tok.shape[1])
    base_mask = (np.arange(tok.shape[1])[None, :] < first[:, None]) & (tok >= 4)
    bases_per_step = int(base_mask.sum())
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    samples = float(lens_np.sum()) * args.steps * world
    value = samples / dt
    res = {
        "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic reads, random-init weights",
        "config": {"workload": workload(args), "chunks_per_gpu_per_step": args.batch,
                   "global_batch": args.batch * world, "seq_len": 512, "parallelism": f"read-shard x{world}"},
        "samples_per_sec_per_gpu": round(value / world, 1),
        "bases_per_sec": round(bases_per_step * args.steps * world / dt, 1),
        "min_length": args.min_length,
    }
    if args.mode == "beam":
        res["decoder_steps_executed"] = int(out["steps"].cpu().item())
    if rank == 0:
        if not args.no_roofline:
            res["roofline"] = kernel_roofline(eng, args.batch, args.mode, beam, args.encoder)
        if args.cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(cfg, W, sig_np, lens_np, args)
        print(json.dumps(res), flush=True)
    eng.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
