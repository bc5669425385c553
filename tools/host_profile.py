"""Host-side profile of the host-inclusive leg (not part of the engine): the bench's configs[1] batches through
Translator.stream_reads on a 3-lane EnginePool, once plain (ms per batch) and once under cProfile (where the
host thread's time goes).   python tools/host_profile.py"""
import cProfile
import pstats
import sys
import time
import types

import torch

sys.path.insert(0, ".")
from nanodecoder_amd import synth  # noqa: E402
from nanodecoder_amd.engine import EnginePool  # noqa: E402
from nanodecoder_amd.translator import Translator  # noqa: E402


def main():
    B, n = 256, 40
    cfg = synth.ModelConfig(encoder_type="transformer")
    W = synth.make_weights(cfg, seed=11, eos_bias=-3.0)
    pool = EnginePool(cfg, W, device=0, lanes=3, max_batch=B, max_src_len=512, max_steps=100)
    opt = types.SimpleNamespace(gpu=0, n_best=1, max_length=100, min_length=57, beam_size=1, batch_size=B,
                                engine_max_batch=B)
    tr = Translator(cfg, None, opt, engine=pool)
    sig = synth.synth_chunk_batch(B, 512, seed=1000, inject_masks=False)
    reads = [[sig[i % B]] for i in range(B * n)]
    list(tr.stream_reads(reads[: 2 * B], batch_size=1))
    torch.cuda.synchronize()
    for rep in range(2):
        t0 = time.perf_counter()
        sum(1 for _ in tr.stream_reads(reads, batch_size=1))
        torch.cuda.synchronize()
        print(f"stream_reads: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per batch", flush=True)
    # the device alone: the same batches as back-to-back engine calls (3 in flight), results left on the device
    sig_d = torch.from_numpy(sig).cuda()
    lens = torch.full((B,), 512, dtype=torch.int32, device="cuda")
    t0 = time.perf_counter()
    outs = [pool.translate_greedy(sig_d, lens, lens, max_len=100, min_len=57) for _ in range(n)]
    torch.cuda.synchronize()
    print(f"engine calls alone: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per batch", flush=True)
    del outs
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    sum(1 for _ in tr.stream_reads(reads, batch_size=1))
    torch.cuda.synchronize()
    pr.disable()
    print(f"under cProfile: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per batch")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
