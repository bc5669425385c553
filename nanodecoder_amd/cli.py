"""translate.py driver (reference translate.py:59-187) on the MI355X engine.

Same inputs, outputs and resume rule: every ``*.signal`` / ``*.fast5`` in
``-src_dir`` whose ``result/<read>.fasta`` does not exist yet is normalised
and windowed in a worker pool (translate.py:131-163), translated, and written
as result/<read>.fasta, segment/<read>.txt and a line of speed.txt
(translate.py:81-98).  One bad read prints ``!!!error!!!`` and the run goes
on (translate.py:97-98).  ``-pack_reads N`` translates N reads per engine pass.
"""
from __future__ import annotations

import logging
import multiprocessing
import codecs
import os
import sys
import time

from . import frontend
from .opts import parse_translate_opts


def init_logger(log_file=None):
    """onmt/utils/logging.py:9-24."""
    fmt = logging.Formatter("[%(asctime)s %(levelname)s] %(message)s")
    logger = logging.getLogger()
    logger.setLevel(logging.INFO)
    h = logging.StreamHandler()
    h.setFormatter(fmt)
    logger.handlers = [h]
    if log_file:
        fh = logging.FileHandler(log_file)
        fh.setFormatter(fmt)
        logger.addHandler(fh)
    return logger


def list_reads(opt):
    """translate.py:134-163: pending reads (resume = skip existing fasta)."""
    todo, done = [], 0
    for name in sorted(os.listdir(opt.src_dir)):
        if name.endswith("fast5"):
            prefix, suffix = name.split(".fast5")[0] + ".txt", "fast5"
        elif name.endswith("signal"):
            prefix, suffix = name.split(".signal")[0] + ".txt", "signal"
        else:
            continue
        if os.path.exists(os.path.join(opt.save_data, "result", prefix.split(".txt")[0] + ".fasta")):
            done += 1
        else:
            todo.append((os.path.join(opt.src_dir, name), prefix, suffix))
    return todo, done


def _read_only(args):
    """-frontend gpu: the worker only reads the raw samples.  An empty read
    yields [prefix] alone and is skipped like the reference's
    (translate.py:102-103)."""
    path, prefix, suffix, norm, length, stride = args
    try:
        raw = frontend.read_raw(path, suffix)
        return [prefix, raw] if len(raw) else [prefix]
    except Exception:
        return ["!" + prefix]


def _gpu_chunks(opt, group):
    """[prefix, raw] reads -> [prefix, chunk, ...] with the device front end,
    on the translator's GPU (-gpu)."""
    sig, lens, rd = frontend.normalize_window_gpu([g[1] for g in group], opt.normalization_raw,
                                                  opt.src_seq_length, opt.src_seq_stride, device=max(0, opt.gpu))
    host = sig.cpu().numpy()
    out = [[g[0]] for g in group]
    for c in range(len(rd)):
        out[rd[c]].append(host[c, : lens[c]].copy())
    return out


def _n_chunks(opt, src, gpu_fe):
    """Chunks a pending read will contribute (for -pack_reads 0)."""
    if not gpu_fe:
        return len(src) - 1
    return len(frontend.windows(len(src[1]), opt.src_seq_length, opt.src_seq_stride))


def _run_group(opt, translator, pending, gpu_fe):
    """Front end (device) + translate for one packed group, with the
    per-group error isolation of translate.py:97-98.  -frontend gpu: the raw
    reads go to the translator, which normalises and windows every engine
    batch on the device right before its call (stream_raw_reads); with
    -attn_debug (its file needs each chunk's samples on the host) the chunks
    come back to the host first."""
    if gpu_fe and not opt.attn_debug:
        return _translate_group(opt, translator, pending, raw=True)
    if gpu_fe:
        try:
            pending = _gpu_chunks(opt, pending)
        except Exception as e:
            for g in pending:
                print("!!!error!!!data src: " + g[0].split(".txt")[0] + " (%r)" % (e,))
            return 0
    return _translate_group(opt, translator, pending)


def _extract(args):
    path, prefix, suffix, norm, length, stride = args
    try:
        return frontend.extract_raw(path, prefix, norm, length, stride, suffix)
    except Exception as e:  # surfaced per read, like the Pool error path
        return ["!" + prefix, repr(e)]


def write_output(opt, file_src, all_predictions, time_translate):
    """translate.py:81-98."""
    try:
        c_bpread = frontend.assemble_read(all_predictions, opt.src_seq_length, opt.src_seq_stride)
        name = file_src.split(".txt")[0]
        with open(os.path.join(opt.save_data, "result", name + ".fasta"), "w") as f:
            f.writelines(">%s\n%s" % (name, c_bpread))
        with open(os.path.join(opt.save_data, "segment", file_src), "w+") as f:
            for n_best_preds in all_predictions:
                f.write("\n".join(n_best_preds) + "\n")
        with open(os.path.join(opt.save_data, "speed.txt"), "a+") as f:
            f.writelines("%s\t%0.2f\t%d\t%0.2f\n" % (name, float(time_translate), len(c_bpread),
                                                     len(c_bpread) / max(float(time_translate), 1e-9)))
    except Exception:
        print("!!!error!!!data src: " + file_src.split(".txt")[0])


def main(opt=None):
    opt = opt or parse_translate_opts()
    logger = init_logger(opt.log_file)
    for sub in ("", "result", "segment") + (("attention",) if opt.attn_debug else ()):  # translate.py:64-71
        os.makedirs(os.path.join(opt.save_data, sub), exist_ok=True)
    from .translator import build_translator
    translator = build_translator(opt, report_score=False, logger=logger)
    todo, done = list_reads(opt)
    logger.info("%d reads have already translated, remains %d read\n" % (done, len(todo)))
    jobs = [(p, pre, suf, opt.normalization_raw, opt.src_seq_length, opt.src_seq_stride) for p, pre, suf in todo]
    ctx = multiprocessing.get_context("spawn")
    t_start = time.time()
    n_done = 0
    gpu_fe = getattr(opt, "frontend", "cpu") == "gpu"
    # -pack_reads 0: flush once the pending reads fill the engine batch
    cap = int(getattr(translator, "max_batch", 0) or 256)
    with ctx.Pool(max(1, opt.thread)) as pool:
        pending, n_chunks = [], 0
        for src in pool.imap(_read_only if gpu_fe else _extract, jobs):
            if src and src[0].startswith("!"):
                print("!!!error!!!data src: " + src[0][1:].split(".txt")[0])
                continue
            if not src or len(src) == 1:   # translate.py:102-103
                continue
            pending.append(src)
            n_chunks += _n_chunks(opt, src, gpu_fe)
            full = len(pending) >= opt.pack_reads if opt.pack_reads > 0 else n_chunks >= cap
            if full:
                n_done += _run_group(opt, translator, pending, gpu_fe)
                pending, n_chunks = [], 0
        if pending:
            n_done += _run_group(opt, translator, pending, gpu_fe)
    logger.info("translated %d reads in %.1f s" % (n_done, time.time() - t_start))
    return n_done


def _translate_attn(opt, translator, group):
    """-attn_debug (translate.py:110-120): read by read, each into its own
    save_data/attention/<read> file (appended)."""
    outs = []
    for g in group:
        with codecs.open(os.path.join(opt.save_data, "attention", g[0]), "a+", "utf-8") as f:
            translator.setAttnFile(f)
            outs.append(translator.translate(src=list(g[1:]), batch_size=opt.batch_size, attn_debug=True))
    return outs


def _translate_group(opt, translator, group, raw=False):
    t0 = time.time()
    try:
        if opt.attn_debug:
            outs = _translate_attn(opt, translator, group)
        elif raw:  # [prefix, raw samples]: the front end runs on the device
            outs = translator.translate_raw_reads([g[1] for g in group], batch_size=opt.batch_size,
                                                  normalization=opt.normalization_raw,
                                                  src_seq_length=opt.src_seq_length,
                                                  src_seq_stride=opt.src_seq_stride)
        else:
            outs = translator.translate_reads([g[1:] for g in group], batch_size=opt.batch_size)
    except Exception as e:
        for g in group:
            print("!!!error!!!data src: " + g[0].split(".txt")[0] + " (%r)" % (e,))
        return 0
    dt = time.time() - t0
    total = max(1, sum(len(preds) for _, preds in outs))
    for g, (_, preds) in zip(group, outs):
        write_output(opt, g[0], preds, dt * len(preds) / total)
    return len(group)


if __name__ == "__main__":
    sys.exit(0 if main() is not None else 1)
