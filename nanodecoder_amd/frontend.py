"""Signal front end and output assembly around the translate path.

Host-side restatement of utils/labelop.py: the
median/MAD normalisation + windowing that produces 512-sample chunks
(extract_fast5_raw, :194-243) and the overlap consensus that joins per-chunk
base strings back into a read (simple_assembly / index2base, :295-352).
Chunks stay float32 arrays end to end — the reference's float -> str -> float
round trip (:231, inputters/nano_dataset.py:52-58) is value-preserving, so it
is skipped.
"""
from __future__ import annotations

import difflib
import math
from typing import List

import numpy as np

from .synth import MAD_SCALE

BASE_KEYS = ["A", "C", "G", "T", "M"]                       # utils/labelop.py:17
BASE_DICT = {"A": 0, "C": 1, "G": 2, "T": 3, "M": 4}        # utils/labelop.py:18


def read_raw(path: str, suffix: str) -> np.ndarray:
    if suffix == "fast5":
        try:
            import h5py  # noqa: F401
        except ImportError as e:  # pragma: no cover - h5py absent in this image
            raise IOError("fast5 input needs h5py, which is not installed; convert reads to .signal text") from e
        import h5py
        with h5py.File(path, "r") as f:
            raw = list(f["/Raw/Reads/"].values())[0]["Signal"][()]
        return np.asarray(raw, dtype=np.float64)
    with open(path) as f:
        return np.asarray(f.read().strip().split(), dtype=np.float64)


def normalize(raw: np.ndarray, normalization: str) -> np.ndarray:
    """utils/labelop.py:220-223 ('mean' divides by std but still centres on
    the median, exactly as the reference does)."""
    raw = np.asarray(raw, dtype=np.float64)
    if normalization == "mean":
        return (raw - np.median(raw)) / float(np.std(raw))
    if normalization == "median":
        med = np.median(raw)
        return (raw - med) / float(np.median(np.abs(raw - med) / MAD_SCALE))
    return raw


def window(sig: np.ndarray, max_length: int, stride: int) -> List[np.ndarray]:
    """utils/labelop.py:225-233."""
    out = []
    for i in range(0, math.ceil(sig.size / stride)):
        s = i * stride
        e = min(s + max_length, len(sig))
        out.append(np.asarray(sig[s:e], dtype=np.float32))
        if e >= len(sig):
            break
    return out


def extract_raw(input_file_path: str, output_prefix: str, normalization: str, max_length: int,
                signal_stride: int, suffix: str):
    """extract_fast5_raw (utils/labelop.py:194-243): [prefix, chunk, ...]."""
    try:
        raw = read_raw(input_file_path, suffix)
        return [output_prefix] + window(normalize(raw, normalization), max_length, signal_stride)
    except Exception as e:
        raise RuntimeError("Raw data is not stored in Raw/Reads/Read_[read#] so new segments cannot be "
                           "identified.") from e


NORM_METHOD = {"none": 0, "None": 0, "median": 1, "mean": 2}


def windows(n: int, max_length: int, stride: int):
    """(start, length) of each chunk window() cuts from an n-sample read
    (utils/labelop.py:225-233)."""
    out = []
    for i in range(0, math.ceil(n / stride)):
        st = i * stride
        e = min(st + max_length, n)
        out.append((st, e - st))
        if e >= n:
            break
    return out


def _pinned(a: np.ndarray):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory()


def device_batch(raws, rd, start, length, normalization: str, B: int, T: int, device):
    """The device front end for one engine batch (nd_normalize_reads +
    nd_window_reads, frontend.hip) on the CURRENT stream: the reads ``raws``
    (float64 arrays) are copied to the device once (pinned, asynchronous),
    normalised in fp64 (median/MAD, median/std or none as
    utils/labelop.py:220-223) and cut into chunk rows c = samples
    [start[c], start[c] + length[c]) of read rd[c] (index into ``raws``), zero
    padded, in a [B, T] float32 batch (rows >= len(rd) zero).  Returns
    (signal [B, T], the device tensors to keep alive until the stream has
    used them)."""
    import ctypes

    import torch

    from . import _lib
    method = NORM_METHOD.get(normalization, 0)  # anything else: the raw read, as labelop.py:220-223
    lens = np.fromiter((r.size for r in raws), np.int64, len(raws))
    if (lens < 1).any():
        raise ValueError("empty read")
    off = np.zeros(len(raws) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    C = len(rd)
    if C > B or (C and int(np.max(length)) > T):
        raise ValueError("chunk descriptors exceed the batch")
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    idx = np.zeros((len(off) * 2 + 3 * C + 1) // 2 * 2, np.int32)  # one pinned block of every index array
    idx.view(np.int64)[: len(off)] = off
    idx[2 * len(off): 2 * len(off) + 3 * C] = np.concatenate([np.asarray(rd, np.int32), np.asarray(start, np.int32),
                                         np.asarray(length, np.int32)])
    raw_d = _pinned(np.concatenate(raws) if len(raws) > 1 else raws[0]).to(dev, non_blocking=True)
    idx_d = _pinned(idx).to(dev, non_blocking=True)
    off_d = idx_d[: 2 * len(off)].view(torch.int64)
    rd_d = idx_d[2 * len(off): 2 * len(off) + C]
    st_d = idx_d[2 * len(off) + C: 2 * len(off) + 2 * C]
    ln_d = idx_d[2 * len(off) + 2 * C: 2 * len(off) + 3 * C]
    norm_d = torch.empty(int(off[-1]), dtype=torch.float32, device=dev)
    sig = torch.zeros(B, T, dtype=torch.float32, device=dev)
    L = _lib.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(L.nd_normalize_reads(p(raw_d), p(off_d), len(raws), method, p(norm_d), stream), "nd_normalize_reads")
    _lib.check(L.nd_window_reads(p(norm_d), p(off_d), p(rd_d), p(st_d), p(ln_d), C, T, p(sig), stream),
               "nd_window_reads")
    return sig, (raw_d, idx_d, norm_d)


def normalize_window_gpu(raws, normalization: str, max_length: int, stride: int, device=0, T: int = None):
    """extract_fast5_raw's normalisation and windowing for many reads on the
    GPU (device_batch over every window of every read).  Returns (signal
    [C, T] device tensor, chunk lengths [C] int32, chunk -> read index [C]
    int32)."""
    raws = [np.asarray(r, dtype=np.float64).reshape(-1) for r in raws]
    rd, st, ln = [], [], []
    for r, x in enumerate(raws):
        for a, b in windows(int(x.size), max_length, stride):
            rd.append(r)
            st.append(a)
            ln.append(b)
    sig, _ = device_batch(raws, rd, st, ln, normalization, len(rd), T or max_length, device)
    return sig, np.array(ln, np.int32), np.array(rd, np.int32)


def index2base(read) -> str:
    """utils/labelop.py:295-307."""
    return "".join(BASE_KEYS[x] for x in read)


def _add_count(consensus, start, segment):
    """utils/labelop.py:310-317."""
    if start < 0:
        segment = segment[-start:]
        start = 0
    for i, base in enumerate(segment):
        consensus[BASE_DICT[base.upper()]][start + i] += 1


def simple_assembly(bpreads, flag_intersection: bool = True):
    """utils/labelop.py:320-352.  ``bpreads`` = all_predictions (lists of
    n_best space-separated strings); with flag_intersection the consecutive
    chunks are aligned by their longest difflib matching block and voted."""
    valid = [x[0].replace(" ", "") for x in bpreads if x[0] != ""]
    if not flag_intersection:
        return "".join(valid)
    consensus = np.zeros([len(BASE_KEYS), 1000])
    pos = 0
    length = 0
    census_len = 1000
    for indx, bpread in enumerate(valid):
        if indx == 0:
            _add_count(consensus, 0, bpread)
            continue
        d = difflib.SequenceMatcher(None, valid[indx - 1], bpread)
        match_block = max(d.get_matching_blocks(), key=lambda x: x[2])
        disp = match_block[0] - match_block[1]
        if disp + pos + len(valid[indx]) > census_len:
            consensus = np.pad(consensus, ((0, 0), (0, 1000)), mode="constant", constant_values=0)
            census_len += 1000
        _add_count(consensus, pos + disp, valid[indx])
        pos += disp
        length = max(length, pos + len(valid[indx]))
    return consensus[:, :length]


def assemble_read(all_predictions, src_seq_length: int, src_seq_stride: int) -> str:
    """translate.py:84-87."""
    if src_seq_stride < src_seq_length:
        return index2base(np.argmax(simple_assembly(all_predictions), axis=0))
    return simple_assembly(all_predictions, flag_intersection=False)
