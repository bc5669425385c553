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
