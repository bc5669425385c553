"""ctypes binding of libnanodec_hip.so (include/nanodec.h).

The library is loaded AFTER ``import torch`` so that its DT_NEEDED
``libamdhip64.so.7`` resolves to the HIP runtime PyTorch-ROCm already mapped
(same SONAME) — one HIP runtime per process, so torch device pointers and
streams are valid inside the engine.  There is no fallback: if the shared
library is missing or fails to load, every engine entry point raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NANODEC_LIB", os.path.join(HERE, "libnanodec_hip.so"))

ND_ENC_TRANSFORMER = 0
ND_ENC_NANO = 1
ND_SELF_SCALED_DOT = 0
ND_SELF_AVERAGE = 1
ND_ERR_ARG, ND_ERR_WEIGHT, ND_ERR_HIP, ND_ERR_STATE = 1, 2, 3, 4  # include/nanodec.h status codes

_CFG_FIELDS = ["encoder_type", "enc_layers", "dec_layers", "d_model", "heads", "d_ff", "vocab", "rnn_hidden",
               "position_encoding", "pad_idx", "bos_idx", "eos_idx", "max_batch", "max_src_len", "max_steps",
               "max_beam", "device", "self_attn_type"]


class NdConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in _CFG_FIELDS]


class NdClassicOpts(ctypes.Structure):
    """include/nanodec.h nd_classic_opts."""
    _fields_ = [("length_penalty", ctypes.c_int32), ("alpha", ctypes.c_float), ("beta", ctypes.c_float),
                ("coverage_penalty", ctypes.c_int32), ("stepwise_penalty", ctypes.c_int32),
                ("block_ngram_repeat", ctypes.c_int32), ("ignore_mask", ctypes.c_uint32)]


_P = ctypes.c_void_p
_I = ctypes.c_int32
_F = ctypes.c_float

# name -> (restype, argtypes); every symbol include/nanodec.h declares
SIGNATURES = {
    "nd_create": (_I, [ctypes.POINTER(NdConfig), ctypes.POINTER(_P)]),
    "nd_load_weight": (_I, [_P, ctypes.c_char_p, _P, ctypes.POINTER(ctypes.c_int64), _I]),
    "nd_finalize": (_I, [_P]),
    "nd_share_weights": (_I, [_P, _P]),
    "nd_translate_greedy": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "nd_translate_greedy_attn": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "nd_translate_sample": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _F, _I, ctypes.c_uint64, _P, _P, _P, _P, _P]),
    "nd_translate_beam": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _F, _I, _I, _P, _P, _P, _P, _P]),
    "nd_translate_beam_attn": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _F, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "nd_translate_beam_classic": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _F, _I, _I, _P, _P, _P, _P, _P]),
    "nd_translate_beam_classic_ex": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, ctypes.POINTER(NdClassicOpts), _I,
                                          _I, _P, _P, _P, _P, _P, _P]),
    "nd_normalize_reads": (_I, [_P, _P, _I, _I, _P, _P]),
    "nd_window_reads": (_I, [_P, _P, _P, _P, _P, _I, _I, _P, _P]),
    "nd_encode": (_I, [_P, _P, _P, _P, _I, _I, _P, _P]),
    "nd_set_graphs": (_I, [_P, _I]),
    "nd_set_timing": (_I, [_P, _I]),
    "nd_set_exact_fp32": (_I, [_P, _I]),
    "nd_set_bank_policy": (_I, [_P, _I]),
    "nd_set_bank_grid": (_I, [_P, _I]),
    "nd_set_gemm_splitk": (_I, [_P, _I]),
    "nd_take_overflow": (_I, [_P, _P, _P]),
    "nd_set_ctx_path": (_I, [_P, _I]),
    "nd_last_timing": (_I, [_P, ctypes.POINTER(_F), ctypes.POINTER(_F)]),
    "nd_set_kernel_stamps": (_I, [_P, _I]),
    "nd_kernel_stamps": (_I, [_P, ctypes.POINTER(_F), ctypes.POINTER(_I)]),
    "nd_stream": (_P, [_P]),
    "nd_gemm_routes": (_I, [ctypes.POINTER(ctypes.c_int64), _I, _I]),
    "nd_switches": (_I, [ctypes.c_char_p, _I]),
    "nd_destroy": (None, [_P]),
    "nd_last_error": (ctypes.c_char_p, []),
    "nd_version": (ctypes.c_char_p, []),
    "nd_op_gemm": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "nd_op_fold_layernorm": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _P]),
    "nd_op_split_weight": (_I, [_P, _I, _I, _P, _P, _P]),
    "nd_op_gemm_split": (_I, [_P, _P, _F, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "nd_op_gemm_p16": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "nd_op_pack_p16": (_I, [_P, _P, _I, _I, _P]),
    "nd_op_pack_p16h": (_I, [_P, _I, _I, _P, _P, _P]),
    "nd_op_gemm_p16_split": (_I, [_P, _P, _F, _P, _P, _P, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "nd_op_enc_ffn": (_I, [_P, _P, _F, _P, _P, _F, _P, _P, _P, _I, _I, _P, _P]),
    "nd_op_enc_ffn_wo": (_I, [_P, _P, _P, _F, _P, _P, _F, _P, _P, _F, _P, _P, _P, _P, _F, _P, _P, _I, _I, _P, _P]),
    "nd_op_dec_ffn": (_I, [_P, _P, _F, _P, _P, _F, _P, _P, _P, _I, _I, _I, _P, _P, _P, _I, _P, _P]),
    "nd_op_dec_ffn_slab_floats": (ctypes.c_int64, [_I, _I]),
    "nd_op_gemm_p16_splitk": (_I, [_P, _P, ctypes.c_float, _P, _P, _P, _I, _I, _I, _P, _P, _P, _I, _P, _P]),
    "nd_op_gemm_p16_splitk_f32": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _I, _P, _P]),
    "nd_op_gemm_p16_split_rm": (_I, [_P, _P, _F, _P, _F, _P, _P, _P, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "nd_op_dec_mem_attention": (_I, [_P, _P, _P, _P, ctypes.c_float, _P, _I, _I, _I, _I, _I, _P]),
    "nd_op_memory_pack": (_I, [_P, _P, _P, _P, _I, _I, _I, _P]),
    "nd_op_bank_pack_d8": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P]),
    "nd_op_dec_bank_d8": (_I, [_P, _P, _P, _P, _P, _P, ctypes.c_float, _P, _I, _I, _P, _I, _P]),
    "nd_bank_form": (_I, [_P]),
    "nd_op_lstm_layer": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _I, _P]),
    "nd_op_enc_attention": (_I, [_P, _P, _P, _P, _I, _I, _P]),
    "nd_op_dec_self_attention": (_I, [_P, _P, _P, _I, _I, _I, _P, _I, _P]),
    "nd_op_dec_self_attention_beam": (_I, [_P, _P, _P, _I, _I, _I, _P, _I, _I, _P, _P]),
    "nd_op_dec_self_attention_q24": (_I, [_P, _P, _P, _I, _I, _I, _P, _I, _I, _P, _P]),
    "nd_op_dec_ctx_attention": (_I, [_P, _P, _I, _I, _P, _P, _F, _P, _I, _I, _I, _P]),
    "nd_op_ctx_pack_q24": (_I, [_P, _I, _I, _P, _P, _I, _I, _P]),
    "nd_op_gemm_split_q24": (_I, [_P, _P, _F, _P, _P, _I, _I, _I, _I, _I, _P]),
    "nd_op_dec_ctx_attention_q24": (_I, [_P, _P, _I, _I, _P, _P, _F, _P, _I, _I, _I, _P]),
    "nd_op_alive_list": (_I, [_P, _I, _P, _I, _P, _P]),
    "nd_op_dec_ctx_attention_list": (_I, [_P, _P, _I, _I, _I, _P, _P, _F, _P, _I, _I, _I, _P, _I, _I, _P, _P, _P]),
}

_lib = None


class NanodecError(RuntimeError):
    pass


def lib():
    """Load (once) and return the library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (map PyTorch's HIP runtime first)
    if not os.path.exists(LIB_PATH):
        raise NanodecError(f"{LIB_PATH} not found: build it with `python -m nanodecoder_amd.build` "
                           "(there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    # an older timing-variant library (NANODEC_LIB) in an A/B run (tools/ab_lib*.sh set NANODEC_AB=1) may lack
    # entry points added since: they stay unbound there.  Anywhere else a missing entry point is a stale or
    # mismatched library, refused at load time
    ab = os.environ.get("NANODEC_AB") == "1"
    missing = []
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is None:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    if missing and not ab:
        raise NanodecError(f"{LIB_PATH} does not export {', '.join(missing)}: rebuild it (or set NANODEC_AB=1 "
                           "for an A/B timing run on an older library)")
    _lib = L
    return L


ROUTES = ["p16_small", "p16_n64", "p16_ln128", "p16s_2x4", "p16s_2x2", "p16_longk", "p16_big", "tile256",
          "tile128", "tile64", "p16_splitk"]  # include/nanodec.h ND_ROUTE_*


def gemm_routes(reset: bool = False):
    """{route: launches enqueued since the last reset} (nd_gemm_routes)."""
    c = (ctypes.c_int64 * len(ROUTES))()
    check(lib().nd_gemm_routes(c, len(ROUTES), int(reset)), "nd_gemm_routes")
    return dict(zip(ROUTES, list(c)))


def switches():
    """{name: value} of the library's A/B switches set to a non-default value
    (nd_switches), plus NANODEC_LIB when it replaces the in-tree library."""
    buf = ctypes.create_string_buffer(4096)
    lib().nd_switches(buf, len(buf))
    out = dict(kv.split("=", 1) for kv in buf.value.decode().split(";") if kv)
    if os.path.realpath(LIB_PATH) != os.path.realpath(os.path.join(HERE, "libnanodec_hip.so")):
        out["NANODEC_LIB"] = LIB_PATH
    return out


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().nd_last_error().decode(errors="replace")
        raise NanodecError(f"{what} failed (code {rc}): {msg}")
