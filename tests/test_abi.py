"""The C-ABI library builds for gfx950, loads without a GPU, and exports every
symbol include/nanodec.h declares (CPU only: no compute calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nanodec.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nd_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from nanodecoder_amd import build, _lib
    build.build()
    return _lib.lib()


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("nd_create", "nd_load_weight", "nd_finalize", "nd_translate_greedy", "nd_translate_beam",
              "nd_encode", "nd_destroy", "nd_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_ctypes_signatures_cover_header():
    from nanodecoder_amd import _lib
    assert set(declared_symbols()) == set(_lib.SIGNATURES)


def test_version_and_error_without_gpu(lib):
    assert b"gfx950" in lib.nd_version()
    # argument validation happens before any HIP call
    from nanodecoder_amd._lib import NdConfig
    c = NdConfig()
    c.d_model, c.heads = 128, 8
    h = ctypes.c_void_p()
    rc = lib.nd_create(ctypes.byref(c), ctypes.byref(h))
    assert rc == 1 and b"d_model" in lib.nd_last_error()


def test_code_object_targets_gfx950(lib):
    so = os.path.join(ROOT, "nanodecoder_amd", "libnanodec_hip.so")
    blob = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_inline_asm_lds_ring_has_no_hazard(tmp_path):
    """ffn.hip's inline-asm LDS read ring: in the compiled gfx950 code no
    instruction touches a ring destination register between its ds_read and
    the s_waitcnt that retires it (tools/lds_ring_check.py)."""
    import subprocess
    import sys
    from nanodecoder_amd import build
    if not os.path.exists(build.HIPCC):
        pytest.skip("no hipcc")
    out = tmp_path / "ffn.s"
    subprocess.run([build.HIPCC] + build.CFLAGS + ["--cuda-device-only", "-S", os.path.join(build.CSRC, "ffn.hip"),
                    "-o", str(out)], check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lds_ring_check.py"), str(out), "enc_ffn"],
                       capture_output=True, text=True)
    assert r.returncode == 0 and "0 hazards" in r.stdout, r.stdout + r.stderr


def test_hot_path_kernels_do_not_drain_loads(tmp_path):
    """The greedy decoder's kernels issue their loads straight-line: no
    `s_waitcnt vmcnt(0)` followed by more loads (hipcc's lowering of a load
    under a runtime condition drains every load in flight; DESIGN.md §3,
    "Straight-line loads").  The P16 GEMMs keep one: the `--fast` beam's
    finished-chunk probe (rows_dead), which runs only with a skip list."""
    import concurrent.futures as cf
    import subprocess
    import sys
    from nanodecoder_amd import build
    if not os.path.exists(build.HIPCC):
        pytest.skip("no hipcc")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from isa_loops import drains

    def asm(name):
        out = tmp_path / (name + ".s")
        subprocess.run([build.HIPCC] + build.CFLAGS + ["--cuda-device-only", "-S", os.path.join(build.CSRC, name + ".hip"),
                        "-o", str(out)], check=True, capture_output=True)
        return out.read_text()

    with cf.ThreadPoolExecutor(4) as ex:
        src = dict(zip(["attention", "mem_attention", "search", "gemm"],
                       ex.map(asm, ["attention", "mem_attention", "search", "gemm"])))
    want = [("attention", r"dec_self_attention_kernelILi\d+ELi\d+ELb0ELb0E", 0),  # no beam ancestry
            # the form that runs the previous step's head: wave 0 waits for the
            # head's own loads, then issues its cache loads (the one allowed)
            ("attention", r"dec_self_attention_kernelILi\d+ELi\d+ELb0ELb1E", 1),
            ("mem_attention", r"dec_bank_h3_kernelILb\dELb0E", 0),  # one chunk per workgroup
            # the walking form (pool lanes): the loop's load schedule drains the
            # first half blocks once per chunk
            ("mem_attention", r"dec_bank_h3_kernelILb\dELb1E", 2),
            # the standalone head (the last step only when the head is fused):
            # the V > 8 generator loop's loads follow the first 8 rows' wait
            ("search", r"greedy_head_kernel", 1),
            ("gemm", r"gemm_p16_kernelILi1ELi8ELi256ELb1ELb0ELb0ELb1E", 1),  # VO / FFN2 (K = 2048)
            ("gemm", r"gemm_p16_kernelILi1ELi4ELi64ELb1ELb0ELb0ELb1E", 1),  # Wo
            ("gemm", r"gemm_p16s_kernelILi2ELi4ELb1ELb1E", 1),  # QK / FFN1
            ("gemm", r"gemm_p16s_kernelILi2ELi2ELb1ELb1ELb0ELb0E", 1)]  # QKV (layers 1, 2)
    for f, rx, most in want:
        found = drains(src[f], rx)
        assert found, rx
        bad = {k: v for k, v in found.items() if v > most}
        assert not bad, bad
