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


@pytest.fixture(scope="module")
def listings(tmp_path_factory):
    """hipcc -S (gfx950, the library's flags) of every csrc/*.hip, compiled once for this module."""
    import concurrent.futures as cf
    import glob
    import subprocess
    from nanodecoder_amd import build
    if not os.path.exists(build.HIPCC):
        pytest.skip("no hipcc")
    tmp = tmp_path_factory.mktemp("asm")
    names = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(build.CSRC, "*.hip")))

    def asm(name):
        out = tmp / (name + ".s")
        subprocess.run([build.HIPCC] + build.CFLAGS + ["--cuda-device-only", "-S", os.path.join(build.CSRC, name + ".hip"),
                        "-o", str(out)], check=True, capture_output=True)
        return str(out)

    with cf.ThreadPoolExecutor(8) as ex:
        return dict(zip(names, ex.map(asm, names)))


@pytest.mark.parametrize("src,kernel", [("ffn", "enc_ffn"), ("attention", "dec_ctx_q24_kernel")])
def test_inline_asm_lds_ring_has_no_hazard(listings, src, kernel):
    """The inline-asm LDS reads (ffn.hip's read ring; the beam context
    attention's reads of its DMA ring, attention.hip): in the compiled gfx950
    code no instruction touches a destination register between its ds_read
    and the s_waitcnt that retires it (tools/lds_ring_check.py)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lds_ring_check.py"), listings[src], kernel],
                       capture_output=True, text=True)
    assert r.returncode == 0 and " 0 hazards" in r.stdout and "hazards" in r.stdout, r.stdout + r.stderr
    assert all(" 0 hazards" in ln for ln in r.stdout.splitlines() if "hazards" in ln), r.stdout


def test_hot_path_kernels_do_not_drain_loads(listings):
    """The greedy decoder's kernels issue their loads straight-line: no
    `s_waitcnt vmcnt(0)` followed by more loads (hipcc's lowering of a load
    under a runtime condition drains every load in flight; DESIGN.md §3,
    "Straight-line loads").  The P16 GEMMs keep one: the `--fast` beam's
    finished-chunk probe (rows_dead), which runs only with a skip list."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from isa_loops import drains
    src = {k: open(v).read() for k, v in listings.items() if k in ("attention", "bank8", "search", "gemm")}
    want = [("attention", r"dec_self_attention_kernelILi\d+ELi\d+ELb0ELb0E", 0),  # no beam ancestry
            # the form that runs the previous step's head: wave 0 waits for the
            # head's own loads, then issues its cache loads (the one allowed)
            ("attention", r"dec_self_attention_kernelILi\d+ELi\d+ELb0ELb1E", 1),
            # beam rows, the bench's beam 5 on the 24-bit history: the one wait is the appends' (vmcnt(0) and a
            # barrier before any wave reads the cache); the keys' loads go straight into the registers the
            # arithmetic reads (composing them made hipcc wait per key: 7 drains before)
            ("attention", r"dec_self_attention_beam_kernelILi5ELi4ELb1E", 1),
            # the 24-bit digit bank: the one-chunk form's two sit in the unrolled key loop: the wait for the
            # last fragment of the half block being multiplied, right before the next half block's loads
            # (reviewed, round 5).  The walking form (pool lanes) holds that body once per chunk and load
            # policy: two chunks straight-line (the second's head loaded during the first's merge, round 6:
            # pooled configs[1] 15.34 -> 15.20 ms, profiles/r06_ab_walk.txt) plus the general loop, each
            # body with the same waits
            ("bank8", r"dec_bank_d8_kernelILb0ELb1E", 3),
            ("bank8", r"dec_bank_d8_kernelILb1ELb1E", 8),
            # (the non-temporal forms hold the chunk body twice: the call's first quarter of chunks keeps the
            # default cache policy, bank_cached in bank8.hip)
            ("bank8", r"dec_bank_d8_kernelILb0ELb0E", 2),
            ("bank8", r"dec_bank_d8_kernelILb1ELb0E", 4),
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


# ----------------------------------------------------------------- MFMA wait states
# DESIGN.md section 3 "MFMA results and wait states" (round 5).  The hardware
# probe (tools/probe_mfma_hazard.py) found one hazard class hipcc 7.2 does not
# pad: an MFMA of another shape accumulating onto an MFMA's destination
# (16x16x32_f16 then 16x16x16_f16, or the reverse) reads half of srcC stale
# unless >= 4 VALU / 5 SALU instructions separate them; the greedy digit-bank
# kernel had such a pair 4 instructions apart (now one shape per accumulator).
# tools/isa_hazard.py walks every path (branches, loop back-edges) after every
# MFMA of every shipped kernel and fails on any instruction that touches the
# MFMA's destination before the form's required wait states (the larger of
# hipcc's own pad and the hardware probe's, tools/probe_mfma_hazard.py).
def _isa_hazard():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_hazard
    return isa_hazard


def test_mfma_hazard_scanner_finds_known_violations():
    """The scanner itself: a VALU read 5 states after a 16x16x32 MFMA is
    flagged; 8 states (the pad) is not; a read reached only through a taken
    branch is flagged; a same-form accumulate chain (srcC only) is not; a
    16x16x16 accumulating onto it is, unless 5 states apart."""
    H = _isa_hazard()
    mf = "\tv_mfma_f32_16x16x32_f16 v[0:3], v[4:7], v[8:11], v[0:3]\n"

    def fn(body):
        return "_Zfoo:\n" + body + "\ts_endpgm\n.Lfunc_end0:\n"
    near = fn(mf + "\ts_nop 3\n\tv_mov_b32_e32 v20, v1\n")
    far = fn(mf + "\ts_nop 7\n\tv_mov_b32_e32 v20, v1\n")
    branch = fn(mf + "\ts_cbranch_scc1 .LBB0_2\n\ts_nop 15\n\ts_nop 15\n.LBB0_2:\n\tv_mov_b32_e32 v20, v3\n")
    chain = fn(mf + "\tv_mfma_f32_16x16x32_f16 v[12:15], v[4:7], v[8:11], v[0:3]\n\ts_nop 15\n")
    # a 16x16x16 accumulating onto the 16x16x32's destination: stale srcC half unless 5 states apart
    mixed = fn(mf + "\tv_mfma_f32_16x16x16_f16 v[0:3], v[4:5], v[8:9], v[0:3]\n\ts_nop 15\n")
    mixed_far = fn(mf + "\ts_nop 4\n\tv_mfma_f32_16x16x16_f16 v[0:3], v[4:5], v[8:9], v[0:3]\n\ts_nop 15\n")
    assert len(H.scan(near)["_Zfoo"]) == 1
    assert H.scan(far)["_Zfoo"] == []
    assert len(H.scan(branch)["_Zfoo"]) == 1
    assert H.scan(chain)["_Zfoo"] == []
    assert len(H.scan(mixed)["_Zfoo"]) == 1
    assert H.scan(mixed_far)["_Zfoo"] == []
    # a VALU result read by the next MFMA: as srcC 0 states apart (needs 1), as srcA 1 apart (needs 2)
    valu_c = fn("\tv_mul_f32_e32 v1, 2.0, v1\n" + mf)
    valu_c_ok = fn("\tv_mul_f32_e32 v1, 2.0, v1\n\ts_nop 0\n" + mf)
    valu_a = fn("\tv_mov_b32_e32 v5, v40\n\ts_nop 0\n" + mf)
    valu_a_ok = fn("\tv_mov_b32_e32 v5, v40\n\ts_nop 1\n" + mf)
    one = lambda a: H.scan_valu_to_mfma(*H.parse(a)["_Zfoo"])
    assert len(one(valu_c)) == 1 and one(valu_c_ok) == []
    assert len(one(valu_a)) == 1 and one(valu_a_ok) == []


def test_mfma_results_respect_wait_states(listings):
    """Every MFMA of every shipped kernel, on every path: no instruction
    reads or writes its destination registers inside the required wait
    states, and no MFMA reads a VALU result as an operand inside the probed
    window (srcC 1 state, srcA / srcB 2).  Covers dec_bank_d8_kernel's
    lazy-rescale branch (bank8.hip, `if (__any(gm > m + B8_THR))` over the U
    accumulators) and every other MFMA consumer; the context attention's
    online_update_lazy runs on VALU accumulators (no MFMA there)."""
    H = _isa_hazard()
    total, bad = 0, {}
    for name, path in listings.items():
        asm = open(path).read()
        total += sum(H.count_mfma(asm).values())
        for k, hz in H.scan(asm).items():
            if hz:
                bad[k] = hz[:3]
        for k, (ins, labels) in H.parse(asm).items():
            vm = H.scan_valu_to_mfma(ins, labels)
            if vm:
                bad[k + " (VALU->MFMA)"] = vm[:3]
    assert total > 1000, total  # the scan saw the kernels' MFMAs
    assert not bad, bad
    d8 = H.count_mfma(open(listings["bank8"]).read(), r"dec_bank_d8_kernel")
    assert d8 and all(n > 0 for n in d8.values())


# ----------------------------------------------------------------- LDS rule
# DESIGN.md section 5 "Co-residency": the closed-form layer-0 encoder attention
# returned wrong chunks beside another engine's kernels exactly when its
# per-wave data past LDS byte 65,536 was accessed by ds_read2* / ds_write2*
# through an address register >= 65,536 (tools/r2_lds.sh, profiles/r04_lds/).
# Every kernel that can hold more than 64 KB of LDS and uses the paired forms
# is listed here with the reason its paired accesses were reviewed, and the
# most paired-form instructions it had when reviewed; a new kernel, or more
# paired accesses in a listed one, fails until it is reviewed again.
DYNAMIC_LDS = {  # kernels launched with dynamic LDS (metadata says 0): bytes at the launch site
    "dec_bank_d8_kernel": 138064,        # bank8.hip B8_LDS
    "dec_mem_attention_kernel": 158208,  # mem_lds_bytes()
    "dec_ctx_attention_kernel": 52224,   # ctx_lds_bytes(6) (the attribute allows 160 KB; launches take this)
    "dec_ctx_q24_kernel": 76992,         # cq_lds_bytes(<= 2 rows): 4 waves x 3 slots x 6416 B
    "gemm_p16s_kernel": 98304,           # 2x4 tiles
}
REVIEWED_PAIRED = {
    # base name: (max paired-form DS instructions per instantiation, reason)
    "enc_attention_h3_kernel": (9, "K / V^T staging with ds_write2st64_b64 from a base below 64 KB, read by the "
                                   "other waves after a barrier; pool-tested bitwise"),
    "enc_ffn_kernel": (8, "row statistics written with ds_write2st64_b32 behind the weight slots, read after a "
                          "barrier; pool-tested"),
    "gemm_f32_kernel": (48, "A / W tile staging (ds_write2_b32 / _b64 / 2st64) read by other waves after a "
                            "barrier; encoder-side GEMMs of the beam / exact / NanoEncoder paths, pool-tested"),
    "gemm_f32d_kernel": (8, "the LayerNorm row statistics (ds_write2st64_b32, one lane per row, mean and rstd) "
                            "read by every wave after a barrier, as gemm_f32_kernel's; the operand ring takes no "
                            "paired form (DMA writes, inline-asm ds_read_b128); exact fp32 pool-tested bitwise at "
                            "the bench's configuration (test_pool_at_bench_config_matches_single_engine)"),
    "dec_ctx_attention_kernel": (36, "the (m, l, acc) merge of the beam context attention (and of its split "
                                     "form); launched with at most 52 KB, listed in case that grows"),
    "dec_ctx_q24_kernel": (26, "the (m, l, acc) merge after a barrier behind the DMA rings' last use; the merge "
                               "image sits at LDS byte 0 (< 22 KB), far below 64 KB (the rings above it take no "
                               "paired form)"),
    "dec_bank_d8_kernel": (15, "the (m, l) merge and the q' digit rows (cross-wave, after a barrier), once per "
                               "chunk body: twice in the non-temporal one-chunk form (bank8.hip bank_cached), up to "
                               "five in the walking non-temporal form (round 6: the two-chunk straight-line path "
                               "per load policy plus the general loop); pool-tested at the bench's configuration "
                               "(profiles/r06_gpu4.log)"),
    "dec_mem_attention_kernel": (92, "the fp32 bank kernel (exact fp32 / short chunks): slab reads after "
                                     "barriers, 23-25 per chunk body; the 512-key form holds four bodies (round 6: "
                                     "the walking form's two-chunk straight-line path, its one-chunk case, the "
                                     "general loop); pool-tested bitwise in exact fp32 at the bench's "
                                     "configuration (test_pool_at_bench_config_matches_single_engine)"),
}


def test_lds_paired_forms_above_64k_are_reviewed():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_meta
    from nanodecoder_amd import build
    build.build()
    seen = {}
    for r in kernel_meta.collect():
        base = re.sub(r"\(.*$", "", re.sub(r"^void ", "", r["name"])).replace("nd::", "")
        base = re.sub(r"<.*$", "", base)
        lds = r.get("lds", 0) + DYNAMIC_LDS.get(base, 0)
        pairs = sum(v for k, v in r["ds"].items() if re.match(r"ds_(read|write)2", k))
        if lds > 65536 and pairs:
            seen[base] = max(seen.get(base, 0), pairs)
    for base, n in seen.items():
        assert base in REVIEWED_PAIRED, f"{base}: {n} paired-form LDS instructions and more than 64 KB of LDS"
        assert n <= REVIEWED_PAIRED[base][0], (base, n, REVIEWED_PAIRED[base])
    # the closed-form layer-0 attention keeps its whole allocation at 64 KB
    r2 = [r for r in kernel_meta.collect() if "enc_attention_rank2_kernel" in r["name"]]
    assert r2 and all(r["lds"] <= 65536 for r in r2)


def test_missing_library_fails_loudly(tmp_path):
    """No HIP library, no engine: with the library path pointing at nothing, the
    product path (an Engine, a Translator's first call) raises NanodecError
    naming the build step; there is no CPU fallback to run instead."""
    import subprocess
    import sys
    code = ("import sys\n"
            "from nanodecoder_amd import _lib, synth\n"
            "from nanodecoder_amd.engine import Engine\n"
            "cfg = synth.ModelConfig()\n"
            "try:\n"
            "    Engine(cfg, synth.make_weights(cfg, seed=1), device=0)\n"
            "except _lib.NanodecError as e:\n"
            "    print('raised:', e)\n"
            "    sys.exit(0)\n"
            "sys.exit(3)\n")
    env = dict(os.environ, NANODEC_LIB=str(tmp_path / "absent.so"))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "not found" in r.stdout and "no CPU fallback" in r.stdout, r.stdout


def test_integration_names_every_entry_point():
    """INTEGRATION.md, the maintainer's binding guide, names every entry point
    include/nanodec.h declares (with the reference interface it replaces, or
    'no reference equivalent')."""
    import re
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    missing = [s for s in sorted(declared_symbols()) if s not in doc]
    assert not missing, missing
