"""Host-code AddressSanitizer run of the C-ABI (SURVEY §5 "race detection /
sanitizers"): tests/asan_driver.cpp linked with engine.hip's host code built
under -fsanitize=address (nanodecoder_amd/build.py build_asan; device code is
not instrumented).  CPU: every entry point's argument validation and the
no-device error path, leak detection on.  GPU: the whole lifecycle (weight
and call errors, finalize, greedy / beam / exact / ungraphed calls, destroy)
on the prebuilt driver."""
import os
import struct
import subprocess

import numpy as np
import pytest

from nanodecoder_amd import build, synth

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1")


def _driver():
    if not os.path.exists(build.ASAN_BIN) or not os.path.exists(build.LIB):
        # the GPU box runs prebuilt binaries only; here (CPU) building is allowed
        if os.environ.get("GRAFT_REPO_ROOT"):
            pytest.fail(f"{build.ASAN_BIN} is not built (python -m nanodecoder_amd.build --asan)")
        build.build_asan()
    return build.ASAN_BIN


def test_asan_abi_validation_no_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("the no-device path needs a machine without a GPU (the GPU test covers the device path)")
    r = subprocess.run([_driver()], capture_output=True, text=True, timeout=300, env=ENV, cwd="/tmp")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed checks" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "ERROR: LeakSanitizer" not in r.stderr, r.stderr


def _write_weights(path, W):
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(W)))
        for name, a in W.items():
            a = np.ascontiguousarray(a, np.float32)
            nb = name.encode()
            f.write(struct.pack("<I", len(nb)) + nb + struct.pack("<I", a.ndim))
            f.write(np.asarray(a.shape, np.int64).tobytes() + a.tobytes())


@pytest.mark.gpu
def test_asan_abi_lifecycle_gpu(tmp_path):
    cfg = synth.ModelConfig()
    W = synth.make_weights(cfg, seed=11, eos_bias=-1.0)
    wp = str(tmp_path / "w.bin")
    _write_weights(wp, W)
    # the HIP runtime's own process-lifetime allocations are not ours: leak checks off on the device path
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")
    r = subprocess.run([_driver(), "--gpu", wp], capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed checks" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr
