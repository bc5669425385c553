"""Build libnanodec_hip.so in-tree with hipcc for gfx950.

Every .hip file under csrc/ is compiled to an object with
``hipcc --offload-arch=gfx950 -O3 -fPIC`` and linked into
``nanodecoder_amd/libnanodec_hip.so``.  Objects are rebuilt when their source
or any csrc header is newer.  Usage: ``python -m nanodecoder_amd.build``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libnanodec_hip.so")
ARCH = os.environ.get("NANODEC_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-Wall",
          "-Wno-unused-function", "-Wno-unused-variable", "-I" + CSRC, "-I" + INCLUDE]


def _newest_dep():
    deps = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return max((os.path.getmtime(p) for p in deps), default=0.0)


def _compile(src, obj, verbose):
    cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(src)}:\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip() and verbose:
        print(r.stderr, file=sys.stderr)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    dep_t = _newest_dep()
    jobs = []
    objs = []
    for src in srcs:
        obj = os.path.join(BUILD, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), dep_t):
            jobs.append((src, obj))
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            list(ex.map(lambda a: _compile(a[0], a[1], verbose), jobs))
    if jobs or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


# Host-side AddressSanitizer build of the C-ABI: engine.hip's host
# code instrumented, device code not (GPU ASan is unavailable); linked with the
# regular objects of the other kernels into tests/asan_driver.cpp's driver.
ASAN_HOST = "-gline-tables-only -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -fno-gpu-sanitize".split()
ASAN_LINK = "-fsanitize=address -fno-gpu-sanitize".split()
ASAN_BIN = os.path.join(HERE, "asan_driver")  # beside the .so: built files under _build/ stay home
ASAN_SRC = os.path.join(os.path.dirname(HERE), "tests", "asan_driver.cpp")


def build_asan(verbose: bool = False) -> str:
    build(verbose=verbose)
    objs = [os.path.join(BUILD, os.path.basename(p)[:-4] + ".o") for p in sorted(glob.glob(os.path.join(CSRC, "*.hip")))
            if os.path.basename(p) != "engine.hip"]
    eng_src, eng_obj = os.path.join(CSRC, "engine.hip"), os.path.join(BUILD, "asan_engine.o")
    drv_obj = os.path.join(BUILD, "asan_driver.o")
    dep_t = _newest_dep()
    jobs = []
    if not os.path.exists(eng_obj) or os.path.getmtime(eng_obj) < max(os.path.getmtime(eng_src), dep_t):
        jobs.append((eng_src, eng_obj))
    if not os.path.exists(drv_obj) or os.path.getmtime(drv_obj) < max(os.path.getmtime(ASAN_SRC), dep_t):
        jobs.append((ASAN_SRC, drv_obj))
    for src, obj in jobs:
        cmd = [HIPCC] + CFLAGS + ASAN_HOST + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc (asan) failed for {os.path.basename(src)}:\n{r.stdout}\n{r.stderr}")
    deps = [eng_obj, drv_obj] + objs
    if jobs or not os.path.exists(ASAN_BIN) or os.path.getmtime(ASAN_BIN) < max(os.path.getmtime(o) for o in deps):
        cmd = [HIPCC, f"--offload-arch={ARCH}"] + ASAN_LINK + ["-o", ASAN_BIN] + deps
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"asan link failed:\n{r.stdout}\n{r.stderr}")
    return ASAN_BIN


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    if "--asan" in sys.argv:
        print(build_asan(verbose=True))
