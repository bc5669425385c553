"""Kernel metadata and LDS instruction census of the shipped gfx950 code
objects (CPU only: no GPU needed).

For every object under nanodecoder_amd/_build/ the gfx950 code object is
pulled out of the .hip_fatbin offload bundle; ``llvm-readelf --notes`` gives
each kernel's metadata (static LDS ``group_segment_fixed_size``, VGPRs,
spills) and ``llvm-objdump -d`` its instructions, from which the DS
(LDS) instruction forms are counted.

    python tools/kernel_meta.py            table of every kernel
    python tools/kernel_meta.py --json     the same as JSON
"""
from __future__ import annotations

import glob
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
BUILD = os.path.join(ROOT, "nanodecoder_amd", "_build")


def code_object(obj: str, out_dir: str) -> str:
    """The gfx950 device code object inside a hipcc host object."""
    fat = os.path.join(out_dir, os.path.basename(obj) + ".fatbin")
    r = subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, obj,
                        os.path.join(out_dir, "scratch.o")], capture_output=True)
    if r.returncode != 0:
        return None  # host code only
    b = open(fat, "rb").read()
    if not b.startswith(b"__CLANG_OFFLOAD_BUNDLE__"):
        raise ValueError(f"{obj}: no offload bundle")
    n = struct.unpack_from("<Q", b, 24)[0]
    off = 32
    for _ in range(n):
        o, sz, tl = struct.unpack_from("<QQQ", b, off)
        off += 24
        triple = b[off: off + tl].decode()
        off += tl
        if "gfx950" in triple:
            co = os.path.join(out_dir, os.path.basename(obj) + ".co")
            with open(co, "wb") as f:
                f.write(b[o: o + sz])
            return co
    raise ValueError(f"{obj}: no gfx950 code object")


def kernel_notes(co: str):
    """{symbol: {lds, vgpr, vgpr_spill, sgpr_spill, private}} from the metadata note."""
    txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                         text=True).stdout
    out, cur, sym = {}, {}, None
    fields = {".group_segment_fixed_size": "lds", ".vgpr_count": "vgpr", ".vgpr_spill_count": "vgpr_spill",
              ".sgpr_spill_count": "sgpr_spill", ".private_segment_fixed_size": "private",
              ".max_flat_workgroup_size": "max_wg", ".agpr_count": "agpr"}
    for line in txt.splitlines():
        s = line.strip().lstrip("- ").strip()
        m = re.match(r"(\.[a-z_]+):\s+(\S+)", s)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == ".args":
            continue
        if k in fields:
            cur[fields[k]] = int(v)
        elif k == ".symbol":
            sym = v[:-3] if v.endswith(".kd") else v
        elif k == ".wavefront_size" and sym:  # the last key of a kernel's (alphabetical) map
            out[sym] = cur
            cur, sym = {}, None
    return out


def ds_census(co: str):
    """{symbol: {ds opcode: count}} from the disassembly."""
    txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.match(r"^\s+(ds_\w+)", line)
        if m and cur is not None:
            cur[m.group(1)] = cur.get(m.group(1), 0) + 1
    return out


def demangle(names):
    import shutil
    tool = shutil.which("c++filt") or shutil.which("llvm-cxxfilt")
    if not tool:
        return {n: n for n in names}
    r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True)
    return dict(zip(names, r.stdout.splitlines())) if r.returncode == 0 else {n: n for n in names}


def collect(build_dir: str = BUILD):
    rows = []
    with tempfile.TemporaryDirectory() as td:
        for obj in sorted(glob.glob(os.path.join(build_dir, "*.o"))):
            if os.path.basename(obj).startswith("asan_"):
                continue
            co = code_object(obj, td)
            if co is None:
                continue
            notes, ds = kernel_notes(co), ds_census(co)
            for sym, meta in notes.items():
                rows.append(dict(object=os.path.basename(obj), symbol=sym, ds=ds.get(sym, {}), **meta))
    names = demangle([r["symbol"] for r in rows])
    for r in rows:
        r["name"] = names.get(r["symbol"], r["symbol"])
    return rows


def main(argv):
    rows = collect()
    if "--json" in argv:
        print(json.dumps(rows, indent=1))
        return
    for r in sorted(rows, key=lambda r: -r.get("lds", 0)):
        pair = sum(v for k, v in r["ds"].items() if re.match(r"ds_(read|write)2", k))
        print(f"{r.get('lds', 0):7d} B  vgpr {r.get('vgpr', 0):3d}  spill {r.get('vgpr_spill', 0):3d}  "
              f"ds2 {pair:3d}  {r['name'][:110]}")


if __name__ == "__main__":
    main(sys.argv[1:])
