"""Instruction mix of the loops of one kernel in a hipcc -S listing.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o x.s file.hip
  python tools/isa_loops.py x.s enc_attention_h3_kernel
  python tools/isa_loops.py --drains x.s REGEX

Prints, per backward branch (a loop), its length, VALU / MFMA / LDS / VMEM
counts and the most common opcodes, plus the kernel's register and spill
counts from the .amdhsa metadata.  --drains lists, for every kernel whose
symbol matches REGEX, the `s_waitcnt vmcnt(0)` followed by another vector
load: a drain of every load in flight before more are issued (hipcc emits
one after a load under a runtime condition whose result is used in the
branch, DESIGN.md §3 "Straight-line loads").
"""
import re
import sys
from collections import Counter


def main(path, name):
    s = open(path).read()
    m = re.search(r"^(_Z\S*%s\S*):" % re.escape(name), s, re.M)
    if not m:
        sys.exit(f"{name}: not found")
    sym = m.group(1)
    body = s[m.end():s.index(".Lfunc_end", m.end())]
    lines = [l.split(";")[0].strip() for l in body.split("\n")]
    lines = [l for l in lines if l and (l.endswith(":") or not l.startswith("."))]
    labels = {l[:-1]: n for n, l in enumerate(lines) if l.endswith(":")}
    for n, l in enumerate(lines):
        b = re.match(r"s_cbranch_\w+ (\S+)|s_branch (\S+)", l)
        tgt = b and (b.group(1) or b.group(2))
        if tgt in labels and labels[tgt] < n:
            seg = [x.split()[0] for x in lines[labels[tgt]:n + 1] if not x.endswith(":")]
            c = Counter(seg)
            mf = sum(v for k, v in c.items() if "mfma" in k)
            va = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
            ds = sum(v for k, v in c.items() if k.startswith("ds_"))
            vm = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_")))
            print(f"loop {tgt}: {len(seg)} instr, valu {va}, mfma {mf}, lds {ds}, vmem {vm}")
            print("   ", ", ".join(f"{k} {v}" for k, v in c.most_common(30)))
    meta = s[s.index(".amdhsa_kernel " + sym):]
    meta = meta[:meta.index(".end_amdhsa_kernel")]
    for key in ("next_free_vgpr", "accum_offset", "next_free_sgpr", "private_segment_fixed_size",
                "group_segment_fixed_size"):
        mm = re.search(r"\.amdhsa_%s (\d+)" % key, meta)
        if mm:
            print(f"{key} {mm.group(1)}")


def drains(asm, regex, window=80):
    """{kernel symbol: number of vmcnt(0) waits followed by a vector load}"""
    out = {}
    for m in re.finditer(r"^(_Z\S+):", asm, re.M):
        name = m.group(1)
        if not re.search(regex, name):
            continue
        body = asm[m.end():asm.index(".Lfunc_end", m.end())]
        lines = [l.split(";")[0].strip() for l in body.split("\n")]
        lines = [l for l in lines if l]
        n = 0
        for i, l in enumerate(lines):
            if l.startswith("s_waitcnt") and "vmcnt(0)" in l:
                for nxt in lines[i + 1:i + window]:
                    if nxt.startswith(("global_load", "buffer_load")):
                        n += 1
                        break
                    if nxt.startswith("s_endpgm"):
                        break
        out[name] = n
    return out


if __name__ == "__main__":
    if sys.argv[1] == "--drains":
        for k, v in sorted(drains(open(sys.argv[2]).read(), sys.argv[3]).items()):
            print(v, k)
    else:
        main(sys.argv[1], sys.argv[2])
