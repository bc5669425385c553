"""Instruction mix of the loops of one kernel in a hipcc -S listing.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o x.s file.hip
  python tools/isa_loops.py x.s enc_attention_h3_kernel

Prints, per backward branch (a loop), its length, VALU / MFMA / LDS / VMEM
counts and the most common opcodes, plus the kernel's register and spill
counts from the .amdhsa metadata.
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


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
