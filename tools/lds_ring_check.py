"""Static check of inline-asm LDS read rings in compiled gfx950 assembly.

A kernel that issues ds_read_b128 from inline asm and waits for it later with
its own `s_waitcnt lgkmcnt(N)` tells the compiler the destination registers
are written at the asm statement; the data really lands at the wait.  If the
register allocator copies or reuses such a register in between, the kernel
reads stale data, intermittently.  This walks every inline-asm ds_read (between
;;#ASMSTART / ;;#ASMEND) forward to the s_waitcnt that retires it (LGKM
operations complete in order for LDS; any scalar-memory load outstanding makes
only lgkmcnt(0) count) and reports any instruction, label or branch that
touches the destination registers, or leaves the block, before then.

    python tools/lds_ring_check.py file.s [kernel-substring]
exit 1 on any hazard.
"""
import re
import sys

REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")


def regs(text):
    out = set()
    for kind, one, lo, hi in REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def functions(lines, want):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", ln)
        if m and not m.group(1).startswith(".L"):
            if cur and want in cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            body.append(ln)
    if cur and want in cur:
        yield cur, body


def check(body):
    ins = []  # (text, in_asm)
    in_asm = False
    for ln in body:
        s = ln.split(";", 1)[0].strip() if ";;#ASM" not in ln else ln.strip()
        if ln.strip().startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if ln.strip().startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith("."):
            if re.match(r"^\.LBB", ln):
                ins.append((ln.strip(), False))
            continue
        ins.append((s, in_asm))
    bad, n_checked = [], 0
    for i, (t, a) in enumerate(ins):
        if not (a and t.startswith("ds_read")):
            continue
        n_checked += 1
        dst = regs(t.split(",")[0])
        younger, smem = 0, False
        for j in range(i + 1, len(ins)):
            u, _ = ins[j]
            if u.startswith(".LBB") or u.startswith("s_cbranch") or u.startswith("s_branch") or u.startswith("s_endpgm"):
                bad.append(f"{t}  leaves the block unretired at `{u}`")
                break
            m = re.search(r"lgkmcnt\((\d+)\)", u)
            if u.startswith("s_waitcnt") and m:
                n = int(m.group(1))
                if n == 0 or (not smem and younger >= n):
                    break
                continue
            if u.startswith("ds_") or u.startswith("s_load") or u.startswith("s_buffer_load"):
                younger += 1
                smem |= not u.startswith("ds_")
            if regs(u) & dst:
                bad.append(f"{t}  destination touched before its wait by `{u}`")
                break
    return n_checked, bad


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    lines = open(path).read().splitlines()
    rc = 0
    for name, body in functions(lines, want):
        n, bad = check(body)
        if not n:
            continue
        print(f"{name}: {n} inline-asm LDS reads, {len(bad)} hazards")
        for b in bad[:20]:
            print("   ", b)
        rc |= bool(bad)
    return rc


if __name__ == "__main__":
    sys.exit(main())
