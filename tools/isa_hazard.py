"""MFMA -> VALU wait-state scan of compiled gfx950 code (hipcc -S listings).

An MFMA writes its destination registers several cycles after it issues.
Until then, gfx950 does not interlock: a VALU, LDS or memory instruction that
reads one of those registers gets the old value, and one that writes it can
be overwritten by the late MFMA result (cdna_hip_programming.md §5.7 item 2).
hipcc pads the code it schedules itself; it does not model inline asm, and
this scan checks what it emitted on EVERY path, across branches and loop
back-edges, not only straight-line code.

For each MFMA in each kernel it walks the control-flow graph forward,
counting wait states (one per instruction, k + 1 for `s_nop k`), until the
form's requirement is met.  Any instruction on the way that names one of the
destination registers is a hazard, except an MFMA of the SAME form that reads
them as its srcC only (an accumulator chain: the matrix pipe forwards it at
no wait state).  An MFMA of another form reading them as srcC is a hazard
inside MIXED_SRCC states: a 16x16x16_f16 accumulating onto a 16x16x32_f16's
destination (or the reverse) reads half of srcC stale with fewer than 4 VALU
/ 5 SALU or s_nop states between them, and hipcc 7.2 emits such pairs back
to back (tools/probe_mfma_hazard.py, profiles/r05_mfma_hazard_probe.json).

Required states per form: the larger of the compiler's own pad (hipcc 7.2,
measured on a VALU read right after the MFMA) and the hardware probe's
(`tools/probe_mfma_hazard.py`, profiles/r05_mfma_hazard.json).

    python tools/isa_hazard.py file.s [KERNEL_REGEX]
"""
import re
import sys

# mnemonic (without v_mfma_) -> required wait states before another instruction touches its destination
REQUIRED = {
    "f32_16x16x16_f16": 8,
    "f32_16x16x32_f16": 8,
    "f32_16x16x32_bf16": 8,
    "f32_16x16x16_bf16": 8,
    "i32_16x16x64_i8": 8,
    "i32_16x16x32_i8": 8,
    "f32_32x32x16_f16": 12,
    "f32_32x32x8_f16": 12,
    "f32_32x32x16_bf16": 12,
    "i32_32x32x32_i8": 12,
    "f32_16x16x4_f32": 10,
    "f32_32x32x2_f32": 18,
    "f32_4x4x1_16b_f32": 4,
    "f32_4x4x4_16b_f16": 4,
}
DEFAULT_REQUIRED = 19  # an unlisted form: the longest (16-pass) requirement
MIXED_SRCC = 5  # states between an MFMA and another form's MFMA taking its destination as srcC

REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")


def regs(text):
    """set of ('v'|'a', index) named in an operand string"""
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(2) is not None:
            out.add((k, int(m.group(2))))
        else:
            out.update((k, i) for i in range(int(m.group(3)), int(m.group(4)) + 1))
    return out


def parse(asm):
    """{kernel symbol: (instructions, labels)}; an instruction is (mnemonic, operand text, source line)"""
    funcs = {}
    for m in re.finditer(r"^(_Z\S+|[A-Za-z_]\w*):\s*(?:;.*)?$", asm, re.M):
        name = m.group(1)
        end = asm.find(".Lfunc_end", m.end())
        if end < 0 or not asm[m.end():end].strip():
            continue
        ins, labels = [], {}
        for raw in asm[m.end():end].split("\n"):
            line = raw.split(";")[0].strip()
            if not line:
                continue
            if line.endswith(":"):
                labels[line[:-1]] = len(ins)
                continue
            if line.startswith("."):
                continue
            parts = line.split(None, 1)
            ins.append((parts[0], parts[1] if len(parts) > 1 else "", raw.strip()))
        if ins:
            funcs[name] = (ins, labels)
    return funcs


def succ(ins, labels, i):
    mn, ops, _ = ins[i]
    if mn == "s_endpgm" or mn.startswith(("s_setpc", "s_swappc")):
        return []
    if mn == "s_branch":
        return [labels[ops.split()[0]]] if ops.split()[0] in labels else []
    if mn.startswith("s_cbranch"):
        t = ops.split()[0]
        return ([labels[t]] if t in labels else []) + ([i + 1] if i + 1 < len(ins) else [])
    return [i + 1] if i + 1 < len(ins) else []


def states(mn, ops):
    if mn == "s_nop":
        return int(ops.split()[0], 0) + 1
    return 1


def split_mfma(ops):
    """dst, srcA, srcB, srcC operand texts of an MFMA"""
    parts = [p.strip() for p in re.split(r",(?![^\[]*\])", ops)]
    return parts[0], parts[1], parts[2], parts[3] if len(parts) > 3 else ""


def scan_function(ins, labels, every=False):
    """[(mfma line, hazard line, states elapsed, required)]; every: report
    every toucher on a path, not only the first"""
    found = []
    for i, (mn, ops, raw) in enumerate(ins):
        if not mn.startswith("v_mfma_"):
            continue
        form = mn[len("v_mfma_"):]
        need = REQUIRED.get(form, DEFAULT_REQUIRED)
        dst = regs(split_mfma(ops)[0])
        dst_text = split_mfma(ops)[0]
        # depth-first over paths: (instruction index, states elapsed before it)
        best = {}
        stack = [(j, 0) for j in succ(ins, labels, i)]
        while stack:
            j, st = stack.pop()
            if st >= need or best.get(j, need) <= st:
                continue  # requirement met, or this point already reached with at most as many states
            best[j] = st
            mn2, ops2, raw2 = ins[j]
            named = regs(ops2) & dst
            if named:
                if mn2.startswith("v_mfma_"):
                    d2, a2, b2, c2 = split_mfma(ops2)
                    if not (regs(a2) | regs(b2)) & dst:
                        if mn2 == mn or st >= MIXED_SRCC:
                            continue  # srcC only, same form (forwarded) or far enough: the chain takes over
                        found.append((raw, raw2, st, MIXED_SRCC))
                        if not every:
                            continue
                        continue
                found.append((raw, raw2, st, need))
                if not every:
                    continue
            st2 = st + states(mn2, ops2)
            for k in succ(ins, labels, j):
                stack.append((k, st2))
    return found


# VALU -> MFMA operand (hardware-probed, tools/probe_mfma_hazard.py valu_srcC /
# valu_srcA rows): a VALU result read by an MFMA as srcC needs 1 intervening
# state, as srcA / srcB 2; gap 0 returned the stale value
VALU_SRCC = 1
VALU_SRCAB = 2


def scan_valu_to_mfma(ins, labels):
    """[(VALU line, MFMA line, states elapsed, required)]: an MFMA reading a
    VALU-written VGPR (as srcC within VALU_SRCC states, as srcA / srcB within
    VALU_SRCAB) on some path"""
    found = []
    horizon = max(VALU_SRCC, VALU_SRCAB)
    for i, (mn, ops, raw) in enumerate(ins):
        if not mn.startswith("v_") or mn.startswith(("v_mfma_", "v_cmp", "v_readlane", "v_readfirstlane")):
            continue
        parts = [p.strip() for p in re.split(r",(?![^\[]*\])", ops)]
        if not parts:
            continue
        dst = regs(parts[0])
        if not dst:
            continue
        best = {}
        stack = [(j, 0) for j in succ(ins, labels, i)]
        while stack:
            j, st = stack.pop()
            if st >= horizon or best.get(j, horizon) <= st:
                continue
            best[j] = st
            mn2, ops2, raw2 = ins[j]
            if mn2.startswith("v_mfma_"):
                d2, a2, b2, c2 = split_mfma(ops2)
                if st < VALU_SRCC and regs(c2) & dst:
                    found.append((raw, raw2, st, VALU_SRCC))
                if st < VALU_SRCAB and (regs(a2) | regs(b2)) & dst:
                    found.append((raw, raw2, st, VALU_SRCAB))
            st2 = st + states(mn2, ops2)
            for k in succ(ins, labels, j):
                stack.append((k, st2))
    return found


def scan(asm, regex=None, every=False):
    """{kernel symbol: [hazards]} for every kernel (matching regex) in a listing"""
    out = {}
    for name, (ins, labels) in parse(asm).items():
        if regex and not re.search(regex, name):
            continue
        out[name] = scan_function(ins, labels, every)
    return out


def count_mfma(asm, regex=None):
    return {name: sum(1 for x in ins if x[0].startswith("v_mfma_")) for name, (ins, _) in parse(asm).items()
            if not regex or re.search(regex, name)}


if __name__ == "__main__":
    res = scan(open(sys.argv[1]).read(), sys.argv[2] if len(sys.argv) > 2 else None)
    n = 0
    for name, hz in sorted(res.items()):
        for mf, h, st, need in hz:
            n += 1
            print(f"{name}: {h!r} {st} states after {mf!r} (needs {need})")
    print(f"{n} hazards in {len(res)} functions")
