"""Hardware probe: how many wait states gfx950 needs between an MFMA and a VALU
read (RAW) or write (WAW) of its destination, per MFMA form the library uses.

The probe source is generated (one kernel per form x wait states x mode,
every instruction inside ONE inline-asm statement, so hipcc pads nothing):
  - the destination registers are preloaded with a sentinel, srcC is a zero
    block in other registers, the operands are all ones;
  - the MFMA writes A*B (= K for the float forms, K for the i8 form);
  - after N wait states (s_nop), RAW: four v_mov_b32 copy destination
    registers 0..3 out (they read at N, N+1, N+2, N+3 states); WAW: one
    v_mov_b32 writes 7.0 into destination register 0, then (after 32 states)
    registers 0..3 are copied out — 7.0 must survive.
A slot that reads the sentinel or any value but the product came too early.

    python tools/probe_mfma_hazard.py build    # here: writes + compiles tools/_hz/probe_mfma_hazard
    python tools/probe_mfma_hazard.py run      # on the GPU box: the table, and a JSON summary

The compiler's own pad for each form (what hipcc inserts before a VALU read
of the destination) is read from a compiled reference kernel and printed
beside the hardware number (tools/isa_hazard.py uses the larger of the two).
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_hz")
SRC = os.path.join(OUT, "probe_mfma_hazard.hip")
BIN = os.path.join(OUT, "probe_mfma_hazard")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
NMAX = 20

# name: (mnemonic, D regs, A regs, B regs, A bits, expected D bits per register, chain-first mnemonic or None)
F16 = "0x3C003C00"
I8 = "0x01010101"
ONE = "0x3F800000"
FORMS = {
    "16x16x16_f16": ("v_mfma_f32_16x16x16_f16", 4, 2, 2, F16, 0x41800000, None),   # 16.0
    "16x16x32_f16": ("v_mfma_f32_16x16x32_f16", 4, 4, 4, F16, 0x42000000, None),   # 32.0
    "16x16x64_i8": ("v_mfma_i32_16x16x64_i8", 4, 4, 4, I8, 64, None),               # int 64
    "32x32x16_f16": ("v_mfma_f32_32x32x16_f16", 16, 4, 4, F16, 0x41800000, None),  # 16.0
    "16x16x4_f32": ("v_mfma_f32_16x16x4_f32", 4, 1, 1, ONE, 0x40800000, None),     # 4.0
    "4x4x1_16b_f32": ("v_mfma_f32_4x4x1_16b_f32", 4, 1, 1, ONE, 0x3F800000, None),  # 1.0
    "32x32x2_f32": ("v_mfma_f32_32x32x2_f32", 16, 1, 1, ONE, 0x40000000, None),     # 2.0
    # the bank kernels' chain: a 16x16x32 then a 16x16x16 on the same accumulator (32 + 16 = 48.0)
    "chain_32_then_16": ("v_mfma_f32_16x16x16_f16", 4, 2, 2, F16, 0x42400000, "v_mfma_f32_16x16x32_f16"),
    "chain_16_then_32": ("v_mfma_f32_16x16x32_f16", 4, 4, 4, F16, 0x42400000, "v_mfma_f32_16x16x16_f16_first"),
    "chain_32_then_32": ("v_mfma_f32_16x16x32_f16", 4, 4, 4, F16, 0x42800000, "v_mfma_f32_16x16x32_f16"),
    "chain_16_then_16": ("v_mfma_f32_16x16x16_f16", 4, 2, 2, F16, 0x42000000, "v_mfma_f32_16x16x16_f16_first"),
}
SENT = "0x7FC0DEAD"
D0, A0, B0, C0 = 100, 116, 120, 124  # register bases (D up to 16, A/B up to 4, C up to 16)


def rng(base, n):
    return f"v{base}" if n == 1 else f"v[{base}:{base + n - 1}]"


def nops(n):
    s = ""
    while n > 0:
        k = min(n, 16)
        s += f"s_nop {k - 1}\\n"
        n -= k
    return s


def filler(kind, g):
    """g wait states of one kind: s_nop states, VALU moves (unrelated registers) or SALU adds"""
    if kind == "nop":
        return nops(g)
    if kind == "valu":
        return "".join("v_mov_b32 v115, v114\\n" for _ in range(g))
    return "".join("s_add_u32 s90, s90, 1\\n" for _ in range(g))


def kernel(name, form, n, mode, gap=0, fill="nop"):
    mn, nd, na, nb, abits, _, first = FORMS[form]
    body = ""
    for i in range(nd):
        body += f"v_mov_b32 v{D0 + i}, {SENT}\\n"
    for i in range(nd):
        body += f"v_mov_b32 v{C0 + i}, 0\\n"
    for i in range(4):
        body += f"v_mov_b32 v{A0 + i}, {abits}\\nv_mov_b32 v{B0 + i}, {abits}\\n"
    body += "s_nop 7\\n"
    if first:  # chain: the 16x16x32 writes D from zero C, the probed MFMA accumulates onto D
        fm = first.replace("_first", "")
        fw = 2 if "16x16x16" in fm else 4
        body += f"{fm} {rng(D0, nd)}, {rng(A0, fw)}, {rng(B0, fw)}, {rng(C0, nd)}\\n" + filler(fill, gap)
        body += f"{mn} {rng(D0, nd)}, {rng(A0, na)}, {rng(B0, nb)}, {rng(D0, nd)}\\n"
    else:
        body += f"{mn} {rng(D0, nd)}, {rng(A0, na)}, {rng(B0, nb)}, {rng(C0, nd)}\\n"
    body += nops(n)
    if mode == "waw":
        body += f"v_mov_b32 v{D0}, 0x40E00000\\n" + nops(32)
    body += "".join(f"v_mov_b32 %{i}, v{D0 + i}\\n" for i in range(4)) + nops(32)
    regs_ = list(range(D0, D0 + nd)) + list(range(A0, A0 + 4)) + list(range(B0, B0 + 4)) + list(range(C0, C0 + nd))
    clob = ", ".join([f'"v{r}"' for r in regs_ + [114, 115]] + ['"s90"'])
    return f"""
extern "C" __global__ void {name}(unsigned* out) {{
  unsigned r0, r1, r2, r3;
  asm volatile("{body}" : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
               : : {clob});
  unsigned* o = out + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 4;
  o[0] = r0; o[1] = r1; o[2] = r2; o[3] = r3;
}}
"""


GAPS = (0, 1, 2, 3, 4, 5, 6, 8, 10, 12, 16)


# VALU write -> MFMA operand read: srcC (or srcA) written by v_mov_b32 in the order
# component 3, 2, 1, 0 (component c written c + 1 states before the gap's end), g wait states, then
# the MFMA; its result read 32 states later.  A component read before its write landed keeps the
# sentinel (srcC) or the stale operand value.
VALU_FORMS = {
    "valu_srcC_16x16x16": ("v_mfma_f32_16x16x16_f16", 2, "C"),
    "valu_srcC_16x16x32": ("v_mfma_f32_16x16x32_f16", 4, "C"),
    "valu_srcA_16x16x32": ("v_mfma_f32_16x16x32_f16", 4, "A"),
}
VGAPS = tuple(range(0, 13))


def valu_kernel(name, form, g):
    mn, w, which = VALU_FORMS[form]
    body = ""
    for i in range(4):
        body += f"v_mov_b32 v{D0 + i}, {SENT}\\nv_mov_b32 v{C0 + i}, {SENT}\\n"
    for i in range(4):
        body += f"v_mov_b32 v{A0 + i}, {F16 if which == 'C' else '0x7C007C00'}\\nv_mov_b32 v{B0 + i}, {F16}\\n"
    body += "s_nop 15\\ns_nop 15\\n"
    if which == "C":  # the real srcC (zeros), component 3 first .. component 0 last
        for i in (3, 2, 1, 0):
            body += f"v_mov_b32 v{C0 + i}, 0\\n"
    else:  # srcA: the real operand (ones) over an inf-filled A, register 3 first .. 0 last
        for i in (3, 2, 1, 0):
            body += f"v_mov_b32 v{A0 + i}, {F16}\\n"
        for i in range(4):
            body += ""
    body += nops(g)
    cop = rng(C0, 4) if which == "C" else "0"
    body += f"{mn} {rng(D0, 4)}, {rng(A0, w)}, {rng(B0, w)}, {cop}\\n" + nops(32)
    body += "".join(f"v_mov_b32 %{i}, v{D0 + i}\\n" for i in range(4)) + nops(32)
    clob = ", ".join(f'"v{r}"' for r in list(range(D0, D0 + 4)) + list(range(A0, A0 + 4)) + list(range(B0, B0 + 4))
                     + list(range(C0, C0 + 4)))
    return f"""
extern "C" __global__ void {name}(unsigned* out) {{
  unsigned r0, r1, r2, r3;
  asm volatile("{body}" : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3) : : {clob});
  unsigned* o = out + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 4;
  o[0] = r0; o[1] = r1; o[2] = r2; o[3] = r3;
}}
"""


def names():
    for form in FORMS:
        for mode in ("raw", "waw"):
            for n in range(NMAX + 1):
                yield form, mode, n, 0, f"hz_{form}_{mode}_{n}".replace("x", "X")
    # chained forms: g wait states between the two MFMAs, the read n states after the second
    for form in [f for f in FORMS if FORMS[f][6]]:
        for g in GAPS:
            for n in range(0, NMAX + 1, 2):
                yield form, f"gap{g}", n, g, f"hz_{form}_gap{g}_{n}".replace("x", "X")
    # mixed-shape chains with VALU / SALU fillers in the gap (the read 20 states after)
    for form in ("chain_32_then_16", "chain_16_then_32"):
        for kind in ("valu", "salu"):
            for g in range(0, 9):
                yield form, f"{kind}{g}", 20, g, f"hz_{form}_{kind}{g}".replace("x", "X")


def build():
    os.makedirs(OUT, exist_ok=True)
    src = ['#include <hip/hip_runtime.h>\n#include <cstdio>\n#include <cstring>\n#include <vector>\n']
    table = []
    for form, mode, n, g, nm in names():
        kind = "valu" if mode.startswith("valu") else "salu" if mode.startswith("salu") else "nop"
        src.append(kernel(nm, form, n, mode if mode in ("raw", "waw") else "raw", g, kind))
        exp = FORMS[form][5]
        table.append(f'  {{"{form}", "{mode}", {n}, {nm}, {exp}u}},')
    for form, (mn, w, which) in VALU_FORMS.items():
        exp = 0x41800000 if "16x16x16" in mn else 0x42000000  # K ones: 16.0 / 32.0
        for g in VGAPS:
            nm = f"hz_{form}_g{g}".replace("x", "X")
            src.append(valu_kernel(nm, form, g))
            table.append(f'  {{"{form}", "vgap", {g}, {nm}, {exp}u}},')
    src.append("""
struct Case { const char* form; const char* mode; int n; void (*k)(unsigned*); unsigned exp; };
static const Case cases[] = {
""" + "\n".join(table) + """
};
int main(int argc, char** argv) {
  const int blocks = 512, reps = 4;
  unsigned* d;
  if (hipMalloc(&d, (size_t)blocks * 256 * 4 * 4) != hipSuccess) return 1;
  std::vector<unsigned> h((size_t)blocks * 256 * 4);
  printf("[\\n");
  bool firstline = true;
  for (const Case& c : cases) {
    for (int threads : {64, 256}) {
      long bad[4] = {0, 0, 0, 0};
      for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(c.k, dim3(blocks), dim3(threads), 0, 0, d);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\\n"); return 1; }
        hipMemcpy(h.data(), d, (size_t)blocks * threads * 16, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < (size_t)blocks * threads; ++i)
          for (int s = 0; s < 4; ++s) {
            const unsigned want = (s == 0 && c.mode[0] == 'w') ? 0x40E00000u : c.exp;
            bad[s] += h[i * 4 + s] != want;
          }
      }
      printf("%s{\\"form\\": \\"%s\\", \\"mode\\": \\"%s\\", \\"n\\": %d, \\"threads\\": %d, \\"bad\\": [%ld, %ld, %ld, %ld]}",
             firstline ? "" : ",\\n", c.form, c.mode, c.n, threads, bad[0], bad[1], bad[2], bad[3]);
      firstline = false;
    }
  }
  printf("\\n]\\n");
  return 0;
}
""")
    open(SRC, "w").write("".join(src))
    subprocess.run([HIPCC, "-O1", "--offload-arch=gfx950", SRC, "-o", BIN], check=True)
    print(BIN)


def run():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-2000:])
        sys.exit(r.returncode)
    rows = json.loads(r.stdout)
    summary = {}
    for form in ("chain_32_then_16", "chain_16_then_32"):
        for kind in ("valu", "salu"):
            sel = [x for x in rows if x["form"] == form and x["mode"].startswith(kind) and x["threads"] == 64]
            need = min([int(x["mode"][len(kind):]) for x in sel
                        if all(sum(y["bad"]) == 0 for y in sel if int(y["mode"][len(kind):]) >= int(x["mode"][len(kind):]))]
                       or [None])
            summary[f"{form}/{kind}_fill"] = {x["mode"]: x["bad"] for x in sel}
            print(f"{form:18s} {kind} fillers: clean from {need} ({[(x['mode'], x['bad']) for x in sel]})")
    for form in VALU_FORMS:
        sel = [x for x in rows if x["form"] == form and x["threads"] == 64]
        for x in sel:
            print(f"{form:20s} gap {x['n']:2d}: bad per component {x['bad']}")
        summary[form] = {x["n"]: x["bad"] for x in sel}
    for form in [f for f in FORMS if FORMS[f][6]]:
        for g in GAPS:
            sel = [x for x in rows if x["form"] == form and x["mode"] == f"gap{g}"]
            clean = [x["n"] for x in sel if sum(x["bad"]) == 0]
            bad01 = [x["n"] for x in sel if x["bad"][0] or x["bad"][1]]
            summary[f"{form}/gap{g}"] = {"clean_reads_at_n": clean, "slots01_bad_at_n": bad01}
            print(f"{form:18s} gap {g:2d}: reads clean at n = {clean}")
    for form in FORMS:
        for mode in ("raw", "waw"):
            sel = [x for x in rows if x["form"] == form and x["mode"] == mode]
            # smallest N from which every later N is clean in every slot (slot s reads at N + s states)
            need = None
            for n in range(NMAX, -1, -1):
                if all(sum(x["bad"]) == 0 for x in sel if x["n"] >= n):
                    need = n
            # per slot: first clean state count (slot s at n + s)
            first = []
            for s in range(4):
                ok = [x["n"] + (s if mode == "raw" else 0) for x in sel if x["bad"][s] == 0 and
                      all(y["bad"][s] == 0 for y in sel if y["n"] >= x["n"])]
                first.append(min(ok) if ok else None)
            summary[f"{form}/{mode}"] = {"clean_from_n": need, "slot_clean_at_states": first,
                                         "bad_at": {x["n"]: x["bad"] for x in sel if sum(x["bad"]) and x["threads"] == 64}}
            print(f"{form:18s} {mode}: clean from N = {need}; per slot first clean state {first}")
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(HERE)), "gpurun_out", "mfma_hazard.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump({"rows": rows, "summary": summary}, open(out, "w"), indent=1)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
