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


def kernel(name, form, n, mode):
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
        body += f"{first} {rng(D0, nd)}, {rng(A0, 4)}, {rng(B0, 4)}, {rng(C0, nd)}\\n"
        body += f"{mn} {rng(D0, nd)}, {rng(A0, na)}, {rng(B0, nb)}, {rng(D0, nd)}\\n"
    else:
        body += f"{mn} {rng(D0, nd)}, {rng(A0, na)}, {rng(B0, nb)}, {rng(C0, nd)}\\n"
    body += nops(n)
    if mode == "waw":
        body += f"v_mov_b32 v{D0}, 0x40E00000\\n" + nops(32)
    body += "".join(f"v_mov_b32 %{i}, v{D0 + i}\\n" for i in range(4)) + nops(32)
    clob = ", ".join(f'"v{r}"' for r in list(range(D0, D0 + nd)) + list(range(A0, A0 + 4)) + list(range(B0, B0 + 4))
                     + list(range(C0, C0 + nd)))
    return f"""
extern "C" __global__ void {name}(unsigned* out) {{
  unsigned r0, r1, r2, r3;
  asm volatile("{body}" : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
               : : {clob});
  unsigned* o = out + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 4;
  o[0] = r0; o[1] = r1; o[2] = r2; o[3] = r3;
}}
"""


def names():
    for form in FORMS:
        for mode in ("raw", "waw"):
            for n in range(NMAX + 1):
                yield form, mode, n, f"hz_{form}_{mode}_{n}".replace("x", "X")


def build():
    os.makedirs(OUT, exist_ok=True)
    src = ['#include <hip/hip_runtime.h>\n#include <cstdio>\n#include <cstring>\n#include <vector>\n']
    table = []
    for form, mode, n, nm in names():
        src.append(kernel(nm, form, n, mode))
        exp = FORMS[form][5]
        table.append(f'  {{"{form}", "{mode}", {n}, {nm}, {exp}u}},')
    src.append("""
struct Case { const char* form; const char* mode; int n; void (*k)(unsigned*); unsigned exp; };
static const Case cases[] = {
""" + "\n".join(table) + """
};
int main(int argc, char** argv) {
  const int blocks = 2048, reps = 8;
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
