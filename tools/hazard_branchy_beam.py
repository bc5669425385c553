"""Round-4 finding, explained: the branchy rescale of the
beam digit-bank kernel.

Rebuilds the two-phase dec_bank_d8_beam_kernel from git history (the last
commit that shipped it), puts back the branch around its accumulator rescale
that round 4 saw return wrong components 0-1 of the second dim block, compiles
both forms for gfx950 and reports, per form, every instruction that reads or
writes a 16x16x16_f16 MFMA's destination within 24 wait states of it, and
every MFMA of another form that accumulates onto an MFMA's destination within
isa_hazard.MIXED_SRCC states (tools/isa_hazard.py's walk over all paths).  CPU only; no GPU run.

    python tools/hazard_branchy_beam.py [COMMIT] > profiles/r05_hazard_branchy_beam.txt
"""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import isa_hazard as H  # noqa: E402
import re  # noqa: E402

COMMIT = sys.argv[1] if len(sys.argv) > 1 else "e81496e"  # round 5, before the kernel's deletion
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
         "-I" + os.path.join(ROOT, "nanodecoder_amd", "csrc"), "-I" + os.path.join(ROOT, "include"),
         "--cuda-device-only", "-S"]
FREE = """      const f32x4 sc4 = *reinterpret_cast<const f32x4*>(lb + BB_SC + b * 64 + 16 * g);
      ua[b][0] *= sc4;
      ua[b][1] *= sc4;"""
BRANCHY = """      const f32x4 sc4 = *reinterpret_cast<const f32x4*>(lb + BB_SC + b * 64 + 16 * g);
      if (__any(sc4[0] != 1.f || sc4[1] != 1.f || sc4[2] != 1.f || sc4[3] != 1.f)) {
        ua[b][0] *= sc4;
        ua[b][1] *= sc4;
      }"""


def listing(src, tmp, name):
    path = os.path.join(tmp, name + ".hip")
    open(path, "w").write(src)
    out = os.path.join(tmp, name + ".s")
    subprocess.run([HIPCC] + FLAGS + [path, "-o", out], check=True, capture_output=True)
    return open(out).read()


def main():
    src = subprocess.run(["git", "-C", ROOT, "show", f"{COMMIT}:nanodecoder_amd/csrc/bank8.hip"], check=True,
                         capture_output=True, text=True).stdout
    assert FREE in src, "the branch-free rescale is not in that commit's bank8.hip"
    H.REQUIRED = {k: 24 for k in H.REQUIRED}  # report every toucher within 24 states
    with tempfile.TemporaryDirectory() as tmp:
        # the kernels live in bank8.hip beside common.hpp etc.: compile from a copy next to csrc's headers
        for tag, text in (("branch-free (shipped in round 4)", src), ("branchy (round 4's wrong results)",
                                                                     src.replace(FREE, BRANCHY))):
            asm = listing(text, tmp, "bank8_" + tag.split()[0].replace("-", "_"))
            res = H.scan(asm, r"dec_bank_d8_beam_kernelILi2E", every=True)
            print(f"== {tag}: dec_bank_d8_beam_kernel<2> (tools/bb_debug.py ran rpc 2)")
            for name, hz in res.items():
                rows = sorted((x for x in hz if "16x16x16" in x[0] and not x[1].startswith("v_mfma")),
                              key=lambda x: x[2])
                if not rows:
                    print("   no instruction touches a 16x16x16_f16 destination within 24 states")
                for mf, h, st, _ in rows[:12]:
                    print(f"   {st:2d} states after {mf}\n      -> {h}")
                # the mixed-form srcC chain (hardware-probed, tools/probe_mfma_hazard.py): an MFMA of
                # another form accumulating onto the destination within MIXED_SRCC states
                mixed = sorted({(mf, h, st) for mf, h, st, need in hz
                                if need == H.MIXED_SRCC and h.startswith("v_mfma")}, key=lambda x: x[2])
                print(f"   mixed-form srcC chains within {H.MIXED_SRCC} states: {len(mixed)}")
                for mf, h, st in mixed[:8]:
                    print(f"   {st:2d} states after {mf}\n      -> {h}")
            # a VALU result read by an MFMA operand too soon (srcC within 1 state, srcA / srcB within 2)
            for name, (ins, labels) in H.parse(asm).items():
                if not re.search(r"dec_bank_d8_beam_kernelILi2E", name):
                    continue
                vm = H.scan_valu_to_mfma(ins, labels)
                print(f"   VALU results read by an MFMA inside the probed window: {len(vm)}")
                for v, mf, st, need in vm[:8]:
                    print(f"   {st} states (needs {need}) from {v}\n      -> {mf}")


if __name__ == "__main__":
    main()
