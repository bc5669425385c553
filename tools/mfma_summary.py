"""Per-kernel MFMA utilisation from one rocprofv3 --pmc pass.

Usage: python tools/mfma_summary.py COUNTER_COLLECTION.csv TAG [out.json]

The pass (tools/gpu.sh mfma) collects, per dispatch:
  SQ_INSTS_VALU_MFMA_MOPS_F16 / _F32   MFMA work in units of 512 FLOP
                                       (rocprofv3's MfmaFlops* = MOPS x 512)
  SQ_VALU_MFMA_BUSY_CYCLES             cycles the matrix cores were busy,
                                       summed over the SIMDs
  SQ_BUSY_CU_CYCLES                    cycles the CUs were busy, summed
  GRBM_GUI_ACTIVE                      GPU-active cycles of the dispatch,
                                       summed over the 8 XCDs (calibrated on
                                       the encoder FFN1 GEMM: 11.6 M for a
                                       0.70 ms dispatch = 8 x 2.07 GHz)
and the dispatch's start/end timestamps.  Per kernel it reports hardware
MFMA FLOP per launch, the achieved rate over the average dispatch span, and
MfmaUtil = MFMA busy cycles / (GUI-active cycles per XCD x 1024 SIMDs)
(rocprofv3's own MfmaUtil expression, reduce(SQ_VALU_MFMA_BUSY_CYCLES,sum)
/ (reduce(GRBM_GUI_ACTIVE,max) * SIMD_NUM), with max over XCDs taken as the
sum / 8), and the CU-busy share SQ_BUSY_CU_CYCLES / (cycles x 256 CUs).  The 'path' entry sums every
kernel of the profiled run: the share of the GPU-active time the matrix
cores were busy.  F16 counts the split-fp16 products as issued (3 fp16
products per fp32 multiply-add), so its FLOPs are 3x the algorithmic fp32
FLOPs of those kernels."""
import collections
import csv
import json
import re
import sys

SIMDS, CUS, XCDS = 1024, 256, 8
F16_PEAK, F32_PEAK = 2516.6, 157.3  # TFLOP/s dense (MI355X_MICROARCH.md)
CTRS = ("SQ_INSTS_VALU_MFMA_MOPS_F16", "SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_VALU_MFMA_BUSY_CYCLES",
        "SQ_BUSY_CU_CYCLES", "GRBM_GUI_ACTIVE")


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("nd::", "")


def main():
    rows = collections.defaultdict(dict)  # dispatch -> {counter: value, name, ns}
    for r in csv.DictReader(open(sys.argv[1])):
        d = rows[r["Dispatch_Id"]]
        d["name"] = short(r["Kernel_Name"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    per = collections.defaultdict(lambda: collections.Counter())
    tot = collections.Counter()
    for d in rows.values():
        k = per[d["name"]]
        k["n"] += 1
        k["ns"] += d["ns"]
        for c in CTRS:
            k[c] += d.get(c, 0.0)
            tot[c] += d.get(c, 0.0)
        tot["ns"] += d["ns"]
    out = {"tag": sys.argv[2], "note": __doc__.split("\n\n")[1].replace("\n", " "), "kernels": {}}
    for name, k in sorted(per.items(), key=lambda kv: -kv[1]["ns"]):
        if k["SQ_INSTS_VALU_MFMA_MOPS_F16"] + k["SQ_INSTS_VALU_MFMA_MOPS_F32"] == 0:
            continue
        n = k["n"]
        f16 = k["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512 / n
        f32 = k["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512 / n
        s = k["ns"] / n * 1e-9
        out["kernels"][name] = {
            "launches": n, "avg_us": round(s * 1e6, 3),
            "f16_flop_per_launch": f16, "f32_flop_per_launch": f32,
            "f16_tflops": round(f16 / s / 1e12, 2), "f32_tflops": round(f32 / s / 1e12, 2),
            "f16_frac_peak": round(f16 / s / 1e12 / F16_PEAK, 4), "f32_frac_peak": round(f32 / s / 1e12 / F32_PEAK, 4),
            "mfma_util": round(k["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, k["GRBM_GUI_ACTIVE"] / XCDS * SIMDS), 4),
            "cu_busy": round(k["SQ_BUSY_CU_CYCLES"] / max(1.0, k["GRBM_GUI_ACTIVE"] / XCDS * CUS), 4),
            # the clock the dispatches ran at: GUI-active cycles per XCD over their span
            "clock_ghz": round(k["GRBM_GUI_ACTIVE"] / XCDS / max(1.0, k["ns"]), 3),
        }
    s = tot["ns"] * 1e-9
    out["path"] = {
        "kernel_seconds": round(s, 6),
        "f16_tflops": round(tot["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512 / s / 1e12, 2),
        "f32_tflops": round(tot["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512 / s / 1e12, 2),
        "mfma_util": round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, tot["GRBM_GUI_ACTIVE"] / XCDS * SIMDS), 4),
        "cu_busy": round(tot["SQ_BUSY_CU_CYCLES"] / max(1.0, tot["GRBM_GUI_ACTIVE"] / XCDS * CUS), 4),
        "note": "every dispatch of the profiled run (weights prep, encoder, decoder steps, search)",
    }
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js)
    print(js[:3000])


if __name__ == "__main__":
    main()
