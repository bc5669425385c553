"""Per-launch view of a rocprofv3 --kernel-trace CSV (run on the GPU box, where the trace is; the summary is small
enough to copy back).  For the busiest kernels: launch count and duration quantiles; for the kernels named by
--series, the durations of their last N launches in order (one decoder step = one launch per layer), so a beam
call's steady part and its tail show separately.

    python tools/trace_steps.py run_kernel_trace.csv [--series ctx_attention self_attention] [--last 300]
"""
import argparse
import csv
from collections import defaultdict

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--series", nargs="*", default=["dec_ctx_attention", "dec_self_attention", "beam_step"])
    ap.add_argument("--last", type=int, default=300)
    ap.add_argument("--top", type=int, default=14)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    name_key = "Kernel_Name" if "Kernel_Name" in rows[0] else "KernelName"
    by = defaultdict(list)
    seq = []
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n = r[name_key]
        by[n].append((int(r["Start_Timestamp"]), d))
        seq.append((int(r["Start_Timestamp"]), n, d))
    tot = sorted(by.items(), key=lambda kv: -sum(d for _, d in kv[1]))
    print("kernel | launches | total ms | p10 p50 p90 max us")
    for n, v in tot[:a.top]:
        d = np.array([x[1] for x in v])
        print(f"{n[:90]} | {len(d)} | {d.sum() / 1e3:.2f} | "
              f"{np.percentile(d, 10):.1f} {np.percentile(d, 50):.1f} {np.percentile(d, 90):.1f} {d.max():.1f}")
    seq.sort()
    for pat in a.series:
        v = [(t, n, d) for t, n, d in seq if pat in n]
        if not v:
            continue
        last = v[-a.last:]
        print(f"\n{pat}: last {len(last)} launches (us, in order; template in brackets when it changes)")
        out, prev = [], None
        for _, n, d in last:
            tag = n[n.find("<"):n.find(">") + 1] if "<" in n else ""
            if tag != prev:
                out.append(f"[{tag}]")
                prev = tag
            out.append(f"{d:.0f}")
        print(" ".join(out))


if __name__ == "__main__":
    main()
