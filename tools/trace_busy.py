"""How busy the GPU is over time in a rocprofv3 --kernel-trace CSV: per window
of W ms, the share of wall time with at least one kernel running (the union
of kernel intervals) and the mean number of kernels running at once; then the
same over the windows whose mean concurrency is >= 1.3 (the pooled leg of a
bench run) and < 1.3 (its one-call leg), and the idle gaps of the pooled
windows by the kernel that follows them.
Usage: python tools/trace_busy.py run_kernel_trace.csv [W_ms]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    W = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 5e6
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 re.sub(r"\(.*$", "", re.sub(r"^void ", "", r["Kernel_Name"])).replace("nd::", "")[:50])
                for r in rows)
    t0, t1 = iv[0][0], max(e for _, e, _ in iv)
    nwin = int((t1 - t0) // W) + 1
    busy = [0.0] * nwin
    conc = [0.0] * nwin
    for s, e, _ in iv:  # summed kernel time per window
        a = s
        while a < e:
            k = int((a - t0) // W)
            b = min(e, t0 + (k + 1) * W)
            conc[k] += (b - a) / W
            a = b
    # union of intervals
    cur_s, cur_e = iv[0][0], iv[0][1]
    unions = []
    gaps = []  # (gap_ns, kernel that ends it, start time)
    for s, e, n in iv[1:]:
        if s > cur_e:
            unions.append((cur_s, cur_e))
            gaps.append((s - cur_e, n, s))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    unions.append((cur_s, cur_e))
    for s, e in unions:
        a = s
        while a < e:
            k = int((a - t0) // W)
            b = min(e, t0 + (k + 1) * W)
            busy[k] += (b - a) / W
            a = b
    print(f"{len(iv)} kernels over {(t1 - t0) / 1e6:.1f} ms, windows of {W / 1e6:g} ms")
    for k in range(nwin):
        print(f"  window {k:3d}: busy {busy[k]:.3f}  kernels at once {conc[k]:.2f}")
    for name, sel in (("pooled (>= 1.3 at once)", lambda k: conc[k] >= 1.3),
                      ("one call (< 1.3 at once)", lambda k: 0.05 < conc[k] < 1.3)):
        ks = [k for k in range(nwin) if sel(k)]
        if ks:
            print(f"{name}: {len(ks)} windows, busy {sum(busy[k] for k in ks) / len(ks):.3f}, "
                  f"kernels at once {sum(conc[k] for k in ks) / len(ks):.2f}")
    pooled = {k for k in range(nwin) if conc[k] >= 1.3}
    by = defaultdict(lambda: [0, 0])
    for g, n, s in gaps:
        if int((s - t0) // W) in pooled and g < 1e6:
            by[n][0] += 1
            by[n][1] += g
    tot = sum(v[1] for v in by.values())
    print(f"idle gaps inside pooled windows: {tot / 1e6:.2f} ms in total; by the kernel that ends them:")
    for n, (c, g) in sorted(by.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {n:50s} n={c:6d} total {g / 1e3:9.1f} us  mean {g / c / 1e3:6.2f} us")


if __name__ == "__main__":
    main()
