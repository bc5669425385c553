"""Cross-queue overlap in a rocprofv3 kernel trace (run_kernel_trace.csv).

  python tools/overlap_analyze.py gpurun_out/TAG/run_kernel_trace.csv [--last-ms 200]

Per queue: kernels, summed kernel time, first/last timestamps.  Overall:
union busy time (any kernel running), time with kernels of >= 2 queues
running at once, and the mean gap between consecutive kernels of one queue
(dispatch boundary).  Only the last ``--last-ms`` of the trace is used (the
timed iterations), so setup kernels do not dilute the numbers.
"""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--last-ms", type=float, default=0.0)
a = ap.parse_args()

rows = []
with open(a.csv) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"]))
rows.sort()
if a.last_ms > 0:
    t_end = max(r[1] for r in rows)
    rows = [r for r in rows if r[0] >= t_end - a.last_ms * 1e6]
byq = defaultdict(list)
for r in rows:
    byq[r[2]].append(r)
t0 = min(r[0] for r in rows)
t1 = max(r[1] for r in rows)
print(f"window {(t1 - t0) / 1e6:.3f} ms, {len(rows)} kernels")
for q, ks in sorted(byq.items()):
    busy = sum(e - s for s, e, _, _ in ks)
    gaps = [ks[i + 1][0] - ks[i][1] for i in range(len(ks) - 1)]
    gpos = [g for g in gaps if g > 0]
    print(f"queue {q}: {len(ks)} kernels, kernel time {busy / 1e6:.3f} ms, "
          f"mean gap {sum(gaps) / max(1, len(gaps)) / 1e3:.2f} us ({len(gpos)} positive), "
          f"span {(ks[-1][1] - ks[0][0]) / 1e6:.3f} ms")
# sweep: count active kernels per queue over time
ev = []
for s, e, q, _ in rows:
    ev.append((s, 1, q))
    ev.append((e, -1, q))
ev.sort(key=lambda x: (x[0], x[1]))
act = defaultdict(int)
last = ev[0][0]
union = multi = 0
for t, d, q in ev:
    dt = t - last
    nq = sum(1 for v in act.values() if v > 0)
    if nq >= 1:
        union += dt
    if nq >= 2:
        multi += dt
    act[q] += d
    last = t
print(f"union busy {union / 1e6:.3f} ms ({union / (t1 - t0):.1%} of window), "
      f">=2 queues active {multi / 1e6:.3f} ms ({multi / max(1, union):.1%} of busy)")
# the top kernels by time per queue
for q, ks in sorted(byq.items()):
    agg = defaultdict(lambda: [0, 0])
    for s, e, _, n in ks:
        agg[n[:60]][0] += 1
        agg[n[:60]][1] += e - s
    top = sorted(agg.items(), key=lambda kv: -kv[1][1])[:6]
    print(f"queue {q} top: " + "; ".join(f"{n} x{c} {t / c / 1e3:.1f}us" for n, (c, t) in top))
