"""Per-kernel durations and the idle gaps before them inside one decoder step
of a rocprofv3 --kernel-trace CSV (one translate call = a dependent chain).
Usage: python tools/trace_gaps.py run_kernel_trace.csv [first_kernel_substring]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: re.sub(r"\(.*$", "", re.sub(r"^void ", "", n)).replace("nd::", "")[:60]
# consecutive kernel pairs within the decode loop (mem-attention neighbourhood)
dur = defaultdict(list)
gap = defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = short(r["Kernel_Name"])
    if prev_end is not None and 0 <= s - prev_end < 20000:
        gap[n].append(s - prev_end)
    dur[n].append(e - s)
    prev_end = e
tot_d = tot_g = 0
for n in sorted(dur, key=lambda k: -sum(dur[k])):
    d = sum(dur[n]) / len(dur[n]) / 1e3
    g = (sum(gap[n]) / len(gap[n]) / 1e3) if gap[n] else float("nan")
    print(f"{n:62s} n={len(dur[n]):6d} dur={d:8.2f} us  gap_before={g:6.2f} us")
