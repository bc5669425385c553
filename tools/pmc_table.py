"""Average PMC counters per kernel from rocprofv3 counter_collection.csv files."""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").replace("nd::", "")[:60]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in acc.items():
    if k.startswith("__amd") or k.startswith("at::"):
        continue
    print(f"{k}  dur~{sum(dur[k])/len(dur[k]):.1f}us")
    for c, v in sorted(cs.items()):
        print(f"    {c:34s} {sum(v)/len(v):16.1f}")
