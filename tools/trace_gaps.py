"""Summarise a rocprofv3 kernel_trace.csv: per-kernel mean duration, and the mean idle gap before
each kernel (start of this kernel - end of the previous one on the same queue)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[skip:]
dur = defaultdict(list)
gap = defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
    dur[name].append(e - s)
    if prev_end is not None:
        gap[name].append(s - prev_end)
    prev_end = e
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
busy = sum(sum(v) for v in dur.values()) / 1e3
print(f"span {span:.1f} us, busy {busy:.1f} us ({100 * busy / span:.1f}%), kernels {len(rows)}")
for name in sorted(dur, key=lambda k: -sum(dur[k])):
    d = dur[name]
    g = gap.get(name, [0])
    print(f"{name:60s} n={len(d):6d} mean={sum(d) / len(d) / 1e3:8.2f}us total={sum(d) / 1e3:10.1f}us "
          f"gap_before={sum(g) / len(g) / 1e3:7.2f}us")
