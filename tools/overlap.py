"""Fraction of kernel time that overlaps another kernel (rocprofv3 kernel_trace.csv), per stream pair."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
    ev.append((s, e, q, r["Kernel_Name"][:40]))
ev.sort()
busy = sum(e - s for s, e, _, _ in ev)
# union of intervals
union = 0
cur_s, cur_e = None, None
for s, e, _, _ in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
span = ev[-1][1] - ev[0][0]
print(f"kernels {len(ev)}  sum of durations {busy/1e6:.1f} ms  union {union/1e6:.1f} ms  span {span/1e6:.1f} ms  "
      f"overlap {(busy-union)/1e6:.1f} ms")
qs = sorted(set(q for _, _, q, _ in ev))
print("streams/queues:", qs[:10])
