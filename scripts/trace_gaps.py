"""Per-step kernel timeline from a rocprofv3 kernel_trace.csv: for every step (a run of
kernels starting at one named first kernel), each kernel's duration and the idle gap
before it, as medians over the steps.  Usage: trace_gaps.py <kernel_trace.csv> <first>"""
import collections
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2]
steps, cur = [], None
for r in rows:
    name = r["Kernel_Name"]
    if first in name:
        cur = []
        steps.append(cur)
    if cur is not None:
        cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
steps = steps[len(steps) // 4:]  # past the warmup
steps = [s[:[i for i, k in enumerate(s) if "rocclr" not in k[0]][-1] + 1] for s in steps]
common = collections.Counter(tuple(k[0] for k in s) for s in steps).most_common(1)[0][0]
shape = [s for s in steps if tuple(k[0] for k in s) == common]
print(f"steps {len(shape)} of {len(steps)} with the commonest kernel sequence")
n = len(shape[0])
for i in range(n):
    d = statistics.median((s[i][2] - s[i][1]) / 1e3 for s in shape)
    g = statistics.median((s[i][1] - s[i - 1][2]) / 1e3 for s in shape) if i else 0.0
    print(f"  gap {g:7.2f} us  run {d:8.2f} us  {shape[0][i][0][:60]}")
span = statistics.median((s[-1][2] - s[0][1]) / 1e3 for s in shape)
nxt = statistics.median((b[0][1] - a[-1][2]) / 1e3 for a, b in zip(shape, shape[1:]))
print(f"  first start -> last end {span:.2f} us; last end -> next step's first start {nxt:.2f} us")
