"""One bench step's kernel timeline from a rocprofv3 kernel trace of bench.py: every kernel
from the second-to-last k_sample_count (training sampler) to the next one, with start
offset, duration and the idle gap before it, then per-kernel totals (diagnostic).
Usage: python tools/step_timeline.py <kernel_trace.csv> [out.txt]"""
import collections
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")))
rows.sort()
starts = [i for i, r in enumerate(rows) if "k_sample_count" in r[2]]
s, e = starts[-2], starts[-1]
out = []
t0 = rows[s][0]
busy = 0
prev_end = t0
tot = collections.OrderedDict()
for st, en, name in rows[s:e]:
    gap = st - prev_end
    out.append(f"{(st - t0) / 1e3:9.1f} us  dur {(en - st) / 1e3:8.1f}  gap {gap / 1e3:7.1f}  {name[:80]}")
    busy += en - st
    prev_end = en
    k = name[:80]
    n, d = tot.get(k, (0, 0))
    tot[k] = (n + 1, d + en - st)
total = rows[e][0] - t0
out.append(f"step {total / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, idle {(total - busy) / 1e3:.1f} us")
out.append("per kernel (launches, total us):")
for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    out.append(f"  {d / 1e3:8.1f} us  x{n:3d}  {k}")
txt = "\n".join(out)
print(txt)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(txt + "\n")
