"""Idle gap before each kernel class over the last frames of a kernel trace (diagnostic): from the last k_render_init on,
mean gap (start minus the previous kernel's end, same trace) per kernel name.
Usage: python tools/gap_summary.py <kernel_trace.csv> [frames]"""
import collections
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
              for r in csv.DictReader(open(sys.argv[1])))
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 2
inits = [i for i, r in enumerate(rows) if "k_render_init" in r[2]]
s = inits[-frames]
gaps = collections.defaultdict(list)
prev_end = rows[s][0]
for st, en, name in rows[s:]:
    gaps[name[:70]].append((st - prev_end) / 1e3)
    prev_end = max(prev_end, en)
tot = 0.0
for name, g in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
    pos = [x for x in g if x > 0]
    tot += sum(pos)
    print(f"{name:70s} n={len(g):4d} mean gap {sum(g) / len(g):7.2f} us  positive sum {sum(pos):8.1f} us")
print(f"total positive gap over {frames} frames: {tot:.1f} us")
