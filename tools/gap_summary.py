"""Idle gap before each kernel class over the last frames of a kernel trace (diagnostic): from the last k_render_init on,
mean gap (start minus the previous kernel's end, same trace) per kernel name.
Usage: python tools/gap_summary.py <kernel_trace.csv> [frames] [anchor kernel, default k_render_init]"""
import collections
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
              for r in csv.DictReader(open(sys.argv[1])))
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 2
anchor = sys.argv[3] if len(sys.argv) > 3 else "k_render_init"
inits = [i for i, r in enumerate(rows) if anchor in r[2]]
s = inits[-frames]
gaps = collections.defaultdict(list)
busy = collections.defaultdict(float)
prev_end = rows[s][0]
for st, en, name in rows[s:]:
    gaps[name[:70]].append((st - prev_end) / 1e3)
    busy[name[:70]] += (en - st) / 1e3
    prev_end = max(prev_end, en)
span = (prev_end - rows[s][0]) / 1e3
print(f"span {span:.1f} us over {frames} frames/steps, kernel time {sum(busy.values()):.1f} us")
for name, b in sorted(busy.items(), key=lambda kv: -kv[1]):
    print(f"  busy {name:70s} {b / frames:8.1f} us per frame/step  n={len(gaps[name]) / frames:.1f}")
tot = 0.0
for name, g in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
    pos = [x for x in g if x > 0]
    tot += sum(pos)
    print(f"{name:70s} n={len(g):4d} mean gap {sum(g) / len(g):7.2f} us  positive sum {sum(pos):8.1f} us")
print(f"total positive gap over {frames} frames: {tot:.1f} us")
