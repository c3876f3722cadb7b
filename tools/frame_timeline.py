"""Summarise a rocprofv3 kernel trace of tools/probe_render.py-style runs: for the last
render frame (k_dense_records .. k_accum_tonemap), list every kernel with its start
offset, duration and the idle gap before it (diagnostic).
Usage: python tools/frame_timeline.py <kernel_trace.csv> [out.txt]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")))
rows.sort()
starts = [i for i, r in enumerate(rows) if "k_dense_records" in r[2]]
s = starts[-2] if len(starts) > 1 else starts[-1]
e = next(i for i in range(s, len(rows)) if "k_shade" in rows[i][2] or "k_accum_tonemap" in rows[i][2])
out = []
t0 = rows[s][0]
busy = 0
prev_end = t0
for st, en, name in rows[s:e + 1]:
    gap = st - prev_end
    out.append(f"{(st - t0) / 1e3:9.1f} us  dur {(en - st) / 1e3:8.1f}  gap {gap / 1e3:7.1f}  {name[:70]}")
    busy += en - st
    prev_end = en
total = rows[e][1] - t0
out.append(f"frame {total / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, idle {(total - busy) / 1e3:.1f} us")
txt = "\n".join(out)
print(txt)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(txt + "\n")
