"""One rendered frame's kernels in launch order from a rocprofv3 kernel trace (diagnostic): start
offset and duration of every launch of the next-to-last frame, with its queue/stream, so the
pipelines' pass chains and their overlap can be read directly.
Usage: python tools/frame_passes.py <kernel_trace.csv> [out.txt]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ngp::", "")
    q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q,
                 int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)))
rows.sort()
starts = [i for i, r in enumerate(rows) if "k_dense_records" in r[2]]
seg = rows[starts[-2]:starts[-1]]
last = max(i for i, r in enumerate(seg) if "k_shade" in r[2])
seg = seg[:last + 1]
t0 = seg[0][0]
lines = [f"frame span {(max(e for _, e, *_ in seg) - t0) / 1e3:.1f} us, {len(seg)} launches"]
for s, e, n, q, g in seg:
    lines.append(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3} grid {g:>9}  {n[:60]}")
txt = "\n".join(lines) + "\n"
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(txt)
print(txt)
