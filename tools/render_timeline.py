"""Overlap of the render's kernels on the GPU from a rocprofv3 kernel trace (diagnostic): for each
of the last frames (k_dense_records .. the last k_shade), the frame span, the time with 0, 1,
2, 3+ kernels in flight, and per kernel class the summed duration and the time it ran alone.
Usage: python tools/render_timeline.py <kernel_trace.csv> [frames] [out.txt]"""
import collections
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ngp::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 3
starts = [i for i, r in enumerate(rows) if "k_dense_records" in r[2]]
out = []


def cls(n):
    for k in ("k_hashgrid_fwd", "k_mlp_infer_rf", "k_render_net", "k_generate", "k_composite", "k_render_init", "k_shade"):
        if k in n:
            return k
    return n[:40]


for fi in range(max(0, len(starts) - nf - 1), len(starts) - 1):
    seg = [r for r in rows[starts[fi]:starts[fi + 1]]]
    # the frame ends at its last k_shade / k_accum_tonemap
    last = max(i for i, r in enumerate(seg) if "k_shade" in r[2] or "k_accum_tonemap" in r[2])
    seg = seg[:last + 1]
    t0, t1 = seg[0][0], max(e for _, e, _ in seg)
    ev = []
    for s, e, n in seg:
        ev.append((s, 1, n))
        ev.append((e, -1, n))
    ev.sort()
    conc = collections.Counter()
    alone = collections.Counter()
    total = collections.Counter()
    running = collections.Counter()
    pairs = collections.Counter()  # time with exactly this multiset of classes in flight (two kernels)
    prev = t0
    for t, d, n in ev:
        k = sum(running.values())
        conc[min(k, 3)] += t - prev
        if k == 1:
            (only,) = [x for x, c in running.items() if c]
            alone[only] += t - prev
        elif k == 2:
            pairs[" + ".join(sorted(x for x, c in running.items() for _ in range(c)))] += t - prev
        prev = t
        running[cls(n)] += d
    for s, e, n in seg:
        total[cls(n)] += e - s
    span = t1 - t0
    out.append(f"frame {fi}: {span / 1e3:.1f} us; in flight 0: {conc[0] / 1e3:.1f}  1: {conc[1] / 1e3:.1f}  2: {conc[2] / 1e3:.1f}  3+: {conc[3] / 1e3:.1f} us")
    for k, v in total.most_common():
        out.append(f"    {k:20s} sum {v / 1e3:8.1f} us  alone {alone[k] / 1e3:8.1f} us")
    for k, v in pairs.most_common(8):
        out.append(f"    pair {k:40s} {v / 1e3:8.1f} us")
txt = "\n".join(out)
print(txt)
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(txt + "\n")
