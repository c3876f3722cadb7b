"""Host-side view of the idle gap in front of each training step (diagnostic): from a rocprofv3
--kernel-trace --hip-trace --memory-copy-trace CSV set, for each of the last steps (anchor: the step's first
k_sample_count), the HIP API calls between the end of the previous GPU operation and the start of the step's
first GPU operation, with their start offset from that end and their duration.
Usage: python tools/host_gap_summary.py <trace dir> [steps]"""
import csv
import glob
import os
import sys


def load(pattern):
    f = glob.glob(os.path.join(sys.argv[1], "**", pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
gpu = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:60])
       for r in load("*kernel_trace.csv")]
gpu += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")) for r in load("*memory_copy_trace.csv")]
gpu.sort()
api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in load("*hip_api_trace.csv"))
anchors = [i for i, g in enumerate(gpu) if "k_sample_count" in g[2]]
for a in anchors[-steps:]:
    # the step's first GPU op: walk back over the ops that start after the previous step's last op
    j = a
    while j > 0 and "k_optimizer" not in gpu[j - 1][2] and "copy" not in gpu[j - 1][2] and "copyBuffer" not in gpu[j - 1][2]:
        j -= 1
    prev_end = max(g[1] for g in gpu[:j]) if j else gpu[0][0]
    first = gpu[j]
    print(f"== step: previous GPU op ({gpu[j - 1][2]}) ends, {(first[0] - prev_end) / 1e3:.1f} us idle before {first[2]}")
    for st, en, fn in api:
        if prev_end - 20000 <= st <= first[0]:
            print(f"   {(st - prev_end) / 1e3:8.1f} us  {(en - st) / 1e3:7.1f} us  {fn}")

# the last full step as one timeline: GPU operations (start, duration, idle gap before) and HIP API calls
a, b = anchors[-2], anchors[-1]
t0 = gpu[a][0]
ev = [(g[0], "GPU", f"{(g[1] - g[0]) / 1e3:7.1f} us  {g[2]}") for g in gpu[a - 3:b + 1]]
ev += [(st, "API", f"{(en - st) / 1e3:7.1f} us  {fn}") for st, en, fn in api if gpu[a - 3][0] <= st <= gpu[b][0]]
print("== last step timeline (us from its k_sample_count)")
for t, kind, txt in sorted(ev):
    print(f"{(t - t0) / 1e3:9.1f}  {kind}  {txt}")
