"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM-side bytes.

Usage: python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>
                                   [bench log of the same run] [fetch calibration json]

FETCH_SIZE / WRITE_SIZE are in KiB (x 1024 = bytes), per dispatch, averaged per launch:
  * fetch_bytes_per_launch: FETCH_SIZE x 1024 as reported (no correction);
  * fetch_bytes_per_launch_corrected: for kernels whose reads are coalesced streams, FETCH_SIZE
    divided by the streams' measured-over-issued ratio from tools/fetch_calib.sh
    (profiles/r02_fetch_calibration.json: 0.50 for 16-B and 4-B per-lane streams on gfx950, as
    MI355X_MICROARCH.md states for 16-B); for random gathers (hash-grid corners) FETCH_SIZE
    counts one 64-B unit per request (calibration: 64 B per random 4-B or 16-B read, and
    Infinity-Cache hits are counted), so the reported value stands: memory-side requests x 64 B,
    a lower bound of the bytes moved and an upper bound of the HBM bytes (the table is
    cache-resident).  Absent calibration: no corrected field;
  * write_bytes_per_launch: WRITE_SIZE x 1024 (exact for 16-B stores and float atomics per the
    guide);
  * per_unit: when the bench log of the same workload is given, bytes per launch divided by the
    device-counted units per launch of the kernel's timer (samples for the encoders / MLPs, rays
    for the march, parameters for the optimizer) -- not Grid_Size, since the launches are sized
    by upper bounds and the encoders handle four levels per thread.
"""
import csv
import json
import re
import sys
from collections import defaultdict

# kernel-name pattern -> (bench timer whose units describe it, access shape of its reads)
KERNELS = [
    (r"k_hashgrid_fwd<\d+u, 1[,>]", "render_encode", "k_gather16"),
    (r"k_hashgrid_fwd<\d+u, 0[,>]", "train_encode", "k_gather16"),
    (r"k_hashgrid_bwd<", "train_encode_bwd", "k_gather4"),
    (r"k_mlp_infer_(rf<.*, true>|sh<.*>)$", "render_mlp", "k_stream16"),
    (r"k_mlp_infer_rf<.*, false, 12, false>$", "train_mlp_infer", "k_stream16"),
    (r"k_mlp_train<", "train_mlp_bwd", "k_stream4"),
    (r"k_optimizer", "optimizer", "k_stream16"),
]


def load(path):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        out[name].append(float(r["Counter_Value"]))
    return out


def bench_units(log):
    if not log:
        return {}
    line = [l for l in open(log) if l.startswith('{"metric"') or l.startswith('{"config_e"')]
    if not line:
        return {}
    d = json.loads(line[-1])
    k = d.get("kernels_calibration") or d.get("config_e", {}).get("kernels_calibration", {})
    return {name: e["units"] / e["launches"] for name, e in k.items() if e.get("launches")}


def main():
    fetch, write, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    units = bench_units(sys.argv[4] if len(sys.argv) > 4 else None)
    calib = json.load(open(sys.argv[5])) if len(sys.argv) > 5 else {}
    f, w = load(fetch), load(write)
    res = {}
    for name in sorted(set(f) | set(w)):
        if not name.startswith("ngp::"):
            continue
        fl, wl = f.get(name, []), w.get(name, [])
        e = {"launches": len(fl) or len(wl)}
        if fl:
            e["fetch_bytes_per_launch"] = 1024 * sum(fl) / len(fl)
        if wl:
            e["write_bytes_per_launch"] = 1024 * sum(wl) / len(wl)
        for pat, timer, shape in KERNELS:
            if not re.search(pat, name):
                continue
            e["timer"] = timer
            e["read_shape"] = shape
            ratio = calib.get(shape, {}).get("measured_over_issued")
            if ratio and "fetch_bytes_per_launch" in e:
                stream = shape.startswith("k_stream")
                e["fetch_bytes_per_launch_corrected"] = e["fetch_bytes_per_launch"] / ratio if stream else e["fetch_bytes_per_launch"]
            if timer in units and units[timer] > 0:
                u = units[timer]
                e["units_per_launch_bench"] = u
                for key in ("fetch_bytes_per_launch", "fetch_bytes_per_launch_corrected", "write_bytes_per_launch"):
                    if key in e:
                        e[key.replace("_per_launch", "_per_unit")] = e[key] / u
            break
        res[name] = e
    json.dump(res, open(dst, "w"), indent=1)
    for k, v in res.items():
        print(k, {a: (round(b, 1) if isinstance(b, float) else b) for a, b in v.items()})


def recompute(path, calib_path):
    """Re-apply the correction rule to a summary written by an earlier version of this script."""
    res, calib = json.load(open(path)), json.load(open(calib_path))
    for e in res.values():
        shape = e.get("read_shape")
        ratio = calib.get(shape, {}).get("measured_over_issued") if shape else None
        if not ratio or "fetch_bytes_per_launch" not in e:
            continue
        stream = shape.startswith("k_stream")
        e["fetch_bytes_per_launch_corrected"] = e["fetch_bytes_per_launch"] / ratio if stream else e["fetch_bytes_per_launch"]
        if e.get("units_per_launch_bench"):
            e["fetch_bytes_per_unit_corrected"] = e["fetch_bytes_per_launch_corrected"] / e["units_per_launch_bench"]
    json.dump(res, open(path, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--recompute":
        recompute(sys.argv[2], sys.argv[3])
    else:
        main()
