"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes.

Usage: python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read (MI355X_MICROARCH.md, HBM section), so fetched bytes are FETCH_SIZE x 1024 x 2;
WRITE_SIZE is exact for 16-B stores and float atomics (x 1024).  Per-kernel results are
normalised per launch and, for the hash-grid kernels, per sample (grid = samples x levels).
"""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        out[name].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    return out


def main():
    fetch, write, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    levels = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    f, w = load(fetch), load(write)
    res = {}
    for name in sorted(set(f) | set(w)):
        if not name.startswith("ngp::"):
            continue
        fl, wl = f.get(name, []), w.get(name, [])
        e = {"launches": len(fl) or len(wl)}
        if fl:
            e["fetch_bytes_per_launch"] = 2 * 1024 * sum(v for _, v in fl) / len(fl)
        if wl:
            e["write_bytes_per_launch"] = 1024 * sum(v for _, v in wl) / len(wl)
        if "hashgrid" in name and fl and wl:
            samples_f = sum(g for g, _ in fl) / levels
            samples_w = sum(g for g, _ in wl) / levels
            e["fetch_bytes_per_sample"] = 2 * 1024 * sum(v for _, v in fl) / samples_f
            e["write_bytes_per_sample"] = 1024 * sum(v for _, v in wl) / samples_w
        res[name] = e
    json.dump(res, open(dst, "w"), indent=1)
    for k, v in res.items():
        print(k, {a: round(b, 1) for a, b in v.items()})


if __name__ == "__main__":
    main()
