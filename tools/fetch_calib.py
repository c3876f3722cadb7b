"""Summarise tools/fetch_calib.sh: FETCH_SIZE (KiB) per dispatch of each access shape against the
bytes the kernel issued.  Only the second repetition of each kernel is used (the first warms).

  measured_over_issued = FETCH_SIZE x 1024 / issued bytes
    stream16 / stream4: issued = the streamed bytes
    gather4 / gather16: issued = reads x 4 / 16 B; FETCH_SIZE also shows the line granularity
    table4: 16 MiB table re-read 16x: ~0 means the Infinity-Cache hits are not counted

Usage: python tools/fetch_calib.py <counter_collection.csv> <run.log> <out.json>"""
import csv
import json
import sys
from collections import defaultdict


def main():
    src, log, dst = sys.argv[1:4]
    meta = json.loads([l for l in open(log) if l.startswith("{")][-1])
    per = defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        per[name].append(float(r["Counter_Value"]))
    issued = {"k_stream16": meta["stream16_bytes"], "k_stream4": meta["stream4_bytes"],
              "k_gather4": 4 * meta["gather4_reads"], "k_gather16": 16 * meta["gather16_reads"],
              "k_table4": 4 * meta["table4_reads"]}
    res = {"source": "tools/fetch_calib.hip under rocprofv3 --pmc FETCH_SIZE (MI355X, gfx950)"}
    for k, b in issued.items():
        vals = per.get(k, [])
        if not vals:
            continue
        fetched = 1024.0 * vals[-1]
        res[k] = {"issued_bytes": b, "fetch_size_bytes": fetched, "measured_over_issued": fetched / b}
    json.dump(res, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
