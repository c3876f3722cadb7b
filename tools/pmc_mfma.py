"""Summarise one rocprofv3 --pmc pass of MFMA / LDS counters per kernel (tools/pmc_mfma.sh).

Usage: python tools/pmc_mfma.py <counter_collection.csv> <out.json>

Per kernel (summed over its dispatches, then per dispatch):
  * mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CU_CYCLES x 4 SIMDs): the share of the
    CU-busy cycles in which a SIMD's matrix core was busy (SQ_BUSY_CU_CYCLES counts, per CU, the
    cycles it had waves; MFMA busy cycles are counted per SIMD);
  * mfma_flop = SQ_INSTS_VALU_MFMA_MOPS_F16 x 512 (the counter tallies fp16 MFMA work in units
    of 512 FLOP), checked against the kernel's algorithmic FLOPs by the caller;
  * lds_wait_frac = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES (both quad-cycles): issue stalls on LDS;
  * clock_ghz_est = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (when the CSV carries it).
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    src, dst = sys.argv[1], sys.argv[2]
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if not name.startswith("ngp::k_mlp"):
            continue
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        n[name].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    res = {}
    for name, c in acc.items():
        d = max(len(n[name]), 1)
        e = {"dispatches": d}
        e.update({k: v / d for k, v in sorted(c.items())})
        busy = c.get("SQ_BUSY_CU_CYCLES", 0.0)
        if busy:
            e["mfma_busy_frac"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (4.0 * busy)
        if c.get("SQ_WAVE_CYCLES"):
            e["lds_wait_frac"] = c.get("SQ_WAIT_INST_LDS", 0.0) / c["SQ_WAVE_CYCLES"]
        e["mfma_flop_per_dispatch"] = 512.0 * c.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0.0) / d
        res[name] = e
    json.dump(res, open(dst, "w"), indent=1)
    for k, v in res.items():
        print(k)
        for a, b in v.items():
            print(f"    {a:32s} {b:.4g}")


if __name__ == "__main__":
    main()
