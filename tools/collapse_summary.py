"""Summarise tools/collapse_sweep.py runs (JSON lines) and their saved density masks into profiles/r06_collapse_sweep.txt:
per scene and background mode the runs that reach the field ("flame" / converged) and those that stay sample-starved
(the 2^18-ray cap; cascade-0 occupancy 0.6-1: the views painted on the box), and, for the scenes with a
reference mosaic, IoU of the >= 2.5 raw-density masks between converged seeds and against the reference.

  python tools/collapse_summary.py OUT.txt sweep1.jsonl[:maskdir] sweep2.jsonl[:maskdir] ...
"""
import itertools
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def collapsed(r):
    """Sample-starved: the rays-per-batch estimate pinned at its 2^18 cap (the occupancy grid stays full, the sample
    cap admits only the first rays) -- the views painted on the box, or on the way there."""
    return r["rays"] >= (1 << 18)


def main():
    out = sys.argv[1]
    runs, masks = [], {}
    for spec in sys.argv[2:]:
        path, _, mdir = spec.partition(":")
        for line in open(path):
            line = line.strip()
            if not line.startswith("{"):
                continue
            r = json.loads(line)
            if "psnr" not in r:
                continue  # a trajectory line
            r.setdefault("random_bg", 1)
            runs.append(r)
            if mdir:
                for name in (f"{r['scene']}_bg{r['random_bg']}_seed{r['seed']}.npz", f"{r['scene']}_seed{r['seed']}.npz"):
                    p = os.path.join(mdir, name)
                    if os.path.exists(p):
                        masks[(r["scene"], r["random_bg"], r["seed"])] = p
                        break
    groups = defaultdict(list)
    for r in runs:
        groups[(r["scene"], r["random_bg"])].append(r)
    lines = []
    for (scene, bg), rs in groups.items():
        ok = [r for r in rs if not collapsed(r)]
        lines.append(f"## {scene} (random_bg_color {bg}): {len(ok)} of {len(rs)} runs converge, {len(rs) - len(ok)} starve (views painted on the box)")
        for r in rs:
            extra = ""
            if "ref_iou" in r:
                extra = (f" | vs reference: IoU {r['ref_iou']:.3f} (1-voxel {r['ref_iou_1voxel']:.3f}), coarse corr "
                         f"{r['ref_corr']:.3f} rank {r['ref_rank']}, occupied ratio {r['occupied_ratio']:.2f}")
            lines.append(f"  seed {r['seed']:5d} {'STARVED  ' if collapsed(r) else 'converged'}: loss {r['loss']:.2e} "
                         f"grid max {r['grid_max']:.3g} occupied {r['occupied']:.3f} rays {r['rays']} batch {r['batch']} "
                         f"PSNR {r['psnr']:.2f} dB ({r['seconds']} s){extra}")
        keys = [(scene, bg, r["seed"]) for r in ok if (scene, bg, r["seed"]) in masks]
        if len(keys) >= 2:
            vol = {k: np.unpackbits(np.load(masks[k])["mask"]).astype(bool) for k in keys}
            ious = [float((vol[a] & vol[b]).sum() / max((vol[a] | vol[b]).sum(), 1)) for a, b in itertools.combinations(keys, 2)]
            lines.append(f"  converged seed vs seed IoU: min {min(ious):.3f} median {float(np.median(ious)):.3f} "
                         f"max {max(ious):.3f} over {len(ious)} pairs")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
