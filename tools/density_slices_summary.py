"""Summarises the reference-mosaic probes (tools/density_slices_probe.py --masks) into one JSON:
per seed the statistics against the reference's mosaic, per pair of seeds the same statistics, and the coarse
(32^3 blocks of 8^3) occupancy correlations with the orientation ranking of tests/density_slices_util.py.

  python tools/density_slices_summary.py gpurun_out/r05c profiles/r05_density_slices.json
"""
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import density_slices_util as D  # noqa: E402


def main(src, dst):
    out = {"protocol": "base.json (fork default L8 F4 T2^19), 35000 steps, random background colours, compute_and_save_png_slices "
                       "defaults (render aabb, 256^3, thresh 2.5, range 4); masks: raw density >= 2.5 (byte >= 129)",
           "scenes": {}}
    for sc in ("test2", "test"):
        probe = json.load(open(os.path.join(src, f"ds_{sc}.json")))
        z = np.load(os.path.join(src, f"masks_{sc}.npz"))
        seeds = sorted({k.split("_")[1] for k in z.files})
        occ = {s: np.unpackbits(z["occ_" + s]).reshape(256, 256, 256).astype(bool) for s in seeds}
        ref = D.reference_volume(sc) >= 129
        cref = D.coarse(ref)
        pairs = {}
        for a, b in itertools.combinations(seeds, 2):
            m = D.compare(occ[a].astype(np.uint8) * 200, occ[b].astype(np.uint8) * 200)
            m["coarse_corr"] = float(np.corrcoef(D.coarse(occ[a]).ravel(), D.coarse(occ[b]).ravel())[0, 1])
            ident, rank = D.orientation_ranking((D.coarse(occ[a]) + D.coarse(occ[b])) / 2, cref)
            m["pair_mean_vs_reference_corr"], m["pair_mean_vs_reference_orientation_rank"] = ident, rank
            pairs[f"{a}/{b}"] = {k: round(v, 4) if isinstance(v, float) else v for k, v in m.items()}
        vs_ref = {}
        for s in seeds:
            r = dict(probe["runs"][f"{s}/35000"])
            r["coarse_corr"] = float(np.corrcoef(D.coarse(occ[s]).ravel(), cref.ravel())[0, 1])
            vs_ref[s] = {k: round(v, 4) if isinstance(v, float) else v for k, v in r.items()}
        out["scenes"][sc] = {"reference": probe["reference"], "seeds_vs_reference": vs_ref, "seed_pairs": pairs}
    out["notes"] = [
        "test2: the data path in the reference's file name (data/nerf/test2/images) is the scene's; trained here at quarter "
        "resolution (180x320, all 300 views).  The scene is a flame animated over the frames on an opaque black background: "
        "this build's own seeds agree at IoU 0.29-0.40 only; against the reference 0.11-0.14.  At the scale the data "
        "determines (32^3 block occupancy) the reference's field correlates best with ours in the identity frame of the 48 "
        "axis permutations / flips for every seed pair (tests/test_gpu_density_slices.py).",
        "test: the reference's file name says its data path was data/nerf/test, while the fire dataset sits in "
        "data/nerf/test/dataset (its log.txt: BlenderNeRF dataset 'dataset' saved under data/nerf/test/); fields trained on "
        "test/dataset agree with each other (IoU 0.44-0.49, coarse correlation 0.70-0.82) and with no orientation of the "
        "reference's mosaic (correlation <= 0.002), so the mosaic was not written from this dataset: not used as a pin.",
    ]
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({sc: {k: v for k, v in d["seed_pairs"].items()} for sc, d in out["scenes"].items()}, indent=None)[:2000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
