"""Trains the fork's base.json on one of the two scenes whose CUDA-trained density mosaics the reference ships and
compares this build's compute_and_save_png_slices mosaics with the reference's (GPU box, repo root).

  python tools/density_slices_probe.py --scene test --seeds 1337 42 --steps 2000 5000 35000 --out gpurun_out/ds_test.json

Per checkpoint and seed: the mosaic's statistics against the reference mosaic (tests/density_slices_util.py) and,
for two seeds, the same statistics between the seeds (the calibration: "as close to the reference as to itself").
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "instant-ngp-rendering_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import density_slices_util as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="test", choices=sorted(D.SCENES))
    ap.add_argument("--seeds", type=int, nargs="+", default=[1337, 42])
    ap.add_argument("--steps", type=int, nargs="+", default=[2000, 5000, 10000, 35000])
    ap.add_argument("--config", default="base.json")
    ap.add_argument("--out", default="gpurun_out/density_slices_probe.json")
    ap.add_argument("--save", default="", help="directory for slice previews (optional)")
    ap.add_argument("--random-bg", type=int, default=1, help="nerf.training.random_bg_color")
    ap.add_argument("--masks", default="", help="npz file for the packed >= 129 / > 0 masks of the last step per seed")
    a = ap.parse_args()
    import pyngp as ngp
    ref = D.reference_volume(a.scene)
    res = {"scene": a.scene, "config": a.config, "random_bg_color": bool(a.random_bg), "reference": D.volume_stats(ref),
           "runs": {}, "seed_vs_seed": {}}
    vols = {}
    if a.save:
        from PIL import Image
        os.makedirs(a.save, exist_ok=True)
        Image.fromarray(D.preview(ref)).save(os.path.join(a.save, f"{a.scene}_reference.png"))
    for seed in a.seeds:
        tb = D.new_testbed(ngp, a.scene, a.config, seed, bool(a.random_bg))
        t0 = time.time()
        for s in a.steps:
            D.train_to(tb, s)
            vol = D.testbed_volume(tb)
            vols[(seed, s)] = vol
            m = D.compare(vol, ref)
            raw = tb.density_on_grid([256, 256, 256], ngp.BoundingBox())
            m["masked"] = float((raw == -10000.0).mean())
            if a.save and s == a.steps[-1]:
                Image.fromarray(D.preview(vol)).save(os.path.join(a.save, f"{a.scene}_bg{a.random_bg}_s{seed}_{s}.png"))
            m["seconds"] = round(time.time() - t0, 1)
            m.update(D.volume_stats(vol))
            res["runs"][f"{seed}/{s}"] = m
            print(json.dumps({"seed": seed, "step": s, **m}), flush=True)
        del tb
    if a.masks:
        pk = {}
        for seed in a.seeds:
            v = vols[(seed, a.steps[-1])]
            pk[f"occ_{seed}"] = np.packbits(v >= 129)
            pk[f"nz_{seed}"] = np.packbits(v > 0)
        np.savez_compressed(a.masks, **pk)
    if len(a.seeds) >= 2:
        for s in a.steps:
            m = D.compare(vols[(a.seeds[0], s)], vols[(a.seeds[1], s)])
            res["seed_vs_seed"][str(s)] = m
            print(json.dumps({"seed_vs_seed": s, **m}), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
