"""Training-collapse sweep: train scenes to N steps with fixed seeds in the DEFAULT training mode
and record, per run, what a collapse to the degenerate "views painted on the box" solution would show:

  * loss      -- mean of the last 64 steps' loss (a collapse drives it to ~0);
  * grid_max  -- largest density-grid value (collapsed fields: 1e6-1e7);
  * grid_mean -- mean density-grid value of cascade 0;
  * occupied  -- fraction of cascade-0 occupancy bits set;
  * batch     -- compacted training samples of the last step, rays of the last step;
  * psnr      -- mean PSNR of `--views` training views rendered at their own resolution against the images
                 (Testbed.render vs render_ground_truth, linear, black background).

Scenes: fire = data/nerf/test/dataset (the bench scene), fox = data/nerf/fox, synthetic = the procedural lego-shaped
surface scene (tests/synthetic.py, 100 views 800^2), test2 = data/nerf/test2 (the scene whose reference mosaic
collapsed in 1 of 4 runs in round 5).  One JSON line per run, flushed as it finishes.

  python tools/collapse_sweep.py --scenes fire,fox --seeds 1337,1,2,3,4,5,6,7 --steps 35000
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), os.path.join(ROOT, "tests"), ROOT]

SCENES = {
    "fire": os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"),
    "fox": os.path.join(ROOT, "data", "nerf", "fox"),
    "test2": os.path.join(ROOT, "data", "nerf", "test2", "images", "transforms_train.json"),
    "test2_half": os.path.join(ROOT, "data", "nerf", "test2_half", "images", "transforms_train.json"),
    "test2_full": os.path.join(ROOT, "data", "nerf", "test2_full", "images", "transforms_train.json"),
}


def load(ngp, scene, seed, config, random_bg=True):
    tb = ngp.Testbed(ngp.TestbedMode.Nerf)
    tb.seed = seed
    if scene == "synthetic":
        import bench
        a = argparse.Namespace(scene="synthetic", views=100, train_res=800)
        bench.make_dataset(ngp, tb, a, "cuda:0")
    else:
        tb.load_training_data(SCENES[scene])
    tb.reload_network_from_file(config)
    tb.nerf.training.random_bg_color = random_bg
    tb.shall_train = True
    return tb


def psnr_views(tb, views):
    ds = tb.nerf.training.dataset
    bg = list(tb.background_color)
    tb.background_color = [0.0, 0.0, 0.0, 1.0]
    out = []
    for v in np.linspace(0, ds.n_images - 1, views).astype(int):
        w, h = (int(x) for x in ds.metadata[int(v)].resolution)
        tb.set_camera_to_training_view(int(v))
        tb.render_ground_truth = True
        gt = tb.render(w, h, 1, True)[..., :3]
        tb.render_ground_truth = False
        img = tb.render(w, h, 1, True)[..., :3]
        mse = float(np.mean((np.clip(img, 0, 1) - np.clip(gt, 0, 1)) ** 2))
        out.append(-10.0 * np.log10(max(mse, 1e-12)))
    tb.background_color = bg
    return float(np.mean(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="fire,fox,synthetic")
    ap.add_argument("--seeds", default="1337,1,2,3,4,5,6,7")
    ap.add_argument("--steps", type=int, default=35000)
    ap.add_argument("--config", default="base.json")
    ap.add_argument("--views", type=int, default=4)
    ap.add_argument("--trajectory", type=int, default=0, help="also print a line every this many steps")
    ap.add_argument("--random-bg", type=int, default=1, help="nerf.training.random_bg_color (the reference's default: 1)")
    ap.add_argument("--mosaic-dir", default="", help="test2 / test2_half / fire: compare the trained field's density "
                    "mosaic with the reference's and save its packed >= 2.5 mask here (seed-versus-seed IoU later)")
    args = ap.parse_args()
    if "synthetic" in args.scenes:
        import torch  # the procedural views are rendered with torch: its HIP runtime starts before pyngp's library

        torch.cuda.set_device(0)
    import pyngp as ngp
    for scene in args.scenes.split(","):
        for seed in (int(s) for s in args.seeds.split(",")):
            t0 = time.time()
            tb = load(ngp, scene, seed, args.config, bool(args.random_bg))
            losses = []
            while tb.training_step < args.steps:
                tb.frame()
                losses.append(tb.loss)
                if args.trajectory and tb.training_step % args.trajectory == 0:
                    st = tb.last_train_stats()
                    g = np.asarray(tb.density_grid())
                    print(json.dumps({"scene": scene, "seed": seed, "step": tb.training_step, "loss": float(np.mean(losses[-64:])),
                                      "batch": int(st["measured_batch_size"]), "before": int(st["measured_batch_size_before_compaction"]),
                                      "rays": int(st["n_rays"]), "grid_max": float(g.max()), "grid_mean": float(g[:128 ** 3].mean())}),
                          flush=True)
            st = tb.last_train_stats()
            g = np.asarray(tb.density_grid())
            bits = np.unpackbits(np.asarray(tb.density_grid_bitfield(), np.uint8)[:128 ** 3 // 8])
            rec = {"scene": scene, "seed": seed, "steps": tb.training_step, "mode": "default", "random_bg": args.random_bg,
                   "loss": float(np.mean(losses[-64:])), "grid_max": float(g.max()), "grid_mean": float(g[:128 ** 3].mean()),
                   "occupied": float(bits.mean()), "batch": int(st["measured_batch_size"]), "rays": int(st["n_rays"]),
                   "psnr": psnr_views(tb, args.views), "seconds": round(time.time() - t0, 1)}
            ref_scene = {"test2": "test2", "test2_half": "test2", "test2_full": "test2", "fire": "test"}.get(scene)
            if args.mosaic_dir and ref_scene:
                import density_slices_util as D
                vol = D.testbed_volume(tb)
                ref = D.reference_volume(ref_scene)
                rec.update({"ref_" + k: v for k, v in D.compare(vol, ref).items()})
                corr, rank = D.orientation_ranking(D.coarse(vol >= 129), D.coarse(ref >= 129))
                rec.update({"ref_corr": corr, "ref_rank": rank,
                            "occupied_ratio": float((vol >= 129).mean() / max((ref >= 129).mean(), 1e-9))})
                os.makedirs(args.mosaic_dir, exist_ok=True)
                np.savez_compressed(os.path.join(args.mosaic_dir, f"{scene}_bg{args.random_bg}_seed{seed}.npz"),
                                    mask=np.packbits(vol >= 129))
            print(json.dumps(rec), flush=True)
            del tb


if __name__ == "__main__":
    main()
