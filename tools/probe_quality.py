"""Diagnostic: train a scene N steps, render training view V and its ground truth, save both
as PNG under gpurun_out/, print PSNR.  Usage: probe_quality.py scene.json network N V [W H]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd")]
import metrics  # noqa: E402
import pyngp as ngp  # noqa: E402
import run  # noqa: E402

scene, net, n, v = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
# variants (env): PROBE_AABB=<int> overrides aabb_scale, PROBE_NOLENS=1 drops the OpenCV parameters
if os.environ.get("PROBE_AABB") or os.environ.get("PROBE_NOLENS"):
    import json
    meta = json.load(open(scene))
    if os.environ.get("PROBE_AABB"):
        meta["aabb_scale"] = int(os.environ["PROBE_AABB"])
    if os.environ.get("PROBE_NOLENS"):
        for k in ("k1", "k2", "k3", "k4", "p1", "p2"):
            meta.pop(k, None)
    scene = os.path.join(os.path.dirname(scene), "_probe.json")
    json.dump(meta, open(scene, "w"))
tb = ngp.Testbed()
tb.load_training_data(scene)
tb.reload_network_from_file(net)
if os.environ.get("PROBE_NIMG"):
    tb.nerf.training.n_images_for_training = int(os.environ["PROBE_NIMG"])
if os.environ.get("PROBE_CONE"):
    tb.nerf.cone_angle_constant = float(os.environ["PROBE_CONE"])
tb.shall_train = True
while tb.training_step < n:
    tb.frame()
md = tb.nerf.training.dataset.metadata[v]
w, h = md.resolution
if len(sys.argv) > 6:
    w, h = int(sys.argv[5]), int(sys.argv[6])
tb.background_color = [0.0, 0.0, 0.0, 1.0]
tb.snap_to_pixel_centers = True
tb.nerf.render_min_transmittance = 1e-4
tb.shall_train = False
tb.render_ground_truth = True
tb.set_camera_to_training_view(v)
ref = tb.render(w, h, 1, True)
tb.render_ground_truth = False
img = tb.render(w, h, 8, True)
psnr, ssim, mse = metrics.psnr_ssim(img, ref)
st = tb.last_train_stats()
print(f"train stats: loss {st['loss']:.6f} batch {st['measured_batch_size']} pre {st['measured_batch_size_before_compaction']} rays {st['rays_per_batch']}")
print(f"aabb {os.environ.get('PROBE_AABB', '-')} nolens {os.environ.get('PROBE_NOLENS', '-')} cone {os.environ.get('PROBE_CONE', '-')} nimg {os.environ.get('PROBE_NIMG', '-')} {net} {os.path.basename(scene)} steps {n} view {v}: PSNR {psnr:.2f} SSIM {ssim:.3f} loss {tb.loss:.6f} "
      f"img mean {img[..., :3].mean():.4f} alpha {img[..., 3].mean():.4f} ref mean {ref[..., :3].mean():.4f}")
tag = os.path.basename(os.path.dirname(scene)) + f"_{n}_{v}"
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
run.write_image(os.path.join(ROOT, "gpurun_out", f"q_{tag}_img.png"), img)
run.write_image(os.path.join(ROOT, "gpurun_out", f"q_{tag}_ref.png"), ref)
