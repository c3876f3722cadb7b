#!/usr/bin/env python3
"""Train / evaluate / screenshot driver over the MI355X `pyngp` (NeRF path).

Command-line compatible with the NeRF subset of the reference driver
(scripts/run.py:28-83): --scene, --network, --load_snapshot/--save_snapshot,
--nerf_compatibility, --test_transforms (PSNR/SSIM, scripts/run.py:210-268),
--near_distance, --exposure, --screenshot_transforms/--screenshot_frames/
--screenshot_dir/--screenshot_spp, --width/--height, --n_steps, --sharpen.
GUI/VR, meshes and camera-path videos are not part of this build.

    python instant-ngp-rendering_amd/run.py --scene data/lego/transforms_train.json \\
        --n_steps 35000 --test_transforms data/lego/transforms_test.json
"""
import argparse
import json
import os
import struct
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import metrics  # noqa: E402
import pyngp as ngp  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Instant-NGP NeRF on MI355X: train, evaluate, screenshot")
    p.add_argument("files", nargs="*", help="scene / network config / snapshot files, loaded in order")
    p.add_argument("--scene", "--training_data", default="", help="NeRF dataset (transforms.json or its directory)")
    p.add_argument("--network", default="", help="network config (configs/nerf/<name>.json or a path)")
    p.add_argument("--load_snapshot", "--snapshot", default="")
    p.add_argument("--save_snapshot", default="")
    p.add_argument("--nerf_compatibility", action="store_true",
                   help="sRGB compositing, no cone tracing, fixed background (original NeRF protocol)")
    p.add_argument("--test_transforms", default="", help="transforms.json of held-out views: report PSNR / SSIM")
    p.add_argument("--near_distance", default=-1, type=float)
    p.add_argument("--exposure", default=0.0, type=float)
    p.add_argument("--screenshot_transforms", default="")
    p.add_argument("--screenshot_frames", nargs="*")
    p.add_argument("--screenshot_dir", default="")
    p.add_argument("--screenshot_spp", type=int, default=16)
    p.add_argument("--width", "--screenshot_w", type=int, default=0)
    p.add_argument("--height", "--screenshot_h", type=int, default=0)
    p.add_argument("--n_steps", type=int, default=-1)
    p.add_argument("--sharpen", default=0)
    p.add_argument("--eval_spp", type=int, default=8, help="samples per pixel of the test-set renders (run.py uses 8)")
    p.add_argument("--quiet", action="store_true")
    return p.parse_args(argv)


def write_image(path, img):
    """Linear premultiplied RGBA -> file: .bin (f16, the reference's raw format) or 8-bit sRGB PNG."""
    if path.endswith(".bin"):
        h, w = img.shape[:2]
        if img.shape[2] < 4:
            img = np.dstack([img, np.ones((h, w, 4 - img.shape[2]), img.dtype)])
        with open(path, "wb") as f:
            f.write(struct.pack("ii", h, w))
            f.write(img.astype(np.float16).tobytes())
        return
    rgb, a = img[..., :3], img[..., 3:4]
    straight = np.divide(rgb, a, out=np.zeros_like(rgb), where=a != 0)
    out = np.concatenate([metrics.linear_to_srgb(np.clip(straight, 0, None)), a], axis=-1)
    write_png(path, (np.clip(out, 0, 1) * 255 + 0.5).astype(np.uint8))


def write_png(path, rgba):
    """RGBA8 [H][W][4] -> PNG (zlib, filter 0)."""
    import zlib

    h, w, _ = rgba.shape
    raw = b"".join(b"\x00" + rgba[y].tobytes() for y in range(h))

    def chunk(t, body):
        return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


def evaluate(testbed, test_transforms, spp=8, log=print):
    """PSNR / SSIM over every view of a transforms.json (scripts/run.py:210-268 protocol)."""
    testbed.background_color = [0.0, 0.0, 0.0, 1.0]
    testbed.snap_to_pixel_centers = True
    testbed.nerf.render_min_transmittance = 1e-4
    testbed.shall_train = False
    testbed.load_training_data(test_transforms)
    psnrs, ssims, mses = [], [], []
    for i in range(testbed.nerf.training.dataset.n_images):
        w, h = testbed.nerf.training.dataset.metadata[i].resolution
        testbed.render_ground_truth = True
        testbed.set_camera_to_training_view(i)
        ref = testbed.render(w, h, 1, True)
        testbed.render_ground_truth = False
        img = testbed.render(w, h, spp, True)
        psnr, ssim, mse = metrics.psnr_ssim(img, ref)
        psnrs.append(psnr)
        ssims.append(ssim)
        mses.append(mse)
    res = {"psnr": float(np.mean(psnrs)), "psnr_min": float(np.min(psnrs)), "psnr_max": float(np.max(psnrs)),
           "psnr_of_mean_mse": float(metrics.mse2psnr(np.mean(mses))), "ssim": float(np.mean(ssims)),
           "n_images": len(psnrs)}
    log(f"PSNR={res['psnr']} [min={res['psnr_min']} max={res['psnr_max']}] SSIM={res['ssim']}")
    return res


def run(args, log=print):
    testbed = ngp.Testbed()
    for f in args.files:
        testbed.load_file(f)
    if args.scene:
        testbed.load_training_data(args.scene)
    if args.load_snapshot:
        testbed.load_snapshot(args.load_snapshot)
    elif args.network:
        testbed.reload_network_from_file(args.network)

    testbed.nerf.sharpen = float(args.sharpen)
    testbed.exposure = args.exposure
    testbed.shall_train = True
    testbed.nerf.render_with_lens_distortion = True
    if args.near_distance >= 0.0:
        testbed.nerf.training.near_distance = args.near_distance
    if args.nerf_compatibility:
        testbed.color_space = ngp.ColorSpace.SRGB
        testbed.nerf.cone_angle_constant = 0
        testbed.nerf.training.random_bg_color = False

    n_steps = args.n_steps
    if n_steps < 0 and not args.load_snapshot:
        n_steps = 35000
    result = {}
    if n_steps > 0:
        t0 = time.perf_counter()
        last = t0
        while testbed.frame():
            if testbed.training_step >= n_steps:
                break
            now = time.perf_counter()
            if not args.quiet and now - last > 5.0:
                log(f"step {testbed.training_step}/{n_steps} loss={testbed.loss:.6f}")
                last = now
        result["train_seconds"] = time.perf_counter() - t0
        result["training_step"] = testbed.training_step
        result["loss"] = testbed.loss
    if args.save_snapshot:
        os.makedirs(os.path.dirname(os.path.abspath(args.save_snapshot)), exist_ok=True)
        testbed.save_snapshot(args.save_snapshot, False)

    if args.test_transforms:
        result.update(evaluate(testbed, args.test_transforms, args.eval_spp, log))

    if args.screenshot_transforms:
        with open(args.screenshot_transforms) as f:
            ref = json.load(f)
        testbed.fov_axis = 0
        testbed.fov = ref["camera_angle_x"] * 180 / np.pi
        frames = args.screenshot_frames or range(len(ref["frames"]))
        for idx in frames:
            fr = ref["frames"][int(idx)]
            testbed.set_nerf_camera_matrix(np.asarray(fr.get("transform_matrix", fr.get("transform_matrix_start")))[:3])
            name = os.path.join(args.screenshot_dir, os.path.basename(fr["file_path"]))
            if not os.path.splitext(name)[1]:
                name += ".png"
            w = args.width or int(ref.get("w", 800))
            h = args.height or int(ref.get("h", 800))
            os.makedirs(os.path.dirname(os.path.abspath(name)), exist_ok=True)
            write_image(name, testbed.render(w, h, args.screenshot_spp, True))
    elif args.screenshot_dir:
        os.makedirs(args.screenshot_dir, exist_ok=True)
        stem = os.path.splitext(os.path.basename(args.network))[0] if args.network else "base"
        name = os.path.join(args.screenshot_dir, f"{os.path.basename(os.path.normpath(args.scene)) or 'scene'}_{stem}.png")
        write_image(name, testbed.render(args.width or 1920, args.height or 1080, args.screenshot_spp, True))
    return result


if __name__ == "__main__":
    print(json.dumps(run(parse_args())))
