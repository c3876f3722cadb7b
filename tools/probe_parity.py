"""Diagnostic: bench scene, train N steps, render a 1080p training view, compare 8-row blocks with
the oracle; dumps gpu/oracle rows to gpurun_out/parity_<N>.npz.  Usage: probe_parity.py N [N ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), os.path.join(ROOT, "tests"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
import pyngp as ngp  # noqa: E402
from scene_util import oracle_frame_rows, testbed_oracle  # noqa: E402

torch.cuda.set_device(0)
tb = ngp.Testbed(ngp.TestbedMode.Nerf)
import argparse
cams, imgs, focal = bench.make_dataset(ngp, tb, argparse.Namespace(scene="synthetic", views=100, train_res=800), "cuda:0")
tb.reload_network_from_file("lego_L16F2.json")
tb.shall_train = True
W, H = 1920, 1080
for n in map(int, sys.argv[1:]):
    while tb.training_step < n:
        tb.train(1 << 18)
    tb.set_camera_to_training_view(3)
    g = tb.render(W, H, 1, True)
    o = testbed_oracle(tb)
    ref = oracle_frame_rows(o, tb, W, H, [67])
    ys = sorted(ref)
    r = np.stack([ref[y] for y in ys])
    gg = g[ys]
    d = np.abs(gg[..., :3] - r[..., :3])
    print(f"step {n}: L1 {d.mean():.5f} max {d.max():.4f} frac>1e-2 {(d.max(-1) > 1e-2).mean():.4f} "
          f"alpha gpu {gg[..., 3].mean():.4f} oracle {r[..., 3].mean():.4f}", flush=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"parity_{n}.npz"), gpu=gg, ref=r, ys=np.array(ys))
