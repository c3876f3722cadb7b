"""Probe (GPU, diagnostic, run under rocprofv3 --kernel-trace): idle gaps between a 1080p frame's kernels with the kernel
timers off or on (ngp_timing_enable), on bench.py's surface scene (one ray pipeline).  Renders 4 frames; summarise the
trace with tools/gap_summary.py.  --train: 8 training steps instead (gap_summary.py ... k_sample_count).
  python tools/probe_gaps.py [--timers MASK] [--train]"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), ROOT, os.path.join(ROOT, "tests")]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--timers", type=int, default=0)
    p.add_argument("--scene", default="synthetic")
    p.add_argument("--train", action="store_true", help="trace 8 training steps instead of frames")
    a = p.parse_args()
    import torch
    torch.cuda.set_device(0)
    import ngp_abi as A
    import pyngp as ngp
    import bench
    tb = ngp.Testbed(ngp.TestbedMode.Nerf)
    if a.scene == "synthetic":
        bench.make_dataset(ngp, tb, argparse.Namespace(scene="synthetic", views=100, train_res=800), "cuda:0")
    else:
        tb.load_training_data(os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"))
    tb.reload_network_from_file(os.path.join(ROOT, "instant-ngp-rendering_amd", "configs", "nerf", "lego_L16F2.json"))
    tb.shall_train = True
    for _ in range(300):
        tb.train(1 << 18)
    lib = A.load()
    h = C.c_void_p(tb.model_handle)
    A.check(lib.ngp_timing_enable(h, a.timers))
    if a.train:
        tb.sync()
        t0 = time.perf_counter()
        for _ in range(8):
            tb.train(1 << 18)
        tb.sync()
        print(f"timers {a.timers}: {(time.perf_counter() - t0) / 8 * 1e6:.1f} us per training step", flush=True)
        return
    tb.shall_train = False
    tb.set_camera_to_training_view(3)
    tb.render_to_device(1920, 1080, 1, True)
    tb.sync()
    t0 = time.perf_counter()
    for _ in range(4):
        tb.render_to_device(1920, 1080, 1, True)
    tb.sync()
    print(f"timers {a.timers}: {(time.perf_counter() - t0) / 4 * 1e3:.3f} ms per frame", flush=True)


if __name__ == "__main__":
    main()
