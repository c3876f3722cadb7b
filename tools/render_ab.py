"""Render-schedule A/B on one box and one set of weights (diagnostic, GPU box).

Trains the bench scene once (bench.py's defaults), then renders the bench's 1080p view under
each setting in turn, round-robin, so box-to-box and run-to-run spread cancel out.  A setting is
a space-separated list of ngp_tuning fields (include/ngp_hip.h; Testbed.set_tuning), applied
before its frames.

Usage: python tools/render_ab.py [--rounds 4] [--frames 5] [--scene synthetic] "" "render_pipelines=1" "render_pass_samples=8388608" ...
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "instant-ngp-rendering_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("settings", nargs="+")
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--frames", type=int, default=5)
    p.add_argument("--pretrain", type=int, default=1500)
    p.add_argument("--config", default=os.path.join(ROOT, "instant-ngp-rendering_amd", "configs", "nerf", "lego_L16F2.json"))
    p.add_argument("--snapshot", default=None, help="load this snapshot if it exists, else train and save it")
    p.add_argument("--pkg", default=None, help="directory holding another build of pyngp + libngp_hip (tools/ab_build_old.sh)")
    p.add_argument("--stats", action="store_true", help="one frame per setting with the march statistics (debug bit 0)")
    p.add_argument("--host", action="store_true", help="time render() into host memory instead of render_to_device(); a "
                   "setting 'hbm' times render_to_device()")
    p.add_argument("--scene", default=os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"))
    a = p.parse_args()
    if a.pkg:
        sys.path.insert(0, os.path.abspath(a.pkg))
    if a.scene == "synthetic":
        import torch  # renders the scene's views: its HIP runtime has to start before pyngp's library loads

        torch.cuda.set_device(0)
    import pyngp as ngp

    print(f"# pyngp from {ngp.__file__}", file=sys.stderr)

    tb = ngp.Testbed(ngp.TestbedMode.Nerf)
    if a.scene == "synthetic":
        # bench.py's procedural lego-shaped surface scene (100 views 800x800)
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import bench
        bench.make_dataset(ngp, tb, argparse.Namespace(scene="synthetic", views=100, train_res=800), "cuda:0")
    else:
        tb.load_training_data(a.scene)
    tb.reload_network_from_file(a.config)
    if a.snapshot and os.path.exists(a.snapshot):
        tb.load_snapshot(a.snapshot)  # the same weights and grid as the run that wrote it
    else:
        tb.shall_train = True
        tb.deterministic = True  # bench.py's reproducible pretraining: the same volume on every box
        for i in range(a.pretrain):
            tb.train(1 << 18)
        tb.deterministic = False
        if a.snapshot:
            tb.save_snapshot(a.snapshot, False)
    n_views = tb.nerf.training.dataset.n_images
    tb.set_camera_to_training_view(3 % n_views)
    base = tb.get_tuning()
    times = {s: [] for s in a.settings}
    for r in range(a.rounds):
        for s in a.settings:
            setting = dict(base)
            kvs = [kv for kv in s.split() if kv != "hbm"]
            for kv in kvs:
                k, v = kv.split("=", 1)
                setting[k] = float(v) if k == "render_budget_scale" else int(v)
            tb.set_tuning(setting)
            host = a.host and "hbm" not in s.split()

            def frame():
                if host:
                    img = tb.render(1920, 1080, 1, True)
                    del img
                else:
                    tb.render_to_device(1920, 1080, 1, True)
            frame()  # warm this setting's buffers
            t0 = time.perf_counter()
            for _ in range(a.frames):
                frame()
            times[s].append((time.perf_counter() - t0) / a.frames * 1e3)
        print(f"# round {r + 1}/{a.rounds}", file=sys.stderr, flush=True)
    if a.stats:
        for s in a.settings:
            setting = dict(base)
            for kv in s.split():
                k, v = kv.split("=", 1)
                setting[k] = float(v) if k == "render_budget_scale" else int(v)
            setting["debug"] = 1  # per-frame march statistics on stderr
            tb.set_tuning(setting)
            print(f"# stats: {s or 'default'}", file=sys.stderr, flush=True)
            tb.render_to_device(1920, 1080, 1, True)
        tb.set_tuning(base)
    for s in a.settings:
        t = times[s]
        print(f"{s or 'default':55s} median {statistics.median(t):7.3f} ms/frame  min {min(t):7.3f}  "
              f"({', '.join(f'{x:.2f}' for x in t)})")


if __name__ == "__main__":
    main()
