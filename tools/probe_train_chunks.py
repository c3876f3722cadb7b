"""Probe (GPU, diagnostic): the training batch's samples per ray against what chunked forward schedules would
evaluate (ngp_tuning.debug bit 1 prints one '[train] ...' line per step) on bench.py's surface scene or the fire scene.
  python tools/probe_train_chunks.py [synthetic|fire] [pretrain steps]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), ROOT, os.path.join(ROOT, "tests")]


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "synthetic"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    if scene == "synthetic":
        import torch
        torch.cuda.set_device(0)
    import pyngp as ngp
    tb = ngp.Testbed(ngp.TestbedMode.Nerf)
    if scene == "synthetic":
        import bench
        bench.make_dataset(ngp, tb, argparse.Namespace(scene="synthetic", views=100, train_res=800), "cuda:0")
    else:
        tb.load_training_data(os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"))
    tb.reload_network_from_file(os.path.join(ROOT, "instant-ngp-rendering_amd", "configs", "nerf", "lego_L16F2.json"))
    tb.shall_train = True
    for _ in range(steps):
        tb.train(1 << 18)
    tb.set_tuning({"debug": 2})
    for _ in range(4):
        tb.train(1 << 18)
    tb.sync()
    tb.set_tuning({"debug": 0})
    print("stats", tb.last_train_stats(), flush=True)


if __name__ == "__main__":
    main()
