"""Writes the procedural lego-shaped scene (instant-ngp-rendering_amd/synthetic.py) in the
nerf_synthetic layout with a TRUE held-out split: 100 training views and 200 test views of the
same static object from different hemisphere cameras, 800x800 RGBA PNG (lego's shape, which is
not available offline).  Usage (GPU box): python tools/make_synthetic_scene.py /tmp/synth"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), os.path.join(ROOT, "tests")]
import synthetic  # noqa: E402

if __name__ == "__main__":
    out = sys.argv[1]
    n_train = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    n_test = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    res = int(sys.argv[4]) if len(sys.argv) > 4 else 800
    dev = "cuda" if os.environ.get("SYNTH_DEVICE", "cuda") == "cuda" else None
    synthetic.write_nerf_synthetic_scene(out, n_train, res, res, seed=0, split="train", device=dev)
    synthetic.write_nerf_synthetic_scene(out, n_test, res, res, seed=1, split="test", device=dev)
    print(f"wrote {n_train} train + {n_test} test views to {out}", file=sys.stderr)
