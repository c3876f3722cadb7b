"""Schedule-independence check (diagnostic, GPU box): trains the bench scene briefly, renders the bench's 1080p
view under each ngp_tuning setting and requires every frame to equal the first bit for bit.
Usage: python tools/same_frame.py [--pretrain 300] "" "render_pipelines=1" ..."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "instant-ngp-rendering_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("settings", nargs="+")
    p.add_argument("--pretrain", type=int, default=300)
    a = p.parse_args()
    import pyngp as ngp
    tb = ngp.Testbed(ngp.TestbedMode.Nerf)
    tb.load_training_data(os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"))
    tb.reload_network_from_file("lego_L16F2.json")
    tb.shall_train = True
    for _ in range(a.pretrain):
        tb.train(1 << 18)
    tb.shall_train = False
    tb.set_camera_to_training_view(3)
    ref = None
    for st in a.settings:
        tu = {}
        for kv in st.split():
            k, v = kv.split("=")
            tu[k] = float(v) if "." in v else int(v)
        tb.set_tuning(tu)
        f = tb.render(1920, 1080, 1, True)
        tb.render(1920, 1080, 1, True)  # a second frame: the adaptive schedule follows the first
        f2 = tb.render(1920, 1080, 1, True)
        if ref is None:
            ref = f2
        same = np.array_equal(f2, ref) and np.array_equal(f, f2)
        print(f"{st or 'default':40s} {'identical' if same else 'DIFFERS'} (max |d| {np.abs(f2 - ref).max():.3g})")
        if not same:
            sys.exit(1)


if __name__ == "__main__":
    main()
