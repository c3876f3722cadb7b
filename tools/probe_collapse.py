"""Probe (GPU, diagnostic): the training trajectory of a seed whose test2 field collapsed in tools/probe_mosaic_stats.py --
loss, batch sizes, rays per batch, occupied density-grid fraction and the parameters' finiteness every 1000 steps.
  python tools/probe_collapse.py SEED [DETERMINISTIC]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), os.path.join(ROOT, "tests")]
import density_slices_util as D  # noqa: E402


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 2024
    det = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    import pyngp as ngp
    tb = D.new_testbed(ngp, "test2", "base.json", seed)
    tb.deterministic = bool(det)
    for target in list(range(500, 5000, 500)) + list(range(5000, 36000, 2500)):
        D.train_to(tb, target)
        st = tb.last_train_stats()
        grid = tb.density_grid()
        bits = tb.density_grid_bitfield()
        p = tb.snapshot_params() if hasattr(tb, "snapshot_params") else None
        print(f"step {tb.training_step:6d} loss {tb.loss:.6f} batch {st['measured_batch_size']:7d} before {st['measured_batch_size_before_compaction']:8d} "
              f"rays {st['n_rays']:6d} grid mean {float(np.mean(grid)):.4f} max {float(np.max(grid)):.3g} finite {bool(np.isfinite(grid).all())} "
              f"occupied {float(np.unpackbits(bits).mean()):.4f}", flush=True)


if __name__ == "__main__":
    main()
