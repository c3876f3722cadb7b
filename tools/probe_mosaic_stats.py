"""Probe (GPU, diagnostic): the statistics test_trained_field_against_the_reference_density_mosaic asserts (test2 scene,
base.json, 35k steps), for several seeds, with nondeterministic (default) and deterministic (fixed-point grid gradient)
training: per seed the occupied ratio to the reference and the identity-orientation correlation / rank of that seed alone,
and per pair of seeds the test's pooled statistics.
  python tools/probe_mosaic_stats.py [--deterministic 0 1] [--seeds 1337 42 7 2024]"""
import argparse
import itertools
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), os.path.join(ROOT, "tests")]
import density_slices_util as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[1337, 42, 7, 2024])
    ap.add_argument("--deterministic", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--steps", type=int, default=35000)
    a = ap.parse_args()
    import pyngp as ngp
    cref = D.coarse(D.reference_volume("test2") >= 129)
    for det in a.deterministic:
        co = {}
        for seed in a.seeds:
            t0 = time.time()
            tb = D.new_testbed(ngp, "test2", "base.json", seed)
            tb.deterministic = bool(det)
            D.train_to(tb, a.steps)
            co[seed] = D.coarse(D.testbed_volume(tb) >= 129)
            ident, rank = D.orientation_ranking(co[seed], cref)
            print(f"det {det} seed {seed}: ratio {co[seed].mean() / cref.mean():.2f} corr {ident:.3f} rank {rank} "
                  f"loss {tb.loss:.5f} ({time.time() - t0:.0f} s)", flush=True)
            del tb
        for s1, s2 in itertools.combinations(a.seeds, 2):
            ours = (co[s1] + co[s2]) / 2
            ident, rank = D.orientation_ranking(ours, cref)
            sc = float(np.corrcoef(co[s1].ravel(), co[s2].ravel())[0, 1])
            print(f"det {det} pair {s1}/{s2}: corr {ident:.3f} rank {rank} seeds_corr {sc:.3f} ratio {ours.mean() / cref.mean():.2f}",
                  flush=True)


if __name__ == "__main__":
    main()
