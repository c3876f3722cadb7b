"""bench.py's config-E leg alone (BASELINE configs[4]'s shape on one GPU: T=2^22 L16F2, aabb_scale 64), so that
rocprofv3 kernel stats and PMC FETCH / WRITE passes see only its kernels.
Takes bench.py's arguments (--steps, --warmup, --config-e-pretrain, ...); prints the leg's JSON object.

    tools/profile_round.sh r06_config_e   with   BENCH_SCRIPT=tools/config_e_leg.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    args = bench.parse()
    import pyngp as ngp
    print(json.dumps({"config_e": bench.config_e(args, ngp)}))


if __name__ == "__main__":
    main()
