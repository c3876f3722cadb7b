"""Per-kernel training-step timings of one build (diagnostic, GPU box): trains the bench scene with
every kernel timer on and prints the mean launch time of each timer class.  Run it once per build
(--pkg: a directory with another build of pyngp + libngp_hip, tools/ab_build_old.sh) to compare
kernels on one box.

Usage: python tools/train_kernels_ab.py [--pkg DIR] [--steps 400] [--settings "" "mlp_workgroups_per_cu=4"] [--scene synthetic]
(--settings: ngp_tuning fields per setting, timed round-robin on the same trained model)
"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "instant-ngp-rendering_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pkg", default=None)
    p.add_argument("--steps", type=int, default=400)
    p.add_argument("--timed", type=int, default=100)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--settings", nargs="*", default=[""])
    p.add_argument("--deterministic", action="store_true", help="fixed-point hash-grid gradients in every step")
    p.add_argument("--config", default=os.path.join(ROOT, "instant-ngp-rendering_amd", "configs", "nerf", "lego_L16F2.json"))
    p.add_argument("--scene", default=os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"))
    a = p.parse_args()
    if a.pkg:
        sys.path.insert(0, os.path.abspath(a.pkg))
    if a.scene == "synthetic":
        import torch  # renders the scene's views: its HIP runtime has to start before pyngp's library loads

        torch.cuda.set_device(0)
    import ngp_abi as A
    import pyngp as ngp

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
    tb.shall_train = True
    tb.deterministic = a.deterministic
    for _ in range(a.steps):
        tb.train(1 << 18)
    lib = A.load(os.path.join(os.path.abspath(a.pkg), "libngp_hip.so")) if a.pkg else A.load()
    h = C.c_void_p(tb.model_handle)
    base = tb.get_tuning()
    print(f"# pyngp {ngp.__file__}")
    acc = {st: {} for st in a.settings}
    for r in range(a.rounds):
        for st in a.settings:
            setting = dict(base)
            for kv in st.split():
                k, v = kv.split("=", 1)
                setting[k] = int(v)
            tb.set_tuning(setting)
            tb.train(1 << 18)
            tb.sync()
            # the step's wall time with the timers off, then the per-kernel pass with them on
            t0 = time.perf_counter()
            for _ in range(a.timed):
                tb.train(1 << 18)
            tb.sync()
            acc[st].setdefault("step_wall", []).append(1e6 * (time.perf_counter() - t0) / a.timed)
            A.check(lib.ngp_timing_enable(h, -1))
            for idx in A.TIMER.values():  # discard what the warm-up step accumulated
                A.check(lib.ngp_timing_read(h, idx, None, None, None, 1))
            for _ in range(a.timed):
                tb.train(1 << 18)
            tb.sync()
            for name, idx in A.TIMER.items():
                ms, units, launches = C.c_double(), C.c_uint64(), C.c_uint32()
                A.check(lib.ngp_timing_read(h, idx, C.byref(ms), C.byref(units), C.byref(launches), 1))
                if launches.value:
                    acc[st].setdefault(name, []).append(1000.0 * ms.value / launches.value)
            A.check(lib.ngp_timing_enable(h, 0))
    for st in a.settings:
        print(f"## {st or 'default'}")
        for name, v in acc[st].items():
            print(f"{name:20s} {sorted(v)[len(v) // 2]:9.2f} us/launch (median of {len(v)} rounds: {', '.join(f'{x:.2f}' for x in v)})")

if __name__ == "__main__":
    main()
