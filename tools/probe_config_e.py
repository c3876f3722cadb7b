"""Probe (GPU, diagnostic): where a config-E frame's time goes -- the T=2^22 L16F2 network on the fox photos with
aabb_scale 64 (tests/test_gpu_config_e.py's scene).  Prints the render's debug statistics (init lattice steps per ray,
passes, generate iterations, slots, samples), the per-class kernel timers and frame times for a few march schedules.

  python tools/probe_config_e.py [pretrain steps]
"""
import ctypes as C
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), os.path.join(ROOT, "tests")]
import ngp_abi as A  # noqa: E402
import pyngp as ngp  # noqa: E402
from test_gpu_config_e import fox_aabb64  # noqa: E402


def frame(tb, lib, h, label, n=3):
    tb.render_to_device(1920, 1080, 1, True)
    A.check(lib.ngp_timing_enable(h, 0))  # frame time without the per-dispatch timer events
    t0 = time.perf_counter()
    for _ in range(n):
        tb.render_to_device(1920, 1080, 1, True)
    dt = (time.perf_counter() - t0) / n
    A.check(lib.ngp_timing_enable(h, -1))
    for name in A.TIMERS:
        lib.ngp_timing_read(h, A.TIMER[name], None, None, None, 1)
    for _ in range(n):
        tb.render_to_device(1920, 1080, 1, True)
    res = {}
    for name in ("render_march", "render_encode", "render_mlp"):
        ms, u, k = C.c_double(), C.c_uint64(), C.c_uint32()
        A.check(lib.ngp_timing_read(h, A.TIMER[name], C.byref(ms), C.byref(u), C.byref(k), 1))
        res[name] = (ms.value / n, u.value / n, k.value / n)
    print(f"{label:36s} frame={dt * 1e3:7.2f}ms " + " ".join(f"{k}={v[0]:.2f}ms/{v[2]:.0f}x/{v[1] / 1e6:.2f}M" for k, v in res.items()),
          flush=True)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    with tempfile.TemporaryDirectory() as d:
        tb = ngp.Testbed(ngp.TestbedMode.Nerf)
        tb.load_training_data(fox_aabb64(d))
        tb.reload_network_from_file("bicycle_L16F2T22.json")
        tb.shall_train = True
        for _ in range(steps):
            tb.train(1 << 18)
        tb.set_camera_to_training_view(3)
        lib = A.load()
        h = C.c_void_p(tb.model_handle)
        tb.set_tuning({"debug": 1})
        tb.render_to_device(1920, 1080, 1, True)  # prints the [render] statistics line
        tb.set_tuning({"debug": 0})
        A.check(lib.ngp_timing_enable(h, -1))
        frame(tb, lib, h, "default")
        variants = ({"render_pipelines": 1}, {"render_pipelines": 3}, {"render_lanes": 1 << 23}, {"render_lanes": 1 << 21},
                    {"render_max_steps": 64}, {"render_max_steps": 16}, {"render_first_steps": 16}, {"render_pass_samples": 10 << 20},
                    {"render_pass_samples": 4 << 20}, {"render_lag": 3}, {"render_exit_cap": 1}, {"mlp_workgroups_per_cu": 8})
        for kw in variants + variants:  # twice: the second round shows the spread
            frame(tb, lib, h, "default")
            tb.set_tuning(kw)
            frame(tb, lib, h, str(kw))
            tb.set_tuning({k: 0 for k in kw})
        A.check(lib.ngp_timing_enable(h, 0))
        del tb


if __name__ == "__main__":
    main()
