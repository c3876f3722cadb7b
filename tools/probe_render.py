"""Probe: render-march cost vs samples-per-pass cap on a briefly trained synthetic scene (diagnostic, GPU)."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd"), os.path.join(ROOT, "tests")]
import torch
import ngp_abi as A
import pyngp as ngp
import synthetic

tb = ngp.Testbed(ngp.TestbedMode.Nerf)
cams = synthetic.hemisphere_cameras(100, seed=0)
focal = synthetic.focal_from_angle(800)
imgs = synthetic.render_views(cams, 800, 800, focal, device="cuda")
tb.create_empty_nerf_dataset(100, aabb_scale=1)
for i in range(100):
    tb.nerf.training.set_image_rgba8(i, imgs[i])
    tb.nerf.training.set_camera_extrinsics(i, cams[i], convert_to_ngp=False)
    tb.nerf.training.set_camera_intrinsics(i, fx=focal, fy=focal)
tb.nerf.training.n_images_for_training = 100
tb.reload_network_from_file("lego_L16F2.json")
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 500):
    tb.train(1 << 18)
lib = A.load()
h = C.c_void_p(tb.model_handle)
A.check(lib.ngp_timing_enable(h, int(os.environ.get("TIMER_MASK", "-1"))))
tb.set_camera_to_training_view(3)
for cap in [int(c) for c in os.environ.get("CAPS", "1,4,8,16,32,64,128").split(",")]:
    tb.set_tuning({"render_max_steps": cap})
    tb.render_to_device(1920, 1080, 1, True)
    for name in A.TIMERS:
        lib.ngp_timing_read(h, A.TIMER[name], None, None, None, 1)
    t0 = time.perf_counter()
    for _ in range(3):
        tb.render_to_device(1920, 1080, 1, True)
    dt = (time.perf_counter() - t0) / 3
    res = {}
    for name in ("render_march", "render_encode", "render_mlp"):
        ms, u, n = C.c_double(), C.c_uint64(), C.c_uint32()
        A.check(lib.ngp_timing_read(h, A.TIMER[name], C.byref(ms), C.byref(u), C.byref(n), 1))
        res[name] = (ms.value / 3, u.value / 3, n.value / 3)
    print(f"cap={cap:4d} frame={dt*1e3:7.2f}ms " + " ".join(f"{k}={v[0]:.2f}ms/{v[2]:.0f}x/{v[1]/1e6:.2f}M" for k, v in res.items()), flush=True)

if os.environ.get("DUMP"):
    import numpy as np
    bits = tb.density_grid_bitfield()
    np.savez(os.path.join(ROOT, "gpurun_out", "render_state.npz"), bits=bits, cam=np.asarray(tb.camera_matrix),
             rel_focal=np.asarray(tb.relative_focal_length), screen_center=np.asarray(tb.screen_center))
