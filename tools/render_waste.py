"""Probe (diagnostic, GPU): the bench scene's 1080p render under several march schedules --
frame time, and (tuning.debug bit 0) the frame's reserved sample slots, filled samples and
composited samples, i.e. how much encoder / MLP work lands past the rays' termination.
Usage: python tools/render_waste.py [pretrain_steps] ; SCHEDULES="first,max,budget,pass;..." overrides."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "instant-ngp-rendering_amd")]
import pyngp as ngp  # noqa: E402

tb = ngp.Testbed(ngp.TestbedMode.Nerf)
tb.load_training_data(os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"))
tb.reload_network_from_file("lego_L16F2.json")
tb.shall_train = True
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1500):
    tb.train(1 << 18)
tb.sync()
tb.set_camera_to_training_view(3)
spec = os.environ.get("SCHEDULES", "4,32,1,0;2,32,1,0;8,32,1,0;4,16,1,0;4,64,1,0;4,32,0.75,0;4,32,1.5,0;4,32,-1,0;4,32,1,2097152;4,32,1,8388608")
for s in spec.split(";"):
    first, mx, budget, ps = s.split(",")
    tu = {"render_first_steps": int(first), "render_max_steps": int(mx), "render_budget_scale": float(budget),
          "render_pass_samples": int(ps), "debug": 0}
    tb.set_tuning(tu)
    for _ in range(2):
        tb.render_to_device(1920, 1080, 1, True)
    t0 = time.perf_counter()
    for _ in range(5):
        tb.render_to_device(1920, 1080, 1, True)
    dt = (time.perf_counter() - t0) / 5
    print(f"schedule first={first} max={mx} budget={budget} pass_samples={ps}: {dt * 1e3:.2f} ms/frame", flush=True)
    tu["debug"] = 1
    tb.set_tuning(tu)
    sys.stderr.flush()
    tb.render_to_device(1920, 1080, 1, True)
    tb.sync()
    sys.stderr.flush()
tb.set_tuning({})
