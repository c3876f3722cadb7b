"""Standalone fused-MLP microbenchmark at SURVEY §8(d)'s sizes.

* render MLP: the renderer's network call (ngp_model_infer_sh_rows -> k_mlp_infer_rf with per-ray SH rows),
  n = 2^21 samples (src/testbed_nerf.cu:1697's render query batch), 32 samples per ray;
* training MLP: k_mlp_train (forward + dgrad + wgrad) through ngp_model_backward, n = 2^18 (the training batch).

Config B network (L16 F2 T2^19: density 32->64->16, rgb 32->64->64->16), Xavier-uniform weights (the model's
init, tcnn's), encodings N(0, 0.1^2) fp16, directions uniform on the sphere, all seeded (pcg-free numpy seed
1337: synthetic inputs, not a trained field).  Times come from the kernel timers (HIP events riding on the MLP
dispatch alone, ngp_timing_read).  Prints one JSON object:
    {"render": {tile: {"us": .., "tflops": .., "frac": ..}}, "train": {...}}
FLOP per sample: 20,480 forward (as executed), 61,440 forward + backward; peak 2.5 PFLOP/s dense
fp16 (MI355X_MICROARCH.md:43).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "instant-ngp-rendering_amd"))
import ngp_abi as A  # noqa: E402

PEAK = 2.5e15
FLOP_FWD, FLOP_TRAIN = 20480, 61440


def sh_deg4(d):
    x, y, z = (2 * d[:, 0] - 1), (2 * d[:, 1] - 1), (2 * d[:, 2] - 1)
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    c = [np.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
         -0.48860251190291987 * x, 1.0925484305920792 * xy, -1.0925484305920792 * yz,
         0.94617469575755997 * z2 - 0.31539156525251999, -1.0925484305920792 * xz,
         0.54627421529603959 * (x2 - y2), 0.59004358992664352 * y * (-3 * x2 + y2), 2.8906114426405538 * xy * z,
         0.45704579946446572 * y * (1 - 5 * z2), 0.3731763325901154 * z * (5 * z2 - 3),
         0.45704579946446572 * x * (1 - 5 * z2), 1.4453057213202769 * z * (x2 - y2),
         0.59004358992664352 * x * (-x2 + 3 * y2)]
    return np.stack(c, 1).astype(np.float16)


def timer(lib, h, idx):
    ms, units, launches = C.c_double(), C.c_uint64(), C.c_uint32()
    A.check(lib.ngp_timing_read(h, idx, C.byref(ms), C.byref(units), C.byref(launches), 1))
    return ms.value, units.value, launches.value


def measure(configs=((0, 0, 0), (3, 2, 4), (2, 2, 4), (2, 4, 2), (1, 4, 0)), n_render=1 << 21, n_train=1 << 18, iters=40,
            samples_per_ray=32, device=0):
    """The render MLP under each (render_mlp_pipeline, render_mlp_tile, mlp_workgroups_per_cu) and the training MLP;
    returns the result dict (see the module docstring).  Every render configuration's output must be bit-identical."""
    torch.cuda.set_device(device)
    lib = A.load()
    cfg = A.default_config()
    h = C.c_void_p()
    A.check(lib.ngp_model_create(device, C.byref(cfg), 1337, C.byref(h)))
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(1337)
    L, F = cfg.n_levels, cfg.n_features_per_level
    out = {"config": "L16F2T19 density 32-64-16 rgb 32-64-64-16, Xavier weights, enc N(0,0.1^2) fp16, "
                     f"{samples_per_ray} samples per SH row", "peak_tflops": PEAK / 1e12, "render": {}, "train": {}}
    try:
        n = n_render
        rays = (n + samples_per_ray - 1) // samples_per_ray
        enc = torch.from_numpy((rng.standard_normal((L, n, F)) * 0.1).astype(np.float16)).cuda()
        d = rng.standard_normal((rays, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        shr = torch.from_numpy(sh_deg4((d + 1) * 0.5)).cuda()
        ri = torch.from_numpy((np.arange(n) // samples_per_ray).astype(np.int32)).cuda()
        o = torch.zeros(n * 4, dtype=torch.float16, device="cuda")
        ref = None
        for pipe, tile, wg in configs:
            t = A.Tuning()
            A.check(lib.ngp_model_get_tuning(h, C.byref(t)))
            t.render_mlp_tile, t.mlp_workgroups_per_cu, t.render_mlp_pipeline = tile, wg, pipe
            A.check(lib.ngp_model_set_tuning(h, C.byref(t)))
            call = lambda: A.check(lib.ngp_model_infer_sh_rows(h, C.c_void_p(enc.data_ptr()), C.c_void_p(shr.data_ptr()),
                                                               C.c_void_p(ri.data_ptr()), n, rays, C.c_void_p(o.data_ptr()),
                                                               0, s))
            A.check(lib.ngp_timing_enable(h, 0))
            # warm-up (the first configuration also brings the clocks up: 3 calls left it 3 % slow)
            for _ in range(10 if ref is not None else 60):
                call()
            torch.cuda.synchronize()
            res = o.clone()
            if ref is None:
                ref = res
            A.check(lib.ngp_timing_enable(h, 1 << A.TIMER["render_mlp"]))
            timer(lib, h, A.TIMER["render_mlp"])  # reset
            for _ in range(iters):
                call()
            torch.cuda.synchronize()
            ms, units, launches = timer(lib, h, A.TIMER["render_mlp"])
            A.check(lib.ngp_timing_enable(h, 0))
            us = ms / max(launches, 1) * 1e3
            tf = FLOP_FWD * n / (us * 1e-6) / 1e12
            key = "default" if not (pipe or tile or wg) else f"pipe{pipe}_tile{tile}" + (f"_wg{wg}" if wg else "")
            out["render"][key] = {"n": n, "us": round(us, 2), "tflops": round(tf, 1), "frac": round(tf * 1e12 / PEAK, 4),
                                  "launches": launches, "equal_to_first": bool(torch.equal(res, ref))}
        best = max(out["render"], key=lambda k: out["render"][k]["frac"])
        out["render_best"] = dict(out["render"][best], tuning=best)
        out["render_default"] = out["render"].get("default")  # the untuned standalone schedule

        n = n_train
        enc = torch.from_numpy((rng.standard_normal((L, n, F)) * 0.1).astype(np.float16)).cuda()
        d = rng.standard_normal((n, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        dirs = torch.from_numpy(((d + 1) * 0.5).astype(np.float32)).cuda()
        dl = torch.from_numpy((rng.standard_normal((n, 4)) * 1e-2).astype(np.float16)).cuda()
        denc = torch.zeros(L * n * F, dtype=torch.float16, device="cuda")
        call = lambda: A.check(lib.ngp_model_backward(h, C.c_void_p(enc.data_ptr()), C.c_void_p(dirs.data_ptr()), n,
                                                      C.c_void_p(dl.data_ptr()), None, C.c_void_p(denc.data_ptr()), s))
        for _ in range(3):
            call()
        A.check(lib.ngp_timing_enable(h, 1 << A.TIMER["train_mlp_bwd"]))
        timer(lib, h, A.TIMER["train_mlp_bwd"])
        for _ in range(max(iters // 4, 5)):
            call()
        torch.cuda.synchronize()
        ms, units, launches = timer(lib, h, A.TIMER["train_mlp_bwd"])
        A.check(lib.ngp_timing_enable(h, 0))
        us = ms / max(launches, 1) * 1e3
        tf = FLOP_TRAIN * n / (us * 1e-6) / 1e12
        out["train"] = {"n": n, "us": round(us, 2), "tflops": round(tf, 1), "frac": round(tf * 1e12 / PEAK, 4),
                        "launches": launches}
    finally:
        torch.cuda.synchronize()
        A.check(lib.ngp_model_destroy(h))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-render", type=int, default=1 << 21)
    ap.add_argument("--n-train", type=int, default=1 << 18)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--tiles", default="4,2,1")
    ap.add_argument("--wg", default="0", help="render-MLP workgroups per CU to sweep (0 = default)")
    ap.add_argument("--pipes", default="1,2,3", help="ngp_tuning.render_mlp_pipeline values to sweep (1 = round 5)")
    ap.add_argument("--samples-per-ray", type=int, default=32)
    args = ap.parse_args()
    configs = [(int(p), int(t), int(w)) for w in args.wg.split(",") for p in args.pipes.split(",") for t in args.tiles.split(",")]
    out = measure(configs, args.n_render, args.n_train, args.iters, args.samples_per_ray)
    for k, v in out["render"].items():
        print(k, v, flush=True)
    print("train", out["train"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
