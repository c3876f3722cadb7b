"""Headline benchmark: Mrays/s of (NeRF training step + 1080p inference) on a
nerf_synthetic/lego-shaped scene (BASELINE.json configs[1]: L=16 F=2 T=2^19,
density 1x64 + rgb 2x64 MLPs) through the pyngp Testbed on MI355X.

One "step" = Testbed.train(2^18) (density-grid update at the reference cadence,
sampler, fused MLP fwd/bwd, hash-grid scatter, Adam) + one 1920x1080 spp=1
render kept in HBM.  value = (training rays + rendered rays, all ranks) / max
over ranks of the timed wall time.  N>1: one process per GPU (torchrun), each
rank trains on its own rays with the gradients all-reduced over RCCL every step
and renders its own 1080p view (weak scaling).

The roofline block is computed from HIP events recorded around each launch
group on the Testbed's stream during the timed region (ngp_timing_read), the
cpu_baseline block from the scalar CPU oracle (oracle/, test infrastructure)
timed on a bounded sample of the same workload on rank 0.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "instant-ngp-rendering_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16/bf16 MFMA, no sparsity (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--pretrain", type=int, default=1500, help="untimed training steps before warmup (grid converges)")
    p.add_argument("--config", default="lego_L16F2.json")
    p.add_argument("--batch", type=int, default=1 << 18)
    p.add_argument("--views", type=int, default=100)
    p.add_argument("--train-res", type=int, default=800)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--kernel-timer", type=int, default=1,
                   help="time the dominant kernel in the timed run (0: diagnostic runs without timer events)")
    p.add_argument("--cpu-rows", type=int, default=8, help="1080p rows rendered by the CPU oracle sample")
    p.add_argument("--cpu-rays", type=int, default=512, help="training rays in the CPU oracle sample")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01_pmc_traffic.json"),
                   help="per-kernel HBM bytes from rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes (tools/pmc_traffic.py)")
    return p.parse_args()


def mlp_macs_per_sample(info_cfg):
    L, F, W = info_cfg["n_levels"], info_cfg["F"], info_cfg["W"]
    dh, rh = info_cfg["dh"], info_cfg["rh"]
    enc = L * F
    dens = enc * W + (dh - 1) * W * W + W * 16
    rgb = 32 * W + (rh - 1) * W * W + W * 16
    return dens + rgb


def kernel_models(cfg):
    """Algorithmic bytes (hbm) or flops (mfma) per unit for each timer (DESIGN.md "Kernels")."""
    L, F = cfg["n_levels"], cfg["F"]
    macs = mlp_macs_per_sample(cfg)
    enc_fwd_bytes = L * 8 * F * 2 + 12 + L * F * 2  # 8 corner gathers (fp16) per level + pos + encoded output
    enc_bwd_bytes = L * 8 * F * 2 * 2 + 12 + L * F * 2  # fp16 packed atomic RMW per corner + pos + dL/denc
    return {
        "train_encode": ("hbm", enc_fwd_bytes),
        "render_encode": ("hbm", enc_fwd_bytes),
        "train_encode_bwd": ("hbm", enc_bwd_bytes),
        "train_mlp_infer": ("mfma", 2 * macs),
        "render_mlp": ("mfma", 2 * macs),
        "train_mlp_bwd": ("mfma", 6 * macs),  # fwd + dgrad + wgrad
        "optimizer": ("hbm", 44),  # w32,g,m,v,step in; w32,w16,m,v,step,ema32,ema16 out
    }


def make_dataset(ngp, tb, n_views, res, device):
    import synthetic

    cams = synthetic.hemisphere_cameras(n_views, seed=0)
    focal = synthetic.focal_from_angle(res)
    imgs = synthetic.render_views(cams, res, res, focal, device=device)
    tb.create_empty_nerf_dataset(n_views, aabb_scale=1)
    for i in range(n_views):
        tb.nerf.training.set_image_rgba8(i, imgs[i])
        tb.nerf.training.set_camera_extrinsics(i, cams[i], convert_to_ngp=False)
        tb.nerf.training.set_camera_intrinsics(i, fx=focal, fy=focal)
    tb.nerf.training.n_images_for_training = n_views  # as the reference's create_empty_nerf_dataset callers do
    return cams, imgs, focal


# timer -> kernel (name pattern) whose PMC counters describe it
TIMER_KERNEL = {"train_encode": r"k_hashgrid_fwd<\d+u, 0[,>]", "render_encode": r"k_hashgrid_fwd<\d+u, 1[,>]",
                "train_encode_bwd": r"k_hashgrid_bwd<", "train_mlp_infer": r"k_mlp_infer_rf<.*, false, \d>$",
                "render_mlp": r"k_mlp_infer_rf<.*, false, \d>$", "train_mlp_bwd": r"k_mlp_train<",
                "optimizer": r"k_optimizer"}


def pmc_traffic(path, timer, units_per_launch):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary (or None).
    The PMC run profiles the same workload, so its mean bytes per launch are used directly
    (launch grids are sized by upper bounds, so per-sample figures from the grid size would
    undercount)."""
    if not os.path.exists(path) or timer not in TIMER_KERNEL:
        return None
    import re

    data = json.load(open(path))
    for name, e in data.items():
        if not re.search(TIMER_KERNEL[timer], name):
            continue
        return round(e.get("fetch_bytes_per_launch", 0) + e.get("write_bytes_per_launch", 0))
    return None


def read_timers(abi, lib, handle):
    out = {}
    for name, idx in abi.TIMER.items():
        ms, units, launches = C.c_double(), C.c_uint64(), C.c_uint32()
        abi.check(lib.ngp_timing_read(C.c_void_p(handle), idx, C.byref(ms), C.byref(units), C.byref(launches), 1))
        out[name] = (ms.value, units.value, launches.value)
    return out


def cpu_baseline(args, tb, cams, imgs, focal, cfg_abi, W, H):
    """Scalar oracle (1 core) on a bounded sample: one training step of --cpu-rays rays
    and --cpu-rows rows of the 1080p frame, with the GPU's trained weights and grid."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ngp_abi as A
    from oracle_abi import Oracle
    from scene_util import HostDataset, pcg_seed, render_args, train_args

    o = Oracle(cfg_abi)
    lib = A.load()
    h = C.c_void_p(tb.model_handle)
    p, n = C.c_void_p(), C.c_size_t()
    A.check(lib.ngp_model_buffer(h, A.PARAMS_FP32, C.byref(p), C.byref(n)))
    import torch

    params = torch.empty(n.value // 4, dtype=torch.float32, device="cuda")
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    tb.sync()
    hip.hipMemcpy(C.c_void_p(params.data_ptr()), p, n.value, 3)
    params = params.cpu().numpy()
    o.set_params(params)
    grid = tb.density_grid()
    o.grid_set(grid)
    o.grid_bitfield(0)

    n_sub = min(len(imgs), 8)
    hd = HostDataset(imgs[:n_sub], cams[:n_sub], focal)
    R = args.cpu_rays
    ta = train_args(hd.ptr, hd.n, R, 1 << 14, 16 * (1 << 14))
    t0 = time.perf_counter()
    o.train_step(ta)
    o.optimizer_step(0, 1, 1)
    t_train = time.perf_counter() - t0

    tb.set_camera_to_training_view(0)
    cam = np.asarray(tb.camera_matrix, np.float32)
    f = tb.relative_focal_length[1] * H
    rows = args.cpu_rows
    ra = render_args(W, H, cam, f, spp=0, snap=0, shard=(H // (2 * rows), H // rows, rows), min_transmittance=0.01)
    t0 = time.perf_counter()
    o.render(ra)
    t_render = time.perf_counter() - t0
    rays = R + W * rows
    secs = t_train + t_render
    return {"value": rays / secs / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"scalar oracle: 1 train step of {R} rays (+Adam over {params.size} params) in {t_train:.2f}s "
                      f"+ {rows} rows of a {W}x{H} frame ({W * rows} rays) in {t_render:.2f}s, same weights/grid"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    if world > 1:
        # host control plane only (unique-id exchange, barriers, max-over-ranks); the data
        # path (gradient / grid all-reduce) runs on the Testbed's own RCCL communicator.
        dist.init_process_group("gloo", rank=rank, world_size=world)

    import ngp_abi as A
    import pyngp as ngp

    tb = ngp.Testbed(ngp.TestbedMode.Nerf)
    cams, imgs, focal = make_dataset(ngp, tb, args.views, args.train_res, f"cuda:{local_rank}")
    tb.reload_network_from_file(args.config)
    if world > 1:
        uid = [ngp.Testbed.nccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        tb.init_distributed(rank, world, uid[0])
    tb.shall_train = True
    W, H = args.width, args.height

    def barrier():
        tb.sync()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    t_pre = time.perf_counter()
    for i in range(args.pretrain):
        tb.train(args.batch)
        if rank == 0 and (i + 1) % 250 == 0:
            print(f"# pretrain {i + 1}/{args.pretrain} loss {tb.loss:.5f} "
                  f"rays/batch {tb.last_train_stats()['rays_per_batch']} ({time.perf_counter() - t_pre:.1f}s)",
                  file=sys.stderr, flush=True)
    view = (rank * 7 + 3) % args.views

    split = {"train_s": 0.0, "render_s": 0.0, "train_rays": 0, "render_rays": 0}

    def step():
        t0 = time.perf_counter()
        tb.train(args.batch)  # returns after the stream is synchronised (Testbed::train)
        t1 = time.perf_counter()
        rays = tb.last_train_stats()["n_rays"]
        tb.set_camera_to_training_view(view)
        tb.render_to_device(W, H, 1, True)  # synchronised as well
        t2 = time.perf_counter()
        split["train_s"] += t1 - t0
        split["render_s"] += t2 - t1
        split["train_rays"] += rays
        split["render_rays"] += W * H
        return rays + W * H

    lib = A.load()
    h = tb.model_handle
    cfg = tb.network_config
    enc = cfg["encoding"]
    mcfg = {"n_levels": int(enc["n_levels"]), "F": int(enc["n_features_per_level"]),
            "W": int(cfg["network"]["n_neurons"]), "dh": int(cfg["network"]["n_hidden_layers"]),
            "rh": int(cfg["rgb_network"]["n_hidden_layers"])}
    models = kernel_models(mcfg)

    # warmup; its last steps run with every kernel timer on to find the dominant kernel
    # (events between launches cost GPU time, so the timed run keeps only that one timer)
    n_cal = min(args.warmup, 3)
    for i in range(args.warmup):
        if i == args.warmup - n_cal:
            A.check(lib.ngp_timing_enable(C.c_void_p(h), -1))
            read_timers(A, lib, h)
        step()
    calib = read_timers(A, lib, h)
    modeled = [k for k in models if calib.get(k, (0, 0, 0))[2] > 0]
    dom = max(modeled, key=lambda k: calib[k][0]) if modeled else "render_encode"
    A.check(lib.ngp_timing_enable(C.c_void_p(h), (1 << A.TIMER[dom]) if args.kernel_timer else 0))
    read_timers(A, lib, h)  # reset

    barrier()
    for k in split:
        split[k] = 0
    t0 = time.perf_counter()
    rays = 0
    for _ in range(args.steps):
        rays += step()
    barrier()
    elapsed = time.perf_counter() - t0
    timers = read_timers(A, lib, h)
    A.check(lib.ngp_timing_enable(C.c_void_p(h), 0))

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays], dtype=torch.float64)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays = int(r.item())

    kernels = {}
    for name, (ms, units, launches) in calib.items():
        if launches == 0:
            continue
        entry = {"ms_total": round(ms, 3), "launches": launches, "units": units,
                 "us_per_launch": round(1000.0 * ms / launches, 2)}
        if name in models and ms > 0:
            bound, per_unit = models[name]
            rate = units * per_unit / (ms / 1000.0)
            if bound == "hbm":
                entry["GB/s"] = round(rate / 1e9, 1)
                entry["frac"] = round(rate / 1e9 / HBM_PEAK_GBS, 4)
            else:
                entry["TFLOP/s"] = round(rate / 1e12, 2)
                entry["frac"] = round(rate / 1e12 / MFMA_F16_PEAK_TFLOPS, 4)
        kernels[name] = entry
    bound, per_unit = models[dom]
    ms, units, launches = timers[dom] if args.kernel_timer else calib[dom]
    achieved = units * per_unit / launches / (ms / launches / 1000.0)
    roofline = {
        "kernel": dom,
        "bound": bound,
        "achieved": round(achieved / (1e9 if bound == "hbm" else 1e12), 2),
        "peak": HBM_PEAK_GBS if bound == "hbm" else MFMA_F16_PEAK_TFLOPS,
        "unit": "GB/s" if bound == "hbm" else "TFLOP/s",
        "traffic": None,
        "per_unit": per_unit,
        "units_per_launch": round(units / launches),
        "us_per_launch": round(1000.0 * ms / launches, 2),
    }
    roofline["frac"] = round(roofline["achieved"] / roofline["peak"], 4)
    roofline["traffic"] = pmc_traffic(args.traffic_json, dom, units / launches)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        from ngp_abi import default_config

        cfg_abi = default_config(n_levels=mcfg["n_levels"], F=mcfg["F"], log2_T=int(enc["log2_hashmap_size"]),
                                 n_neurons=mcfg["W"], density_hidden=mcfg["dh"], rgb_hidden=mcfg["rh"])
        cpu = cpu_baseline(args, tb, cams, imgs, focal, cfg_abi, W, H)

    value = rays / elapsed / 1e6
    if rank == 0:
        line = {
            "metric": "Mrays/sec (train step + 1080p inference), nerf_synthetic/lego, 1→8 MI355X",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f16-mfma/f32-accum",
            "data": f"synthetic lego-shaped scene ({args.views} views {args.train_res}x{args.train_res} RGBA8, "
                    f"random-init weights trained {args.pretrain} steps before timing)",
            "config": {"workload": "lego L16F2T19 MLP 64 (1x density + 2x rgb hidden): Testbed.train(2^18) "
                                   f"+ {W}x{H} spp1 render per step", "batch": args.batch, "config_file": args.config,
                       "parallelism": f"dp{world} (RCCL grad all-reduce) + per-rank 1080p view"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "split": {"train_Mrays_s": round(split["train_rays"] / split["train_s"] / 1e6, 3),
                      "render_Mrays_s": round(split["render_rays"] / split["render_s"] / 1e6, 3),
                      "train_ms_per_step": round(1e3 * split["train_s"] / args.steps, 3),
                      "render_ms_per_frame": round(1e3 * split["render_s"] / args.steps, 3),
                      "note": "rank 0; per-part wall time inside the timed region (SURVEY 8(d) counts train and inference separately)"},
            "kernels_calibration": kernels,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
