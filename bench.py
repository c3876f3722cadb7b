"""Headline benchmark: Mrays/s of (NeRF training step + 1080p inference) on a
nerf_synthetic/lego-shaped scene (BASELINE.json configs[1]: L=16 F=2 T=2^19,
density 1x64 + rgb 2x64 MLPs) through the pyngp Testbed on MI355X.

One "step" = Testbed.train(2^18) (density-grid update at the reference cadence,
sampler, fused MLP fwd/bwd, hash-grid scatter, Adam) + one Testbed.render(1920,
1080, spp=1) -- the float frame read back to host memory, as BASELINE.md counts
inference.  value = (training rays + rendered rays, all ranks) / max over ranks
of the timed wall time.  N>1: one process per GPU (torchrun), each
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
TESTS = os.path.join(ROOT, "tests")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16/bf16 MFMA, no sparsity (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--pretrain", type=int, default=1500, help="untimed training steps before warmup (grid converges)")
    p.add_argument("--deterministic-pretrain", type=int, default=1,
                   help="pretrain with bit-reproducible hash-grid gradients (Testbed.deterministic), so every run times "
                        "the same trained scene (its samples per 1080p frame otherwise vary by +-10 %% run to run); "
                        "the timed steps use the default fp16-atomic path")
    p.add_argument("--config", default="lego_L16F2.json")
    p.add_argument("--scene", default=os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"),
                   help="transforms.json of the scene to train on, or 'synthetic' for the procedural lego-shaped one")
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
    p.add_argument("--surface-scene", type=int, default=1,
                   help="N=1: also time the procedural lego-shaped SURFACE scene (train + 1080p render) -> surface_scene")
    p.add_argument("--config-e", type=int, default=1,
                   help="N=1: also time BASELINE config E's shape (T=2^22 L16F2 network, aabb_scale 64 scene) -> config_e")
    p.add_argument("--config-e-pretrain", type=int, default=500)
    p.add_argument("--mlp-microbench", type=int, default=1,
                   help="time the fused MLPs alone at 2^21 / 2^18 samples after the timed region (tools/mlp_microbench.py)")
    p.add_argument("--render-in-hbm", type=int, default=5,
                   help="N=1: 1080p renders timed through render_to_device() (the frame stays in HBM) -> render_in_hbm")
    p.add_argument("--surface-traffic-json", default=os.path.join(ROOT, "profiles", "r06_final_surface_pmc_traffic.json"),
                   help="PMC traffic summary of the surface-scene bench (tools/pmc_traffic.py)")
    p.add_argument("--config-e-traffic-json", default=os.path.join(ROOT, "profiles", "r06_config_e_final_pmc_traffic.json"),
                   help="PMC FETCH/WRITE summary of the config-E leg alone (tools/config_e_leg.py under tools/profile_round.sh)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r06_final_pmc_traffic.json"),
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
        # init/generate/composite/shade: 28 B per filled sample + 36 B per ray;
        # units are rays, the per-sample part comes from the render's filled-sample count
        "render_march": ("hbm", None),
    }


MARCH_B_PER_SAMPLE, MARCH_B_PER_RAY = 28, 36


def model_bytes(name, per_unit, units, timers):
    """Algorithmic bytes (or flops) of a timer's launches."""
    if name == "render_march":
        return units * MARCH_B_PER_RAY + timers["render_encode"][1] * MARCH_B_PER_SAMPLE
    return units * per_unit


def make_dataset(ngp, tb, args, device):
    """The bench scene: a transforms.json through the Testbed's loader (default: the reference's
    data/nerf/test/dataset, SURVEY 8(d)'s stand-in for lego), or the procedural lego-shaped scene.
    Returns (cams [3x4 NGP], RGBA8 images, focal) for the CPU oracle's sample."""
    if args.scene != "synthetic":
        tb.load_training_data(args.scene)
        ds = tb.nerf.training.dataset
        cams = [np.asarray(x, np.float32) for x in ds.transforms]
        imgs = np.stack([ds.image(i) for i in range(ds.n_images)])
        return cams, imgs, float(ds.metadata[0].focal_length[0])
    sys.path.insert(0, TESTS)  # the procedural scene generator is a test fixture
    import synthetic

    cams = synthetic.hemisphere_cameras(args.views, seed=0)
    focal = synthetic.focal_from_angle(args.train_res)
    imgs = synthetic.render_views(cams, args.train_res, args.train_res, focal, device=device)
    tb.create_empty_nerf_dataset(args.views, aabb_scale=1)
    for i in range(args.views):
        tb.nerf.training.set_image_rgba8(i, imgs[i])
        tb.nerf.training.set_camera_extrinsics(i, cams[i], convert_to_ngp=False)
        tb.nerf.training.set_camera_intrinsics(i, fx=focal, fy=focal)
    tb.nerf.training.n_images_for_training = args.views  # as the reference's create_empty_nerf_dataset callers do
    return cams, imgs, focal


# timer -> kernel (name pattern) whose PMC counters describe it
TIMER_KERNEL = {"train_encode": r"k_hashgrid_fwd<\d+u, 0[,>]", "render_encode": r"k_hashgrid_fwd<\d+u, 1[,>]",
                "train_encode_bwd": r"k_hashgrid_bwd<", "train_mlp_infer": r"k_mlp_infer_rf<.*, false, \d+, false>$",
                "render_mlp": r"k_mlp_infer_(rf<.*, true>|sh<.*>)$", "train_mlp_bwd": r"k_mlp_train<",
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
        # FETCH corrected by the measured ratio of the kernel's read shape (tools/fetch_calib.sh) where
        # the summary carries it, as reported otherwise; WRITE as reported (exact per the guide)
        fetch = e.get("fetch_bytes_per_launch_corrected", e.get("fetch_bytes_per_launch", 0))
        return round(fetch + e.get("write_bytes_per_launch", 0))
    return None


def read_timers(abi, lib, handle):
    out = {}
    for name, idx in abi.TIMER.items():
        ms, units, launches = C.c_double(), C.c_uint64(), C.c_uint32()
        abi.check(lib.ngp_timing_read(C.c_void_p(handle), idx, C.byref(ms), C.byref(units), C.byref(launches), 1))
        out[name] = (ms.value, units.value, launches.value)
    return out


def kernel_table(calib, models):
    """Per timer: time, launches, units and the roofline fraction of its algorithmic bytes / flops."""
    kernels = {}
    for name, (ms, units, launches) in calib.items():
        if launches == 0:
            continue
        entry = {"ms_total": round(ms, 3), "launches": launches, "units": units,
                 "us_per_launch": round(1000.0 * ms / launches, 2)}
        if name in models and ms > 0:
            bound, per_unit = models[name]
            rate = model_bytes(name, per_unit, units, calib) / (ms / 1000.0)
            if bound == "hbm":
                entry["GB/s"] = round(rate / 1e9, 1)
                entry["frac"] = round(rate / 1e9 / HBM_PEAK_GBS, 4)
            else:
                entry["TFLOP/s"] = round(rate / 1e12, 2)
                entry["frac"] = round(rate / 1e12 / MFMA_F16_PEAK_TFLOPS, 4)
        kernels[name] = entry
    return kernels


def roofline_of(dom, tsrc, models):
    """The roofline block of timer `dom` from (ms, units, launches) timers: algorithmic work per launch / launch time."""
    bound, per_unit = models[dom]
    ms, units, launches = tsrc[dom]
    work = model_bytes(dom, per_unit, units, tsrc)
    achieved = work / launches / (ms / launches / 1000.0)
    r = {"kernel": dom, "bound": bound, "achieved": round(achieved / (1e9 if bound == "hbm" else 1e12), 2),
         "peak": HBM_PEAK_GBS if bound == "hbm" else MFMA_F16_PEAK_TFLOPS,
         "unit": "GB/s" if bound == "hbm" else "TFLOP/s", "traffic": None,
         "per_unit": per_unit if per_unit is not None else f"{MARCH_B_PER_SAMPLE} B/filled sample + {MARCH_B_PER_RAY} B/ray",
         "units_per_launch": round(units / launches), "bytes_or_flops_per_launch": round(work / launches),
         "us_per_launch": round(1000.0 * ms / launches, 2)}
    r["frac"] = round(r["achieved"] / r["peak"], 4)
    return r, work


def testbed_models(tb):
    cfg = tb.network_config
    enc = cfg["encoding"]
    return kernel_models({"n_levels": int(enc["n_levels"]), "F": int(enc["n_features_per_level"]),
                          "W": int(cfg["network"]["n_neurons"]), "dh": int(cfg["network"]["n_hidden_layers"]),
                          "rh": int(cfg["rgb_network"]["n_hidden_layers"])})


def timed_leg(args, tb, step):
    """Warmup (its last calibration steps with every kernel timer on), then args.steps timed steps with only the
    dominant kernel's timer; returns (seconds, step results, kernel table, roofline of the dominant kernel)."""
    import ngp_abi as A
    lib = A.load()
    h = C.c_void_p(tb.model_handle)
    models = testbed_models(tb)
    n_cal = min(args.warmup, 3)
    for i in range(args.warmup):
        if i == args.warmup - n_cal:
            A.check(lib.ngp_timing_enable(h, -1))
            read_timers(A, lib, tb.model_handle)
        step()
    calib = read_timers(A, lib, tb.model_handle)
    modeled = [k for k in models if calib.get(k, (0, 0, 0))[2] > 0 and k != "render_march"]
    dom = max(modeled, key=lambda k: calib[k][0]) if modeled else "render_encode"
    A.check(lib.ngp_timing_enable(h, 1 << A.TIMER[dom]))
    read_timers(A, lib, tb.model_handle)
    tb.sync()
    t0 = time.perf_counter()
    out = [step() for _ in range(args.steps)]
    tb.sync()
    elapsed = time.perf_counter() - t0
    timers = read_timers(A, lib, tb.model_handle)
    A.check(lib.ngp_timing_enable(h, 0))
    roof, _ = roofline_of(dom, timers, models)
    return elapsed, out, kernel_table(calib, models), roof


def cpu_baseline(args, tb, cams, imgs, focal, view, W, H, calib, n_cal):
    """The scalar C++ oracle (tests/cpu_baseline.py) on bounded samples, timed single-threaded and
    with OpenMP on min(16, hardware_concurrency) threads (the GPU box's CPU share):
      * value: one training step of --cpu-rays rays + --cpu-rows rows of the 1080p frame with the
        GPU's trained weights (EMA inference weights for the render, as the GPU renders) and grid,
        all-core; the same rows of the GPU's frame are compared with the oracle's (north_star:
        rendered RGB within 1e-3 mean L1) -> "parity";
      * config A (BASELINE configs[0]) end to end: 16 training steps + a 64x64 render;
      * config B per kernel at 2^15 samples, extrapolated to one bench step."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cpu_baseline as cb
    from scene_util import HostDataset, testbed_oracle

    tb.set_camera_to_training_view(view)
    gpu_frame = tb.render(W, H, 1, True)  # the timed workload's frame, copied to the host
    o = testbed_oracle(tb)
    hw, nth = cb.threads_for_box()
    n_sub = min(len(imgs), 8)
    hd = HostDataset(imgs[:n_sub], cams[:n_sub], focal)
    R = args.cpu_rays
    # all-core first: its rows are the parity check (the training step after them moves the weights)
    t_train, t_render, rays, ref = cb.bench_sample(o, tb, W, H, args.cpu_rows, hd, R, nth)
    ys = sorted(ref)
    l1 = float(np.abs(gpu_frame[ys, :, :3] - np.stack([ref[y] for y in ys])[..., :3]).mean())
    t1_train, t1_render, _, _ = cb.bench_sample(o, tb, W, H, args.cpu_rows, hd, R, 1)
    # single-threaded, on the box's CPU share (nth) and on every hardware thread (hw; VERDICT r05
    # item 8).  The box's scheduler share is reported beside it: threads beyond it time-slice the same cores
    legs = [("single_thread", 1), ("all_core", nth)] + ([("hardware_concurrency", hw)] if hw > nth else [])
    cfg_a = {label: cb.config_a_end_to_end(th) for label, th in legs}
    train_samples = calib["train_mlp_infer"][1] / max(n_cal, 1)
    render_samples = calib["render_encode"][1] / max(n_cal, 1)
    train_rays = calib["train_sampler"][1] / max(n_cal, 1)
    cfg_b = {}
    for label, th in legs:
        e = cb.config_b_kernels(o, th, train_samples, render_samples, n=1 << 15)
        e["Mrays_s_extrapolated"] = (train_rays + W * H) / e["extrapolated_s_per_step"] / 1e6
        cfg_b[label] = e
    cpu = {"value": rays / (t_train + t_render) / 1e6, "unit": "Mrays/s", "cores": nth, "kind": "port",
           "sample": f"scalar C++ oracle, OpenMP on {nth} threads (hardware_concurrency {hw}): 1 train step of {R} rays "
                     f"(+Adam over {o.n_params} params) in {t_train:.2f}s + {len(ys)} rows of the {W}x{H} frame "
                     f"({W * len(ys)} rays) in {t_render:.2f}s, same weights/grid as the GPU",
           "hardware_concurrency": hw, "cpu_share": cb.cpu_share(),
           "single_thread": {"value": rays / (t1_train + t1_render) / 1e6, "cores": 1, "train_s": round(t1_train, 3),
                             "render_s": round(t1_render, 3)},
           "config_a_end_to_end": cfg_a,
           "config_b_per_kernel_extrapolated": cfg_b}
    parity = {"rgb_mean_l1_vs_oracle": l1, "rows": [ys[0], ys[-1]], "tolerance": 1e-3, "ok": l1 < 1e-3,
              "object_pixels_frac": float((gpu_frame[ys, :, 3] > 0.01).mean())}
    return cpu, parity


def surface_scene(args, ngp):
    """The procedural lego-shaped surface scene (synthetic.py: 100 hemisphere views of 800x800, opaque
    primitives) -- nerf_synthetic/lego's workload shape (a few samples per 1080p ray) next to the
    volumetric headline scene: pretrain, then args.steps of train(2^18) + one 1080p spp1 render."""
    sub_args = argparse.Namespace(**vars(args))
    sub_args.scene = "synthetic"
    tb = ngp.Testbed(ngp.TestbedMode.Nerf)
    cams, _, _ = make_dataset(ngp, tb, sub_args, "cuda:0")
    tb.reload_network_from_file(args.config)
    tb.shall_train = True
    tb.deterministic = bool(args.deterministic_pretrain)
    for _ in range(args.pretrain):
        tb.train(args.batch)
    tb.deterministic = False
    W, H = args.width, args.height
    view = 3 % len(cams)

    def step():
        t0 = time.perf_counter()
        tb.train(args.batch)
        t1 = time.perf_counter()
        tb.set_camera_to_training_view(view)
        img = tb.render(W, H, 1, True)  # to host memory, as the headline step
        del img
        return tb.last_train_stats()["n_rays"], t1 - t0, time.perf_counter() - t1

    elapsed, out, kernels, roof = timed_leg(args, tb, step)
    rays = sum(r + W * H for r, _, _ in out)
    train_s = sum(a for _, a, _ in out)
    render_s = sum(b for _, _, b in out)
    roof["traffic"] = pmc_traffic(args.surface_traffic_json, roof["kernel"], roof["units_per_launch"])
    return {"Mrays_s": round(rays / elapsed / 1e6, 3), "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "roofline": roof, "kernels_calibration": kernels,
            "train_ms_per_step": round(1e3 * train_s / args.steps, 3), "render_ms_per_frame": round(1e3 * render_s / args.steps, 3),
            "render_Mrays_s": round(W * H * args.steps / render_s / 1e6, 3),
            "workload": f"synthetic lego-shaped surface scene ({args.views} views {args.train_res}x{args.train_res}), same network, "
                        f"{args.pretrain} pretrain steps, then train(2^18) + render({W}, {H}, spp 1) to host memory per step"}


def config_e(args, ngp):
    """BASELINE config E's shape on one GPU: the T=2^22 L16F2 network (configs/nerf/bicycle_L16F2T22.json) on a scene
    with aabb_scale 64 (the fox's real photos with aabb_scale raised to 64: mip-nerf360/bicycle is not available
    offline), pretrained, then args.steps of train(2^18) + render(1920, 1080, spp 1) to host memory."""
    import tempfile

    sys.path.insert(0, TESTS)
    from test_gpu_config_e import fox_aabb64

    hip = C.CDLL("libamdhip64.so")

    def used():
        free, total = C.c_size_t(), C.c_size_t()
        hip.hipMemGetInfo(C.byref(free), C.byref(total))
        return total.value - free.value

    used0 = used()
    with tempfile.TemporaryDirectory() as d:
        tb = ngp.Testbed(ngp.TestbedMode.Nerf)
        tb.load_training_data(fox_aabb64(d))
        tb.reload_network_from_file("bicycle_L16F2T22.json")
        tb.shall_train = True
        for _ in range(args.config_e_pretrain):
            tb.train(args.batch)
        W, H = args.width, args.height

        def step():
            t0 = time.perf_counter()
            tb.train(args.batch)
            t1 = time.perf_counter()
            tb.set_camera_to_training_view(3)
            img = tb.render(W, H, 1, True)
            del img
            return tb.last_train_stats()["n_rays"], t1 - t0, time.perf_counter() - t1

        elapsed, out, kernels, roof = timed_leg(args, tb, step)
        roof["traffic"] = pmc_traffic(args.config_e_traffic_json, roof["kernel"], roof["units_per_launch"])
        mem = used() - used0
        del tb
    rays = sum(r + W * H for r, _, _ in out)
    return {"Mrays_s": round(rays / elapsed / 1e6, 3), "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "train_ms_per_step": round(1e3 * sum(a for _, a, _ in out) / args.steps, 3),
            "render_ms_per_frame": round(1e3 * sum(b for _, _, b in out) / args.steps, 3),
            "device_memory_GiB": round(mem / 2**30, 3), "roofline": roof, "kernels_calibration": kernels,
            "workload": f"T=2^22 L16F2 64-wide MLPs, fox photos with aabb_scale 64 (max_cascade 6), {args.config_e_pretrain} "
                        f"pretrain steps, then train(2^18) + render({W}, {H}, spp 1) to host memory per step"}


def launch_ranks(args):
    """--gpus N without a torchrun environment: start N ranks as a CHILD torchrun (nothing here has
    touched the GPU yet), relay its output and exit with its status."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "WORLD_SIZE" in os.environ and args.gpus != 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
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
    cams, imgs, focal = make_dataset(ngp, tb, args, f"cuda:{local_rank}")
    n_views = len(cams)
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
    tb.deterministic = bool(args.deterministic_pretrain)
    for i in range(args.pretrain):
        tb.train(args.batch)
        if rank == 0 and (i + 1) % 250 == 0:
            print(f"# pretrain {i + 1}/{args.pretrain} loss {tb.loss:.5f} "
                  f"rays/batch {tb.last_train_stats()['rays_per_batch']} ({time.perf_counter() - t_pre:.1f}s)",
                  file=sys.stderr, flush=True)
    tb.deterministic = False  # the timed steps run the default path
    view = (rank * 7 + 3) % n_views

    split = {"train_s": 0.0, "render_s": 0.0, "train_rays": 0, "render_rays": 0}

    def step():
        t0 = time.perf_counter()
        tb.train(args.batch)  # returns after the stream is synchronised (Testbed::train)
        t1 = time.perf_counter()
        rays = tb.last_train_stats()["n_rays"]
        tb.set_camera_to_training_view(view)
        # render() as BASELINE.md:30-31 counts inference: the float frame read back to host memory (render_to_cpu,
        # src/python_api.cu:124-202; here into pooled page-locked numpy arrays)
        img = tb.render(W, H, 1, True)
        del img
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
    # the dominant KERNEL: render_march times a family of kernels (init, generate, composite,
    # shade) with events around them, and with several ray pipelines on their own streams
    # (render.hip render_pipes) those brackets also span the other pipelines' kernels; its
    # fraction is still reported under kernels_calibration
    modeled = [k for k in models if calib.get(k, (0, 0, 0))[2] > 0 and k != "render_march"]
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

    # config C (BASELINE configs[2]): ONE 1080p frame per step, row-sharded over the ranks in
    # 8-row blocks and gathered to rank 0 over RCCL -- strong scaling of inference
    config_c = None
    if world > 1:
        tb.set_camera_to_training_view(3 % n_views)
        for _ in range(2):
            tb.render_distributed(W, H, 1, True, False)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tb.render_distributed(W, H, 1, True, False)
        barrier()
        tc = time.perf_counter() - t0
        t = torch.tensor([tc], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tc = float(t.item())
        config_c = {"workload": f"one {W}x{H} spp1 frame per step, 8-row blocks interleaved over {world} ranks, "
                                "gathered to rank 0 (RCCL send/recv)",
                    "Mrays_s": round(W * H * args.steps / tc / 1e6, 3), "ms_per_frame": round(1e3 * tc / args.steps, 3),
                    "scaling": "strong"}

    kernels = kernel_table(calib, models)
    bound, per_unit = models[dom]
    tsrc = timers if args.kernel_timer else calib
    ms, units, launches = tsrc[dom]
    work = model_bytes(dom, per_unit, units, tsrc)
    if per_unit is None:
        per_unit = f"{MARCH_B_PER_SAMPLE} B/filled sample + {MARCH_B_PER_RAY} B/ray"
    achieved = work / launches / (ms / launches / 1000.0)
    roofline = {
        "kernel": dom,
        "bound": bound,
        "achieved": round(achieved / (1e9 if bound == "hbm" else 1e12), 2),
        "peak": HBM_PEAK_GBS if bound == "hbm" else MFMA_F16_PEAK_TFLOPS,
        "unit": "GB/s" if bound == "hbm" else "TFLOP/s",
        "traffic": None,
        "per_unit": per_unit,
        "units_per_launch": round(units / launches),
        "bytes_or_flops_per_launch": round(work / launches),
        "us_per_launch": round(1000.0 * ms / launches, 2),
    }
    roofline["frac"] = round(roofline["achieved"] / roofline["peak"], 4)
    # the PMC summary of the same scene (bench.py --scene synthetic profiles the surface scene)
    roofline["traffic"] = pmc_traffic(args.surface_traffic_json if args.scene == "synthetic" else args.traffic_json,
                                      dom, units / launches)
    if dom == "render_encode" and split["render_s"] > 0:
        # the same algorithmic bytes over a whole frame: one frame's encode bytes / the frame's wall time
        frame_s = split["render_s"] / args.steps
        per_frame = work / args.steps
        roofline["per_frame"] = {"bytes": round(per_frame), "frame_ms": round(1e3 * frame_s, 3),
                                 "GB/s": round(per_frame / frame_s / 1e9, 1),
                                 "frac": round(per_frame / frame_s / 1e9 / HBM_PEAK_GBS, 4),
                                 "note": "algorithmic encode bytes of one 1080p frame / its render() wall time (host copy included)"}

    # the same view through render() (the timed step's call) and render_to_device() (the frame stays in HBM):
    # the read-back's share of a frame, reported beside value
    render_in_hbm = None
    if world == 1 and args.render_in_hbm > 0:
        tb.set_camera_to_training_view(view)
        tb.render(W, H, 1, True)
        t0 = time.perf_counter()
        for _ in range(args.render_in_hbm):
            img = tb.render(W, H, 1, True)
            del img
        tr = (time.perf_counter() - t0) / args.render_in_hbm
        t0 = time.perf_counter()
        for _ in range(args.render_in_hbm):
            tb.render_to_device(W, H, 1, True)
        td = (time.perf_counter() - t0) / args.render_in_hbm
        render_in_hbm = {"ms_per_frame": round(1e3 * td, 3), "Mrays_s": round(W * H / td / 1e6, 3),
                         "ms_per_frame_render": round(1e3 * tr, 3), "readback_ms": round(1e3 * (tr - td), 3),
                         "readback_GB_s": round(W * H * 16 / max(tr - td, 1e-9) / 1e9, 1),
                         "note": f"{args.render_in_hbm} renders of the bench view through render_to_device() (frame kept in "
                                 "HBM) vs render() (numpy float32 [H,W,4] on pooled pinned host memory, the timed step's call)"}

    cpu = parity = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu, parity = cpu_baseline(args, tb, cams, imgs, focal, view, W, H, calib, n_cal)

    surface = cfg_e = None
    if world == 1 and (args.surface_scene or args.config_e):
        del tb
    if world == 1 and args.surface_scene:
        surface = surface_scene(args, ngp)
    if world == 1 and args.config_e:
        cfg_e = config_e(args, ngp)
    mlp_standalone = None
    if world == 1 and args.mlp_microbench:
        # the fused MLPs alone at SURVEY 8(d)'s sizes (tools/mlp_microbench.py): the render MLP over 2^21 samples under
        # the frame's tunings and the training MLP over 2^18, after the timed region
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import mlp_microbench
        mlp_standalone = mlp_microbench.measure(iters=20)

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
            "data": (f"real scene {os.path.relpath(args.scene, ROOT)} ({n_views} views {imgs.shape[2]}x{imgs.shape[1]} "
                     f"RGBA8; the reference's data/nerf/test/dataset, nerf_synthetic/lego is not available offline)"
                     if args.scene != "synthetic" else
                     f"synthetic lego-shaped scene ({n_views} views {args.train_res}x{args.train_res} RGBA8)")
                    + f", random-init weights trained {args.pretrain} steps before timing"
                    + (" (bit-reproducible hash-grid gradients: the same trained scene every run; timed steps on the "
                       "default fp16-atomic path)" if args.deterministic_pretrain else ""),
            "config": {"workload": "lego L16F2T19 MLP 64 (1x density + 2x rgb hidden): Testbed.train(2^18) "
                                   f"+ Testbed.render({W}, {H}, spp 1) to host memory per step", "batch": args.batch, "config_file": args.config,
                       "parallelism": f"dp{world} (RCCL grad all-reduce) + per-rank 1080p view"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
            "split": {"train_Mrays_s": round(split["train_rays"] / split["train_s"] / 1e6, 3),
                      "render_Mrays_s": round(split["render_rays"] / split["render_s"] / 1e6, 3),
                      "train_ms_per_step": round(1e3 * split["train_s"] / args.steps, 3),
                      "render_ms_per_frame": round(1e3 * split["render_s"] / args.steps, 3),
                      "note": "rank 0; per-part wall time inside the timed region (SURVEY 8(d) counts train and inference separately)"},
            "kernels_calibration": kernels,
            "render_in_hbm": render_in_hbm,
            "surface_scene": surface,
            "config_e": cfg_e,
            "config_c": config_c,
            "mlp_standalone": mlp_standalone,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
