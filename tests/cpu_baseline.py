"""CPU baseline of the bench: the scalar C++ oracle (oracle/, test
infrastructure; the reference has no CPU path) timed on the host cores, single-threaded and
with OpenMP over the independent loops (render rows, per-sample encoding and inference).

Three measurements, all on bounded samples so the default bench finishes in minutes:
  * the bench workload itself: one training step of R rays + K rows of the 1080p frame, on the
    GPU's trained weights and density grid;
  * config A end to end (BASELINE configs[0]: 64x64, L=4 F=2 T=2^14, 16-wide MLP): a few
    training steps with density-grid updates, then one 64x64 render;
  * config B per kernel at 2^16 samples (encode, inference, MLP backward, encode backward),
    extrapolated linearly to one bench step (labelled "extrapolated").
Only bench.py's cpu_baseline leg calls this; the oracle is never the thing measured as `value`.
"""
import os
import time

import numpy as np

import ngp_abi as A
import synthetic as S
from oracle_abi import Oracle, load
from scene_util import HostDataset, grid_args, oracle_frame_rows, render_args, sphere_bitfield, train_args


def threads_for_box(cap=16):
    """All-core thread count: the host's hardware concurrency, capped at the GPU box's CPU share."""
    hw = int(load().oref_hardware_concurrency())
    return hw, max(1, min(cap, hw))


def cpu_share():
    """The CPUs this process may actually run on: its affinity mask and the cgroup CPU quota (cpu.max), if any."""
    out = {"affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        out["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        out["cgroup_cpu_quota"] = None
    return out


def _timed(fn):
    t0 = time.perf_counter()
    r = fn()
    return time.perf_counter() - t0, r


def bench_sample(o, tb, W, H, rows, hd, R, threads):
    """One training step of R rays + `rows` rows of the W x H frame; returns (train_s, render_s, rays, frame rows)."""
    lib = load()
    lib.oref_set_threads(threads)
    try:
        block = H // (2 * rows)
        t_render, ref = _timed(lambda: oracle_frame_rows(o, tb, W, H, [block], rows))
        ta = train_args(hd.ptr, hd.n, R, 1 << 14, 16 * (1 << 14))
        t_train, _ = _timed(lambda: (o.train_step(ta), o.optimizer_step(0, 1, 1)))
    finally:
        lib.oref_set_threads(1)
    return t_train, t_render, R + W * len(ref), ref


def config_a_end_to_end(threads, steps=16, rays=1024, res=64, views=8):
    """BASELINE configs[0] end to end on the oracle: `steps` training steps (density-grid update
    every 16 steps, as training_prep_nerf after warm-up) of `rays` rays on a res x res scene,
    then one res x res render.  Returns the timing and Mrays/s."""
    lib = load()
    cams = S.hemisphere_cameras(views, seed=0)
    focal = S.focal_from_angle(res)
    imgs = S.render_views(cams, res, res, focal)
    hd = HostDataset(imgs, cams, focal)
    o = Oracle(A.default_config(n_levels=4, F=2, log2_T=14, n_neurons=16))
    rng = np.random.default_rng(0)
    p = np.zeros(o.n_params, np.float32)
    p[: o.n_mlp] = rng.normal(0, 0.2, o.n_mlp)
    p[o.n_mlp:] = rng.uniform(-1e-4, 1e-4, o.n_params - o.n_mlp)
    o.set_params(p)
    o.set_inference_params(p)
    o.grid_set(sphere_bitfield(0.4))
    o.grid_bitfield(0)
    lib.oref_set_threads(threads)
    try:
        t0 = time.perf_counter()
        for s in range(steps):
            if s % 16 == 0:
                ga = grid_args(hd.ptr, hd.n, 1 << 14, 1 << 14, ema_step=s // 16, mark=int(s == 0), clear=int(s == 0))
                o.grid_evaluate(ga)
                o.grid_finish(ga)
            o.train_step(train_args(hd.ptr, hd.n, rays, 1 << 14, 16 * (1 << 14), step=s))
            o.optimizer_step(s, 1, 1)
        t_train = time.perf_counter() - t0
        ra = render_args(res, res, cams[0], focal)
        t_render, _ = _timed(lambda: o.render(ra))
    finally:
        lib.oref_set_threads(1)
    total = steps * rays + res * res
    return {"train_s": round(t_train, 3), "render_s": round(t_render, 4), "steps": steps, "rays_per_step": rays,
            "render": f"{res}x{res}", "Mrays_s": total / (t_train + t_render) / 1e6}


def config_b_kernels(o, threads, train_samples, render_samples, n=1 << 16):
    """Per-kernel oracle timings at n samples on the bench's model (config B), extrapolated
    linearly to one bench step: training = encode + MLP forward/backward + encode backward over
    the 2^18-sample batch (plus its forward over the samples the early-terminated forward
    evaluates, counted as `train_samples`), render = encode + inference over the frame's
    `render_samples` network-evaluated samples."""
    lib = load()
    rng = np.random.default_rng(1)
    pos = rng.random((n, 3), dtype=np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    dirs = ((d + 1.0) * 0.5).astype(np.float32)
    coords = np.concatenate([pos, np.full((n, 1), 0.01, np.float32), dirs, np.zeros((n, 1), np.float32)], 1)
    dloss = rng.normal(0, 1e-3, (n, 4)).astype(np.float16).astype(np.float32)
    lib.oref_set_threads(threads)
    try:
        t_enc, enc = _timed(lambda: o.encode(pos, use_inf=True))
        t_inf, _ = _timed(lambda: o.infer(coords, use_inf=True))
        t_bwd, denc = _timed(lambda: o.backward(enc, dirs, dloss))
        t_ebwd, _ = _timed(lambda: o.encode_backward(pos, denc))
    finally:
        lib.oref_set_threads(1)
    per = {"encode": t_enc / n, "inference": t_inf / n, "mlp_backward": t_bwd / n, "encode_backward": t_ebwd / n}
    step_s = (train_samples * per["inference"] + (1 << 18) * (per["mlp_backward"] + per["encode_backward"])
              + render_samples * per["inference"])
    return {"samples_timed": n, "us_per_sample": {k: round(v * 1e6, 3) for k, v in per.items()},
            "train_samples_per_step": int(train_samples), "render_samples_per_frame": int(render_samples),
            "extrapolated_s_per_step": round(step_s, 3)}
