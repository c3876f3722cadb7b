"""Data-parallel decomposition of the path on CPU (gloo, world_size 2).

The GPU build splits a training step over ranks by global ray index (rank r owns rays
[r·R, (r+1)·R) of the shared pcg32 stream, src/testbed_nerf.cu:715), all-reduces the
gradient sum and runs the identical optimizer step everywhere; the density-grid update
evaluates 1/N of the samples per rank and max-reduces the evaluation buffer before the
EMA.  These tests run that exact decomposition with the CPU oracle as
each rank's device and gloo as the collective, and check it against one process doing
the whole job.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ctypes as C

import ngp_abi as A
from oracle_abi import Oracle
from scene_util import HostDataset, grid_args, make_views, train_args

CFG = dict(n_levels=4, F=2, log2_T=14, n_neurons=16)
CELLS = 128 ** 3
# ngp_train_args.allreduce_i32: (user, int32 words, n, stream) -> status
ALLREDUCE_I32 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int32), C.c_uint32, C.c_void_p)
# global (sample cap, compaction cap) pairs of the exact-decomposition runs: the sample cap drops
# rays of the second rank / the compaction cap ends inside the first rank's samples / neither
EXACT_CAPS = {"sample_cap": (1 << 12, 1 << 16), "compaction_cap": (1 << 20, 1 << 11), "rollover": (1 << 20, 1 << 16)}


def _exact_args(hd, R_global, caps):
    ta = train_args(hd.ptr, hd.n, R_global, caps[1], caps[0])
    ta.n_rays_global = R_global
    return ta


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(seed=0):
    o = Oracle(A.default_config(**CFG))
    rng = np.random.default_rng(seed)
    p = np.zeros(o.n_params, np.float32)
    p[: o.n_mlp] = rng.normal(0, 0.3, o.n_mlp)
    p[o.n_mlp:] = rng.uniform(-0.5, 0.5, o.n_params - o.n_mlp)
    o.set_params(p)
    return o


def _sphere_grid():
    from scene_util import sphere_bitfield
    return sphere_bitfield(0.32)


def _per_ray(o, R):
    ns = o.scratch(A.SCRATCH_RAY_NUMSTEPS, np.uint32).reshape(-1, 2)[:R]
    coords = o.scratch(A.SCRATCH_COORDS, np.float32).reshape(-1, 8)
    return [coords[b:b + n].copy() for n, b in ns]


def _worker(rank, world, port, R, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        imgs, cams, focal = make_views(6, 24, 24)
        hd = HostDataset(imgs, cams, focal)
        o = _model()
        o.grid_set(_sphere_grid())
        o.grid_bitfield(0)
        # --- density grid: evaluate 1/world of the samples, max all-reduce, finish
        ga = grid_args(hd.ptr, hd.n, 1 << 14, 1 << 14, ema_step=3, mark=1, clear=1)
        ga.rank, ga.world_size = rank, world
        o.grid_evaluate(ga)
        tmp = torch.from_numpy(o.grid_tmp(CELLS))
        dist.all_reduce(tmp, op=dist.ReduceOp.MAX)
        o.grid_tmp(CELLS, tmp.numpy())
        o.grid_finish(ga)
        grid, bits, mean = o.grid_get(CELLS)
        o.grid_set(_sphere_grid())  # training below uses the same grid as the single-process check
        o.grid_bitfield(0)
        # --- training step: this rank's slice of the global rays
        ta = train_args(hd.ptr, hd.n, R, 1 << 16, 1 << 20)
        ta.ray_index_offset = rank * R
        ta.n_rays_global = world * R
        o.train_step(ta)
        rays = _per_ray(o, R)
        g = torch.from_numpy(o.get(A.GRADS_FP32).copy())
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        o.set_grads(g.numpy())
        o.optimizer_step(0, 1, 1)
        params = torch.from_numpy(o.get(A.PARAMS_FP32).copy())
        gathered = [torch.zeros_like(params) for _ in range(world)]
        dist.all_gather(gathered, params)
        # --- the exact decomposition (ngp_train_args.world_size): the step learns every rank's sample
        # and compacted totals through the all-reduce callback, so the caps and the rollover follow the
        # global ray order of one process
        def allreduce_i32(user, words, n, stream):
            arr = np.ctypeslib.as_array(words, shape=(n,))
            t = torch.from_numpy(arr.copy())
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            arr[:] = t.numpy()
            return 0
        cb = ALLREDUCE_I32(allreduce_i32)
        exact = {}
        for name, caps in EXACT_CAPS.items():
            o2 = _model()
            o2.grid_set(_sphere_grid())
            o2.grid_bitfield(0)
            ta = _exact_args(hd, world * R, caps)
            ta.n_rays = R
            ta.ray_index_offset = rank * R
            ta.rank, ta.world_size = rank, world
            ta.allreduce_i32 = C.cast(cb, C.c_void_p)
            o2.train_step(ta)
            g2 = torch.from_numpy(o2.get(A.GRADS_FP32).copy())
            dist.all_reduce(g2, op=dist.ReduceOp.SUM)
            st = o2.stats()
            cp = o2.scratch(A.SCRATCH_RAY_COMPACTED, np.uint32).reshape(-1, 2)[:R, 0].copy()
            ns = o2.scratch(A.SCRATCH_RAY_NUMSTEPS, np.uint32).reshape(-1, 2)[:R, 0].copy()
            exact[name] = dict(grads=g2.numpy(), loss=float(st.loss), compacted=cp, numsteps=ns,
                               totals=(st.measured_batch_size_before_compaction, st.measured_batch_size))
        out_q.put((rank, rays, g.numpy(), [x.numpy() for x in gathered], grid, bits, mean, exact))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def dp_run():
    world, R = 2, 96
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, R, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=300)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return world, R, res


def test_rank_rays_are_slices_of_the_global_stream(dp_run):
    world, R, res = dp_run
    imgs, cams, focal = make_views(6, 24, 24)
    hd = HostDataset(imgs, cams, focal)
    o = _model()
    o.grid_set(_sphere_grid())
    o.grid_bitfield(0)
    o.train_step(train_args(hd.ptr, hd.n, world * R, 1 << 16, 1 << 20))
    full = _per_ray(o, world * R)
    assert sum(len(c) for c in full) > 100
    for r in range(world):
        for i, c in enumerate(res[r][0]):
            np.testing.assert_array_equal(c, full[r * R + i])


def test_replicas_stay_identical_after_allreduce_and_step(dp_run):
    world, R, res = dp_run
    for r in range(world):
        params = res[r][2]
        for p in params[1:]:
            np.testing.assert_array_equal(params[0], p)
    np.testing.assert_array_equal(res[0][1], res[1][1])  # all-reduced gradients identical
    assert np.abs(res[0][1]).sum() > 0


@pytest.mark.parametrize("case", list(EXACT_CAPS))
def test_exact_decomposition_matches_one_process_with_all_rays(dp_run, case):
    """world_size ranks of R rays each == one process of world x R rays and the global caps: the
    same rays dropped by the sample cap, the same samples kept by the compaction cap, the rollover
    weights of the global batch -- so the summed gradients and losses equal the single-process ones
    (float association aside)."""
    world, R, res = dp_run
    imgs, cams, focal = make_views(6, 24, 24)
    hd = HostDataset(imgs, cams, focal)
    o = _model()
    o.grid_set(_sphere_grid())
    o.grid_bitfield(0)
    caps = EXACT_CAPS[case]
    o.train_step(_exact_args(hd, world * R, caps))
    st = o.stats()
    g = o.get(A.GRADS_FP32)
    ns = o.scratch(A.SCRATCH_RAY_NUMSTEPS, np.uint32).reshape(-1, 2)[: world * R, 0]
    cp = o.scratch(A.SCRATCH_RAY_COMPACTED, np.uint32).reshape(-1, 2)[: world * R, 0]
    total_samples, total_compacted = st.measured_batch_size_before_compaction, st.measured_batch_size
    if case == "sample_cap":
        assert total_samples > caps[0] and (ns == 0).sum() > (ns[:R] == 0).sum()  # rays dropped past the cap
    elif case == "compaction_cap":
        assert total_compacted > caps[1] and cp.sum() == caps[1]
    else:
        assert total_compacted < caps[1]  # rollover over the whole batch
    ex = [res[r][6][case] for r in range(world)]
    np.testing.assert_array_equal(np.concatenate([e["numsteps"] for e in ex]), ns)
    np.testing.assert_array_equal(np.concatenate([e["compacted"] for e in ex]), cp)
    assert sum(e["totals"][0] for e in ex) == total_samples and sum(e["totals"][1] for e in ex) == total_compacted
    assert sum(e["loss"] for e in ex) == pytest.approx(st.loss, rel=1e-5)
    for e in ex:
        np.testing.assert_array_equal(e["grads"], ex[0]["grads"])  # every rank holds the same sum
    rel = np.linalg.norm(ex[0]["grads"] - g) / np.linalg.norm(g)
    assert rel < 1e-5, rel


def test_sliced_density_grid_update_matches_single_process(dp_run):
    world, R, res = dp_run
    imgs, cams, focal = make_views(6, 24, 24)
    hd = HostDataset(imgs, cams, focal)
    o = _model()
    o.grid_set(_sphere_grid())
    o.grid_bitfield(0)
    ga = grid_args(hd.ptr, hd.n, 1 << 14, 1 << 14, ema_step=3, mark=1, clear=1)
    o.grid_update(ga)
    grid, bits, mean = o.grid_get(CELLS)
    for r in range(world):
        np.testing.assert_array_equal(res[r][3], grid)
        np.testing.assert_array_equal(res[r][4], bits)
        assert res[r][5] == mean
