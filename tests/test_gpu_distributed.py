"""The Testbed's data-parallel path (m_world > 1) on the GPU, with two processes sharing one
MI355X.  RCCL refuses two ranks on one device, so the collectives go through the Testbed's
host-staged test backend (init_distributed_host) over torch.distributed/gloo; everything else
is the product path: per-rank ray offsets, the density-grid evaluation split over ranks with a
max all-reduce of the evaluation buffer, the fp32 MLP + fp16 hash-grid gradient all-reduce, the
reduced batch statistics, the error-map, exposure and extrinsic-gradient all-reduces, and the
row-sharded frame gathered to rank 0.

Checks: the density grid after the split update is bit-identical to one process doing the
whole update; after 130 steps (one error-map CDF rebuild, eight camera updates) every rank
holds bit-identical parameters, grid and camera offsets (the replicas do not drift); the
gathered frame equals rank 0's own full render bit for bit.  And the decomposition is exact:
two ranks of batch B train like ONE process of batch 2B (the same rays, sample / compaction caps
and rollover over the global ray order, ngp_train_args.world_size), compared in deterministic
mode (fixed-point hash-grid gradients, so the gradient all-reduce is an exact integer sum).

The RCCL calls themselves run in test_rccl_world_size_one_matches_plain_testbed: a real RCCL
communicator of one rank on the box's GPU drives the same data-parallel path (ncclAllReduce of the
per-rank totals, gradients, violation word, grid evaluation, statistics; ncclSend / ncclRecv of the
frame rows), bit-identical to a Testbed without a communicator.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import synthetic as S

pytestmark = pytest.mark.gpu

STEPS = 130
BATCH = 1 << 14
W, H = 96, 72


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _params(tb):
    import ctypes as C
    import ngp_abi as A
    lib = A.load()
    p, n = C.c_void_p(), C.c_size_t()
    A.check(lib.ngp_model_buffer(C.c_void_p(tb.model_handle), A.PARAMS_FP32, C.byref(p), C.byref(n)))
    out = torch.empty(n.value // 4, dtype=torch.float32, device="cuda")
    tb.sync()
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(C.c_void_p(out.data_ptr()), p, n.value, 3) == 0
    return out.cpu().numpy()


def _testbed(scene_dir, config="tiny_L4F2.json"):
    import pyngp as ngp
    tb = ngp.Testbed()
    tb.load_training_data(os.path.join(scene_dir, "transforms_train.json"))
    tb.reload_network_from_file(config)
    tb.training_batch_size = BATCH
    return tb


def _host_allreduce(dist):
    def allreduce(arr, op):
        t = torch.from_numpy(arr)
        rop = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
        if t.dtype == torch.float16:  # gloo reduces fp32; a 2-rank fp16 sum rounds exactly once either way
            t32 = t.float()
            dist.all_reduce(t32, op=rop)
            t.copy_(t32.half())
        else:
            dist.all_reduce(t, op=rop)
    return allreduce


EQ_STEPS = 24
EQ_EXACT = (1, 2)  # frames after which the two sides are compared to rounding
EQ_WINDOW = 12  # the last frames whose (global-batch) losses are averaged on both sides


def _equivalence_worker(rank, world, port, scene_dir, q, config="tiny_L4F2.json", tuning=None):
    """Deterministic data-parallel training: state after the first frame and after EQ_STEPS."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tb = _testbed(scene_dir, config)
        if tuning:
            tb.set_tuning(tuning)
        tb.init_distributed_host(rank, world, _host_allreduce(dist))
        tb.deterministic = True
        tb.shall_train = True
        out = dict(rank=rank, losses=[])
        while tb.training_step < EQ_STEPS:
            tb.frame()
            if tb.training_step > EQ_STEPS - EQ_WINDOW:
                out["losses"].append(tb.last_train_stats()["loss"])
            if tb.training_step in EQ_EXACT + (EQ_STEPS,):
                out[tb.training_step] = dict(params=_params(tb), grid=tb.density_grid(), bits=tb.density_grid_bitfield(),
                                             stats=tb.last_train_stats(), loss=tb.loss)
        out["violations_total"] = tb.last_train_stats()["forward_early_stop_violations_total"]
        q.put(out)
    finally:
        dist.destroy_process_group()


def _worker(rank, world, port, scene_dir, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tb = _testbed(scene_dir)
        tb.init_distributed_host(rank, world, _host_allreduce(dist))
        assert tb.world_size == world and tb.rank == rank
        tr = tb.nerf.training
        tr.optimize_exposure = True
        tr.optimize_extrinsics = True
        tb.shall_train = True
        tb.frame()  # step 0: density grid over all cells (split over the ranks) + one training step
        grid0 = tb.density_grid()
        losses = []
        while tb.training_step < STEPS:
            tb.frame()
            losses.append(tb.last_train_stats()["loss"])  # this step's (rank-reduced) loss
        tb.background_color = [0.0, 0.0, 0.0, 1.0]
        tb.set_camera_to_training_view(1)
        gathered = tb.render_distributed(W, H, 1, True)
        local = tb.render(W, H, 1, True) if rank == 0 else None
        ds = tb.nerf.training.dataset
        q.put(dict(rank=rank, grid0=grid0, grid=tb.density_grid(), bits=tb.density_grid_bitfield(), params=_params(tb),
                   losses=np.array(losses), gathered=gathered, local=local,
                   xforms=np.stack([np.asarray(tr.get_camera_extrinsics(i)) for i in range(ds.n_images)]),
                   stats=tb.last_train_stats()))
    finally:
        dist.destroy_process_group()


def _extra_dims_worker(rank, world, port, scene_dir, q):
    """optimize_extra_dims under data parallelism: every rank all-reduces the per-image code gradients and applies
    the same VarAdam step, so codes and parameters stay identical on the ranks."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tb = _testbed(scene_dir, "lego_L16F2.json")
        tb.init_distributed_host(rank, world, _host_allreduce(dist))
        tr = tb.nerf.training
        tr.optimize_extra_dims = True
        tb.shall_train = True
        tb.frame()
        n = tr.dataset.n_images
        c0 = np.stack([np.asarray(tr.get_extra_dims(i)) for i in range(n)])
        while tb.training_step < 16:
            tb.frame()
        c1 = np.stack([np.asarray(tr.get_extra_dims(i)) for i in range(n)])
        q.put(dict(rank=rank, c0=c0, c1=c1, params=_params(tb), loss=tb.loss, dims=tr.dataset.n_extra_dims()))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def scene(tmp_path_factory):
    root = tmp_path_factory.mktemp("dp_scene")
    S.write_nerf_synthetic_scene(str(root), 10, 48, 48, seed=5, split="train")
    return str(root)


def _spawn(target, scene, world=2, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, scene, q) + tuple(extra)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            d = q.get(timeout=240)
            res[d["rank"]] = d
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


def test_data_parallel_testbed_two_processes_one_gpu(scene):
    world = 2
    res = _spawn(_worker, scene, world)
    r0, r1 = res[0], res[1]

    # the split density-grid update (1/N of the samples per rank + max all-reduce) equals one
    # process evaluating every sample
    torch.cuda.set_device(0)
    tb = _testbed(scene)
    tb.shall_train = True
    tb.frame()
    np.testing.assert_array_equal(r0["grid0"], tb.density_grid())
    np.testing.assert_array_equal(r1["grid0"], r0["grid0"])

    # replicas stay bit-identical: parameters, grid, bitfield and optimised camera poses
    np.testing.assert_array_equal(r0["params"], r1["params"])
    np.testing.assert_array_equal(r0["grid"], r1["grid"])
    np.testing.assert_array_equal(r0["bits"], r1["bits"])
    np.testing.assert_array_equal(r0["xforms"], r1["xforms"])
    assert r0["stats"]["measured_batch_size"] == r1["stats"]["measured_batch_size"]
    # every rank saw the same reduced loss, and the camera offsets moved (the reduced camera
    # gradients were applied)
    assert np.isfinite(r0["losses"]).all() and r0["losses"].max() > 0
    np.testing.assert_array_equal(r0["losses"], r1["losses"])
    assert np.abs(r0["xforms"] - np.stack([np.asarray(tb.nerf.training.get_camera_extrinsics(i))
                                           for i in range(r0["xforms"].shape[0])])).max() > 0
    # the row-sharded frame gathered to rank 0 is rank 0's full-frame render
    assert r1["gathered"] is None
    np.testing.assert_array_equal(r0["gathered"], r0["local"])
    assert r0["local"][..., 3].max() > 0.5


@pytest.mark.parametrize("world,config,tuning", [
    (2, "tiny_L4F2.json", None),
    # config D at its own shape: the config-B network (L16 F2 T2^19, 64-wide MLPs)
    (2, "lego_L16F2.json", None),
    (4, "lego_L16F2.json", None),
    # 4 ranks whose sample buffers start too small (debug bit 3: every rank's share overflows, the step is
    # discarded and re-run with grown buffers) and whose chunked forward stops rays far too early (bit 2:
    # violations on the first step, discarded and re-run with the full forward): the same training
    (4, "lego_L16F2.json", {"debug": 12}),
    # config D's full width: eight ranks (the per-rank sample caps at twice the even share of 1/8 of the global cap,
    # and the capacity-overflow regrowth, at the world size the node runs)
    (8, "lego_L16F2.json", None),
    (8, "lego_L16F2.json", {"debug": 12}),
], ids=["2-tiny", "2-lego", "4-lego", "4-lego-retries", "8-lego", "8-lego-retries"])
def test_ranks_train_like_one_process_with_world_times_the_batch(scene, world, config, tuning):
    """rank r of N owns global rays [r R, (r+1) R) of one batch; with the exact
    decomposition the N ranks' step is one process's step of N x the batch.  Deterministic mode on
    both sides: the hash-grid gradients are integer sums (identical), the MLP gradients sums over
    different partitions (float association).  After the first frames the parameters therefore agree
    to rounding and the batch statistics, density grid and bitfield exactly; later, a training
    trajectory amplifies the association differences (a ray's compacted count can move by one
    sample), so at EQ_STEPS only the statistics and losses are compared, within a percent."""
    res = _spawn(_equivalence_worker, scene, world, config, tuning)
    if tuning and tuning.get("debug", 0) & 4:
        assert all(res[r]["violations_total"] > 0 for r in range(world))  # the retry path ran
    torch.cuda.set_device(0)
    tb = _testbed(scene, config)
    tb.training_batch_size = world * BATCH
    tb.deterministic = True
    tb.shall_train = True
    single = {}
    single_losses = []
    while tb.training_step < EQ_STEPS:
        tb.frame()
        if tb.training_step > EQ_STEPS - EQ_WINDOW:
            single_losses.append(tb.last_train_stats()["loss"])
        if tb.training_step in EQ_EXACT + (EQ_STEPS,):
            single[tb.training_step] = dict(params=_params(tb), grid=tb.density_grid(), bits=tb.density_grid_bitfield(),
                                            stats=tb.last_train_stats(), loss=tb.loss)
    n_mlp = _n_mlp(tb)
    for step in EQ_EXACT:
        s = single[step]
        for r in range(world):
            d = res[r][step]
            # the global batch statistics are the single process's
            for k in ("measured_batch_size", "measured_batch_size_before_compaction", "rays_per_batch"):
                assert d["stats"][k] == s["stats"][k], (step, k, d["stats"][k], s["stats"][k])
            assert d["stats"]["loss"] == pytest.approx(s["stats"]["loss"], rel=1e-5)
            np.testing.assert_array_equal(d["bits"], s["bits"])
            np.testing.assert_allclose(d["grid"], s["grid"], rtol=1e-4, atol=1e-6)
            # replicas identical; against one process: MLP weights to float association, the hash grid
            # (whose gradients are exact) to the rounding the MLP differences feed through
            np.testing.assert_array_equal(d["params"], res[0][step]["params"])
            np.testing.assert_allclose(d["params"][:n_mlp], s["params"][:n_mlp], rtol=1e-3, atol=1e-6)
            # step 2 runs on step-1 MLP weights that differ in association: a grid gradient sum close to zero
            # can change sign, and Adam's early steps turn that into a full step (lr) of the other sign
            # (two ranks: < 0.5 % of the grid; four ranks' partitions differ more: measured 0.65 %)
            far = ~np.isclose(d["params"][n_mlp:], s["params"][n_mlp:], rtol=1e-3, atol=1e-6)
            print("world", world, "step", step, "grid params off", far.mean())
            assert far.mean() < {2: 5e-3, 4: 1e-2}.get(world, 2e-2), (step, far.mean())
    # after the first step the hash-grid parameters are bit-identical (integer-summed gradients, the
    # same Adam step); the step-1 MLP gradients only differ in association
    np.testing.assert_array_equal(res[0][1]["params"][n_mlp:], single[1]["params"][n_mlp:])
    s, d = single[EQ_STEPS], res[0][EQ_STEPS]
    if tuning:
        # the retried steps are the steps a run without retries takes: the same ranks, partition and integer /
        # fixed-order sums, so after EQ_STEPS the parameters, statistics and losses are bit-identical to it (the
        # retry-free four-rank run is compared with one process by the 4-lego case)
        plain = _spawn(_equivalence_worker, scene, world, config, None)
        for r in range(world):
            for step in EQ_EXACT + (EQ_STEPS,):
                np.testing.assert_array_equal(res[r][step]["params"], plain[r][step]["params"], err_msg=f"rank {r} step {step}")
                np.testing.assert_array_equal(res[r][step]["bits"], plain[r][step]["bits"])
                assert res[r][step]["stats"]["measured_batch_size"] == plain[r][step]["stats"]["measured_batch_size"]
            np.testing.assert_array_equal(res[r]["losses"], plain[r]["losses"])
        return
    # the trajectories drift apart with the association of the MLP sums (measured 1.6 % in the batch sizes at four
    # ranks); one frame's loss is one batch's and moves with the drift (a single step read 19 % apart at four
    # ranks), so the losses are compared as the mean over the last EQ_WINDOW frames' global batches
    losses = res[0]["losses"]
    print("batch", [(d["stats"][k], s["stats"][k]) for k in ("measured_batch_size", "measured_batch_size_before_compaction")],
          "window loss", np.mean(losses), np.mean(single_losses))
    for k in ("measured_batch_size", "measured_batch_size_before_compaction"):
        assert d["stats"][k] == pytest.approx(s["stats"][k], rel={2: 1e-2, 4: 3e-2}.get(world, 5e-2)), k
    assert len(losses) == len(single_losses) == EQ_WINDOW
    assert np.mean(losses) == pytest.approx(np.mean(single_losses), rel={2: 3e-2, 4: 8e-2}.get(world, 1.2e-1))


def _n_mlp(tb):
    import ctypes as C
    import ngp_abi as A
    info = A.ModelInfo()
    A.check(A.load().ngp_model_get_info(C.c_void_p(tb.model_handle), C.byref(info)))
    return int(info.n_mlp_params)


def test_rccl_world_size_one_matches_plain_testbed(scene):
    """The RCCL path on the one GPU of the box (a world_size-1 communicator): a Testbed
    with init_distributed(0, 1, uid) runs every data-parallel collective through RCCL -- the per-rank
    totals (ncclInt32), the fixed-point gradient all-reduce (ngp_allreduce_grads, ncclInt64 + fp32),
    the violation max, the density-grid max all-reduce, the statistics, and render_distributed's
    ncclSend / ncclRecv of the frame rows -- and must match a Testbed without a communicator bit for
    bit (deterministic mode on both)."""
    import pyngp as ngp
    torch.cuda.set_device(0)
    out = {}
    for name in ("plain", "rccl"):
        tb = _testbed(scene)
        if name == "rccl":
            tb.init_distributed(0, 1, ngp.Testbed.nccl_unique_id())
            assert tb.distributed and tb.world_size == 1
        tb.deterministic = True
        tb.shall_train = True
        while tb.training_step < 50:
            tb.frame()
        tb.background_color = [0.0, 0.0, 0.0, 1.0]
        tb.set_camera_to_training_view(1)
        frame = tb.render_distributed(W, H, 1, True) if name == "rccl" else tb.render(W, H, 1, True)
        out[name] = dict(params=_params(tb), grid=tb.density_grid(), bits=tb.density_grid_bitfield(), frame=frame,
                         stats=tb.last_train_stats())
        del tb
    a, b = out["plain"], out["rccl"]
    assert a["stats"] == b["stats"]
    np.testing.assert_array_equal(a["params"], b["params"])
    np.testing.assert_array_equal(a["grid"], b["grid"])
    np.testing.assert_array_equal(a["bits"], b["bits"])
    np.testing.assert_array_equal(a["frame"], b["frame"])
    assert a["frame"][..., 3].max() > 0.5


def test_deterministic_steps_are_bit_reproducible(scene):
    """SURVEY §5 deterministic mode: two Testbeds training the same scene from the same seed end
    bit-identical (fixed-point hash-grid gradients, fixed-order MLP reductions).  The default
    fp16-atomic mode trains the same scene to the same loss; its parameters are not comparable
    element-wise (Adam turns the rounding of near-zero gradient sums into full-size steps of either
    sign), so only the first step is compared: where both modes move a parameter, Adam's first update
    (lr * sign(g)) has the same sign.  The modes do differ in WHICH parameters move: fp16 atomics round
    every run of corner contributions to fp16, so sums of contributions below the fp16 subnormal range
    vanish (the optimizer's sparse skip then leaves the parameter alone), while the fixed-point sum keeps
    them until its single rounding."""
    torch.cuda.set_device(0)
    runs, first, losses = [], [], []
    for det in (True, True, False):
        tb = _testbed(scene)
        tb.deterministic = det
        tb.shall_train = True
        init = _params(tb)
        tb.frame()
        first.append(_params(tb) - init)
        while tb.training_step < 100:
            tb.frame()
        runs.append(_params(tb))
        losses.append(tb.loss)
        n_mlp = _n_mlp(tb)
        del tb
    np.testing.assert_array_equal(runs[0], runs[1])
    np.testing.assert_array_equal(first[0], first[1])
    both = (first[0] != 0) & (first[2] != 0)
    assert both[:n_mlp].mean() > 0.5 and both[n_mlp:].sum() > 1000
    agree = np.sign(first[0][both]) == np.sign(first[2][both])
    assert agree.mean() > 0.99, agree.mean()
    assert losses[2] == pytest.approx(losses[0], rel=0.1)


def test_deterministic_mode_switches_off_between_steps(scene):
    """bench.py pretrains with the deterministic hash-grid gradients and times the default path: a
    Testbed switched from one mode to the other between steps keeps training (the fixed-point and the
    fp16 gradient buffers are each zeroed by the optimizer step that consumes them), and the switched
    run's first deterministic steps are the deterministic run's."""
    torch.cuda.set_device(0)
    out = []
    for switch in (False, True):
        tb = _testbed(scene)
        tb.deterministic = True
        tb.shall_train = True
        while tb.training_step < 40:
            tb.frame()
        at40 = _params(tb)
        if switch:
            tb.deterministic = False
        while tb.training_step < 80:
            tb.frame()
        out.append((at40, _params(tb), tb.loss))
        del tb
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert np.isfinite(out[1][1]).all() and np.isfinite(out[1][2])
    assert out[1][2] == pytest.approx(out[0][2], rel=0.25)



def test_extra_dims_train_identically_on_every_rank(scene):
    """The per-image latent codes (extra dims) under data parallelism: the ranks draw the same initial codes, sum
    their code gradients and take the same VarAdam step, so after 16 steps codes and parameters are bit-identical
    on both ranks, and the codes have moved."""
    res = _spawn(_extra_dims_worker, scene, 2)
    r0, r1 = res[0], res[1]
    assert r0["dims"] == r1["dims"] == 16
    np.testing.assert_array_equal(r0["c0"], r1["c0"])
    np.testing.assert_array_equal(r0["c1"], r1["c1"])
    np.testing.assert_array_equal(r0["params"], r1["params"])
    assert np.isfinite(r0["loss"]) and np.abs(r0["c1"] - r0["c0"]).max() > 1e-4
