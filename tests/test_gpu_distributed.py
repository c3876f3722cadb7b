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
gathered frame equals rank 0's own full render bit for bit.
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


def _testbed(scene_dir):
    import pyngp as ngp
    tb = ngp.Testbed()
    tb.load_training_data(os.path.join(scene_dir, "transforms_train.json"))
    tb.reload_network_from_file("tiny_L4F2.json")
    tb.training_batch_size = BATCH
    return tb


def _worker(rank, world, port, scene_dir, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tb = _testbed(scene_dir)

        def allreduce(arr, op):
            t = torch.from_numpy(arr)
            rop = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
            if t.dtype == torch.float16:  # gloo reduces fp32; a 2-rank fp16 sum rounds exactly once either way
                t32 = t.float()
                dist.all_reduce(t32, op=rop)
                t.copy_(t32.half())
            else:
                dist.all_reduce(t, op=rop)

        tb.init_distributed_host(rank, world, allreduce)
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


@pytest.fixture(scope="module")
def scene(tmp_path_factory):
    root = tmp_path_factory.mktemp("dp_scene")
    S.write_nerf_synthetic_scene(str(root), 10, 48, 48, seed=5, split="train")
    return str(root)


def test_data_parallel_testbed_two_processes_one_gpu(scene):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scene, q)) for r in range(world)]
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
