"""HIP path against the committed golden fixtures (no oracle run on the GPU box).

Tolerances as in test_gpu_kernels / test_gpu_pipeline: hash indices, weights,
features, occupancy bitfield, training sample counts and coordinates bit-exact; network
outputs within fp16 MFMA tolerance; rendered RGB <= 1e-3 mean L1 (north_star)."""
import ctypes as C
import json
import os

import numpy as np
import pytest
import torch

import ngp_abi as A
import golden_util as G
from gpu_util import GpuModel, cuda_memcpy_d2h, cuda_memcpy_h2d, stream
from scene_util import DeviceDataset

pytestmark = pytest.mark.gpu


def fixture(name):
    return np.load(os.path.join(G.GOLDEN, name))


def gpu_model(cfg_kw, seed, **kw):
    g = GpuModel(A.default_config(**cfg_kw))
    g.set_params(G.seeded_params(g.n_params, g.n_mlp, seed, **kw))
    return g


def set_grid(g, grid):
    gp, bp, tp, mp = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
    A.check(g.lib.ngp_density_grid_bitfield(g.h, 0, stream()))
    A.check(g.lib.ngp_density_grid_buffers(g.h, C.byref(gp), C.byref(bp), C.byref(tp), C.byref(mp)))
    cuda_memcpy_h2d(gp.value, np.ascontiguousarray(grid, np.float32))
    A.check(g.lib.ngp_density_grid_bitfield(g.h, 0, stream()))
    torch.cuda.synchronize()
    return bp.value, mp.value


@pytest.mark.parametrize("name", ["L16F2T19", "L8F4T19", "L4F2T14", "L16F2T22A64"])
def test_encode_golden(name):
    f = fixture(f"encode_{name}.npz")
    g = gpu_model(json.loads(str(f["cfg"])), int(f["params_seed"]))
    try:
        idx, w = g.encode_indices(f["pos"])
        np.testing.assert_array_equal(idx, f["idx"])
        np.testing.assert_array_equal(w, f["w"])
        np.testing.assert_array_equal(g.encode(f["pos"]).astype(np.float32), f["feat"])
    finally:
        g.close()


@pytest.mark.parametrize("name", ["A", "B"])
def test_mlp_golden(name):
    f = fixture(f"mlp_{name}.npz")
    g = gpu_model(json.loads(str(f["cfg"])), int(f["params_seed"]), mlp_scale=0.25, grid_scale=0.5)
    try:
        out = g.infer(f["coords"])
        err = np.abs(out - f["out"])
        assert (err <= 4e-3 + 8e-3 * np.abs(f["out"])).mean() > 0.999 and err.mean() < 1e-3
        np.testing.assert_allclose(g.density(f["coords"][:, :3]), f["density"], atol=4e-3, rtol=8e-3)
        g.zero_grads()
        enc = g.encode(f["coords"][:, :3]).astype(np.float32)
        denc = g.backward(enc, f["coords"][:, 4:7], f["dloss"].astype(np.float32))
        assert np.linalg.norm(denc - f["denc"]) / np.linalg.norm(f["denc"]) < 1e-2
        gg = g.get(A.GRADS_FP32)[: g.n_mlp]
        assert np.linalg.norm(gg - f["mlp_grads"]) / np.linalg.norm(f["mlp_grads"]) < 1e-2
    finally:
        g.close()


def test_bitfield_golden():
    f = fixture("bitfield.npz")
    g = GpuModel(A.default_config(**G.CFG_A))
    try:
        bp, mp = set_grid(g, G.seeded_grid(int(f["grid_seed"])))
        bits = np.zeros(G.CELLS // 8 * 8, np.uint8)
        cuda_memcpy_d2h(bits, bp)
        mean = np.zeros(1, np.float32)
        cuda_memcpy_d2h(mean, mp)
        assert mean[0] == f["mean"]
        assert G.digest(bits) == str(f["sha256"])
    finally:
        g.close()


def test_train_golden():
    f = fixture("train_A.npz")
    g = gpu_model(G.CFG_A, int(f["params_seed"]))
    try:
        set_grid(g, G.sphere_grid())
        dd = DeviceDataset(f["imgs"], f["cams"], float(f["focal"]))
        ta = G.golden_train_args(dd.ptr, dd.n, int(f["R"]), int(f["B"]), int(f["MS"]))
        g.zero_grads()
        A.check(g.lib.ngp_train_step(g.h, C.byref(ta), stream()))
        st = A.TrainStats()
        A.check(g.lib.ngp_train_read_stats(g.h, C.byref(st), stream()))
        assert st.measured_batch_size_before_compaction == int(f["n_before"])
        p, nb = C.c_void_p(), C.c_size_t()
        A.check(g.lib.ngp_train_scratch(g.h, A.SCRATCH_RAY_NUMSTEPS, C.byref(p), C.byref(nb)))
        ns = np.zeros(nb.value // 4, np.uint32)
        cuda_memcpy_d2h(ns, p.value)
        np.testing.assert_array_equal(ns.reshape(-1, 2), f["numsteps"])
        n = int(f["n_before"])
        A.check(g.lib.ngp_train_scratch(g.h, A.SCRATCH_COORDS, C.byref(p), C.byref(nb)))
        coords = np.zeros(nb.value // 4, np.float32)
        cuda_memcpy_d2h(coords, p.value)
        np.testing.assert_array_equal(coords.reshape(-1, 8)[:n], f["coords"])
        np.testing.assert_allclose(st.loss, float(f["loss"]), rtol=2e-2)
    finally:
        g.close()


def test_render_golden():
    f = fixture("render_A.npz")
    g = gpu_model(G.CFG_A, int(f["params_seed"]), grid_scale=1.0)
    try:
        set_grid(g, G.sphere_grid(0.3))
        ra = G.golden_render_args()
        frame = torch.zeros(ra.height * ra.width * 4, dtype=torch.float32, device="cuda")
        depth = torch.zeros(ra.height * ra.width, dtype=torch.float32, device="cuda")
        A.check(g.lib.ngp_render(g.h, C.byref(ra), C.c_void_p(frame.data_ptr()), C.c_void_p(depth.data_ptr()), stream()))
        torch.cuda.synchronize()
        gf = frame.cpu().numpy().reshape(ra.height, ra.width, 4)
        assert np.abs(gf - f["frame"]).mean() < 1e-3
    finally:
        g.close()
