"""The oracle still reproduces the committed golden fixtures (tests/golden/*.npz, made by
tests/golden/make_golden.py).  CPU only; the GPU side is tests/test_gpu_golden.py."""
import json
import os

import numpy as np
import pytest

import ngp_abi as A
import golden_util as G
from oracle_abi import Oracle, load, ptr

FIX = G.GOLDEN


def fixture(name):
    path = os.path.join(FIX, name)
    if not os.path.exists(path):
        pytest.fail(f"missing golden fixture {name}: run tests/golden/make_golden.py")
    return np.load(path)


@pytest.mark.parametrize("name", ["L16F2T19", "L8F4T19", "L4F2T14", "L16F2T22A64"])
def test_encode_fixture(name):
    g = fixture(f"encode_{name}.npz")
    o = Oracle(A.default_config(**json.loads(str(g["cfg"]))))
    o.set_params(G.seeded_params(o.n_params, o.n_mlp, int(g["params_seed"])))
    idx, w = o.encode_indices(g["pos"])
    np.testing.assert_array_equal(idx, g["idx"])
    np.testing.assert_array_equal(w, g["w"])
    np.testing.assert_array_equal(o.encode(g["pos"]), g["feat"])


@pytest.mark.parametrize("name", ["A", "B"])
def test_mlp_fixture(name):
    g = fixture(f"mlp_{name}.npz")
    o = Oracle(A.default_config(**json.loads(str(g["cfg"]))))
    o.set_params(G.seeded_params(o.n_params, o.n_mlp, int(g["params_seed"]), mlp_scale=0.25, grid_scale=0.5))
    c = g["coords"]
    np.testing.assert_array_equal(o.infer(c), g["out"])
    np.testing.assert_array_equal(o.density(c[:, :3]), g["density"])
    denc = o.backward(o.encode(c[:, :3]), c[:, 4:7], g["dloss"].astype(np.float32))
    np.testing.assert_array_equal(denc, g["denc"])
    np.testing.assert_array_equal(o.get(A.GRADS_FP32)[: o.n_mlp], g["mlp_grads"])


def test_sh_fixture():
    g = fixture("sh4.npz")
    lib = load()
    for d, ref in zip(g["dirs"], g["sh"]):
        out = np.zeros(16, np.float32)
        lib.oref_sh4(ptr(np.ascontiguousarray(d)), ptr(out))
        np.testing.assert_array_equal(out, ref)


def test_bitfield_fixture():
    g = fixture("bitfield.npz")
    o = Oracle(A.default_config(**G.CFG_A))
    o.grid_set(G.seeded_grid(int(g["grid_seed"])))
    o.grid_bitfield(0)
    _, bits, mean = o.grid_get(G.CELLS)
    assert np.float32(mean) == g["mean"]
    assert G.digest(bits) == str(g["sha256"])


def test_train_fixture():
    g = fixture("train_A.npz")
    o = Oracle(A.default_config(**G.CFG_A))
    o.set_params(G.seeded_params(o.n_params, o.n_mlp, int(g["params_seed"])))
    o.grid_set(G.sphere_grid())
    o.grid_bitfield(0)
    hd = G.host_dataset(g["imgs"], g["cams"], float(g["focal"]))
    o.train_step(G.golden_train_args(hd.ptr, hd.n, int(g["R"]), int(g["B"]), int(g["MS"])))
    st = o.stats()
    assert st.measured_batch_size_before_compaction == int(g["n_before"])
    assert st.measured_batch_size == int(g["n_after"])
    np.testing.assert_array_equal(o.scratch(A.SCRATCH_RAY_NUMSTEPS, np.uint32).reshape(-1, 2), g["numsteps"])
    n = int(g["n_before"])
    np.testing.assert_array_equal(o.scratch(A.SCRATCH_COORDS, np.float32).reshape(-1, 8)[:n], g["coords"])
    np.testing.assert_array_equal(o.scratch(A.SCRATCH_RAY_COMPACTED, np.uint32).reshape(-1, 2), g["compacted"])
    assert np.float32(st.loss) == g["loss"]


def test_render_fixture():
    g = fixture("render_A.npz")
    o = Oracle(A.default_config(**G.CFG_A))
    o.set_params(G.seeded_params(o.n_params, o.n_mlp, int(g["params_seed"]), grid_scale=1.0))
    o.grid_set(G.sphere_grid(0.3))
    o.grid_bitfield(0)
    frame, depth = o.render(G.golden_render_args())
    np.testing.assert_array_equal(frame, g["frame"])
    assert (frame[..., 3] > 0.01).mean() > 0.2
