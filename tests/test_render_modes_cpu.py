"""CPU checks of the oracle's render API restatement (the HIP side is compared with it in
test_gpu_render_modes.py): the crop box's identity frame, an aperture of zero, the Slice mode's depth
buffer, Cost counts as integers, and AO / Positions colours in their ranges."""
import numpy as np
import pytest

import ngp_abi as A
from oracle_abi import Oracle
from scene_util import make_views, render_args, sphere_bitfield

W, H = 24, 20


@pytest.fixture(scope="module")
def model():
    o = Oracle(A.default_config(n_levels=4, F=2, log2_T=14, n_neurons=16))
    rng = np.random.default_rng(0)
    p = np.zeros(o.n_params, np.float32)
    p[: o.n_mlp] = rng.normal(0, 0.3, o.n_mlp)
    p[o.n_mlp:] = rng.uniform(-1.0, 1.0, o.n_params - o.n_mlp)
    o.set_params(p)
    o.grid_set(sphere_bitfield(0.3))
    o.grid_bitfield(0)
    return o


def _args(**kw):
    cam = make_views(1, 8, 8)[1][0]
    ra = render_args(W, H, cam, 0.5 * W / np.tan(0.5 * 0.69), spp=1)
    ra.depth_scale = 1.0 / 0.33
    for k, v in kw.items():
        setattr(ra, k, v)
    return ra


def test_identity_frame_and_zero_aperture_change_nothing(model):
    base, bd = model.render(_args())
    ra = _args(aperture_size=0.0, focus_z=1.5)
    for k, x in enumerate(np.eye(3, dtype=np.float32).reshape(-1)):
        ra.render_aabb_to_local[k] = float(x)
    f, d = model.render(ra)
    np.testing.assert_array_equal(f, base)
    np.testing.assert_array_equal(d, bd)
    assert (base[..., 3] > 0.01).mean() > 0.1


def test_modes_ranges(model):
    ao, _ = model.render(_args(render_mode=A.RENDER_AO))
    assert ao[..., :3].min() >= 0 and ao[..., :3].max() <= 1.0 + 1e-6
    pos, _ = model.render(_args(render_mode=A.RENDER_POSITIONS))
    hit = pos[..., 3] > 0.01
    assert hit.any()
    # positions in the unit cube map to [0.25, 0.75] ((p - 0.5) / 2 + 0.5); the colour is their
    # weight-sum, alpha the weights' sum
    mean = pos[hit, :3] / pos[hit, 3:4]
    assert mean.min() > 0.2 and mean.max() < 0.8
    cost, _ = model.render(_args(render_mode=A.RENDER_COST))
    hitc = cost[..., 3] == 1.0
    assert hitc.any()
    counts = cost[hitc, 0] * 128.0
    np.testing.assert_array_equal(counts, np.round(counts))
    assert counts.max() >= 1


def test_slice_depth_buffer(model):
    f, d = model.render(_args(render_mode=A.RENDER_SLICE, focus_z=1.3))
    d = np.asarray(d).reshape(H, W)
    np.testing.assert_array_equal(d, np.float32(1.3))
    assert (f[..., 3] > 0).all()


def test_crop_removes_samples(model):
    full, _ = model.render(_args())
    ra = _args()
    for k in range(3):
        ra.aabb_min[k], ra.aabb_max[k] = 0.45, 0.55
    crop, _ = model.render(ra)
    assert (crop[..., 3] > 0.01).sum() < (full[..., 3] > 0.01).sum()
