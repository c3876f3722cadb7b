"""The tracer's render API beyond the default Shade mode, HIP against the oracle (a28-a30):

* the render crop box (Testbed::m_render_aabb in the frame of m_render_aabb_to_local;
  src/testbed_nerf.cu:335-381, 421-469, 1465-1475; nerf_device.cuh:461-494), rotated;
* the render modes of composite_kernel_nerf / shade_kernel_nerf (src/testbed_nerf.cu:626-638,
  1327-1338): AO, Normals (the density gradient through the network, :1715-1717), Positions,
  Depth (soft and with render_gbuffer_hard_edges), Cost, and Slice (render_nerf's 2-D path,
  :1842-1845, 1908-1932);
* depth of field (uv_to_ray, common_device.cuh:450-456);
* the glow of composite_kernel_nerf (nerf.glow_mode / glow_y_cutoff, src/testbed_nerf.cu:540-628): grid and
  cut lines below the cutoff, mask to alpha, radial distance, grid mode.

Every case renders a 72 x 66 frame of a config-A/B network over a sphere of occupancy and compares
RGBA with the oracle within the north-star 1e-3 mean L1 (Normals, a gradient through fp16
activations: 1e-2); Cost values are counts and must match exactly.
"""
import ctypes as C

import numpy as np
import pytest
import torch

import ngp_abi as A
from gpu_util import stream
from scene_util import make_views, render_args, sphere_bitfield
from test_gpu_pipeline import CFG_A, CFG_B, pair, set_bitfield_both

pytestmark = pytest.mark.gpu

W, H = 72, 66


def rot_z(deg):
    a = np.deg2rad(deg)
    return np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]], np.float32)


def _render(g, o, ra):
    frame = torch.zeros(H * W * 4, dtype=torch.float32, device="cuda")
    depth = torch.zeros(H * W, dtype=torch.float32, device="cuda")
    A.check(g.lib.ngp_render(g.h, C.byref(ra), C.c_void_p(frame.data_ptr()), C.c_void_p(depth.data_ptr()), stream()))
    torch.cuda.synchronize()
    of, od = o.render(ra)
    return frame.cpu().numpy().reshape(H, W, 4), depth.cpu().numpy().reshape(H, W), of, np.asarray(od).reshape(H, W)


CASES = {
    "crop_rotated": dict(crop=((0.32, 0.3, 0.35), (0.68, 0.7, 0.6)), R=rot_z(30)),
    "ao": dict(mode=A.RENDER_AO),
    "positions": dict(mode=A.RENDER_POSITIONS),
    "depth": dict(mode=A.RENDER_DEPTH),
    "depth_hard_edges": dict(mode=A.RENDER_DEPTH, hard=1),
    "positions_hard_edges": dict(mode=A.RENDER_POSITIONS, hard=1),
    "cost": dict(mode=A.RENDER_COST),
    "normals": dict(mode=A.RENDER_NORMALS, tol=1e-2),
    "slice": dict(mode=A.RENDER_SLICE, focus=1.3),
    "dof": dict(aperture=0.04, focus=2.4, spp=3),
    "dof_crop": dict(aperture=0.04, focus=2.4, crop=((0.25, 0.25, 0.25), (0.75, 0.7, 0.75)), R=rot_z(-20)),
    # Nerf::glow_mode / glow_y_cutoff (composite_kernel_nerf's glow, src/testbed_nerf.cu:540-628)
    "glow_grid_cutline": dict(glow=1 | 2, cutoff=0.55),
    "glow_mask_to_alpha": dict(glow=1 | 2 | 4, cutoff=0.5),
    # radial: dist = min(|pos - camera|, (4.5 - y) / 3), 1.03-1.33 on the sphere's visible side; the glow lives in
    # the shell dist in (cutoff - 21/80, cutoff)
    "glow_radial": dict(glow=1 | 2 | 8, cutoff=1.3),
    "glow_grid_mode": dict(glow=16),
    "glow_positions": dict(glow=1 | 4, cutoff=0.6, mode=A.RENDER_POSITIONS),
}


@pytest.mark.parametrize("case", list(CASES))
def test_render_mode_matches_oracle(case):
    c = CASES[case]
    g, o, rng = pair(CFG_B if case == "normals" else CFG_A, grid_scale=1.0)
    try:
        set_bitfield_both(g, o, sphere_bitfield(0.3))
        cam = make_views(1, 8, 8)[1][0]
        focal = 0.5 * W / np.tan(0.5 * 0.69)
        ra = render_args(W, H, cam, focal, spp=c.get("spp", 1), snap=0)
        ra.render_mode = c.get("mode", A.RENDER_SHADE)
        ra.depth_scale = 1.0 / 0.33
        ra.gbuffer_hard_edges = c.get("hard", 0)
        ra.aperture_size = c.get("aperture", 0.0)
        ra.focus_z = c.get("focus", 0.0)
        ra.glow_mode = c.get("glow", 0)
        ra.glow_y_cutoff = c.get("cutoff", 0.0)
        if "crop" in c:
            lo, hi = c["crop"]
            for k in range(3):
                ra.aabb_min[k], ra.aabb_max[k] = lo[k], hi[k]
        if "R" in c:
            for k, x in enumerate(c["R"].reshape(-1)):
                ra.render_aabb_to_local[k] = float(x)
        gf, gd, of, od = _render(g, o, ra)
        assert np.isfinite(gf).all()
        cover = (of[..., 3] > 0.01).mean()
        assert cover > 0.05, cover
        if ra.render_mode == A.RENDER_COST:
            np.testing.assert_array_equal(gf, of)
            assert of[..., 0].max() > 0
        else:
            err = np.abs(gf - of).mean()
            assert err < c.get("tol", 1e-3), err
        if ra.render_mode == A.RENDER_SLICE:
            np.testing.assert_array_equal(gd[gd < 1e4], np.float32(ra.focus_z))
        if ra.glow_mode:
            # the glow changes the frame
            ra.glow_mode = 0
            plain, _, _, _ = _render(g, o, ra)
            assert np.abs(plain - gf).mean() > 1e-3
        if "crop" in c:
            # the crop removes part of the sphere: fewer covered pixels than the uncropped render
            ra2 = render_args(W, H, cam, focal, spp=c.get("spp", 1), snap=0)
            ra2.aperture_size, ra2.focus_z = ra.aperture_size, ra.focus_z
            full, _, _, _ = _render(g, o, ra2)
            assert (gf[..., 3] > 0.01).sum() < (full[..., 3] > 0.01).sum()
    finally:
        g.close()


def test_testbed_render_api_properties():
    """pyngp surface of the same features: render_mode, render_aabb / render_aabb_to_local, aperture_size /
    dof, slice_plane_z, nerf.render_gbuffer_hard_edges -- a Depth render of a trained scene has the
    depth buffer's values in its colour channels (hard edges), a crop box to nothing renders nothing."""
    import os
    import pyngp as ngp
    import synthetic as S
    import tempfile
    root = tempfile.mkdtemp()
    S.write_nerf_synthetic_scene(root, 8, 48, 48, seed=3, split="train")
    tb = ngp.Testbed()
    tb.load_training_data(os.path.join(root, "transforms_train.json"))
    tb.reload_network_from_file("tiny_L4F2.json")
    tb.shall_train = True
    for _ in range(64):
        tb.frame()
    tb.set_camera_to_training_view(0)
    tb.background_color = [0.0, 0.0, 0.0, 0.0]
    shade = tb.render(48, 48, 1, True)
    assert shade[..., 3].max() > 0.5
    tb.render_mode = ngp.RenderMode.Depth
    tb.nerf.render_gbuffer_hard_edges = True
    dep = tb.render(48, 48, 1, True)
    hit = dep[..., 3] > 0.5
    assert hit.any() and np.all(dep[hit, 0] > 0)
    tb.render_mode = ngp.RenderMode.Shade
    box = tb.render_aabb
    assert np.allclose(box.min, tb.aabb.min) and np.allclose(box.max, tb.aabb.max)
    np.testing.assert_array_equal(tb.render_aabb_to_local, np.eye(3, dtype=np.float32))
    tb.render_aabb = ngp.BoundingBox([0.0, 0.0, 0.0], [0.01, 0.01, 0.01])
    assert tb.render(48, 48, 1, True)[..., 3].max() == 0
    tb.render_aabb = box
    tb.aperture_size = 0.0
    np.testing.assert_array_equal(tb.render(48, 48, 1, True), shade)
    with pytest.raises(RuntimeError, match="Distortion"):
        tb.render_mode = ngp.RenderMode.Distortion
        tb.render(48, 48, 1, True)
