"""Testbed.compute_and_save_png_slices / get_density_on_grid on the GPU (src/python_api.cu:451-459,
src/testbed.cu:534-559, src/testbed_nerf.cu:147-160, 234-250, 3026-3075, src/marching_cubes.cu:40-47, 957-1020):
the lattice densities against the oracle with the same weights and density grid, the written mosaic byte for byte
against the oracle's mosaic of the same densities."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FOX = os.path.join(ROOT, "data", "nerf", "fox", "transforms.json")


@pytest.fixture(scope="module")
def fox():
    """base.json trained 300 steps on the fox (aabb_scale 4: three occupancy cascades, OpenCV lens)."""
    import pyngp as ngp
    tb = ngp.Testbed()
    tb.load_training_data(FOX)
    tb.reload_network_from_file("base.json")
    tb.shall_train = True
    while tb.training_step < 300:
        tb.frame()
    assert tb.nerf.max_cascade == 2
    return ngp, tb


def _query(tb, res, lo, hi, to_local=None):
    import ngp_abi as A
    q = A.GridQuery()
    for k in range(3):
        q.res[k] = res[k]
        q.box_min[k], q.box_max[k] = lo[k], hi[k]
        q.aabb_min[k], q.aabb_max[k] = tb.aabb.min[k], tb.aabb.max[k]
    m = np.eye(3, dtype=np.float32) if to_local is None else np.asarray(to_local, np.float32)
    for k in range(9):
        q.box_to_local[k] = float(m.reshape(-1)[k])
    q.max_cascade = int(tb.nerf.max_cascade)
    q.mask_with_grid = 1
    q.use_inference_params = 1
    return q


def _rot(axis, angle):
    c, s = np.cos(angle), np.sin(angle)
    i, j = [k for k in range(3) if k != axis]
    R = np.eye(3, dtype=np.float32)
    R[i, i], R[i, j], R[j, i], R[j, j] = c, -s, s, c
    return R


@pytest.mark.parametrize("box", ["render_aabb", "sub_box", "rotated"])
def test_density_on_grid_matches_oracle(fox, box):
    """get_density_on_grid: raw density outputs within the fp16 tolerance of the MLP parity tests, the -10000 mask
    of cells the cascaded density grid holds below NERF_MIN_OPTICAL_THICKNESS identical."""
    from scene_util import testbed_oracle
    ngp, tb = fox
    res = (40, 36, 28)
    bb = ngp.BoundingBox()
    orig_box, orig_local = tb.render_aabb, np.array(tb.render_aabb_to_local, np.float32)
    if box == "sub_box":
        bb = ngp.BoundingBox([-0.4, 0.1, 0.0], [1.7, 1.2, 0.9])
    if box == "rotated":
        tb.render_aabb = ngp.BoundingBox([-0.5, -0.5, -0.5], [1.5, 1.5, 1.5])
        tb.render_aabb_to_local = _rot(1, 0.3) @ _rot(0, -0.2)
    try:
        g = tb.density_on_grid(list(res), bb)
        if bb.is_empty():
            lo, hi, R = tb.render_aabb.min, tb.render_aabb.max, np.asarray(tb.render_aabb_to_local)
        else:
            lo, hi, R = bb.min, bb.max, None
        o = testbed_oracle(tb)
        r = o.density_on_grid(_query(tb, res, lo, hi, R), tb.density_grid())
    finally:
        tb.render_aabb = orig_box
        tb.render_aabb_to_local = orig_local
    assert g.shape == (res[2], res[1], res[0])
    masked_g, masked_r = g == -10000.0, r == -10000.0
    np.testing.assert_array_equal(masked_g, masked_r)
    assert 0.02 < masked_g.mean() < 0.98, masked_g.mean()  # both kinds of lattice points occur
    np.testing.assert_allclose(g[~masked_g], r[~masked_r], atol=4e-3, rtol=8e-3)


def test_png_slices_are_the_oracle_mosaic(fox, tmp_path):
    """The written file: filename + '.density_slices_{x}x{y}x{z}.png', 8-bit gray, byte-identical to the oracle's
    save_density_grid_to_png mosaic of the same lattice densities, for the defaults (render aabb, thresh =
    mesh_thresh 2.5, range 4), a non-cubic box (get_marching_cubes_res rounds each axis up to 16), another
    threshold / range and flip_y_and_z_axes; the return value is the lattice resolution."""
    from oracle_abi import density_slices_mosaic
    from density_slices_util import read_png_gray
    ngp, tb = fox
    cases = [
        (dict(), None, (64, 64, 64)),
        (dict(aabb=ngp.BoundingBox([-0.4, 0.2, 0.1], [1.6, 1.1, 1.3])), ngp.BoundingBox([-0.4, 0.2, 0.1], [1.6, 1.1, 1.3]),
         (64, 32, 48)),
        (dict(thresh=1.0, density_range=8.0), None, (64, 64, 64)),
        (dict(flip_y_and_z_axes=True, aabb=ngp.BoundingBox([0.0, 0.0, 0.0], [1.0, 0.5, 1.0])),
         ngp.BoundingBox([0.0, 0.0, 0.0], [1.0, 0.5, 1.0]), (64, 32, 64)),
    ]
    assert tb.mesh_thresh == 2.5
    for i, (kw, bb, want) in enumerate(cases):
        prefix = str(tmp_path / f"slices{i}")
        res = tuple(int(v) for v in tb.compute_and_save_png_slices(prefix, 64, **kw))
        assert res == want, (kw, res)
        path = prefix + ".density_slices_{}x{}x{}.png".format(*res)
        assert os.path.exists(path), path
        png = read_png_gray(path)
        d = tb.density_on_grid(list(res), bb if bb is not None else ngp.BoundingBox())
        ref, _ = density_slices_mosaic(d, kw.get("thresh", 2.5), kw.get("flip_y_and_z_axes", False),
                                       kw.get("density_range", 4.0))
        np.testing.assert_array_equal(png, ref, err_msg=str(kw))
        assert (png >= 129).any() and (png == 0).any()


def _training_view_psnr(tb, views=4):
    """Mean PSNR of `views` training views rendered at their own resolution against the images (black background)."""
    ds = tb.nerf.training.dataset
    tb.background_color = [0.0, 0.0, 0.0, 1.0]
    out = []
    for v in np.linspace(0, ds.n_images - 1, views).astype(int):
        w, h = (int(x) for x in ds.metadata[int(v)].resolution)
        tb.set_camera_to_training_view(int(v))
        tb.render_ground_truth = True
        gt = tb.render(w, h, 1, True)[..., :3]
        tb.render_ground_truth = False
        img = tb.render(w, h, 1, True)[..., :3]
        out.append(-10.0 * np.log10(max(float(np.mean((np.clip(img, 0, 1) - np.clip(gt, 0, 1)) ** 2)), 1e-12)))
    return float(np.mean(out))


def test_trained_field_at_the_reference_resolution_against_its_density_mosaic():
    """The same pin at the resolution the reference trained at (720x1280, data/nerf/test2_full): there the default mode
    has one outcome.  tools/collapse_sweep.py, 8 fixed seeds, base.json, 35 k steps, random background colours
    (profiles/r06_collapse_sweep_test2_full.jsonl, last section of r06_collapse_sweep.txt): 8 of 8 form the flame and
    its backdrop (three starved at 5 k steps and recovered by 15 k): occupied volume 1.50-1.80x the reference's, the
    reference's field correlating best with ours in the identity frame of the 48 axis orders / flips (0.17-0.23), IoU
    of the >= 2.5 masks 0.13-0.16 against the reference and 0.38-0.45 seed versus seed.  Seeds 1337 and 1 (the sweep's
    first two, fixed before measuring); thresholds: the measured ranges widened by about a third.  Voxel-level
    agreement with the reference's single run at the seed-versus-seed level is not claimed (0.14 vs 0.42).
    At lower resolution the default mode is bimodal (half: 6 of 8 form the flame, quarter: 2 of 8; the rest stay sample-
    starved and paint the views on the box), which is why the pin trains the reference's resolution.
    The other shipped mosaic (data/nerf/test.density_slices_...) names the data path data/nerf/test, not test/dataset
    where the fire scene sits, and matches no orientation of fields trained on it: it is not compared."""
    import density_slices_util as D
    import pyngp as ngp
    ref = D.reference_volume("test2") >= 129
    cref = D.coarse(ref)
    occs = []
    for seed in (1337, 1):
        tb = D.new_testbed(ngp, "test2_full", "base.json", seed)
        D.train_to(tb, 35000)
        rays = tb.last_train_stats()["n_rays"]
        occ = D.testbed_volume(tb) >= 129
        ident, rank = D.orientation_ranking(D.coarse(occ), cref)
        ratio = float(occ.mean() / ref.mean())
        iou = float((occ & ref).sum() / max((occ | ref).sum(), 1))
        print(f"test2_full seed {seed}: rays {rays}, occupied ratio {ratio:.2f}, corr vs reference {ident:.3f} "
              f"(rank {rank} of 48), IoU vs reference {iou:.3f}")
        assert rays < (1 << 18), rays  # not sample-starved
        assert 1.0 < ratio < 2.4, ratio
        assert rank == 0 and ident > 0.11, (ident, rank)
        assert iou > 0.09, iou
        occs.append(occ)
        del tb
    a, b = occs
    iou_seeds = float((a & b).sum() / max((a | b).sum(), 1))
    print(f"test2_full seed vs seed IoU {iou_seeds:.3f}")
    assert iou_seeds > 0.25, iou_seeds


def test_black_background_training_on_the_reference_scene_has_no_backdrop():
    """The mosaic pins' control: test2 at the reference's resolution (720x1280) trained with a black background
    (random_bg_color False, default mode, seeds 1337 and 1) forms the flame alone -- the reference's 13.3 % is the flame
    plus the backdrop density random-background training builds.  The sweep measured it first (8 of 8 seeds, no density
    excursion on the way: occupied volume 0.037-0.039x the reference's, seed-versus-seed IoU 0.85-0.89, training-view
    PSNR 32.1-35.8 dB; profiles/r06_collapse_sweep_test2_full_black_bg.jsonl, r06_collapse_sweep.txt).  Thresholds: the
    measured ranges widened by about a third.
    This control first trained the quarter-resolution copy, where black-background runs are not stable: they pass
    through transient density excursions (2 of 5 trajectories) and 2 of 17 ended inside one or painted on the box
    (21.0 dB; ratio 6.9 at 25.6 dB -- the round-6 suite runs, profiles/r06_gpu_tests_suite*.txt), as random-background
    runs do more often at low resolution."""
    import density_slices_util as D
    import pyngp as ngp
    ref = D.reference_volume("test2") >= 129
    occ_black, psnr = [], []
    for seed in (1337, 1):
        tb = D.new_testbed(ngp, "test2_full", "base.json", seed, random_bg_color=False)
        D.train_to(tb, 35000)
        rays = tb.last_train_stats()["n_rays"]
        occ_black.append(D.testbed_volume(tb) >= 129)
        psnr.append(round(_training_view_psnr(tb), 2))
        assert rays < (1 << 18), rays
        del tb
    a, b = occ_black
    iou = float((a & b).sum() / max((a | b).sum(), 1))
    ratios = [float(o.mean() / ref.mean()) for o in occ_black]
    print(f"test2_full black background: seed vs seed IoU {iou:.3f}, occupied ratios {ratios}, training-view PSNR {psnr}")
    assert iou > 0.55, iou
    assert max(ratios) < 0.1, ratios
    assert min(psnr) > 24.0, psnr
