"""Error map (Nerf::Training::ErrorMap) on the CPU oracle: the CDF construction against a
numpy restatement of construct_cdf_2d/1d (src/testbed_nerf.cu:1493-1546), and the
bilinear error deposit of compute_loss_kernel_train_nerf (:1028-1054) by mass
conservation over one training step."""
import ctypes as C

import numpy as np

import ngp_abi as A
from error_map_util import build_cdf_numpy, normalise_image_cdf
from oracle_abi import Oracle, load, ptr
from scene_util import HostDataset, make_views, sphere_bitfield, train_args

CFG_A = dict(n_levels=4, F=2, log2_T=14, n_neurons=16)


def test_cdf_construction_matches_numpy():
    rng = np.random.default_rng(3)
    err = rng.exponential(1.0, (5, 11, 13)).astype(np.float32)
    err[2] = 0.0  # an image with no error yet: the 1e-10 floor keeps its CDFs well-formed
    cx = np.zeros_like(err)
    cy = np.zeros(err.shape[:2], np.float32)
    ci = np.zeros(5, np.float32)
    load().oref_error_map_build_cdf(ptr(err), 5, 13, 11, ptr(cx), ptr(cy), ptr(ci))
    ex, ey, ei = build_cdf_numpy(err)
    np.testing.assert_allclose(cx, ex, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(cy, ey, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ci, ei, rtol=1e-6)
    assert np.all(np.diff(cx, axis=2) > 0) and np.allclose(cx[..., -1], 1.0, atol=1e-6)
    assert np.all(np.diff(cy, axis=1) > 0) and np.allclose(cy[..., -1], 1.0, atol=1e-6)
    pmf, cdf = normalise_image_cdf(ci)
    assert np.isclose(pmf.sum(), 1.0, atol=1e-5) and np.isclose(cdf[-1], 1.0, atol=1e-6)
    assert pmf.min() >= 0.1 / 5 - 1e-7  # MIN_PMF floor


def test_error_deposit_conserves_mean_loss():
    imgs, cams, focal = make_views(4, 16, 16)
    hd = HostDataset(imgs, cams, focal)
    o = Oracle(A.default_config(**CFG_A))
    o.set_params(np.random.default_rng(5).uniform(-0.2, 0.2, o.n_params).astype(np.float32))
    o.grid_set(sphere_bitfield(0.32))
    o.grid_bitfield(0)
    R = 96
    a = train_args(hd.ptr, hd.n, R, 4096, 1 << 14)
    err = np.zeros((hd.n, 5, 7), np.float32)
    a.error_map = err.ctypes.data
    a.error_map_res[0], a.error_map_res[1] = 7, 5
    o.train_step(a)
    st = o.stats()
    # every ray with kept samples deposits its mean loss with bilinear weights summing to 1;
    # the reported loss is sum(mean_loss) / n_rays
    assert err.sum() > 0
    np.testing.assert_allclose(err.sum(), st.loss * R, rtol=1e-4)


def test_importance_sampling_follows_error_map():
    """With the CDFs of a one-hot error map, image choice follows the normalised image CDF
    and the non-uniform half of the pixels lands in the hot texel (sample_cdf_2d, image_idx),
    with the pdf the loss is divided by."""
    imgs, cams, focal = make_views(4, 16, 16)
    hd = HostDataset(imgs, cams, focal)
    err = np.zeros((4, 4, 4), np.float32)
    err[2, 1, 3] = 1000.0
    cx = np.zeros_like(err)
    cy = np.zeros((4, 4), np.float32)
    ci = np.zeros(4, np.float32)
    lib = load()
    lib.oref_error_map_build_cdf(ptr(err), 4, 4, 4, ptr(cx), ptr(cy), ptr(ci))
    pmf_img, cdf_img = normalise_image_cdf(ci)
    R = 4000
    a = train_args(hd.ptr, hd.n, R, 1 << 15, 1 << 16)
    a.cdf_x_cond_y, a.cdf_y, a.cdf_img = cx.ctypes.data, cy.ctypes.data, cdf_img.ctypes.data
    a.cdf_res[0], a.cdf_res[1] = 4, 4
    u, v, pdf = C.c_float(), C.c_float(), C.c_float()
    imgs_, hot = [], 0
    for gi in range(R):
        img = lib.oref_pick_pixel(C.byref(a), gi, C.byref(u), C.byref(v), C.byref(pdf))
        imgs_.append(img)
        if img == 2 and 0.75 <= u.value < 1.0 and 0.25 <= v.value < 0.5:
            hot += 1
        assert pdf.value > 0
    frac = np.bincount(imgs_, minlength=4) / R
    np.testing.assert_allclose(frac, pmf_img, atol=0.03)  # low-discrepancy draws track the pmf closely
    n2 = frac[2] * R
    # half uniform (1/16 of it in the texel), half from the CDF (0.99 of it + the floor)
    assert 0.45 < hot / n2 < 0.6
