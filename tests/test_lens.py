"""Camera lens models of uv_to_ray (common_device.cuh:248-460) on the CPU oracle: the
iterative OpenCV / OpenCV-fisheye undistortion inverts the distortion polynomial, and the
panoramic models give unit directions with the reference's axis conventions."""
import numpy as np
import pytest

from oracle_abi import load, ptr


def lens_dir(u, v, mode, params, res=(64, 48), focal=(50.0, 52.0), pp=(0.5, 0.5)):
    p = np.zeros(7, np.float32)
    p[:len(params)] = params
    out = np.zeros(3, np.float32)
    ok = load().oref_lens_direction(u, v, float(res[0]), float(res[1]), focal[0], focal[1], pp[0], pp[1], mode, ptr(p),
                                    ptr(out))
    return bool(ok), out


def opencv_distort(x, y, k):
    k1, k2, p1, p2 = k
    r2 = x * x + y * y
    radial = k1 * r2 + k2 * r2 * r2
    return (x + x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x),
            y + y * radial + 2 * p2 * x * y + p1 * (r2 + 2 * y * y))


def fisheye_distort(x, y, k):
    r = np.hypot(x, y)
    th = np.arctan(r)
    thd = th * (1 + k[0] * th ** 2 + k[1] * th ** 4 + k[2] * th ** 6 + k[3] * th ** 8)
    return x * thd / r, y * thd / r


@pytest.mark.parametrize("mode,k,distort", [(1, (-0.12, 0.03, 0.001, -0.002), opencv_distort),
                                            (4, (0.05, -0.01, 0.002, -0.0005), fisheye_distort)])
def test_undistortion_inverts_distortion(mode, k, distort):
    rng = np.random.default_rng(0)
    for u, v in rng.uniform(0.05, 0.95, (64, 2)):
        ok, d = lens_dir(float(u), float(v), mode, k)
        assert ok and d[2] == 1.0
        # the undistorted point re-distorts to the pinhole coordinates of the pixel
        x0, y0 = (u - 0.5) * 64 / 50.0, (v - 0.5) * 48 / 52.0
        xd, yd = distort(float(d[0]), float(d[1]), k)
        assert abs(xd - x0) < 2e-5 and abs(yd - y0) < 2e-5


def test_perspective_and_panoramic_directions():
    ok, d = lens_dir(0.75, 0.25, 0, ())
    np.testing.assert_allclose(d, [(0.25) * 64 / 50.0, (-0.25) * 48 / 52.0, 1.0], rtol=1e-6)
    ok, d = lens_dir(0.5, 0.5, 3, ())  # latlong centre looks down +z
    np.testing.assert_allclose(d, [0, 0, 1], atol=1e-6)
    ok, d = lens_dir(0.75, 0.5, 3, ())  # quarter turn: +x
    np.testing.assert_allclose(d, [1, 0, 0], atol=1e-6)
    ok, d = lens_dir(0.5, 1.0, 5, ())  # equirectangular bottom row: +y
    np.testing.assert_allclose(d, [0, 1, 0], atol=1e-6)
    for u, v in np.random.default_rng(1).uniform(0, 1, (16, 2)):
        for mode in (3, 5):
            assert abs(np.linalg.norm(lens_dir(float(u), float(v), mode, ())[1]) - 1) < 1e-5
    # F-Theta beyond its field of view yields no ray
    ok, _ = lens_dir(0.9, 0.9, 2, (0.0, 0.06, 0.0, 0.0, 0.0, 64, 48))  # alpha = 1.92 rad
    assert not ok
    ok, d = lens_dir(0.6, 0.5, 2, (0.0, 0.06, 0.0, 0.0, 0.0, 64, 48))  # 6.4 px off-axis: alpha = 0.384 rad
    assert ok and abs(np.linalg.norm(d) - 1) < 1e-6 and abs(d[2] - np.cos(0.384)) < 1e-5
