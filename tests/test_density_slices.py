"""CPU side of compute_and_save_png_slices (src/testbed.cu:534-559, src/marching_cubes.cu:957-1020): the oracle's
mosaic against a numpy restatement, and the two mosaics the reference ships (data/nerf/test.density_slices_256x256x256.png,
data/nerf/test2/images.density_slices_256x256x256.png, held byte for byte under tests/golden/ref_density_slices/)."""
import hashlib

import numpy as np
import pytest

import density_slices_util as D
from oracle_abi import density_slices_mosaic


def np_mosaic(d, thresh=2.5, swap=False, density_range=4.0):
    """save_density_grid_to_png restated with numpy (float32 arithmetic as the C++): the slices of a [z][y][x] grid
    (y slices, unflipped, with swap_y_z; z slices with rows flipped otherwise) tiled floor(sqrt(n)) rows down."""
    vol = d.transpose(1, 0, 2) if swap else d[:, ::-1, :]
    T, R, X = vol.shape
    ndown = int(np.sqrt(np.float32(T)))
    nacross = (T + ndown - 1) // ndown
    scale = np.float32(128.0) / np.float32(density_range)
    b = (vol.astype(np.float32) - np.float32(thresh)) * scale + np.float32(128.5)
    b = np.clip(b, np.float32(0), np.float32(255)).astype(np.uint8)
    out = np.zeros((R * ndown, X * nacross), np.uint8)
    for t in range(T):
        out[(t // nacross) * R:(t // nacross + 1) * R, (t % nacross) * X:(t % nacross + 1) * X] = b[t]
    return out


def np_counts(d, thresh):
    below = d < thresh
    Z, Y, X = d.shape
    c = np.zeros((Z - 2, Y - 2, X - 2), np.int32)
    for dz in (0, 1):
        for dy in (0, 1):
            for dx in (0, 1):
                c += below[1 + dz:Z - 1 + dz, 1 + dy:Y - 1 + dy, 1 + dx:X - 1 + dx]
    me = below[1:-1, 1:-1, 1:-1]
    diff = np.zeros_like(me)
    for sl in ((slice(2, None), slice(1, -1), slice(1, -1)), (slice(0, -2), slice(1, -1), slice(1, -1)),
               (slice(1, -1), slice(2, None), slice(1, -1)), (slice(1, -1), slice(0, -2), slice(1, -1)),
               (slice(1, -1), slice(1, -1), slice(2, None)), (slice(1, -1), slice(1, -1), slice(0, -2))):
        diff |= below[sl] != me
    return int(((c > 0) & (c < 8)).sum()), int(diff.sum())


@pytest.mark.parametrize("shape,swap", [((16, 16, 16), False), ((48, 32, 64), False), ((48, 32, 64), True),
                                        ((20, 12, 8), False), ((7, 5, 3), True)])
def test_oracle_mosaic_matches_numpy_restatement(shape, swap):
    rng = np.random.default_rng(sum(shape))
    d = rng.normal(2.5, 3.0, shape).astype(np.float32)
    d[rng.random(shape) < 0.2] = -10000.0
    for thresh, rng_ in ((2.5, 4.0), (0.0, 1.0)):
        m, counts = density_slices_mosaic(d, thresh, swap, rng_)
        np.testing.assert_array_equal(m, np_mosaic(d, thresh, swap, rng_))
        assert counts == np_counts(d, thresh)


@pytest.mark.parametrize("scene", sorted(D.REFERENCE_SHA256))  # the two shipped mosaics (test2_half shares test2's)
def test_reference_mosaics_are_the_shipped_files_and_round_trip(scene):
    """The fixtures are the reference's files (sha256); each is a 16 x 16 mosaic of 256 slices of 256^2; a volume
    whose bytes map back to the same bytes re-encodes to the identical mosaic (the layout inverse is exact)."""
    path = D.SCENES[scene][1]
    assert hashlib.sha256(open(path, "rb").read()).hexdigest() == D.REFERENCE_SHA256[scene]
    mosaic = D.read_png_gray(path)
    assert mosaic.shape == (4096, 4096)
    vol = D.reference_volume(scene)
    # byte b <- raw density 2.5 + (b - 128) / 32 (the middle of the byte's interval), -10000 for 0
    raw = np.where(vol == 0, np.float32(-10000), np.float32(2.5) + (vol.astype(np.float32) - 128) / 32).astype(np.float32)
    again, _ = density_slices_mosaic(raw)
    np.testing.assert_array_equal(again, mosaic)
    st = D.volume_stats(vol)
    assert 0.01 < st["occupied"] < 0.2 and st["nonzero"] > st["occupied"]


def test_compare_statistics_basics():
    rng = np.random.default_rng(0)
    a = (rng.random((32, 32, 32)) < 0.1).astype(np.uint8) * 200
    a[:, :, -1] = 0
    assert D.compare(a, a) == {"iou": 1.0, "iou_1voxel": 1.0, "iou_nonzero": 1.0, "mean_abs_byte_diff": 0.0}
    b = np.zeros_like(a)
    b[:, :, 1:] = a[:, :, :-1]  # one voxel off: exact IoU drops, the tolerant one stays 1
    m = D.compare(a, b)
    assert m["iou"] < 0.2 and m["iou_1voxel"] == 1.0
