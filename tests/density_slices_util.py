"""Density-slice mosaics (Testbed.compute_and_save_png_slices, src/testbed.cu:534-559 and
src/marching_cubes.cu:957-1020) and their comparison with the two mosaics the reference's CUDA build wrote from
models trained on the fork's own scenes (test infrastructure: tests/ and tools/ only).

A mosaic byte is clamp((raw density - 2.5) * 32 + 128.5): >= 129 means a raw density output >= 2.5 (sigma >= e^2.5,
the marching-cubes threshold), 0 means raw <= -1.5 or a cell the occupancy grid marks empty (-10000).
"""
import os
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "ref_density_slices")

# scene -> (training transforms, the reference's mosaic).  The reference trained at full resolution on every
# frame; these are data/nerf copies at half (test, test2_half), quarter (test2) and full (test2_full) resolution
# (tools/make_real_data.py).
SCENES = {
    "test": (os.path.join(ROOT, "data", "nerf", "test", "dataset", "transforms_all.json"), os.path.join(GOLDEN, "test.png")),
    "test2": (os.path.join(ROOT, "data", "nerf", "test2", "images", "transforms_train.json"), os.path.join(GOLDEN, "test2.png")),
    # the same 300 views at half resolution (360x640; the reference trained at 720x1280)
    "test2_half": (os.path.join(ROOT, "data", "nerf", "test2_half", "images", "transforms_train.json"),
                   os.path.join(GOLDEN, "test2.png")),
    # ... and at the reference's own training resolution (720x1280, lossless RGB)
    "test2_full": (os.path.join(ROOT, "data", "nerf", "test2_full", "images", "transforms_train.json"),
                   os.path.join(GOLDEN, "test2.png")),
}
# sha256 of the reference's files (data/nerf/test.density_slices_256x256x256.png,
# data/nerf/test2/images.density_slices_256x256x256.png), checked by tests/test_density_slices.py
REFERENCE_SHA256 = {
    "test": "cf8568b5c1e98a91eaed7209a30275eb6f399189bd7cf8a48bcc31667aa006a7",
    "test2": "acae4d4cce12bbe7f92db6d45f6a38f734f7af85acd7fcaa0707749394762448",
}


def read_png_gray(path):
    from PIL import Image
    im = Image.open(path)
    assert im.mode == "L", (path, im.mode)
    return np.array(im)


def mosaic_to_volume(mosaic, res=(256, 256, 256)):
    """Inverse of the unswapped mosaic layout: tile z at column z % nacross, row z // nacross, rows flipped."""
    X, Y, Z = res
    ndown = int(np.sqrt(np.float32(Z)))
    nacross = (Z + ndown - 1) // ndown
    assert mosaic.shape == (Y * ndown, X * nacross), mosaic.shape
    vol = np.zeros((Z, Y, X), np.uint8)
    for z in range(Z):
        tile = mosaic[(z // nacross) * Y:(z // nacross + 1) * Y, (z % nacross) * X:(z % nacross + 1) * X]
        vol[z] = tile[::-1]
    return vol


def reference_volume(scene):
    return mosaic_to_volume(read_png_gray(SCENES[scene][1]))


def volume_stats(vol):
    return {"occupied": float((vol >= 129).mean()), "nonzero": float((vol > 0).mean())}


def _iou(a, b):
    u = np.logical_or(a, b).sum()
    return float(np.logical_and(a, b).sum() / u) if u else 1.0


def compare(a, b):
    """Statistics of two [z][y][x] uint8 mosaic volumes: IoU of the >= 129 masks (raw density >= 2.5), the same
    with one voxel of tolerance (a voxel counts as matched when the other mask has one within its 3^3
    neighbourhood: (matched a + matched b) / (|a| + |b|)), IoU of the non-zero masks and the mean |byte
    difference| over their union."""
    from scipy.ndimage import binary_dilation
    ma, mb = a >= 129, b >= 129
    st = np.ones((3, 3, 3), bool)
    da, db = binary_dilation(ma, st), binary_dilation(mb, st)
    n = ma.sum() + mb.sum()
    tol = float((np.logical_and(ma, db).sum() + np.logical_and(mb, da).sum()) / n) if n else 1.0
    nza, nzb = a > 0, b > 0
    u = np.logical_or(nza, nzb)
    mad = float(np.abs(a.astype(np.int16) - b.astype(np.int16))[u].mean()) if u.any() else 0.0
    return {"iou": _iou(ma, mb), "iou_1voxel": tol, "iou_nonzero": _iou(nza, nzb), "mean_abs_byte_diff": mad}


def new_testbed(ngp, scene, config="base.json", seed=1337, random_bg_color=True):
    tb = ngp.Testbed()
    tb.seed = seed
    tb.load_training_data(SCENES[scene][0])
    tb.reload_network_from_file(config)
    tb.nerf.training.random_bg_color = random_bg_color
    tb.shall_train = True
    return tb


def preview(vol, zs=range(16, 256, 32), step=2):
    """A strip of slices z in zs (every `step`-th pixel), rows flipped as in the mosaic: for looking at fields."""
    return np.concatenate([vol[z, ::-1][::step, ::step] for z in zs], axis=1)


def train_to(tb, steps):
    while tb.training_step < steps:
        tb.frame()


def testbed_volume(tb, save_prefix=None, resolution=256):
    """compute_and_save_png_slices at its defaults (the render aabb, thresh 2.5, range 4), read back."""
    if save_prefix:
        os.makedirs(os.path.dirname(os.path.abspath(save_prefix)), exist_ok=True)
        res = tb.compute_and_save_png_slices(save_prefix, resolution)
        path = save_prefix + ".density_slices_{}x{}x{}.png".format(*res)
        return mosaic_to_volume(read_png_gray(path), tuple(int(r) for r in res))
    with tempfile.TemporaryDirectory() as d:
        return testbed_volume(tb, os.path.join(d, "field"), resolution)


def coarse(mask, block=8):
    """Fraction of set voxels per block^3 block of a cubic mask."""
    n = mask.shape[0] // block
    return mask.astype(np.float32).reshape(n, block, n, block, n, block).mean((1, 3, 5))


def orientation_ranking(ours, ref):
    """Correlation of two coarse occupancy grids under each of the 48 axis permutations / flips of `ref`; returns
    (correlation at the identity, its rank among the 48: 0 = best)."""
    import itertools
    cs = []
    ident = None
    for perm in itertools.permutations(range(3)):
        for flips in itertools.product((0, 1), repeat=3):
            r = ref.transpose(perm)
            for ax, f in enumerate(flips):
                if f:
                    r = np.flip(r, ax)
            c = float(np.corrcoef(r.ravel(), ours.ravel())[0, 1])
            cs.append(c)
            if perm == (0, 1, 2) and flips == (0, 0, 0):
                ident = c
    return ident, sorted(cs, reverse=True).index(ident)
