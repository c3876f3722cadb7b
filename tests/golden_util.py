"""Seeded inputs shared by tests/golden/make_golden.py and the golden-fixture tests.

Large inputs (parameter vectors, 128^3 occupancy grids) are regenerated here from the
seeds stored in the fixtures (numpy PCG64 streams are stable across numpy versions),
so the committed .npz files stay small.
"""
import hashlib
import os

import numpy as np

import ngp_abi as A

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
CELLS = 128 ** 3
CFG_A = dict(n_levels=4, F=2, log2_T=14, n_neurons=16)
CFG_B = dict(n_levels=16, F=2, log2_T=19, n_neurons=64)


def seeded_params(n_params, n_mlp, seed, mlp_scale=0.25, grid_scale=0.5):
    rng = np.random.default_rng(seed)
    p = np.empty(n_params, np.float32)
    p[:n_mlp] = rng.uniform(-mlp_scale, mlp_scale, n_mlp)
    p[n_mlp:] = rng.uniform(-grid_scale, grid_scale, n_params - n_mlp)
    return p


def seeded_positions(n, seed):
    return np.random.default_rng(seed).uniform(0, 1, (n, 3)).astype(np.float32)


def seeded_coords(n, seed):
    """NerfCoordinate rows: pos(3), dt(1), warped direction(3)."""
    rng = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0, 1, (n, 3))
    c[:, 3] = rng.uniform(0, 0.05, n)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    c[:, 4:7] = (d + 1) * 0.5
    return c


def seeded_grid(seed):
    rng = np.random.default_rng(seed)
    g = rng.exponential(0.01, CELLS).astype(np.float32)
    g[rng.random(CELLS) < 0.1] = -1.0
    return g


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def sphere_grid(radius=0.32):
    from scene_util import sphere_bitfield
    return sphere_bitfield(radius)


def golden_views():
    """6 views of the synthetic scene at 24x24 (stored in train_A.npz once generated)."""
    path = os.path.join(GOLDEN, "train_A.npz")
    if os.path.exists(path):
        g = np.load(path)
        return g["imgs"], g["cams"], float(g["focal"])
    from scene_util import make_views
    return make_views(6, 24, 24)


def host_dataset(imgs, cams, focal):
    from scene_util import HostDataset
    return HostDataset(imgs, cams, focal)


def golden_train_args(images_ptr, n_images, R, B, MS):
    from scene_util import train_args
    return train_args(images_ptr, n_images, R, B, MS)


def golden_render_args():
    from scene_util import render_args
    import synthetic as S
    W, H = 40, 32
    cam = S.hemisphere_cameras(1, seed=0)[0]
    focal = 0.5 * W / np.tan(0.5 * 0.69)
    return render_args(W, H, cam, focal, spp=0, snap=1, shard=(0, 1, 8))
