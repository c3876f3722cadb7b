"""The stepping lattice against a literal transcription of the reference's sampling loop
(generate_training_samples_nerf, src/testbed_nerf.cu:779-795: t += calc_dt(t) on a sample,
t = advance_to_next_voxel(t, ...) past an empty cell at mip_from_dt; nerf_device.cuh:378-453),
on the CPU oracle.  The fast paths (HIP sampler and oracle) define a sample as lattice point
n0 + k of stepping space and reproduce the reference's jumps on the lattice; the literal loop
chains floats.  Both must visit the same lattice points: for every ray the literal loop's
samples, mapped back to stepping space, round to exactly the fast path's lattice points.
Cascaded scenes (aabb_scale 16, cone angle 1/256) exercise mip_from_dt and the jumps; aabb 1
the uniform-step case."""
import numpy as np
import pytest

import ngp_abi as A
from oracle_abi import Oracle
from scene_util import HostDataset, make_views, train_args

CELLS = 128 ** 3


def _oracle_with_grid(max_cascade, density, seed):
    o = Oracle(A.default_config(n_levels=4, F=2, log2_T=14, n_neurons=16))
    rng = np.random.default_rng(seed)
    nc = max_cascade + 1
    grid = np.where(rng.random(CELLS * nc) < density, 1.0, 0.0).astype(np.float32)
    # a solid core in cascade 0 so that rays also run through long occupied stretches
    from scene_util import sphere_bitfield
    grid[:CELLS] = np.maximum(grid[:CELLS], sphere_bitfield(0.18))
    o.grid_set(grid)
    o.grid_bitfield(max_cascade)
    return o


@pytest.mark.parametrize("aabb_scale,density", [(1, 0.003), (16, 0.003), (16, 0.05), (64, 0.01)])
def test_lattice_walk_matches_literal_reference_loop(aabb_scale, density):
    max_cascade = int(np.log2(aabb_scale))
    o = _oracle_with_grid(max_cascade, density, seed=aabb_scale)
    imgs, cams, focal = make_views(6, 24, 24)
    hd = HostDataset(imgs, cams, focal)
    R = 192
    a = train_args(hd.ptr, hd.n, R, 1 << 16, 1 << 20, aabb_scale=aabb_scale)
    total, rays_with_samples, exact = 0, 0, 0
    for i in range(R):
        fast, n0 = o.train_ray_samples(a, i, literal=False)
        lit, _ = o.train_ray_samples(a, i, literal=True)
        k_fast = np.round(fast - n0).astype(np.int64)
        k_lit = np.round(lit - n0).astype(np.int64)
        np.testing.assert_allclose(fast - n0, k_fast, atol=1e-3)  # fast samples sit on the lattice
        total += len(fast)
        rays_with_samples += len(fast) > 0
        exact += np.array_equal(k_fast, k_lit)
        if not np.array_equal(k_fast, k_lit):
            # the chained floats stay within a small fraction of a step of the lattice
            assert abs(len(k_fast) - len(k_lit)) <= 1, (i, len(k_fast), len(k_lit))
    assert rays_with_samples > R // 4 and total > 1000
    assert exact == R, f"{R - exact} of {R} rays differ"
