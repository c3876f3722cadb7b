"""The render march's stepping lattice against a literal transcription of the reference's tracer
(CPU, oracle): advance_pos_nerf (src/testbed_nerf.cu:333-362) from the payload's t, then
generate_next_nerf_network_inputs passes (:421-469) with t += calc_dt(t) chained through payload.t,
and if_unoccupied_advance_to_next_occupied_voxel with its mip climb (nerf_device.cuh:462-494).

The HIP renderer and the oracle's render() define a sample as lattice point n0 + k of stepping space
(n0 = to_stepping_space(t_entry) + jitter) and cross empty space in verified jumps; the literal march
chains floats.  For every ray the literal march's samples, mapped back to stepping space, round to
exactly the lattice march's points -- except where the ray passes a decision point lying on a cell face
to within float rounding (< 1e-3 of a cell): there the reference's own occupancy lookup (grid_idx) and
jump (distance_to_next_voxel) put the point in different cells, the chained floats and the lattice may
fall on either side, and the samples of that ray can differ past it (< 1 % of the rays; the lattice
march's verified jumps never skip an occupied point, the literal one can).  The pass length (n_steps per
generate pass) does not matter.  Covered: aabb_scale 1, 4 and 64 (1, 3 and 7 cascades), cone angle 0 and 1/256, floaters in
every cascade, a rotated crop box, depth of field.  The GPU suite pins the HIP march to the lattice
march (test_render_*_matches_oracle) and renders against the literal oracle too
(test_render_matches_literal_reference_march)."""
import numpy as np
import pytest

import ngp_abi as A
from oracle_abi import Oracle
from scene_util import make_views, render_args, sphere_bitfield

CELLS = 128 ** 3


def _oracle(max_cascade, density, seed):
    o = Oracle(A.default_config(n_levels=4, F=2, log2_T=14, n_neurons=16))
    rng = np.random.default_rng(seed)
    nc = max_cascade + 1
    grid = np.where(rng.random(CELLS * nc) < density, 1.0, 0.0).astype(np.float32)
    grid[:CELLS] = np.maximum(grid[:CELLS], sphere_bitfield(0.15))  # a solid core: long occupied stretches
    o.grid_set(grid)
    o.grid_bitfield(max_cascade)
    return o


# a lattice point this close to a cell face (in cells of its mip) is a knife edge: the reference's own two
# cell computations -- grid_idx's ((p - 0.5) 2^-mip + 0.5) 128 for the occupancy and distance_to_next_voxel's
# 128 2^-mip (p - 0.5) for the jump -- round it into different cells, and so do the chained floats vs the lattice
KNIFE_EDGE = 1e-3


def _compare(o, ra, W, H, stride=1):
    """Per ray: the lattice march's and the literal march's sample sets on the lattice n0 + k.  Returns
    (rays, rays with identical samples, samples, max off-lattice drift of the literal chain, the largest face
    distance found in a differing ray's divergence window)."""
    rays = exact = total = 0
    max_drift = edge = 0.0
    for y in range(0, H, stride):
        for x in range(0, W, stride):
            lat, n0 = o.render_ray_samples(ra, x, y)
            lit, _, tr = o.render_ray_samples(ra, x, y, literal=True, n_steps=1 + (x + y) % 8, trace=True)
            if len(lat) == 0 and len(lit) == 0:
                continue
            rays += 1
            total += len(lat)
            k_lat = np.round(lat - n0).astype(np.int64)
            k_lit = np.round(lit - n0).astype(np.int64)
            np.testing.assert_allclose(lat - n0, k_lat, atol=2e-3)  # the lattice march sits on the lattice
            if len(lit):
                max_drift = max(max_drift, float(np.abs(lit - n0 - k_lit).max()))
            if np.array_equal(k_lat, k_lit):
                exact += 1
                continue
            # the two marches share every sample before the divergence; the literal march's visited points
            # between the last shared sample and the first differing one include a knife-edge point
            m = min(len(k_lat), len(k_lit))
            i = next((j for j in range(m) if k_lat[j] != k_lit[j]), m)
            lo = k_lat[i - 1] if i > 0 else -(1 << 30)
            hi = min(int(v[i]) for v in (k_lat, k_lit) if i < len(v))
            kt = tr[:, 0] - n0
            window = (kt >= lo - 0.5) & (kt <= hi + 0.5)
            edge = max(edge, float(tr[window, 1].min()) if window.any() else 1.0)
    return rays, exact, total, max_drift, edge


@pytest.mark.parametrize("aabb_scale,density,cone", [(1, 0.003, 0.0), (1, 0.05, 0.0), (4, 0.01, 0.0), (4, 0.01, 1 / 256),
                                                     (64, 0.01, 1 / 256), (64, 0.002, 0.0)],
                         ids=["aabb1-sparse", "aabb1-dense", "aabb4", "aabb4-cone", "aabb64-cone", "aabb64"])
def test_render_lattice_march_matches_literal_reference_march(aabb_scale, density, cone):
    max_cascade = int(np.log2(aabb_scale))
    o = _oracle(max_cascade, density, seed=aabb_scale + int(cone * 1024))
    W, H = 48, 36
    imgs, cams, focal = make_views(3, W, H)
    ra = render_args(W, H, cams[1], focal, spp=1, aabb_scale=aabb_scale)
    ra.cone_angle_constant = cone
    rays, exact, total, drift, edge = _compare(o, ra, W, H)
    assert rays > W * H // 4 and total > 2000, (rays, total)
    # the chained floats stay a fraction of a step off the lattice (aabb 64 at cone 0: ~2e4 chained steps,
    # t ~ 30, drift < 0.1 step), so rounding to the nearest lattice point is unambiguous
    assert drift < 0.25, drift
    # characterised bound: every ray samples exactly the literal march's lattice points, except rays that
    # pass within KNIFE_EDGE of a cell face at a decision point (< 1 % of the rays)
    assert edge < KNIFE_EDGE, edge
    assert rays - exact <= max(1, rays // 100), f"{rays - exact} of {rays} rays differ"


def test_literal_march_does_not_depend_on_the_pass_length():
    """generate_next_nerf_network_inputs carries t in payload.t between passes: 1, 2, 3, 8 or 64 samples
    per pass give the same samples bit for bit."""
    o = _oracle(2, 0.01, seed=11)
    W, H = 24, 18
    imgs, cams, focal = make_views(2, W, H)
    ra = render_args(W, H, cams[0], focal, spp=2, aabb_scale=4)
    ra.cone_angle_constant = 1 / 256
    n = 0
    for y in range(H):
        for x in range(W):
            ref, _ = o.render_ray_samples(ra, x, y, literal=True, n_steps=8)
            n += len(ref)
            for ns in (1, 2, 3, 64):
                got, _ = o.render_ray_samples(ra, x, y, literal=True, n_steps=ns)
                np.testing.assert_array_equal(got, ref)
    assert n > 500


def test_render_lattice_march_matches_literal_with_crop_box_and_depth_of_field():
    """A rotated, shrunk crop box (render_aabb + render_aabb_to_local: the containment test in the box's
    frame, init_rays_with_payload_kernel_nerf:1465-1475) and a lens aperture (uv_to_ray's depth of field)."""
    o = _oracle(0, 0.01, seed=5)
    W, H = 40, 30
    imgs, cams, focal = make_views(3, W, H)
    ra = render_args(W, H, cams[2], focal, spp=3, aabb_scale=1)
    th = 0.4
    R = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]], np.float32)
    for k in range(9):
        ra.render_aabb_to_local[k] = float(R.reshape(-1)[k])
    lo = R @ np.array([0.5, 0.5, 0.5]) - 0.3
    for k in range(3):
        ra.aabb_min[k], ra.aabb_max[k] = float(lo[k]), float(lo[k] + 0.6)
    ra.aperture_size = 0.02
    ra.focus_z = 1.3
    rays, exact, total, drift, edge = _compare(o, ra, W, H)
    assert rays > 100 and total > 500, (rays, total)
    assert edge < KNIFE_EDGE and rays - exact <= max(1, rays // 100), (rays, exact, edge)


def test_oracle_frames_lattice_and_literal_agree():
    """The oracle's frame with the literal march equals its lattice-march frame within the north_star
    tolerance (the sample positions differ by the chained floats' rounding only)."""
    o = Oracle(A.default_config(n_levels=4, F=2, log2_T=14, n_neurons=16))
    rng = np.random.default_rng(3)
    p = np.zeros(o.n_params, np.float32)
    p[: o.n_mlp] = rng.normal(0, 0.3, o.n_mlp)
    p[o.n_mlp:] = rng.uniform(-1.0, 1.0, o.n_params - o.n_mlp)
    o.set_params(p)
    o.set_inference_params(p)
    o.grid_set(sphere_bitfield(0.3))
    o.grid_bitfield(0)
    W, H = 32, 24
    imgs, cams, focal = make_views(2, W, H)
    ra = render_args(W, H, cams[0], focal, spp=1)
    try:
        f_lat, _ = o.render(ra)
        o.set_render_literal(True)
        f_lit, _ = o.render(ra)
    finally:
        o.set_render_literal(False)
    assert f_lat[..., 3].max() > 0.3
    assert np.abs(f_lat - f_lit).mean() < 1e-4
