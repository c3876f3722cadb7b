"""HIP kernels vs the scalar oracle, through the C-ABI (needs an MI355X).

Tolerances: hash indices and trilinear weights bit-exact; hash features
bit-exact (both accumulate with fmaf in corner order); MLP outputs within a
few fp16 ulps (MFMA sums 32 products per instruction in its own order, the
oracle sums sequentially); gradients within 1e-2 relative of the gradient norm.
"""
import numpy as np
import pytest

import ngp_abi as A
from oracle_abi import Oracle

pytestmark = pytest.mark.gpu

CONFIGS = {
    "B_L16F2T19": dict(n_levels=16, F=2, log2_T=19, n_neurons=64),
    "base_L8F4T19": dict(n_levels=8, F=4, log2_T=19, n_neurons=64),
    "A_L4F2T14": dict(n_levels=4, F=2, log2_T=14, n_neurons=16),
    "E_L16F2T22": dict(n_levels=16, F=2, log2_T=22, n_neurons=64, aabb_scale=64),
}


def make(name, seed=0, grid_scale=0.5):
    from gpu_util import GpuModel, random_params
    cfg = A.default_config(**CONFIGS[name])
    g = GpuModel(cfg)
    o = Oracle(cfg)
    rng = np.random.default_rng(seed)
    p = random_params(g.n_params, g.n_mlp, g.info, rng, grid_scale)
    g.set_params(p)
    o.set_params(p)
    return g, o, rng


def random_coords(rng, n):
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0, 1, (n, 3))
    c[:, 3] = rng.uniform(0, 0.05, n)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    c[:, 4:7] = (d + 1) * 0.5
    return c


@pytest.mark.parametrize("name", list(CONFIGS))
def test_hashgrid_indices_and_features_bit_exact(name):
    g, o, rng = make(name)
    try:
        pos = rng.uniform(0, 1, (4096, 3)).astype(np.float32)
        pos[:8] = [[0, 0, 0], [1, 1, 1], [0.5, 0.5, 0.5], [1, 0, 1], [0.999999, 1e-7, 0.5], [0.25, 0.75, 0.125],
                   [0.0625, 0.0625, 0.0625], [1 / 3, 2 / 3, 1 / 7]]
        gi, gw = g.encode_indices(pos)
        oi, ow = o.encode_indices(pos)
        np.testing.assert_array_equal(gi, oi)
        np.testing.assert_array_equal(gw, ow)
        ge = g.encode(pos).astype(np.float32)
        oe = o.encode(pos)
        np.testing.assert_array_equal(ge, oe)
        if CONFIGS[name]["n_levels"] % 4 == 0 and CONFIGS[name]["F"] == 2:
            # both XCD chunk mappings (ngp_tuning.encode_xcd_regions) and plain / non-temporal stores, also on a
            # count that is not a multiple of 8 chunks of 256
            for kw in (dict(encode_xcd_regions=1), dict(encode_xcd_regions=0, encode_streaming=1), dict(encode_streaming=0)):
                g.set_tuning(**kw)
                np.testing.assert_array_equal(g.encode(pos).astype(np.float32), oe, err_msg=str(kw))
                np.testing.assert_array_equal(g.encode(pos[:3001]).astype(np.float32), oe[:, :3001], err_msg=str(kw))
    finally:
        g.close()


@pytest.mark.parametrize("name", ["B_L16F2T19", "base_L8F4T19", "A_L4F2T14"])
def test_infer_matches_oracle(name):
    g, o, rng = make(name)
    try:
        coords = random_coords(rng, 3000)
        go = g.infer(coords)
        oo = o.infer(coords)
        assert np.isfinite(go).all()
        err = np.abs(go - oo)
        tol = 4e-3 + 8e-3 * np.abs(oo)
        assert (err <= tol).mean() > 0.999, f"max err {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
        assert np.abs(go - oo).mean() < 1e-3
    finally:
        g.close()


@pytest.mark.parametrize("name", ["B_L16F2T19", "A_L4F2T14"])
def test_infer_sh_rows_matches_oracle_under_every_render_mlp_tuning(name):
    """ngp_model_infer_sh_rows -- the renderer's network call (src/testbed_nerf.cu:1720) on given encodings with the
    degree-4 SH of each ray's direction precomputed once per ray (k_mlp_infer_sh / k_mlp_infer_rf's SH-row path) --
    against the oracle's NerfNetwork::inference of the same samples; the output is bit-identical across the render-MLP
    load pipelines (round 5's ring and the decoupled one), wave steps and workgroup counts, and a sample count that
    is not a multiple of any tile (past-the-end tiles read through an empty descriptor) leaves the rows after it
    untouched."""
    import torch
    from gpu_util import dev, stream, vp
    g, o, rng = make(name)
    try:
        n, per_ray = 5001, 7
        rays = (n + per_ray - 1) // per_ray
        d = rng.normal(size=(rays, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        wd = ((d + 1) * 0.5).astype(np.float32)
        coords = random_coords(rng, n)
        coords[:, 4:7] = wd[np.arange(n) // per_ray]
        enc = o.encode(coords[:, :3]).astype(np.float16)  # [L][n][F]
        oo = o.infer(coords)
        # the rows: the device's own SH of each direction (one ngp_model_infer_sh_rows input per ray)
        x, y, z = (2 * wd[:, 0] - 1), (2 * wd[:, 1] - 1), (2 * wd[:, 2] - 1)
        sh = np.stack([np.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
                       -0.48860251190291987 * x, 1.0925484305920792 * x * y, -1.0925484305920792 * y * z,
                       0.94617469575755997 * z * z - 0.31539156525251999, -1.0925484305920792 * x * z,
                       0.54627421529603959 * (x * x - y * y), 0.59004358992664352 * y * (-3 * x * x + y * y),
                       2.8906114426405538 * x * y * z, 0.45704579946446572 * y * (1 - 5 * z * z),
                       0.3731763325901154 * z * (5 * z * z - 3), 0.45704579946446572 * x * (1 - 5 * z * z),
                       1.4453057213202769 * z * (x * x - y * y), 0.59004358992664352 * x * (-x * x + 3 * y * y)],
                      1).astype(np.float16)
        e, r, ri = dev(enc.view(np.int16)), dev(sh.view(np.int16)), dev((np.arange(n) // per_ray).astype(np.int32))
        outs = {}
        for pipe, tile, wg in ((0, 0, 0), (1, 4, 0), (2, 4, 0), (2, 4, 2), (2, 2, 0), (2, 1, 0), (3, 4, 0), (3, 2, 4)):
            g.set_tuning(render_mlp_pipeline=pipe, render_mlp_tile=tile, mlp_workgroups_per_cu=wg)
            out = torch.full(((n + 64) * 4,), -7.0, dtype=torch.float16, device="cuda")
            A.check(g.lib.ngp_model_infer_sh_rows(g.h, vp(e), vp(r), vp(ri), n, rays, vp(out), 0, stream()))
            torch.cuda.synchronize()
            h = out.float().cpu().numpy().reshape(n + 64, 4)
            assert np.all(h[n:] == -7.0), (pipe, tile, wg)  # nothing written past the n samples
            outs[(pipe, tile, wg)] = h[:n]
        first = next(iter(outs.values()))
        for k, v in outs.items():
            np.testing.assert_array_equal(v, first, err_msg=str(k))
        err = np.abs(first - oo)
        tol = 4e-3 + 8e-3 * np.abs(oo)
        assert (err <= tol).mean() > 0.999, f"max err {err.max()}"
        assert err.mean() < 1e-3
    finally:
        g.close()


@pytest.mark.parametrize("layout_rm", [0, 1])
@pytest.mark.parametrize("name", ["B_L16F2T19", "A_L4F2T14"])
def test_infer_padded_output_matches_oracle(name, layout_rm):
    """The reference's 16-row padded network output (padded_output_width(), row 3 = density via
    extract_density, nerf_network.h:32-43,132-138), column-major as training reads it
    (src/testbed_nerf.cu:2801) and row-major as the renderer does (:1720), with a row stride
    larger than the minimum; rows 0-3 equal the compact output bit for bit."""
    g, o, rng = make(name)
    try:
        coords = random_coords(rng, 2500)
        gp = g.infer_padded(coords, layout_rm, pad=7)
        op = o.infer_padded(coords)
        assert np.isfinite(gp).all()
        err = np.abs(gp - op)
        tol = 4e-3 + 8e-3 * np.abs(op)
        assert (err <= tol).mean() > 0.999, f"max err {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
        np.testing.assert_array_equal(gp[:, :4], g.infer(coords))
        # the 16-row rgb output tile is the rgb network's real output, not padding
        assert np.abs(op[:, 4:]).max() > 0
    finally:
        g.close()


def make_extra(n_extra, seed=3):
    from gpu_util import GpuModel, random_params
    cfg = A.default_config(**CONFIGS["B_L16F2T19"], n_extra_dims=n_extra)
    g = GpuModel(cfg)
    o = Oracle(cfg)
    rng = np.random.default_rng(seed)
    p = random_params(g.n_params, g.n_mlp, g.info, rng, 0.5)
    g.set_params(p)
    o.set_params(p)
    return g, o, rng


@pytest.mark.parametrize("n_extra", [16, 3, 19, 32])
def test_extra_dims_infer_matches_oracle(n_extra):
    """NerfNetwork with n_extra_dims (nerf_network.h:81-93): the records' extra dims (floats 7 .. 7 + E, the latent
    code) enter the rgb network after the SH (rgb input next_multiple(32 + E, 16) = 48 or 64 wide; 19 = light
    direction + the 16-wide code of optimize_extra_dims, src/testbed.cu:4046-4053); against the oracle, and a zero
    code differs from a random one only in the rgb outputs."""
    g, o, rng = make_extra(n_extra)
    try:
        assert g.info.layer_in[2] == (48 if n_extra <= 16 else 64)
        n = 3000
        coords = np.zeros((n, 7 + n_extra), np.float32)
        coords[:, :7] = random_coords(rng, n)
        coords[:, 7:] = rng.normal(0, 1, (n, n_extra))
        go = g.infer(coords)
        oo = o.infer(coords)
        err = np.abs(go - oo)
        tol = 4e-3 + 8e-3 * np.abs(oo)
        assert (err <= tol).mean() > 0.999, f"max err {err.max()}"
        assert err.mean() < 1e-3
        zero = coords.copy()
        zero[:, 7:] = 0
        gz = g.infer(zero)
        np.testing.assert_array_equal(gz[:, 3], go[:, 3])  # density does not see the code
        assert np.abs(gz[:, :3] - go[:, :3]).mean() > 1e-3
        gp = g.infer_padded(coords, 1)
        np.testing.assert_array_equal(gp[:, :4], go)
        with pytest.raises(RuntimeError, match="floats_per_coord"):
            g.infer(coords[:, :7])
    finally:
        g.close()


@pytest.mark.parametrize("n_extra", [16, 19, 32])
def test_extra_dims_mlp_backward_matches_oracle(n_extra):
    """The fused training MLP with the latent-code rows (Net XE 1: 48-row rgb input, XE 2: 64 rows; the images' code
    segment last): weight gradients (incl. the rgb first layer's code columns) and dL/denc against the oracle, and
    dL/d(code) of each sample's own row (the input gradient compute_extra_dims_gradient_train_nerf sums)."""
    g, o, rng = make_extra(n_extra)
    try:
        n = 1000
        coords = random_coords(rng, n)
        enc = o.encode(coords[:, :3])
        extra = rng.normal(0, 1, (n, n_extra)).astype(np.float32)
        dl = (rng.normal(0, 1e-2, (n, 4))).astype(np.float16).astype(np.float32)
        w = rng.uniform(1, 2, n).astype(np.float32)
        g.zero_grads()
        gd, gx = g.backward_extra(enc, coords[:, 4:7], extra, dl, w)
        od, ox = o.backward_extra(enc, coords[:, 4:7], extra, dl, w)
        gg = g.get(A.GRADS_FP32)[: g.n_mlp]
        og = o.get(A.GRADS_FP32)[: o.n_mlp]
        rel = np.linalg.norm(gg - og) / np.linalg.norm(og)
        assert rel < 1e-2, rel
        # the rgb first layer's code columns (32 .. 32 + E of its 48 / 64) carry gradient, every one of them
        off, lin = g.info.layer_param_offset[2], g.info.layer_in[2]
        wcode = gg[off:off + 64 * lin].reshape(64, lin)[:, 32:32 + n_extra]
        assert np.abs(wcode).max(axis=0).min() > 0
        dr = np.linalg.norm(gd - od) / max(np.linalg.norm(od), 1e-12)
        assert dr < 1e-2, dr
        xr = np.linalg.norm(gx - ox) / max(np.linalg.norm(ox), 1e-12)
        assert np.abs(ox).max() > 0 and xr < 1e-2, xr
        # the tiny network has no latent-code instance; n_extra_dims > 32 is refused
        from gpu_util import GpuModel
        cfg = A.default_config(**CONFIGS["A_L4F2T14"], n_extra_dims=4)
        with pytest.raises(RuntimeError, match="n_extra_dims"):
            GpuModel(cfg)
        cfg = A.default_config(**CONFIGS["B_L16F2T19"], n_extra_dims=33)
        with pytest.raises(RuntimeError, match="n_extra_dims"):
            GpuModel(cfg)
    finally:
        g.close()


@pytest.mark.parametrize("name", ["B_L16F2T19", "A_L4F2T14"])
def test_density_matches_oracle_and_infer(name):
    g, o, rng = make(name)
    try:
        coords = random_coords(rng, 2000)
        gd = g.density(coords[:, :3])
        od = o.density(coords[:, :3])
        np.testing.assert_allclose(gd, od, atol=4e-3, rtol=8e-3)
        # density head of the full network equals NerfNetwork::density
        gi = g.infer(coords)
        np.testing.assert_array_equal(gi[:, 3], gd)
    finally:
        g.close()


@pytest.mark.parametrize("name", ["B_L16F2T19", "A_L4F2T14", "E_L16F2T22"])
def test_mlp_backward_matches_oracle(name):
    """The fused training MLP (8 waves, wave-shared weight gradients) against the oracle's NerfNetwork
    backward (nerf_network.h:189-268)."""
    g, o, rng = make(name)
    try:
        n = 1000
        coords = random_coords(rng, n)
        enc = o.encode(coords[:, :3])  # fp16 values
        dl = (rng.normal(0, 1e-2, (n, 4))).astype(np.float16).astype(np.float32)
        w = rng.uniform(1, 2, n).astype(np.float32)
        g.zero_grads()
        gd = g.backward(enc, coords[:, 4:7], dl, w)
        od = o.backward(enc, coords[:, 4:7], dl, w)
        gg = g.get(A.GRADS_FP32)[: g.n_mlp]
        og = o.get(A.GRADS_FP32)[: o.n_mlp]
        rel = np.linalg.norm(gg - og) / np.linalg.norm(og)
        assert rel < 1e-2, rel
        dr = np.linalg.norm(gd - od) / max(np.linalg.norm(od), 1e-12)
        assert dr < 1e-2, dr
    finally:
        g.close()


@pytest.mark.parametrize("name", ["B_L16F2T19", "base_L8F4T19"])
def test_mlp_backward_deterministic_at_batch_size(name):
    """At a full 2^18 batch (+ a ragged tail: every workgroup runs many persistent chunks and the last
    chunk is partial) the weight gradients -- per-workgroup partials summed by k_mlp_reduce in a fixed
    order -- and the input gradients are bit-identical from run to run."""
    g, o, rng = make(name)
    try:
        n = (1 << 18) + 77
        coords = random_coords(rng, n)
        enc = g.encode(coords[:, :3])
        dl = (rng.normal(0, 1e-2, (n, 4))).astype(np.float16).astype(np.float32)
        w = rng.uniform(1, 2, n).astype(np.float32)
        out = []
        for _ in range(2):
            g.zero_grads()
            gd = g.backward(enc, coords[:, 4:7], dl, w)
            out.append((g.get(A.GRADS_FP32)[: g.n_mlp].copy(), gd.copy()))
        (g1, d1), (g2, d2) = out
        assert np.abs(g1).max() > 0
        np.testing.assert_array_equal(g1, g2)
        np.testing.assert_array_equal(d1, d2)
    finally:
        g.close()


@pytest.mark.parametrize("name", ["B_L16F2T19", "base_L8F4T19", "E_L16F2T22"])
def test_hashgrid_backward_matches_oracle(name):
    """Hash-grid backward (tcnn GridEncoding backward: packed half2 atomics of run-merged corner contributions)
    against the oracle's fp32 sums.  Half the samples lie on short ray segments, so coarse levels see long runs
    of the same corner (the contention case); a second call adds into the first."""
    g, o, rng = make(name)
    try:
        n = 6000
        pos = rng.uniform(0, 1, (n, 3)).astype(np.float32)
        # rays: 60 segments of 50 consecutive points, 1/1024 apart
        o0 = rng.uniform(0.2, 0.8, (60, 3))
        d0 = rng.normal(size=(60, 3))
        d0 /= np.linalg.norm(d0, axis=1, keepdims=True)
        t = np.arange(50) / 1024.0
        pos[: 3000] = (o0[:, None, :] + t[None, :, None] * d0[:, None, :]).reshape(-1, 3).astype(np.float32)
        denc = rng.normal(0, 1, (g.L, n, g.F)).astype(np.float16)
        denc[:, 100:200] = 0  # samples with no gradient (skipped)
        g.zero_grads()
        g.encode_backward(pos, denc)
        o.encode_backward(pos, denc.astype(np.float32))
        gg = g.grads()[g.n_mlp:]
        og = o.get(A.GRADS_FP32)[o.n_mlp:]
        # fp16 gradients: the atomics round the running sum to half at each add
        assert np.linalg.norm(gg - og) / np.linalg.norm(og) < 2e-3
        big = np.abs(og) > 1e-2
        close = np.abs(gg[big] - og[big]) <= 5e-2 * np.abs(og[big])
        assert close.mean() > 0.999, (close.mean(), np.abs(gg - og).max())
        assert ((gg != 0) == (og != 0)).mean() > 0.9999
        g.encode_backward(pos, denc)
        g2 = g.grads()[g.n_mlp:]
        assert np.linalg.norm(g2 - 2 * og) / np.linalg.norm(2 * og) < 3e-3
    finally:
        g.close()
