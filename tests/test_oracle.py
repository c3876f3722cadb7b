"""CPU tests of the scalar oracle against published known answers and the
hash-grid level tables derived in SURVEY.md Appendix A (parity unpinned for the
tcnn-side arithmetic: the reference ships no tests or golden vectors)."""
import json
import os

import numpy as np
import pytest

import ngp_abi as A
from oracle_abi import Oracle, load, ptr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def test_pcg32_known_answer():
    # pcg32-demo (pcg-c-basic) output for pcg32_srandom_r(&rng, 42u, 54u), round 1;
    # tcnn's pcg32 (Jakob) seed(initstate, initseq) is the same generator.
    lib = load()
    out = np.zeros(6, np.uint32)
    lib.oref_pcg32(42, 54, 6, ptr(out))
    assert [hex(x) for x in out] == ["0xa15c02b7", "0x7b47f409", "0xba1d3330", "0x83d2f293", "0xbfa4784b", "0xcbed606e"]


def test_pcg32_advance_matches_stepping():
    lib = load()
    a = np.zeros(40, np.float32)
    lib.oref_pcg32_floats_advanced(0x853c49e6748fea9b, 0xda3e39cb94b95bdb, 0, 40, ptr(a))
    b = np.zeros(8, np.float32)
    lib.oref_pcg32_floats_advanced(0x853c49e6748fea9b, 0xda3e39cb94b95bdb, 32, 8, ptr(b))
    np.testing.assert_array_equal(a[32:40], b)
    assert (a >= 0).all() and (a < 1).all()


def test_sobol_direction_numbers():
    lib = load()
    # dim 0 = van der Corput, dim 1 = random_val.cuh:176-179 direction numbers
    assert [lib.oref_sobol(i, 0) for i in range(1, 5)] == [0x80000000, 0x40000000, 0xC0000000, 0x20000000]
    assert [lib.oref_sobol(i, 1) for i in range(1, 5)] == [0x80000000, 0xC0000000, 0x40000000, 0xA0000000]


def test_scrambled_sobol_is_stratified():
    # Owen scrambling keeps the (0, m, 2)-net property: 2^k points, one per 1/2^k interval per dim
    lib = load()
    for dim in (0, 1):
        v = np.array([lib.oref_ld_random_val(i, 0xdeadbeef, dim) for i in range(256)])
        assert sorted(np.floor(v * 256).astype(int)) == list(range(256))


def test_morton():
    lib = load()
    assert lib.oref_morton3D(1, 0, 0) == 1 and lib.oref_morton3D(0, 1, 0) == 2 and lib.oref_morton3D(0, 0, 1) == 4
    assert lib.oref_morton3D(127, 127, 127) == 128 ** 3 - 1
    # bijective on the 128^3 grid
    s = {lib.oref_morton3D(x, y, z) for x in range(0, 128, 7) for y in range(0, 128, 11) for z in range(0, 128, 13)}
    assert len(s) == len(range(0, 128, 7)) * len(range(0, 128, 11)) * len(range(0, 128, 13))


def test_f16_conversion_matches_numpy():
    lib = load()
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.normal(0, 3, 2000), rng.normal(0, 1e-5, 500), [0.0, -0.0, 65504.0, 70000.0, 6e-8, 1e-9]])
    x = x.astype(np.float32)
    h = np.array([lib.oref_f2h(float(v)) for v in x], np.uint16)
    np.testing.assert_array_equal(h, x.astype(np.float16).view(np.uint16))
    back = np.array([lib.oref_h2f(int(v)) for v in h], np.float32)
    np.testing.assert_array_equal(back, x.astype(np.float16).astype(np.float32))


def test_spherical_harmonics_vs_scipy():
    # tcnn's degree-4 SH basis equals the real SH of scipy up to the Condon-Shortley sign (-1)^m
    from scipy.special import sph_harm_y
    lib = load()
    rng = np.random.default_rng(1)
    for _ in range(20):
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        wd = ((d + 1) * 0.5).astype(np.float32)
        out = np.zeros(16, np.float32)
        lib.oref_sh4(ptr(wd), ptr(out))
        x, y, z = (wd.astype(np.float64) * 2 - 1)
        theta, phi = np.arccos(np.clip(z / np.linalg.norm([x, y, z]), -1, 1)), np.arctan2(y, x)
        ref = []
        for l in range(4):
            for m in range(-l, l + 1):
                if m == 0:
                    v = np.real(sph_harm_y(l, 0, theta, phi))
                elif m > 0:
                    v = np.sqrt(2) * (-1) ** m * np.real(sph_harm_y(l, m, theta, phi))
                else:
                    v = np.sqrt(2) * (-1) ** m * np.imag(sph_harm_y(l, -m, theta, phi))
                ref.append(v * (-1) ** m)
        np.testing.assert_allclose(out, np.array(ref), atol=2e-3, rtol=2e-3)


# SURVEY.md Appendix A / §8 derived sizes (tcnn level formula)
@pytest.mark.parametrize("L,F,T,aabb,entries,dense_res", [
    (16, 2, 19, 1, 6_098_120, [16, 23, 31, 43, 59]),
    (8, 4, 19, 1, 2_920_448, [16, 32, 64]),
    (4, 2, 14, 1, 53_248, [16]),
    (16, 2, 22, 64, 51_461_400, [16, 30, 54, 98]),
])
def test_level_tables(L, F, T, aabb, entries, dense_res):
    cfg = A.default_config(n_levels=L, F=F, log2_T=T, aabb_scale=aabb,
                           n_neurons=16 if T == 14 else 64)
    o = Oracle(cfg)
    s, r, off, size, hashed = o.level_table()
    assert int(size.sum()) == entries
    nd = len(dense_res)
    assert list(r[:nd]) == dense_res and not hashed[:nd].any() and hashed[nd:].all()
    assert r[-1] == (2048 * aabb if T != 22 else 131072) or r[-1] >= 2048
    assert o.n_params == o.n_mlp + entries * F
    assert o.n_mlp == 3072 + 7168 if cfg.n_neurons == 64 else True
