"""The ExponentialDecay learning-rate schedule shared by the network optimizer, the distortion
map and the camera updates (ngp_math.h exp_decay_learning_rate; configs/nerf/base.json:9-14).

PARITY UNPINNED: tcnn's ExponentialDecay source is not in the reference mount,
so these values pin the restated spec -- the first decay applies at decay_start, one more every
decay_interval steps, none at or after decay_end -- and make any later correction visible."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def ngp():
    import pyngp
    return pyngp


def test_schedule_boundaries(ngp):
    lr = lambda step: ngp.exponential_decay_learning_rate(1e-2, 0.33, 20000, 10000, 45000, step)
    f = np.float32
    assert lr(0) == f(1e-2)
    assert lr(19999) == f(1e-2)                       # decay_start - 1: undecayed
    assert lr(20000) == pytest.approx(1e-2 * 0.33, rel=1e-6)   # first decay at decay_start
    assert lr(29999) == lr(20000)
    assert lr(30000) == pytest.approx(1e-2 * 0.33 ** 2, rel=1e-6)  # decay_start + interval
    assert lr(40000) == pytest.approx(1e-2 * 0.33 ** 3, rel=1e-6)
    # decay_end: the last decay is the one below decay_end; none at or after it
    assert lr(44999) == lr(40000) == lr(45000) == lr(10 ** 6)


def test_schedule_without_end_or_interval(ngp):
    # the network optimizer (base.json has no decay_end)
    lr = lambda step: ngp.exponential_decay_learning_rate(1e-2, 0.33, 20000, 10000, 2 ** 32 - 1, step)
    assert lr(35000) == pytest.approx(1e-2 * 0.33 ** 2, rel=1e-6)
    assert lr(10 ** 6) == pytest.approx(1e-2 * 0.33 ** 99, rel=1e-5)
    # interval 0 = no decay; distortion map defaults (testbed.h: start 10000, interval 5000, end 25000)
    assert ngp.exponential_decay_learning_rate(1e-4, 0.33, 0, 0, 100, 50) == np.float32(1e-4)
    d = lambda step: ngp.exponential_decay_learning_rate(1e-4, 0.33, 10000, 5000, 25000, step)
    assert d(9999) == np.float32(1e-4) and d(24999) == d(30000) == pytest.approx(1e-4 * 0.33 ** 3, rel=1e-6)
