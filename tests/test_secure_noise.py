"""Secure (granularity-snapped) noise: host parameters, the oracle's
restatement of the samplers, and the host sampler (CPU tests).

The reference adds noise through PyDP's LaplaceMechanism / GaussianMechanism
(dp_computations.py:439-440, 456-457, 489-491, 508-509), i.e. Google's
differential-privacy samplers: the value is rounded to a power-of-two grid
and a grid-valued discrete sample (two-sided geometric / centred binomial) is
added.  PyDP is not installed (parity unpinned for the draws themselves), so
these tests pin the published construction: the grid, the distribution
(KS against the continuous mechanism, p > 1e-4 on 30k samples as
dp_computations_test.py:472-545 does), and that every output is a multiple
of the grid.  GPU bit-exactness against this oracle is in test_gpu_api.py /
test_gpu_kernels.py.
"""
import math

import numpy as np
import pytest
from scipy import stats

from oracle import columnar as O
from oracle import pydp_restatement as pydp
from pipelinedp_amd import dp_computations as dpc


@pytest.mark.parametrize("eps,l1", [(1.0, 1.0), (0.1, 3.0), (1 / 3, 16.0), (5.0, 0.25), (1e5, 1.0)])
def test_laplace_params_match_oracle_restatement(eps, l1):
    got = dpc.laplace_noise_params(eps, l1).as_dict()
    want = pydp.laplace_params(eps, l1)
    assert got == want
    b = l1 / eps
    g = got["granularity"]
    assert math.log2(g).is_integer()
    assert b / 2 ** 40 <= g < 2 * b / 2 ** 40  # next power of two of b / 2^40


@pytest.mark.parametrize("sigma", [1.0, 2.5, 114.375, 1e-3, 5e4])
def test_gaussian_params_match_oracle_restatement(sigma):
    got = dpc.gaussian_noise_params(sigma).as_dict()
    want = pydp.gaussian_params(sigma)
    assert got == want
    sqrt_n = 2 * sigma / got["granularity"]
    assert 2 ** 27.5 <= sqrt_n <= 2 ** 28.5 + 1e-6
    assert got["step"] < 2 ** 32


def test_zero_scale_is_no_noise():
    assert dpc.laplace_noise_params(1.0, 0.0).granularity == 0.0
    assert dpc.gaussian_noise_params(0.0).granularity == 0.0
    x = np.array([1.25, -3.0, 7.0])
    np.testing.assert_array_equal(O.secure_add_noise(pydp.laplace_params(1.0, 0.0), x, 1, np.arange(3), 5), x)


@pytest.mark.parametrize("make", [lambda: dpc.laplace_noise_params(1.0, math.inf),
                                  lambda: dpc.laplace_noise_params(5e-324, 1.0),
                                  lambda: dpc.laplace_noise_params(1.0, math.nan),
                                  lambda: dpc.gaussian_noise_params(math.inf),
                                  lambda: dpc.gaussian_noise_params(math.nan),
                                  lambda: dpc.gaussian_noise_params(-1.0)])
def test_non_finite_scale_fails_closed(make):
    """A scale that is not finite must raise, never become granularity 0
    (which the kernels read as "no noise" and release raw values)."""
    with pytest.raises(ValueError):
        make()


def test_abi_rejects_zero_granularity_with_scale():
    """check_noise (pdp_select.hip) refuses granularity 0 unless the scale is
    exactly 0; runs before any device work, so it needs no GPU."""
    import ctypes
    from pipelinedp_amd import _native as N
    lib = N.lib()
    bad = dpc.NoiseParams(kind=0, scale=2.0, granularity=0.0).to_c()
    rc = lib.pdp_add_noise(None, N.VALUE_F64, 0, ctypes.byref(bad), 1, 0, None, None)
    assert rc == -1 and b"granularity 0" in lib.pdp_last_error()
    inf = dpc.NoiseParams(kind=1, scale=math.inf, granularity=0.0).to_c()
    assert lib.pdp_add_noise(None, N.VALUE_F64, 0, ctypes.byref(inf), 1, 0, None, None) == -1
    ok = dpc.NoiseParams(kind=0, scale=0.0, granularity=0.0).to_c()
    assert lib.pdp_add_noise(None, N.VALUE_F64, 0, ctypes.byref(ok), 1, 0, None, None) == 0


def test_round_to_multiple_ties_toward_zero():
    g = 0.5
    xs = np.array([0.25, -0.25, 0.26, -0.26, 1.0, 0.74, 0.75, -0.75])
    got = O.round_to_multiple(xs, g)
    np.testing.assert_array_equal(got, [0.0, 0.0, 0.5, -0.5, 1.0, 0.5, 0.5, -0.5])
    assert [dpc.round_to_multiple(float(x), g) for x in xs] == got.tolist()


def _ks(samples, cdf):
    return stats.kstest(samples, cdf).pvalue


@pytest.mark.parametrize("eps,l1", [(1.0, 1.0), (0.5, 4.0)])
def test_oracle_laplace_distribution_and_grid(eps, l1):
    p = pydp.laplace_params(eps, l1)
    x = np.full(30000, 3.0)
    y = O.secure_add_noise(p, x, 12345, np.arange(30000), 7)
    assert np.all(np.fmod(y, p["granularity"]) == 0.0)
    assert _ks(y - 3.0, stats.laplace(scale=l1 / eps).cdf) > 1e-4


@pytest.mark.parametrize("sigma", [1.0, 17.1826171875])
def test_oracle_gaussian_distribution_and_grid(sigma):
    p = pydp.gaussian_params(sigma)
    x = np.full(30000, -2.0)
    y = O.secure_add_noise(p, x, 999, np.arange(30000), 3)
    assert np.all(np.fmod(y, p["granularity"]) == 0.0)
    assert _ks(y + 2.0, stats.norm(scale=sigma).cdf) > 1e-4
    # 1 / 2 sigma mass within a 4-sigma binomial CI (dp_computations_test.py:99-130)
    z = np.abs(y + 2.0) / sigma
    for k, mass in ((1, 0.6827), (2, 0.9545)):
        got = np.mean(z <= k)
        assert abs(got - mass) < 4 * math.sqrt(mass * (1 - mass) / len(z))


def test_oracle_streams_are_counter_based():
    """A draw depends only on (seed, index, slot): subsets agree with the whole."""
    p = pydp.laplace_params(1.0, 2.0)
    idx = np.arange(1000, 3000)
    whole = O.secure_add_noise(p, np.zeros(2000), 5, idx, 9)
    part = O.secure_add_noise(p, np.zeros(500), 5, idx[700:1200], 9)
    np.testing.assert_array_equal(whole[700:1200], part)
    other = O.secure_add_noise(p, np.zeros(2000), 6, idx, 9)
    assert np.mean(whole == other) < 0.01


def test_output_independent_of_low_bits_of_input():
    """The attack the snapping prevents: two inputs that differ below the grid
    give the same output for the same randomness."""
    p = pydp.laplace_params(1.0, 1.0)
    g = p["granularity"]
    a = O.secure_add_noise(p, np.full(100, 10.0), 3, np.arange(100), 1)
    b = O.secure_add_noise(p, np.full(100, 10.0 + g / 4), 3, np.arange(100), 1)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("kind", ["laplace", "gaussian"])
def test_host_sampler_distribution(kind):
    p = dpc.laplace_noise_params(1.0, 2.0) if kind == "laplace" else dpc.gaussian_noise_params(3.0)
    smp = dpc.secure_sampler()
    y = np.array([smp.add_noise(p, 0.0) for _ in range(4000)])
    assert np.all(np.fmod(y, p.granularity) == 0.0)
    dist = stats.laplace(scale=2.0) if kind == "laplace" else stats.norm(scale=3.0)
    assert _ks(y, dist.cdf) > 1e-4


def test_mechanism_add_noise_uses_secure_sampler():
    m = dpc.LaplaceMechanism.create_from_epsilon(1.0, 1.0)
    g = m.secure_params().granularity
    v = m.add_noise(5)
    assert isinstance(v, float) and math.fmod(v, g) == 0.0
    gm = dpc.GaussianMechanism.create_from_epsilon_delta(1.0, 1e-5, 1.0)
    v = gm.add_noise(5)
    assert math.fmod(v, gm.secure_params().granularity) == 0.0
