"""CPU tests of the arithmetic / random-stream contract shared by the oracle
and the HIP kernels (include/ptmi_math.h, include/ptmi_rng.h)."""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def ulp_err(got, ref64):
    ref32 = ref64.astype(np.float32)
    sp = np.spacing(np.abs(ref32)).astype(np.float64)
    return float(np.max(np.abs(got.astype(np.float64) - ref64) / sp))


@pytest.fixture(scope='module')
def rng():
    return np.random.default_rng(1)


def test_sincos_accuracy(rng):
    x = rng.uniform(0, 2 * np.pi, 100000).astype(np.float32)  # random_cosine_direction phi range
    assert ulp_err(oracle.math_probe('sin', x), np.sin(x.astype(np.float64))) < 2.0
    assert ulp_err(oracle.math_probe('cos', x), np.cos(x.astype(np.float64))) < 2.0
    x = rng.uniform(-500, 500, 100000).astype(np.float32)      # noise texture argument range
    assert np.max(np.abs(oracle.math_probe('sin', x) - np.sin(x.astype(np.float64)))) < 2e-7


def test_log_acos_atan2_accuracy(rng):
    x = np.exp(rng.uniform(np.log(1e-10), 0, 100000)).astype(np.float32)  # kernels.py:441 domain
    assert ulp_err(oracle.math_probe('log', x), np.log(x.astype(np.float64))) < 1.5
    c = rng.uniform(-1, 1, 100000).astype(np.float32)
    assert ulp_err(oracle.math_probe('acos', c), np.arccos(c.astype(np.float64))) < 2.0
    y = rng.uniform(-1, 1, 100000).astype(np.float32)
    x = rng.uniform(-1, 1, 100000).astype(np.float32)
    assert ulp_err(oracle.math_probe('atan2', y, x), np.arctan2(y.astype(np.float64), x.astype(np.float64))) < 4.0


def test_atan2_signed_zero_and_axes():
    y = np.array([0.0, -0.0, 0.0, -0.0, 1.0, -1.0], np.float32)
    x = np.array([1.0, 1.0, -1.0, -1.0, 0.0, 0.0], np.float32)
    got = oracle.math_probe('atan2', y, x)
    ref = np.arctan2(y, x)
    assert np.array_equal(np.signbit(got), np.signbit(ref))
    assert np.allclose(got, ref, rtol=0, atol=3e-7)


def test_pow5_definition(rng):
    x = rng.uniform(0, 1, 1000).astype(np.float32)
    x2 = x * x
    assert np.array_equal(oracle.math_probe('pow5', x), (x2 * x2) * x)


# --- independent Python restatement of include/ptmi_rng.h -----------------
M32 = 0xffffffff


def mix32(x):
    x &= M32
    x ^= x >> 16
    x = (x * 0x7feb352d) & M32
    x ^= x >> 15
    x = (x * 0x846ca68b) & M32
    x ^= x >> 16
    return x


def path_key(seed, pixel, sample):
    h = mix32(seed + 0x68e31da4)
    h = mix32(h ^ ((pixel * 0x9e3779b9) & M32))
    h = mix32(h + ((sample * 0x85ebca6b) & M32) + 0xc2b2ae35)
    return h


def rand(key, n):
    u = mix32(key ^ mix32((n * 0x9e3779b9 + 0x632be5ab) & M32))
    return np.float32(u >> 8) * np.float32(2.0 ** -24)


def test_rng_matches_python_restatement():
    for seed, pix, s in [(0, 0, 0), (0, 639999, 1023), (7, 12345, 3), (0xffffffff, 1, 65535)]:
        vals, key = oracle.rng_probe(seed, pix, s, 64)
        assert key == path_key(seed, pix, s)
        assert np.array_equal(vals, np.array([rand(key, n) for n in range(64)], np.float32))


def test_rng_known_answers():
    """Pins the stream: any change to ptmi_rng.h changes every rendered pixel."""
    with open(os.path.join(GOLD, 'rng_vectors.json')) as f:
        gold = json.load(f)
    for case in gold:
        vals, key = oracle.rng_probe(case['seed'], case['pixel'], case['sample'], len(case['u24']))
        assert key == case['key']
        assert [int(v * 2 ** 24) for v in vals] == case['u24']


def test_rng_statistics():
    n = 200000
    vals, _ = oracle.rng_probe(0, 42, 0, n)
    assert vals.min() >= 0.0 and vals.max() < 1.0
    assert abs(vals.mean() - 0.5) < 0.005
    hist, _ = np.histogram(vals, bins=64, range=(0, 1))
    chi2 = np.sum((hist - n / 64) ** 2 / (n / 64))
    assert chi2 < 130  # 63 dof, p ~ 1e-6
    # first draws of neighbouring pixels / samples are not correlated
    firsts = np.array([oracle.rng_probe(0, p, 0, 1)[0][0] for p in range(4000)])
    assert abs(np.corrcoef(firsts[:-1], firsts[1:])[0, 1]) < 0.05


def _div_cases(rng, n):
    """(x, a) pairs for the shared-reciprocal division: log-uniform magnitudes
    over and past the guard range, the megakernel's a = |d|^2 ~ 1 regime, and
    the IEEE special values."""
    def logu(lo, hi, k):
        return (2.0 ** rng.uniform(lo, hi, k)) * rng.choice([-1.0, 1.0], k)
    xs = [logu(-70, 70, n), logu(-30, 30, n), logu(-10, 14, n)]
    as_ = [np.abs(logu(-60, 60, n)), np.abs(logu(-8, 8, n)),
           (1.0 + rng.integers(-64, 64, n) * 2.0 ** -23)]  # a within 64 ulp of 1
    x = np.concatenate(xs).astype(np.float32)
    a = np.concatenate(as_).astype(np.float32)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.1754942e-38, 3.4028235e38,
                   2.0 ** -50, 2.0 ** 50, 2.0 ** -50 * 0.99999994, 2.0 ** 50 * 1.0000001, 1.0, 3.0],
                  np.float32)
    gx, ga = np.meshgrid(sp, np.abs(sp))
    return np.concatenate([x, gx.ravel(), sp]), np.concatenate([a, ga.ravel(), -np.abs(sp)])


def test_shared_reciprocal_division_is_exact(rng):
    """pt_div_by (include/ptmi_math.h; the HIP sphere test's division of both
    roots by the per-ray a) equals the IEEE quotient x / a bit for bit."""
    x, a = _div_cases(rng, 1_000_000)
    got = oracle.math_probe('div_by', x, a)
    with np.errstate(all='ignore'):
        ref = x / a
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), ref[~nan].view(np.uint32))


def test_shared_reciprocal_division_near_midpoints(rng):
    """Quotients close to a rounding midpoint: x = RN(a * m) for m with a
    25th significant bit set, so x / a lies near a tie of m's neighbours."""
    n = 500_000
    m = (rng.integers(2 ** 24, 2 ** 25, n) | 1).astype(np.float64) * 2.0 ** rng.integers(-60, -10, n)
    a = (2.0 ** rng.uniform(-20, 20, n)).astype(np.float32)
    x = (m * a.astype(np.float64)).astype(np.float32)
    got = oracle.math_probe('div_by', x, a)
    assert np.array_equal(got.view(np.uint32), (x / a).view(np.uint32))
