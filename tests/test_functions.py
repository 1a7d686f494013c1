"""Function-level pin of the oracle against the reference's own Python.

tests/golden/functions.npz holds known-answer vectors made by
tests/golden/gen_functions.py from the reference's core/perlin.py (noise,
turb), core/sphere.py (get_sphere_uv, hit), core/quad.py, core/triangle.py,
core/material.py (Schlick) and util/vec3.py (reflect, refract), evaluated in
float64 on float32 inputs. The oracle evaluates the kernels.py versions of the
same functions (or_func_probe) in float32, so the bound is float32 rounding:
relative 1e-5 (absolute 2e-6 for the Perlin values, which pass through 0 and
are O(1) at most). Hit flags must agree exactly (the vectors keep only rays
whose hit/miss margins are far from float32 rounding).

The negative control rebuilds the oracle without the Perlin Hermite smoothing
(kernels.py:125-127) and checks that the same comparison then fails.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle
from ptmi import scene_data as sd

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, 'golden', 'functions.npz'), allow_pickle=False)


@pytest.fixture(scope='module')
def oscene():
    return oracle.OracleScene(sd.load_fixture('vol2_final_scene'))


def _cmp(got, want, rel=1e-5, abs_=0.0):
    got = np.asarray(got, np.float64).reshape(want.shape)
    err = np.abs(got - want)
    bound = rel * np.abs(want) + abs_
    bad = err > bound
    return int(bad.sum()), float(err.max()) if err.size else 0.0


@pytest.mark.parametrize('fn, abs_', [('perlin_noise', 2e-6), ('perlin_turb', 2e-6)])
def test_perlin_matches_reference_python(oscene, fn, abs_):
    """core/perlin.py noise / turb (depth 3 and 7) with the fixture tables,
    including negative lattice coordinates (Q29) and 2p / 4p octave points."""
    x = G[f'{fn}_in']
    assert (x[:, :3] < 0).any() and len(x) >= 2000
    bad, mx = _cmp(oracle.func_probe(oscene, fn, x)[:, 0], G[f'{fn}_out'], 1e-5, abs_)
    assert bad == 0, f'{fn}: {bad} of {len(x)} values off, max error {mx}'


def test_perlin_turb_covers_the_noise_texture_depth():
    d = G['perlin_turb_in'][:, 3]
    assert (d == 3).sum() >= 1000 and (d == 7).sum() >= 100


def test_sphere_uv_matches_reference_python(oscene):
    bad, mx = _cmp(oracle.func_probe(oscene, 'sphere_uv', G['sphere_uv_in']), G['sphere_uv_out'], 1e-5, 1e-6)
    assert bad == 0, f'sphere_uv: {bad} off, max error {mx}'


@pytest.mark.parametrize('fn', ['reflect', 'refract', 'reflectance'])
def test_fresnel_helpers_match_reference_python(oscene, fn):
    bad, mx = _cmp(oracle.func_probe(oscene, fn, G[f'{fn}_in']), G[f'{fn}_out'], 1e-5, 1e-6)
    assert bad == 0, f'{fn}: {bad} off, max error {mx}'


@pytest.mark.parametrize('fn', ['hit_sphere', 'hit_quad', 'hit_triangle'])
def test_primitive_hits_match_reference_python(oscene, fn):
    got = oracle.func_probe(oscene, fn, G[f'{fn}_in']).astype(np.float64)
    want = G[f'{fn}_out']
    assert 0.1 * len(want) < want[:, 0].sum() < 0.9 * len(want)  # hits and misses both covered
    assert np.array_equal(got[:, 0], want[:, 0]), f'{fn}: hit flags differ on {(got[:, 0] != want[:, 0]).sum()} rays'
    h = want[:, 0] == 1
    bad, mx = _cmp(got[h, 1], want[h, 1], 1e-5)
    assert bad == 0, f'{fn}: {bad} t values off, max relative error {mx}'


def test_perlin_pin_rejects_a_broken_perlin(oscene, tmp_path):
    """Negative control: the oracle built without the Hermite smoothing
    (uu = u etc.) must fail the Perlin comparison above."""
    src = os.path.join(os.path.dirname(oracle.__file__), 'pt_oracle.c')
    so = str(tmp_path / 'libptoracle_nohermite.so')
    subprocess.run(['gcc', '-O1', '-std=c11', '-fPIC', '-shared', '-ffp-contract=off', '-fno-fast-math',
                    '-DOR_NEGATIVE_CONTROL_NO_HERMITE', '-o', so, src, '-lm'], check=True)
    lib = C.CDLL(so)
    lib.or_func_probe.argtypes = [C.POINTER(oracle.OrScene), C.c_int, C.c_void_p, C.c_void_p, C.c_int]
    lib.or_func_probe.restype = C.c_int
    x = np.ascontiguousarray(G['perlin_noise_in'], np.float32)
    out = np.zeros(len(x), np.float32)
    assert lib.or_func_probe(C.byref(oscene.s), 0, x.ctypes.data, out.ctypes.data, len(x)) == 3
    bad, _ = _cmp(out, G['perlin_noise_out'], 1e-5, 2e-6)
    assert bad > len(x) // 2
