"""CPU tests of the oracle itself: closest-hit traversal against a brute-force
scan, and BASELINE config 1 (wavefront_comparison 400x225 @ 4 spp, the
reference's ti.cpu plumbing case) end to end on the CPU."""
import numpy as np
import pytest

import oracle
from parity_helpers import BG, fixture, oracle_render, scene_inputs
from ptmi import scene_data as sd


def dot(a, b):
    """(x + y) + z in f32, the contract's dot (no BLAS/FMA reordering)."""
    return np.float32(np.float32(a[0] * b[0]) + np.float32(a[1] * b[1])) + np.float32(a[2] * b[2])


def cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], np.float32)


def brute_force(sa, o, d, tmin=np.float32(0.001), tmax=np.float32(1e10)):
    """Closest hit over every primitive with the reference formulas (f32)."""
    best_t, best = tmax, (-1, -1)
    for i, s in enumerate(sa.sphere_data):
        c, r = s[:3], s[3]
        oc = c - o
        a = dot(d, d)
        h = dot(d, oc)
        cc = dot(oc, oc) - r * r
        disc = h * h - a * cc
        if disc >= 0:
            sq = np.sqrt(disc)
            for root in ((h - sq) / a, (h + sq) / a):
                if tmin <= root <= tmax:
                    if root < best_t:
                        best_t, best = root, (0, i)
                    break
    q = sa.quads
    for i in range(sa.num_quads):
        n = q['quad_normal'][i]
        den = dot(n, d)
        if abs(den) >= 1e-8:
            t = (q['quad_D'][i] - dot(n, o)) / den
            if tmin <= t <= tmax:
                p = (o + t * d) - q['quad_Q'][i]
                w = q['quad_w'][i]
                al = dot(w, cross(p, q['quad_v'][i]))
                be = dot(w, cross(q['quad_u'][i], p))
                if 0 <= al <= 1 and 0 <= be <= 1 and t < best_t:
                    best_t, best = t, (2, i)
    tr = sa.tris
    if sa.num_triangles:  # kernels.py:252-307, vectorised over triangles (elementwise f32, same op order)
        v0, e1, e2 = tr['triangle_v0'], tr['triangle_edge1'], tr['triangle_edge2']
        f = np.float32

        def vdot(a, b):
            return (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]

        def vcross(a, b):
            return np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                             a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], axis=1)
        dd = np.broadcast_to(d, e2.shape).astype(f)
        hv = vcross(dd, e2)
        det = vdot(e1, hv)
        ok = np.abs(det) >= f(1e-8)
        with np.errstate(divide='ignore', invalid='ignore', over='ignore'):
            inv = f(1.0) / det
            sv = (o - v0).astype(f)
            u = inv * vdot(sv, hv)
            q = vcross(sv, e1)
            v = inv * vdot(dd, q)
            t = inv * vdot(e2, q)
        ok &= (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= tmin) & (t <= tmax)
        for i in np.nonzero(ok)[0]:  # in index order: first-found on equal t, like the scan above
            if t[i] < best_t:
                best_t, best = t[i], (1, int(i))
    return best_t, best


@pytest.mark.parametrize('traversal', ['stack', 'stackless'])
@pytest.mark.parametrize('name', ['wavefront_comparison', 'cornell_smoke', 'coverage'])
def test_traversal_matches_brute_force(name, traversal):
    """Both of the reference's traversals (traverse_bvh_legacy, kernels.py:625,
    and traverse_bvh_stackless, :453) find the brute-force closest hit."""
    sa, cam, _ = scene_inputs(name, 800 if name != 'coverage' else 160)
    osc = oracle.OracleScene(sa)
    rng = np.random.default_rng(5)
    agree = 0
    n = 300
    tri_hits = 0
    for _ in range(n):
        o = cam['center'] + rng.normal(0, 0.5, 3).astype(np.float32)
        d = (cam['pixel00'] + rng.uniform(0, cam['width']) * cam['delta_u'] + rng.uniform(0, cam['height']) * cam['delta_v']
             - o).astype(np.float32)
        hit, t, ty, ix = oracle.traverse(osc, o, d, traversal=traversal)
        tri_hits += bool(hit and ty == 1)
        bt, (bty, bix) = brute_force(sa, o.astype(np.float32), d)
        if bty < 0:
            assert not hit
            agree += 1
        else:
            assert hit
            assert t == bt
            agree += (ty, ix) == (bty, bix)
    assert agree >= n - 2  # exact float ties may resolve differently
    if sa.num_triangles:
        assert tri_hits >= 5


@pytest.fixture(scope='module')
def config1():
    """BASELINE configs[0]: wavefront_comparison 400x225 @ 4 spp, both variants."""
    out = {}
    for v in ('mk', 'wf'):
        out[v] = oracle_render('wavefront_comparison', 400, v, (0, 0, 400, 225), 0, 4)
    return out


def test_config1_plumbing(config1):
    for v, (acc, st) in config1.items():
        img = acc / 4
        assert np.isfinite(img).all()
        assert st['paths'] == 400 * 225 * 4
        assert 1.5 < st['segments'] / st['paths'] < 3.5
        assert 0.3 < img.mean() < 0.7
        # sky (bg 0.7,0.8,1.0) dominates the top rows
        top = img[:20].reshape(-1, 3).mean(0)
        assert top[2] > top[0]


def test_config1_megakernel_vs_wavefront_statistically_equal(config1):
    """Q1/Q11/Q14 make the variants differ per path, not in expectation."""
    a = config1['mk'][0] / 4
    b = config1['wf'][0] / 4
    ca, cb = a.reshape(-1, 3).mean(0), b.reshape(-1, 3).mean(0)
    assert np.all(np.abs(ca - cb) < 0.01)
    # blurred images agree
    k = 25
    ba = a[:225 // k * k, :400 // k * k].reshape(225 // k, k, 400 // k, k, 3).mean((1, 3))
    bb = b[:225 // k * k, :400 // k * k].reshape(225 // k, k, 400 // k, k, 3).mean((1, 3))
    assert np.max(np.abs(ba - bb)) < 0.08


def test_oracle_deterministic_and_window_local():
    a, _ = oracle_render('vol2_final_scene', 64, 'mk', (8, 8, 16, 16), 0, 3)
    b, _ = oracle_render('vol2_final_scene', 64, 'mk', (8, 8, 16, 16), 0, 3, threads=1)
    assert np.array_equal(a, b)
    full, _ = oracle_render('vol2_final_scene', 64, 'mk', (0, 0, 64, 64), 0, 3)
    assert np.array_equal(full[8:24, 8:24], a[8:24, 8:24])
    assert not a[:8].any()


def test_stackless_traversal_iterations_cover_a_full_walk():
    """kernels.py:487-491 caps the stackless loop at 2 * num_bvh_nodes
    iterations; a walk of every node takes 3 per internal node + 1 per leaf =
    4L - 3 < 4L - 2, so the cap never cuts a traversal short: a ray from inside
    the root box that must visit every node still finds the brute-force hit."""
    sa, cam, _ = scene_inputs('wavefront_comparison', 800)
    osc = oracle.OracleScene(sa)
    c = (sa.bvh['bvh_bbox_min'][0] + sa.bvh['bvh_bbox_max'][0]) * np.float32(0.5)
    for d in (np.array([0.3, -1.0, 0.2], np.float32), np.array([0.0, 1.0, 0.0], np.float32)):
        a = oracle.traverse(osc, c, d, traversal='stack')
        b = oracle.traverse(osc, c, d, traversal='stackless')
        assert a[:2] == b[:2]


def test_stackless_render_matches_stack_statistically():
    """USE_STACKLESS_TRAVERSAL changes only the leaf visiting order (left first,
    kernels.py:572-577): the closest hit differs only on exact ties, so the
    two renders agree on almost every pixel."""
    a, _ = oracle_render('vol2_final_scene', 64, 'mk', (0, 0, 64, 64), 0, 2)
    b, _ = oracle_render('vol2_final_scene', 64, 'mk', (0, 0, 64, 64), 0, 2, traversal='stackless')
    assert np.mean(np.all(a == b, axis=2)) > 0.99
