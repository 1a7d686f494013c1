"""Orbit-camera math of the headless InteractiveViewer
(reference: src/render_server/interactive_viewer.py:52-129)."""
import math

from ptmi.core import point3
from ptmi.interactive_viewer import orbit_step, spherical_from, spherical_offset


def test_spherical_roundtrip():
    lf, la = point3(478, 278, -600), point3(278, 278, 0)
    r, th, ph = spherical_from(lf, la)
    x, y, z = spherical_offset(r, th, ph)
    assert math.isclose(la.x + x, lf.x, abs_tol=1e-9)
    assert math.isclose(la.y + y, lf.y, abs_tol=1e-9)
    assert math.isclose(la.z + z, lf.z, abs_tol=1e-9)


def test_orbit_step_matches_reference_formula():
    th, ph = orbit_step(0.25, 0.1, 30, -15)
    assert th == 0.25 + math.radians(30 * 0.3)
    assert ph == 0.1 + math.radians(-15 * 0.3)
    _, ph = orbit_step(0.0, 0.0, 0, 10_000)
    assert ph == math.radians(89.0)
    _, ph = orbit_step(0.0, 0.0, 0, -10_000)
    assert ph == -math.radians(89.0)
