"""Pins the oracle's turtlelib restatement with the reference's own known-answer tests.

Transcribed from turtlelib/tests/test_geometry2d.cpp:8-17, test_se2d.cpp:152-251 and
test_diff_drive.cpp:7-99 (same inputs, same expected values, same tolerances). The product's own
geometry (ekf-slam_amd/csrc/geom.hpp) is checked against the oracle on the GPU side and through
slam_integrate_odometry here.
"""
import math

import numpy as np
import pytest

import ekf_numpy as npo
import orc

PI = math.pi


@pytest.mark.parametrize("impl", ["c", "numpy"])
def test_normalize_angle_kat(impl):
    f = orc.normalize_angle if impl == "c" else npo.normalize_angle
    cases = [(0, 0), (PI, PI), (-PI, PI), (-PI / 4, -PI / 4), (3 * PI / 2, -PI / 2),
             (-3 * PI / 2, PI / 2), (-5 * PI / 2, -PI / 2), (5 * PI / 2, PI / 2)]
    for a, want in cases:
        assert abs(f(a) - want) < 1e-8, (a, f(a), want)


@pytest.mark.parametrize("impl", ["c", "numpy"])
def test_transform_inv_compose_kat(impl):
    comp = orc.tf_compose if impl == "c" else npo.tf_compose
    inv = orc.tf_inv if impl == "c" else npo.tf_inv
    tf = (0.6, 1.2, -2.2)
    r = inv(tf)                                           # test_se2d.cpp:152-160
    assert abs(r[0] + 0.6) < 1e-3 and abs(r[1] - 0.252) < 1e-3 and abs(r[2] - 2.493) < 1e-3
    r = comp(tf, inv(tf))                                 # :162-170
    assert max(abs(v) for v in r) < 1e-3
    r = comp((0.6, 1.2, -2.2), (-0.1, 0.3, 4.1))          # :172-194
    assert abs(r[0] - 0.5) < 1e-3 and abs(r[1] + 0.867) < 1e-3 and abs(r[2] - 1.353) < 1e-3


@pytest.mark.parametrize("impl", ["c", "numpy"])
def test_integrate_twist_kat(impl):
    it = orc.integrate_twist if impl == "c" else npo.integrate_twist
    r = it(0.0, 1.0, -1.1)                                # test_se2d.cpp:226-251
    assert abs(r[0]) < 1e-3 and abs(r[1] - 1.0) < 1e-3 and abs(r[2] + 1.1) < 1e-3
    r = it(1.0, 0.0, 0.0)
    assert abs(r[0] - 1.0) < 1e-3 and abs(r[1]) < 1e-3 and abs(r[2]) < 1e-3
    r = it(1.0, 1.0, -1.0)
    w = 1.0
    assert abs(r[0] - 1.0) < 1e-3
    assert abs(r[2] - (-math.cos(w) - math.sin(w) + 1)) < 1e-3
    assert abs(r[1] - (-math.cos(w) + math.sin(w) + 1)) < 1e-3


def _fkin_cases():
    q = (0.1 * PI / 4.0) / (2.0 * PI * 0.2) * 2.0 * PI
    arc_l = (0.4 * PI / 4.0) / (2.0 * PI * 0.2) * 2.0 * PI
    arc_r = (0.2 * PI / 4.0) / (2.0 * PI * 0.2) * 2.0 * PI
    return [  # (track, radius, wheel sequence, expected (x, y, θ)) — test_diff_drive.cpp:7-99
        (0.1, 0.05, [(PI, PI)], (PI * 0.05, 0.0, 0.0)),
        (0.1, 0.05, [(-PI, -PI)], (-PI * 0.05, 0.0, 0.0)),
        (0.1, 0.05, [(PI / 4, PI / 4), (0.0, 0.0)], (0.0, 0.0, 0.0)),
        (0.1, 0.2, [(q, -q)], (0.0, 0.0, -PI / 2)),
        (0.1, 0.2, [(-q, q)], (0.0, 0.0, PI / 2)),
        (0.1, 0.2, [(arc_l, arc_r)], (0.15, -0.15, -PI / 2)),
        (0.1, 0.2, [(-arc_l, -arc_r)], (-0.15, -0.15, PI / 2)),
        (0.1, 0.2, [(arc_l, arc_r), (0.0, 0.0)], (0.0, 0.0, 0.0)),
    ]


@pytest.mark.parametrize("impl", ["c", "numpy", "product"])
@pytest.mark.parametrize("case", range(8))
def test_fkin_kat(impl, case):
    track, radius, seq, (ex, ey, et) = _fkin_cases()[case]
    if impl == "product":
        import pyekf
        from pyekf import synth
        wheel = np.array(seq, dtype=np.float64).reshape(1, len(seq), 2)
        sc = synth.Scenario(1, np.zeros((0, 2)), wheel, np.zeros((1, 0), np.int32),
                            np.zeros((1, 0), np.int32), np.zeros((1, 0, 2)),
                            np.zeros(1, np.int32), np.zeros((1, 3)), track, radius)
        th, x, y = pyekf.odometry(sc)[0]
    else:
        dd = orc.DiffDrive(track, radius) if impl == "c" else npo.DiffDrive(track, radius)
        for l, r in seq:
            out = dd.fkin(l, r)
        th, x, y = out
    assert abs(x - ex) < 1e-8 and abs(y - ey) < 1e-8 and abs(th - et) < 1e-8


def test_product_normalize_angle_bit_exact_with_oracle():
    """geom.hpp's fast fmod(x, 2π) path returns fmod's bits (normalize_angle is on every step)."""
    import pyekf
    L = pyekf.lib()
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(-40, 40, 20000), rng.uniform(-7, 7, 20000),
                         np.array([0.0, -0.0, PI, -PI, 2 * PI, -2 * PI, 3 * PI, -3 * PI, 4 * PI,
                                   -4 * PI, 5 * PI, -5 * PI, 1e-300, -1e-300, 1e6, -1e6]),
                         np.nextafter(np.array([PI, -PI, 3 * PI, -3 * PI]), 10.0),
                         np.nextafter(np.array([PI, -PI, 3 * PI, -3 * PI]), -10.0)])
    for v in xs:
        a, b = L.ekf_normalize_angle(float(v)), orc.normalize_angle(float(v))
        assert a == b and np.signbit(a) == np.signbit(b), (v, a, b)
