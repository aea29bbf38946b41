"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers on
the CPU restatement). `make -C oracle sanitize` links the sanitizer runtimes into a standalone
driver (oracle/orc_sanitize_main.c); it replays every golden fixture the way orc.run_scenario does
(wheel ticks through DiffDrive::FKin, then fake_sensor_cb / sensor_cb of slam.cpp), in the literal
dense, structured and Joseph modes, plus the error paths (id ≥ N, map full). Any invalid access,
leak or undefined operation aborts the driver (-fno-sanitize-recover=all); its outputs must match
the golden fixtures at the tolerances of tests/test_oracle_golden.py."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN_CASES, load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
EXE = os.path.join(ORACLE, "_build", "orc_sanitized")
POSE_TOL = SIGMA_TOL = 1e-8


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], check=True)
    return EXE


def _run(exe, tmp_path, sc, assoc, literal=False, joseph=False, name="s"):
    N, T, M = sc.n_landmarks, sc.n_messages, sc.ids.shape[1]
    W = sc.wheel.shape[1]
    src, dst = tmp_path / f"{name}.in", tmp_path / f"{name}.out"
    with open(src, "wb") as fh:
        fh.write(np.array([N, T, M, W, int(assoc), int(literal), int(joseph), 0], np.int32).tobytes())
        fh.write(np.array([sc.track, sc.radius], np.float64).tobytes())
        for t in range(T):
            fh.write(np.ascontiguousarray(sc.wheel[t], np.float64).tobytes())
            fh.write(np.array([sc.count[t]], np.int32).tobytes())
            fh.write(np.ascontiguousarray(sc.ids[t], np.int32).tobytes())
            fh.write(np.ascontiguousarray(sc.actions[t], np.int32).tobytes())
            fh.write(np.ascontiguousarray(sc.rel[t], np.float64).tobytes())
    # the harness may preload a library of its own: ASan must not insist on coming first
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="2")
    r = subprocess.run([exe, str(src), str(dst)], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    buf = open(dst, "rb").read()
    n = 3 + 2 * N
    o, out = 0, {}
    for key, dt, cnt in (("poses", np.float64, 3 * T), ("tmo", np.float64, 3 * T),
                         ("rcs", np.int32, T), ("assoc_j", np.int32, T * M),
                         ("assoc_new", np.int32, T * M), ("state", np.float64, n),
                         ("sigma", np.float64, n * n), ("tmo_final", np.float64, 3),
                         ("counter", np.uint32, 1)):
        a = np.frombuffer(buf, dt, cnt, o)
        o += a.nbytes
        out[key] = a
    assert o == len(buf)
    out["poses"] = out["poses"].reshape(T, 3)
    out["tmo"] = out["tmo"].reshape(T, 3)
    out["assoc_j"] = out["assoc_j"].reshape(T, M)
    out["assoc_new"] = out["assoc_new"].reshape(T, M)
    out["sigma"] = out["sigma"].reshape(n, n)
    out["counter"] = int(out["counter"][0])
    return out


@pytest.mark.parametrize("literal", [False, True], ids=["structured", "literal"])
@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_sanitized_oracle_matches_golden(exe, tmp_path, name, literal):
    sc, g = load_golden(name)
    assoc = bool(g["assoc"])
    o = _run(exe, tmp_path, sc, assoc, literal=literal)
    assert np.all(o["rcs"] == 0)
    assert np.abs(o["poses"] - g["poses"]).max() < POSE_TOL
    assert np.abs(o["tmo"] - g["tmo"]).max() < POSE_TOL
    assert np.abs(o["state"] - g["state"]).max() < POSE_TOL
    assert np.abs(o["sigma"] - g["sigma"]).max() < SIGMA_TOL
    assert o["counter"] == int(g["counter"])
    if assoc:
        assert np.array_equal(o["assoc_j"], g["assoc_j"])
        assert np.array_equal(o["assoc_new"], g["assoc_new"])


@pytest.mark.parametrize("assoc", [False, True], ids=["known", "assoc"])
def test_sanitized_oracle_joseph(exe, tmp_path, assoc):
    """The Joseph mode's two forms under the sanitizers (synth scenario of test_oracle_golden's
    Joseph test)."""
    from pyekf import synth
    sc = synth.synthetic(20, 30, seed=7, max_markers=6, shuffle=assoc)
    js = _run(exe, tmp_path, sc, assoc, joseph=True, name="js")
    jl = _run(exe, tmp_path, sc, assoc, joseph=True, literal=True, name="jl")
    assert js["counter"] == jl["counter"]
    assert np.abs(js["sigma"] - jl["sigma"]).max() < 1e-8


def test_sanitized_oracle_error_paths(exe, tmp_path):
    """Bad ids (EKF_E_RANGE before anything changes) and a full map (the reference indexes past
    the state, slam.cpp:351-356): the bounds checks themselves must stay inside the arrays."""
    from pyekf import synth
    sc = synth.synthetic(6, 12, seed=3, max_markers=5)
    ids = sc.ids.copy()
    ids[4, 0] = 6                                     # id = N
    bad = synth.Scenario(sc.n_landmarks, sc.landmarks, sc.wheel, ids, sc.actions, sc.rel,
                         sc.count, sc.truth, sc.track, sc.radius)
    o = _run(exe, tmp_path, bad, False, name="bad")
    assert o["rcs"][4] == -2 and np.all(np.delete(o["rcs"], 4) == 0)
    tiny = synth.Scenario(2, sc.landmarks, sc.wheel, sc.ids, sc.actions, sc.rel, sc.count,
                          sc.truth, sc.track, sc.radius)
    o = _run(exe, tmp_path, tiny, True, name="full")  # more landmarks in view than 2 slots
    assert np.any(o["rcs"] == -2) and o["counter"] == 2
