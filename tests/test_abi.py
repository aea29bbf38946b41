"""The C-ABI library loads (no GPU needed) and exports every symbol include/*.h declares."""
import os
import re

import pyekf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in ("ekf.h", "slam_core.h", "landmarks.h", "ekf_sim.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b((?:ekf|slam|lm)_\w+)\s*\(",
                             src, flags=re.M):
            names.add(m.group(1))
    return names


def test_header_symbols_exported():
    L = pyekf.lib()
    declared = _declared()
    assert len(declared) >= 30
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    assert declared == set(pyekf.EXPORTS)


def test_config_defaults_match_reference():
    c = pyekf.make_config()
    # slam.cpp:665-671 and the literal 10e6 at :130
    assert (c.n_landmarks, c.q_noise, c.r_noise, c.init_var, c.mah_gate) == (50, 1e-2, 1e-2,
                                                                             1e7, 2.0)


def test_strerror_table():
    L = pyekf.lib()
    for rc in (0, -1, -2, -3, -4, -5, -6, -7):
        assert L.ekf_strerror(rc)


def test_no_cpu_fallback_in_product():
    """The product package never imports the oracle."""
    pkg = os.path.join(ROOT, "ekf-slam_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".hpp")):
                text = open(os.path.join(dirpath, fn)).read()
                for banned in ("import orc", "ekf_numpy", "ekf_oracle", "libekf_oracle",
                               "orc_ekf", "landmarks_numpy"):
                    assert banned not in text, (fn, banned)
