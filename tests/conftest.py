import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _make(path):
    subprocess.run(["make", "-s", "-C", path], check=True)


@pytest.fixture(scope="session", autouse=True)
def built_libraries():
    """The oracle (test infrastructure) and the product library must both exist."""
    _make(os.path.join(ROOT, "oracle"))
    lib = os.path.join(ROOT, "ekf-slam_amd", "libekfslam.so")
    if not os.path.exists(lib):
        _make(os.path.join(ROOT, "ekf-slam_amd"))
    yield


GOLDEN = os.path.join(ROOT, "tests", "golden")
GOLDEN_CASES = ["basic_world_known", "basic_world_assoc", "synth16_known", "synth16_assoc",
                "crowded_assoc", "mixed_actions_known"]


def load_golden(name):
    import numpy as np
    from pyekf import synth
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    sc = synth.Scenario(int(g["n_landmarks"]), g["landmarks"], g["wheel"], g["ids"], g["actions"],
                        g["rel"], g["count"], g["truth"], float(g["track"]), float(g["radius"]))
    return sc, g
