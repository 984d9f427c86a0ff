import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and the built libnbx.so")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"))
    return load


@pytest.fixture(scope="session")
def hip_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a HIP device")
    import nbody_amd._lib as L
    L.lib()  # loud failure if the extension is missing
    return torch.device("cuda:0")


def assert_cols(got, ref, rel=1e-5, abs_=1e-7, label=""):
    """The per-output-column tolerance of the SEGNN parity tests, shared by every family:
    max_r |got[r, c] - ref[r, c]| <= rel * max_r |ref[r, c]| + abs_ for each column c (the last axis);
    prints the worst column's error / scale so the margin is on record."""
    import numpy as np
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    g, r = got.reshape(-1, got.shape[-1]), ref.reshape(-1, ref.shape[-1])
    err = np.abs(g - r).max(0)
    scale = np.abs(r).max(0)
    ratio = (err / np.maximum(scale, 1e-30)).max()
    if label:
        print(f"[cols] {label}: worst column error / scale {ratio:.2e} (tolerance {rel:.0e})")
    bad = err > rel * scale + abs_
    assert not bad.any(), f"{label}: column errors {err} vs scales {scale} (rel {rel})"
    return ratio
