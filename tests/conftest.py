"""pytest configuration: the `gpu` marker and shared fixture loaders."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "game-of-life-distributed_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# The GPU suites pin every plan the A/B tuning knobs select (skew_*, lds_*,
# persist_* ...) against the oracle, so the session consents to them
# (GOLHIP_TUNING=1; the product refuses them without it:
# tests/test_gpu_parity.py::test_wrong_result_options_need_measurement_consent).
# Wrong-result options and test hooks still need their own consent per test.
os.environ.setdefault("GOLHIP_TUNING", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def fixtures():
    with np.load(os.path.join(GOLDEN, "fixtures.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture
def test_hooks(monkeypatch):
    """Consent for the library's test hooks (resident_fault, flip_debug 4):
    GOLHIP_TEST_HOOKS=1 for this test only."""
    monkeypatch.setenv("GOLHIP_TEST_HOOKS", "1")
