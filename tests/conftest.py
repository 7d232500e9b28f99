import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import pytest  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (HIP device) and the built libvihmc.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a visible HIP device")
    return torch.device("cuda", 0)


def pytest_sessionfinish(session, exitstatus):
    """Measured parity errors of the GPU tests (tests/parity.py) -> $VIHMC_PARITY_LOG, default
    gpurun_out/parity_errors.json (copied into profiles/ as the round's record)."""
    import parity
    parity.write(os.environ.get("VIHMC_PARITY_LOG", os.path.join(ROOT, "gpurun_out", "parity_errors.json")))
