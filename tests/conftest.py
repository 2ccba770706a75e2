"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs the oracle-vs-golden, host-logic, ABI-load and gloo tests on
CPU; `-m gpu` runs the parity tests through the C ABI on a real MI355X.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests through the C ABI")


def _gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure libcts_engine.so and the oracle exist (builds in-tree if missing)."""
    need = [os.path.join(ROOT, "ctstraffic_amd", "libcts_engine.so"), os.path.join(ROOT, "oracle", "libcts_oracle.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-s", "-C", ROOT, "-j8"], check=True)
    yield


@pytest.fixture(scope="session")
def engine():
    if not _gpu_available():
        pytest.fail("gpu test selected but no HIP device is visible (the engine has no CPU fallback)")
    from ctstraffic_amd import Engine

    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="session")
def tuning_engine():
    """An engine of the tuning build (libcts_engine_tuning.so: every launch variant) for the variant parity tests;
    the product library compiles one kernel per path."""
    if not _gpu_available():
        pytest.fail("gpu test selected but no HIP device is visible (the engine has no CPU fallback)")
    from ctstraffic_amd import Engine

    e = Engine(0, tuning=True)
    yield e
    e.close()
