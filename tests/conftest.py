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


class RioFake:
    """tests/cpp/rio_fake.c loaded with ctypes: the RIORegisterBuffer/RIODeregisterBuffer fakes and their
    bookkeeping queries."""

    def __init__(self, path):
        import ctypes

        L = ctypes.CDLL(path)
        u64, P = ctypes.c_uint64, ctypes.c_void_p
        for name, args, res in [("rio_fake_lookup", [u64, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_uint32)],
                                 ctypes.c_int),
                                ("rio_fake_live", [], u64), ("rio_fake_errors", [], u64),
                                ("rio_fake_registered", [], u64), ("rio_fake_reset", [u64], None)]:
            fn = getattr(L, name)
            fn.argtypes, fn.restype = args, res
        self.lib = L
        self.register_ptr = ctypes.cast(L.rio_fake_register, P).value
        self.deregister_ptr = ctypes.cast(L.rio_fake_deregister, P).value

    def lookup(self, buffer_id):
        import ctypes

        p, n = ctypes.c_uint64(), ctypes.c_uint32()
        return (int(p.value), int(n.value)) if self.lib.rio_fake_lookup(buffer_id, ctypes.byref(p), ctypes.byref(n)) \
            else None

    def live(self):
        return int(self.lib.rio_fake_live())

    def errors(self):
        return int(self.lib.rio_fake_errors())

    def registered(self):
        return int(self.lib.rio_fake_registered())

    def reset(self, fail_after=(1 << 64) - 1):
        self.lib.rio_fake_reset(fail_after)


@pytest.fixture(scope="session")
def rio_fake(tmp_path_factory):
    """Build the RIO fakes (gcc, seconds) and install them as the pattern mirror's rioFunctions."""
    from ctstraffic_amd.pattern import rio_functions_set

    so = str(tmp_path_factory.mktemp("rio") / "librio_fake.so")
    subprocess.run(["gcc", "-std=c11", "-O1", "-shared", "-fPIC", "-pthread",
                    os.path.join(ROOT, "tests", "cpp", "rio_fake.c"), "-o", so], check=True)
    fake = RioFake(so)
    rio_functions_set(fake.register_ptr, fake.deregister_ptr)
    yield fake
    rio_functions_set(None, None)
