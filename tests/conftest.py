"""Test configuration: paths, markers, build of the native pieces.

`-m "not gpu"` runs everywhere (oracle vs independent model, C-ABI exports,
host logic); `-m gpu` needs an MI355X and compares the HIP path with the
oracle bit for bit.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "qpsk-modulator-demodulator_amd")
for p in (os.path.join(ROOT, "oracle"), PKG, os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


@pytest.fixture(scope="session", autouse=True)
def _native_builds():
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "liboracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if not os.path.exists(os.path.join(PKG, "_build", "libqpsk_demod.so")):
        subprocess.check_call(["make", "-s", "-j8", "-C", PKG])
    yield
