"""pytest configuration: the `gpu` marker and a session-wide native build.

CPU tests (`-m "not gpu"`) exercise the oracle, the host logic and the C ABI
surface; `-m gpu` tests are the engine-vs-oracle parity tests proper.
"""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session", autouse=True)
def _native_build():
    import mpenv_testlib

    mpenv_testlib.ensure_built()
    yield
