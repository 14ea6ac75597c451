"""Shared pytest configuration.

GPU tests (marker `gpu`) call the HIP path through the C ABI and compare it with the CPU
oracle (oracle/, test infrastructure). CPU tests cover the oracle against golden vectors and
the reference's deterministic unit tests, the host logic, and the C ABI's exported symbols.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "node-replication_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libnrgpu.so)")


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def nrg():
    import nrgpu

    nrgpu.load()
    if nrgpu.device_count() < 1:
        pytest.fail("gpu test selected but no HIP device is visible")
    return nrgpu
