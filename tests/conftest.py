"""Test configuration.

`-m "not gpu"` (CPU, this container): oracle vs committed golden vectors,
host-side logic, C-ABI library loading / exported symbols, gloo multi-process.
`-m gpu` (MI355X): parity of the HIP path (through the C-ABI) against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "roborts-edu-slam_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libroborts_csm.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
