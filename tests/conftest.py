"""Shared pytest setup: the `gpu` marker and import paths.

`-m "not gpu"` runs on the CPU-only dev container (oracle vs golden vectors,
host logic, C-ABI symbol exports); `-m gpu` runs the HIP parity tests on an
MI355X through the C-ABI library.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gpu-bpe_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
