import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FIX = os.path.join(ROOT, "tests", "fixtures")
GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def sup():
    import superman_amd
    superman_amd._lib.load()
    return superman_amd


@pytest.fixture(scope="session")
def orc():
    import oracle
    oracle.load()
    return oracle


def fixture_path(name: str) -> str:
    return os.path.join(FIX, name)


def rel(a: float, b: float) -> float:
    if a == b:
        return 0.0
    return abs(a - b) / max(abs(a), abs(b), 1e-300)
