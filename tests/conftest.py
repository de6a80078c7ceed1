"""Shared fixtures.  GPU tests are marked @pytest.mark.gpu; everything else runs on CPU."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def patterns():
    with open(os.path.join(GOLDEN, "patterns.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def refgold():
    with open(os.path.join(GOLDEN, "refgold.json")) as f:
        return json.load(f)
