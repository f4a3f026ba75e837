"""Shared fixtures.  ``-m gpu`` tests need an MI355X; everything else runs on CPU."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "erasure-coding-crust_amd")
for p in (os.path.join(ROOT, "oracle"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    """The byte-output checker: the reference ec-cpp (oracle/_ref, built from
    /root/reference by oracle/Makefile; it travels to the GPU box with the
    tree) when present, else the C restatement; internals from the restatement
    (oracle.Checker).  test_oracle.py pins the restatement itself."""
    import oracle as orc
    orc.build()
    return orc.Checker.default()


@pytest.fixture(scope="session")
def restatement():
    """The C restatement alone (oracle/ec_oracle.c), for the tests that pin it."""
    import oracle as orc
    orc.build()
    return orc.Oracle()


@pytest.fixture(scope="session")
def golden_vectors():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def golden_tables():
    with open(os.path.join(GOLDEN, "tables.json")) as f:
        return json.load(f)
