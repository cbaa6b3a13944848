"""Shared fixtures. `gpu`-marked tests need a real MI355X (run with `-m gpu`); the rest run on CPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); parity tests through the C ABI")


@pytest.fixture(scope="session")
def evam():
    import __graft_entry__ as g

    return g.import_package()


@pytest.fixture(scope="session")
def O():
    import oracle

    return oracle


@pytest.fixture(scope="session")
def coracle():
    import oracle

    oracle.build_c_oracle()
    return oracle.COracle()


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
