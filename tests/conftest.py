import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hsig-picotls_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    from oracle_lib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import json
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    out = {}
    for name in ("kats", "sweep", "configs"):
        with open(os.path.join(d, name + ".json")) as f:
            out[name] = json.load(f)
    return out


@pytest.fixture(scope="session")
def engine():
    import torch
    import ptls_hip
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    e = ptls_hip.Engine(0)
    yield e
    e.close()
