import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgsa.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU check")


@pytest.fixture(scope="session")
def golden():
    from tests import _data
    return _data.Golden()


@pytest.fixture(scope="session")
def engine():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import gpuseqalign_amd as gsa
    e = gsa.Engine(0)
    yield e
    e.close()


@pytest.fixture
def knobs(engine, monkeypatch):
    """Set library knobs for one test: on the session engine (gsa_set_knob -- a context reads the
    environment only when it is created) and in the environment, for the engines the test creates
    itself (shard.gpu_batch_align and the like).  Both are undone after the test."""
    names = []

    def set_knob(name, value):
        if value is None:  # unset: the library's own choice
            monkeypatch.delenv(name, raising=False)
            engine.set_knob(name, None)
            return
        value = str(value)
        monkeypatch.setenv(name, value)
        engine.set_knob(name, value)
        names.append(name)

    yield set_knob
    for n in names:
        engine.set_knob(n, None)
