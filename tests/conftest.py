"""Shared fixtures. `-m "not gpu"` runs here (no GPU); `-m gpu` on an MI355X."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def _ensure_built():
    import __graft_entry__ as g
    g._load_build_module().build_all(verbose=False)


_ensure_built()


@pytest.fixture(scope="session")
def lvkv():
    import __graft_entry__ as g
    return g.load_package()


@pytest.fixture(scope="session")
def oracle():
    import oracle as o  # test infrastructure: the checker
    return o


@pytest.fixture(scope="session")
def golden():
    def load(name):
        p = GOLDEN / name
        if p.suffix == ".json":
            return json.loads(p.read_text())
        return np.fromfile(p, dtype=np.uint8)
    return load


@pytest.fixture(scope="session")
def corpus_buf(golden, oracle):
    spec = golden("corpus.json")
    return oracle.splitmix_bytes(spec["seed"], spec["buffer_bytes"])


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(params=[1, 2, 3], ids=["fused", "two_launch", "spec"])
def sst_form(request, lvkv, gpu):
    """Whole-SSTable verify form under test: 1 = one fused launch, 2 = the
    two-launch form, 3 = the speculative launch (CRC workgroups decode their
    own index entries; lvkv_debug_set_sst_form); back to by-size afterwards."""
    assert lvkv.lib.lvkv_debug_set_sst_form(request.param) == 0
    yield request.param
    lvkv.lib.lvkv_debug_set_sst_form(0)


