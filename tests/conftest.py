import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "deferred_only: test_gpu_tree_ops runs it with deferred running sums only")


def _build_oracle():
    src = os.path.join(ROOT, "oracle", "fold_ref.c")
    out = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(out) or os.path.getmtime(src) > os.path.getmtime(out):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                        "-pthread", src, "-o", out, "-lm"], check=True)
    return out


@pytest.fixture(scope="session")
def coracle():
    """The C restatement (oracle/fold_ref.c) via ctypes."""
    from tests import coracle as co
    return co.load(_build_oracle())


@pytest.fixture()
def tu_settings(monkeypatch):
    """Set fedjax_amd.tree_util's module settings (_PIPELINE_FRAC, _NATIVE_MEAN, ...) for one
    test. The builtin tree_mean (fjhost.tree_mean) holds its own copy of them, so it is
    re-configured (tree_util._mean_config) on every set and after the test's monkeypatches
    are undone."""
    from fedjax_amd import tree_util as tu

    def set_(**kw):
        for k, v in kw.items():
            monkeypatch.setattr(tu, k, v)
        tu._mean_config()
    yield set_
    monkeypatch.undo()
    tu._mean_config()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fedjax_amd import _lib
    _lib.load()
    return torch.device("cuda:0")


def pytest_sessionstart(session):
    # (re)build libfjagg.so / liboracle.so in-tree if a source is newer (no-op otherwise)
    import __graft_entry__
    __graft_entry__.build()
