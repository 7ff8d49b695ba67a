import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kernel-methods-for-genomics_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
# every Gram output is pre-filled with garbage, so a kernel that silently does not run
# cannot pass by leaving a previous (correct) result in a reused device buffer
os.environ.setdefault("KMG_POISON", "1")
# every neighbourhood-list fill is followed by the metadata check (KMG_EINTERNAL instead of a
# Gram kernel reading past a list: DESIGN §7)
os.environ.setdefault("KMG_CHECK", "1")
for p in (PKG, ORACLE, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and libkmgram.so")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    import golden_io
    return golden_io.Golden()


@pytest.fixture(scope="session")
def ctx():
    from kmgram import _lib as L
    c = L.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def engine():
    from kmgram import GramEngine
    e = GramEngine(0)
    yield e
    e.close()


@pytest.fixture
def tune(ctx, monkeypatch):
    """Set KMG_* tuning variables for one test: the library reads them once per context
    (kmg_create / kmg_reload_tuning), so every change is followed by a reload."""
    def set_(**kv):
        for k, v in kv.items():
            if v is None:
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, str(v))
        ctx.reload_tuning()
    yield set_
    monkeypatch.undo()
    ctx.reload_tuning()
