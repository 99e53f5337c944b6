import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built libivc.so")


@pytest.fixture
def tune():
    """tune(name, value): an ivc_set_tuning override (chunk counts, the symbols -> image
    fallback) for this test only; every key it touched is restored at teardown."""
    from ivclab_amd import _native as N
    saved = {}

    def set_(name, value):
        prev = N.set_tuning(name, value)
        saved.setdefault(name, prev)
    yield set_
    for name, prev in saved.items():
        N.set_tuning(name, prev)


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    return load
