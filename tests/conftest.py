import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "marl-maze_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


def pytest_runtest_setup(item):
    if "gpu" in item.keywords:
        import torch
        if not torch.cuda.is_available():
            pytest.fail("gpu test selected but no GPU is visible (no CPU fallback exists)")


class _Fixture(dict):
    """npz contents decompressed once (NpzFile re-reads the zip on every access)."""

    @property
    def files(self):
        return list(self.keys())


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
                d = {k: z[k] for k in z.files}
            cache[name] = _Fixture(d)
        return cache[name]

    return load
