import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def pytest_collection_modifyitems(config, items):
    # Without a visible GPU the gpu-marked tests cannot run here; on the GPU
    # box they run (the driver selects them with -m gpu).
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden_ref():
    import numpy as np
    with np.load(os.path.join(GOLDEN, "golden_reference.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden_edge():
    import numpy as np
    with np.load(os.path.join(GOLDEN, "golden_edge.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
