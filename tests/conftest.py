import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: full-size property tests")


def _ensure_built():
    so = os.path.join(ROOT, "weaviate_amd", "libwvgpu.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "weaviate_amd", "csrc")], check=True)
    orc = os.path.join(ROOT, "oracle", "_build", "libwvoracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def ctx():
    import torch

    # torch ships its own HIP runtime under the same soname: initialise it first
    # so the process holds ONE runtime that both torch and libwvgpu.so use.
    torch.cuda.init()
    from weaviate_amd.device import Context

    c = Context(0)  # raises on a box without a GPU: GPU tests never silently skip
    yield c
    c.close()


@pytest.fixture(scope="session")
def orc():
    from oracle import wv_oracle

    wv_oracle.lib()
    return wv_oracle
