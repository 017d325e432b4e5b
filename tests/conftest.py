import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libspec_amd.so on cuda:0)")


# BASELINE-size tests (1M-record configs 2-4, the 16M config 5, 100k+ trees) take most of the
# GPU suite's time: run them after everything else, so under -x a quick test's failure is
# reported first and the small tests never wait behind them.
FULL_SIZE = ("full_size", "config5", "at_scale", "131072")


def pytest_collection_modifyitems(config, items):
    items.sort(key=lambda it: any(k in it.nodeid for k in FULL_SIZE))  # stable: file order otherwise


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (and the engine if it is missing) once per session."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = os.path.join(ROOT, "spec_amd", "libspec_amd.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "spec_amd", "csrc")], check=True)
    yield


@pytest.fixture(scope="session")
def dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
