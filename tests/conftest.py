import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)

# Under tests/test_sanitized.py this process runs with the ASan runtime
# preloaded (for the sanitized check library); the compilers and tools the
# tests start need none of it, so it is taken out of their environment.
if os.environ.get("MK_CHECK_LIB") and "libasan" in os.environ.get("LD_PRELOAD", ""):
    _keep = [p for p in os.environ["LD_PRELOAD"].replace(":", " ").split() if "libasan" not in p]
    if _keep:
        os.environ["LD_PRELOAD"] = " ".join(_keep)
    else:
        del os.environ["LD_PRELOAD"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built():
    import __graft_entry__ as g

    g.build_native()
    from oracle import pyoracle

    pyoracle.build()
    yield


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        # -m gpu runs only on the GPU box: a missing GPU there is a failure, not a skip
        pytest.fail("no GPU visible to torch (HIP)")
    torch.cuda.init()
    return torch.device("cuda:0")
