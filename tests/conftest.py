import os
import sys

# before anything initialises HIP (see distributed_training_and_deepspeed_amd/__init__.py)
os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")

import pytest  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _install_segv_backtrace():
    """DTD_SEGV_BT=1: native backtrace of a host-side SIGSEGV (scripts/diag/native/segv_bt.c)."""
    if os.environ.get("DTD_SEGV_BT") != "1":
        return
    import ctypes
    lib = os.path.join(ROOT, "scripts", "diag", "native", "libsegv_bt.so")
    if os.path.exists(lib):
        ctypes.CDLL(lib).segv_bt_install()


def pytest_configure(config):
    _install_segv_backtrace()
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def pick_free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture
def free_port():
    return pick_free_port()
