import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def free_port() -> int:
    """An unused TCP port on 127.0.0.1 for a torchrun rendezvous (tests may run under xdist).

    Picked below the kernel's ephemeral range (32768+): gloo opens many outgoing
    connections there, and one of them can take an ephemeral port between this
    probe and torchrun's bind (EADDRINUSE). Each xdist worker draws from its own
    slice of 20000-32000."""
    import random
    import socket

    wid = os.environ.get("PYTEST_XDIST_WORKER", "gw0")
    slot = int(wid[2:]) if wid[2:].isdigit() else 0
    lo = 20000 + (slot % 8) * 1500
    for _ in range(200):
        port = random.randrange(lo, lo + 1500)
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
