import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "experiments: A/B or diagnostic kernels that only a "
                                       "PDMB_EXPERIMENTS=1 build carries (deselected otherwise)")


def _experiment_kernels():
    try:
        from pytorch_distributed_matmul_benchmark_amd.ops.gemm import EXPERIMENT_KERNELS

        return set(EXPERIMENT_KERNELS)
    except Exception:  # pragma: no cover
        return set()


@pytest.hookimpl(tryfirst=True)
def pytest_collection_modifyitems(config, items):
    # Experiment-kernel cases (a ``kernel`` parameter naming an experiment
    # kernel, or an explicit ``experiments`` mark) run only against a
    # PDMB_EXPERIMENTS=1 build: deselected otherwise, so the shipping build's
    # ``-m gpu`` run reports only real skips. Runs before -m filtering, so
    # ``-m "gpu and experiments"`` selects them on an experiment build.
    exp = _experiment_kernels()
    for item in items:
        cs = getattr(item, "callspec", None)
        k = cs.params.get("kernel") if cs is not None else None
        if isinstance(k, str) and k in exp:
            item.add_marker(pytest.mark.experiments)
    if os.environ.get("PDMB_EXPERIMENTS") != "1":
        drop = [it for it in items if it.get_closest_marker("experiments") is not None]
        if drop:
            config.hook.pytest_deselected(items=drop)
            items[:] = [it for it in items if it.get_closest_marker("experiments") is None]
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
