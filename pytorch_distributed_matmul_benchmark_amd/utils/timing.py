"""Device-side timing: HIP events on GPU, ``perf_counter`` on CPU.

The reference brackets its hot loops with ``torch.cuda.Event`` pairs
(matmul_benchmark.py:54-68, matmul_scaling_benchmark.py:85-99) but also
calls ``torch.cuda.synchronize()`` before and after every compute and comm
segment inside the timed loops (:140,144,152), which adds host
latency to every measured interval. ``SegmentTimer`` records an event at
every segment boundary on the stream the work runs on and reads them all
once, after the loop — no host synchronisation inside the timed region.
"""
from __future__ import annotations

import contextlib
import time
from typing import Dict, List, Optional

import torch


def synchronize(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


class Stopwatch:
    """Elapsed time between ``start()`` and ``stop()`` on one stream (ms)."""

    def __init__(self, device: torch.device):
        self.device = device
        self._gpu = device.type == "cuda"
        self._t0 = self._t1 = None

    def start(self, stream=None) -> None:
        if self._gpu:
            self._t0 = torch.cuda.Event(enable_timing=True)
            self._t0.record(stream)
        else:
            self._t0 = time.perf_counter()

    def stop(self, stream=None) -> None:
        if self._gpu:
            self._t1 = torch.cuda.Event(enable_timing=True)
            self._t1.record(stream)
        else:
            self._t1 = time.perf_counter()

    def elapsed_ms(self) -> float:
        if self._gpu:
            self._t1.synchronize()
            return float(self._t0.elapsed_time(self._t1))
        return (self._t1 - self._t0) * 1e3


class SegmentTimer:
    """Accumulates named segments (e.g. ``compute`` / ``comm``) per iteration.

    ``mark(name)`` closes the segment that started at the previous mark.
    On GPU each mark is an event on ``stream`` (default: current stream);
    on CPU a wall-clock reading (the CPU ops themselves are synchronous).
    """

    def __init__(self, device: torch.device):
        self.device = device
        self._gpu = device.type == "cuda"
        self._marks: List[tuple] = []  # (name or None, event|time)

    def begin(self, stream=None) -> None:
        self._marks.append((None, self._stamp(stream)))

    def mark(self, name: str, stream=None) -> None:
        self._marks.append((name, self._stamp(stream)))

    def _stamp(self, stream):
        if self._gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            return e
        return time.perf_counter()

    def totals_ms(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        if self._gpu and self._marks:
            self._marks[-1][1].synchronize()
        prev = None
        for name, st in self._marks:
            if name is not None and prev is not None:
                dt = prev.elapsed_time(st) if self._gpu else (st - prev) * 1e3
                out[name] = out.get(name, 0.0) + float(dt)
            prev = st
        return out


def time_loop_ms(fn, iters: int, warmup: int, device: torch.device, stream=None,
                 sync_fn=None) -> float:
    """Total ms of ``iters`` back-to-back ``fn()`` calls after ``warmup`` untimed ones.

    ``sync_fn`` (e.g. a barrier) runs after the warmup so every rank starts the
    timed region together (matmul_scaling_benchmark.py:78-82)."""
    for _ in range(warmup):
        fn()
    synchronize(device)
    if sync_fn is not None:
        sync_fn()
    sw = Stopwatch(device)
    sw.start(stream)
    for _ in range(iters):
        fn()
    sw.stop(stream)
    return sw.elapsed_ms()


@contextlib.contextmanager
def marker(name: str, enabled: bool = True):
    """A named range in the profiler timeline (roctx on PyTorch-ROCm:
    ``torch.cuda.nvtx`` is routed to roctx). Visible with
    ``rocprofv3 --marker-trace --kernel-trace``. No-op when disabled."""
    if not enabled:
        yield
        return
    import torch.cuda.nvtx as nvtx

    nvtx.range_push(name)
    try:
        yield
    finally:
        nvtx.range_pop()
