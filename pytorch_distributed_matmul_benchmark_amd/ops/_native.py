"""Loader for the in-tree native extension (``ops/_C*.so``).

Policy: on a machine with a GPU the native path is mandatory — if the
extension is missing, or its source stamp (``_C.sources.sha256``, a content
hash of every source + build flag) does not match the current sources, it
is (re)built in-tree once (``ops/build.py``) and, if that fails or
autobuild is off (``PDMB_NO_AUTOBUILD=1`` / ``build_if_missing=False``),
every GPU op raises: a stale library is never imported silently. There is no silent eager fallback for
GPU tensors. CPU tensors never need the extension.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def load(build_if_missing: bool = True):
    """Return the ``_C`` module, building it in-tree if needed. Raises on failure."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        import torch  # noqa: F401  (loads torch's HIP runtime first)

        from . import build as _build

        stale = _build.is_stale()
        if not stale:
            try:
                _mod = importlib.import_module(f"{__package__}._C")
                return _mod
            except ImportError as e:  # not built yet
                _err = e
        else:
            _err = RuntimeError(
                f"{_build.lib_path().name} is missing or was built from different sources "
                f"(stamp {_build.stamp_path().name} does not match)")
        if build_if_missing and os.environ.get("PDMB_NO_AUTOBUILD", "0") != "1":
            # One builder at a time: torchrun starts one process per GPU and all of
            # them may find the extension missing; the others wait on the lock and
            # then import what the first one built.
            import fcntl

            lock_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), ".build.lock")
            with open(lock_path, "w") as lk:
                fcntl.flock(lk, fcntl.LOCK_EX)
                try:
                    _build.build()
                finally:
                    fcntl.flock(lk, fcntl.LOCK_UN)
            importlib.invalidate_caches()
            _mod = importlib.import_module(f"{__package__}._C")
            return _mod
        raise RuntimeError(
            "pytorch_distributed_matmul_benchmark_amd: native extension _C is not built or is "
            "stale (python -m pytorch_distributed_matmul_benchmark_amd.ops.build)") from _err


def available() -> bool:
    try:
        load(build_if_missing=False)
        return True
    except Exception:
        return False
