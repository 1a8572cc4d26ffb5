"""Test-only fault-injection switches (``PDMB_TEST_*`` environment variables).

The negative controls of the overlap / IPC checks remove a producer
dependency on purpose (parallel/overlap.py ``PDMB_TEST_SKIP_READY_WAIT``,
parallel/ipc.py ``PDMB_TEST_IPC_SKIP_B0``), so a run with one of them set
computes racy collectives and meaningless timings. ``bench.py`` refuses to
run with any of them set; the CLIs (runner.py) print a warning and record
them in every JSON record, so such a run can never pass for a measurement.
"""
from __future__ import annotations

import os
from typing import Dict

PREFIX = "PDMB_TEST_"


def active() -> Dict[str, str]:
    """The ``PDMB_TEST_*`` variables set (non-empty) in this process's environment."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(PREFIX) and v != ""}
