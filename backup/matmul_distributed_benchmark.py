#!/usr/bin/env python3
"""CLI-compatible entry point (reference: /root/reference/backup/matmul_distributed_benchmark.py).

Same flags, defaults and output lines as the reference, with the
reference's bugs fixed. See
pytorch_distributed_matmul_benchmark_amd/runner.py.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_matmul_benchmark_amd.runner import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main("distributed"))
