"""Process groups (RCCL over xGMI), partitioning and event-ordered comm streams."""
from .dist import (DistContext, all_ok, barrier, cleanup_distributed, reduce_scalar,  # noqa: F401
                   setup_distributed, verify_collectives)
