"""When to issue collectives.

Every collective in this package is skipped in a 1-rank job — except with
``FOREMAST_FORCE_COLLECTIVES=1``, where a 1-rank process group runs them all
(all-gather, all-reduce, all-to-all, broadcast) exactly as N ranks would.  On
one GPU that exercises the real RCCL path (backend ``nccl``: communicator
set-up, the dtypes and split sizes each call uses, stream ordering) that the
driver's 8-GPU run depends on — ``tests/test_rccl_gpu.py``.
"""

from __future__ import annotations

import os

import torch.distributed as dist


def force_collectives() -> bool:
    return os.environ.get("FOREMAST_FORCE_COLLECTIVES", "0") == "1"


def world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def active(group=None) -> bool:
    """A process group exists and has more than one rank (or collectives are forced)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or force_collectives()
