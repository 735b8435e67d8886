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


class CollectiveTimeout(RuntimeError):
    """A collective did not complete within its deadline (a peer is dead or stopped)."""


def wait_bounded(work, timeout_s: float, what: str = "collective") -> None:
    """Wait for an ``async_op=True`` work handle on the HOST with a deadline.

    ``work.wait()`` on an RCCL (``nccl``) work only makes the current stream wait;
    the host then blocks in the next D2H copy until the watchdog fires and, by
    default, tears the process down.  Polling ``is_completed()`` (a non-blocking
    event query) keeps the host in control: a dead or stopped peer surfaces as
    :class:`CollectiveTimeout` after ``timeout_s``, the caller aborts the
    communicator and re-forms the group (``parallel/elastic.py``)."""
    import time
    t_end = time.monotonic() + timeout_s
    spin_until = time.monotonic() + 0.002
    while not work.is_completed():
        now = time.monotonic()
        if now > t_end:
            raise CollectiveTimeout(f"{what} did not complete within {timeout_s:.1f} s")
        time.sleep(0 if now < spin_until else 0.0005)
    try:
        work.wait()  # completed: returns at once, or raises the backend's error
    except Exception as e:  # noqa: BLE001 - the peer's death surfaces as a backend error
        raise CollectiveTimeout(f"{what} failed: {e}") from e


def exchange_timeout_s() -> float:
    """Deadline of the per-tick exchange (``FOREMAST_EXCHANGE_TIMEOUT_S``, default
    ``FOREMAST_HEARTBEAT_S``): with 2 x heartbeat as the staleness horizon, the
    survivors re-form within about 2 x heartbeat of a peer's death."""
    return float(os.environ.get("FOREMAST_EXCHANGE_TIMEOUT_S", os.environ.get("FOREMAST_HEARTBEAT_S", "5")))


_FAULT_COUNTS: dict = {}


def fault_point(name: str) -> None:
    """Fault injection: ``FOREMAST_FAULT=<name>:<n>`` SIGSTOPs this
    process at the n-th time it reaches point ``name`` — e.g. ``exchange:3``
    freezes a rank INSIDE its 3rd health exchange, after its all-gather was
    issued, to test how the survivors' deadlines and re-formation behave."""
    spec = os.environ.get("FOREMAST_FAULT", "")
    if not spec.startswith(name + ":"):
        return
    n = _FAULT_COUNTS.get(name, 0) + 1
    _FAULT_COUNTS[name] = n
    if n == int(spec.split(":", 1)[1]):
        import signal
        os.kill(os.getpid(), signal.SIGSTOP)
