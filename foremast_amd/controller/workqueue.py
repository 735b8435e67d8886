"""Rate-limited work queue + worker pool (the client-go ``workqueue`` pattern).

The reference wires a ``RateLimitingInterface`` and 2 workers into Barrelman
whose ``syncHandler`` only records a "Synced" event
(``foremast-barrelman/pkg/controller/Barrelman.go:906-1062``).  This is the
asyncio equivalent with the semantics that matter:

* a key is queued at most once while waiting (dedup), and never processed by
  two workers at once — a key re-added while in flight is re-queued when its
  worker calls :meth:`done`;
* per-key exponential backoff on failure (``base * 2**n`` capped at ``cap``),
  reset by :meth:`forget`; ``max_retries`` drops a poison key.
"""

from __future__ import annotations

import asyncio
import logging
from typing import Awaitable, Callable, Dict, Hashable, List, Optional, Set

log = logging.getLogger("foremast.workqueue")


class RateLimitingQueue:
    def __init__(self, base_delay: float = 0.005, max_delay: float = 1000.0) -> None:
        self._q: asyncio.Queue = asyncio.Queue()
        self._waiting: Set[Hashable] = set()
        self._processing: Set[Hashable] = set()
        self._dirty: Set[Hashable] = set()
        self._failures: Dict[Hashable, int] = {}
        self.base, self.cap = base_delay, max_delay
        self._shutdown = False

    def add(self, key: Hashable) -> None:
        if self._shutdown:
            return
        if key in self._processing:
            self._dirty.add(key)
            return
        if key in self._waiting:
            return
        self._waiting.add(key)
        self._q.put_nowait(key)

    def add_rate_limited(self, key: Hashable) -> float:
        n = self._failures.get(key, 0)
        self._failures[key] = n + 1
        delay = min(self.base * (2 ** n), self.cap)
        asyncio.get_running_loop().call_later(delay, self.add, key)
        return delay

    def num_requeues(self, key: Hashable) -> int:
        return self._failures.get(key, 0)

    def forget(self, key: Hashable) -> None:
        self._failures.pop(key, None)

    async def get(self) -> Optional[Hashable]:
        key = await self._q.get()
        if key is None:
            return None
        self._waiting.discard(key)
        self._processing.add(key)
        return key

    def done(self, key: Hashable) -> None:
        self._processing.discard(key)
        if key in self._dirty:
            self._dirty.discard(key)
            self.add(key)

    def __len__(self) -> int:
        return len(self._waiting)

    def shutdown(self, workers: int) -> None:
        self._shutdown = True
        for _ in range(workers):
            self._q.put_nowait(None)


async def run_workers(queue: RateLimitingQueue, handler: Callable[[Hashable], Awaitable[None]],
                      workers: int = 2, max_retries: int = 5) -> List[asyncio.Task]:
    """Start ``workers`` tasks draining ``queue`` into ``handler``."""

    async def worker(i: int) -> None:
        while True:
            key = await queue.get()
            if key is None:
                return
            try:
                await handler(key)
                queue.forget(key)
            except Exception as e:  # noqa: BLE001 — retry with backoff, then drop
                if queue.num_requeues(key) < max_retries:
                    log.info("sync %s failed (%s), retrying", key, e)
                    queue.add_rate_limited(key)
                else:
                    log.warning("dropping %s after %d retries: %s", key, max_retries, e)
                    queue.forget(key)
            finally:
                queue.done(key)

    return [asyncio.create_task(worker(i)) for i in range(workers)]
