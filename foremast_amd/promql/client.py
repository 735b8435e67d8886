"""Prometheus ``query_range`` client used by the brain.

The job documents already carry fully-built URLs (``alias== <endpoint>
query_range?query=...&start=..&end=..&step=..``, built by the service); the
client fetches them concurrently (asyncio + httpx), decodes the matrix with
the native parser, and returns columnar arrays.  A pluggable ``transport``
routes requests to an in-process fake Prometheus in tests.
"""

from __future__ import annotations

import asyncio
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

import httpx
import numpy as np

from ..ingest import native


@dataclass
class Series:
    labels: Dict[str, str]
    ts: np.ndarray      # float64 seconds
    values: np.ndarray  # float32


class FetchError(RuntimeError):
    pass


class PromClient:
    def __init__(self, transport: Any = None, timeout: float = 90.0, concurrency: int = 32) -> None:
        self.transport = transport
        self.timeout = timeout
        self._sem = asyncio.Semaphore(concurrency)
        self.bytes_fetched = 0
        self.requests = 0

    def _client(self) -> httpx.AsyncClient:
        kw: Dict[str, Any] = {"timeout": self.timeout}
        if self.transport is not None:
            kw["transport"] = self.transport
        return httpx.AsyncClient(**kw)

    async def fetch(self, url: str, client: Optional[httpx.AsyncClient] = None) -> List[Series]:
        async with self._sem:
            try:
                if client is None:
                    async with self._client() as c:
                        resp = await c.get(url)
                else:
                    resp = await client.get(url)
            except httpx.HTTPError as e:
                raise FetchError(f"GET {url}: {e}") from e
        self.requests += 1
        self.bytes_fetched += len(resp.content)
        if resp.status_code != 200:
            raise FetchError(f"GET {url}: HTTP {resp.status_code}")
        try:
            parsed = native.parse_matrix(resp.content)
        except native.ParseError as e:
            raise FetchError(f"GET {url}: {e}") from e
        return [Series(labels=l, ts=t, values=v) for l, t, v in parsed]

    async def fetch_raw(self, url: str, client: httpx.AsyncClient) -> bytes:
        """Body of one query_range call (decoded by the caller, e.g. the keyed
        native scatter straight into a staging block)."""
        async with self._sem:
            try:
                resp = await client.get(url)
            except httpx.HTTPError as e:
                raise FetchError(f"GET {url}: {e}") from e
        self.requests += 1
        self.bytes_fetched += len(resp.content)
        if resp.status_code != 200:
            raise FetchError(f"GET {url}: HTTP {resp.status_code}")
        return resp.content

    async def fetch_raw_many(self, urls: Sequence[str]) -> List[Any]:
        """Bodies (or the exception) of concurrent query_range calls."""
        async with self._client() as c:
            return await asyncio.gather(*(self.fetch_raw(u, c) for u in urls), return_exceptions=True)

    async def fetch_many(self, urls: Sequence[str]) -> List[Any]:
        """Fetch concurrently; each result is a list of Series or the exception."""
        async with self._client() as c:
            return await asyncio.gather(*(self.fetch(u, c) for u in urls), return_exceptions=True)
