"""Ingest: Prometheus matrix parsing (native C++) and HBM ring buffers."""

from .ringbuffer import HistoryRing, WindowRing  # noqa: F401
