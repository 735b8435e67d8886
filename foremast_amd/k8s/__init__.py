"""Kubernetes access: protocol, in-memory fake cluster, HTTP adapter."""
from .api import ApiError, Conflict, KubeAPI, NotFound  # noqa: F401
