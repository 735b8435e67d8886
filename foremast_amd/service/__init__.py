"""foremast-service equivalent: REST job API + Prometheus query proxy."""

from .app import create_app, lookup, register, status_response  # noqa: F401
