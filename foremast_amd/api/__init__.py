"""Wire-compatible API types (CRDs, REST models, status tables)."""

from . import crd, rest, status  # noqa: F401
from .gojson import from_go, to_go  # noqa: F401
