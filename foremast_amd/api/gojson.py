"""Go ``encoding/json`` semantics for dataclasses.

The reference's wire formats are defined by Go structs whose JSON shape is
decided by struct tags (``json:"name,omitempty"``).  To stay wire-compatible
we declare each type as a dataclass whose fields carry the Go tag, and
serialise with Go's rules:

* ``omitempty`` drops ``false``, ``0``, ``""``, ``None`` and empty
  lists/maps — but never a nested struct (Go never treats a struct value as
  empty);
* a nil slice/map without ``omitempty`` marshals as ``null``;
* map keys are emitted in sorted order (Go sorts map keys).

Malformed tags in the reference such as ``json:"anomaly",omitempty``
(``foremast-service/pkg/models/models.go:71``) parse in Go as the name with
*no* options, so those fields are declared here without ``omitempty``.
"""

from __future__ import annotations

import dataclasses
import typing
from typing import Any, Dict, Optional, get_args, get_origin, get_type_hints


def gofield(name: str, omitempty: bool = False, default: Any = dataclasses.MISSING,
            default_factory: Any = dataclasses.MISSING) -> Any:
    """A dataclass field carrying a Go JSON tag."""
    md = {"json": name, "omitempty": omitempty}
    if default_factory is not dataclasses.MISSING:
        return dataclasses.field(default_factory=default_factory, metadata=md)
    if default is dataclasses.MISSING:
        default = None
    return dataclasses.field(default=default, metadata=md)


def _is_empty(v: Any) -> bool:
    if v is None:
        return True
    if isinstance(v, bool):
        return v is False
    if isinstance(v, (int, float)):
        return v == 0
    if isinstance(v, (str, list, tuple, dict)):
        return len(v) == 0
    return False  # structs are never empty


def to_go(v: Any) -> Any:
    """Convert a value to its Go-JSON-compatible Python representation."""
    if dataclasses.is_dataclass(v) and not isinstance(v, type):
        out: Dict[str, Any] = {}
        for f in dataclasses.fields(v):
            name = f.metadata.get("json")
            if name is None:
                continue
            val = getattr(v, f.name)
            if name == "":  # inline (e.g. TypeMeta)
                inner = to_go(val)
                if isinstance(inner, dict):
                    out.update(inner)
                continue
            if f.metadata.get("omitempty") and _is_empty(val):
                continue
            out[name] = to_go(val)
        return out
    if isinstance(v, dict):
        return {k: to_go(v[k]) for k in sorted(v)}
    if isinstance(v, (list, tuple)):
        return [to_go(x) for x in v]
    return v


_HINTS_CACHE: Dict[type, Dict[str, Any]] = {}


def _hints(cls: type) -> Dict[str, Any]:
    h = _HINTS_CACHE.get(cls)
    if h is None:
        h = get_type_hints(cls)
        _HINTS_CACHE[cls] = h
    return h


def _coerce(tp: Any, v: Any) -> Any:
    if v is None:
        return None
    origin = get_origin(tp)
    if origin is typing.Union:
        args = [a for a in get_args(tp) if a is not type(None)]
        return _coerce(args[0], v) if args else v
    if origin in (list, typing.List):
        (et,) = get_args(tp) or (Any,)
        return [_coerce(et, x) for x in v]
    if origin in (dict, typing.Dict):
        args = get_args(tp)
        vt = args[1] if len(args) == 2 else Any
        return {k: _coerce(vt, x) for k, x in v.items()}
    if isinstance(tp, type) and dataclasses.is_dataclass(tp):
        return from_go(tp, v)
    if tp is int and isinstance(v, (int, float)) and not isinstance(v, bool):
        return int(v)
    if tp is float and isinstance(v, (int, float)) and not isinstance(v, bool):
        return float(v)
    return v


def from_go(cls: type, d: Optional[Dict[str, Any]]) -> Any:
    """Build dataclass ``cls`` from a decoded JSON object (unknown keys ignored,
    as Go's decoder does)."""
    if d is None:
        d = {}
    hints = _hints(cls)
    kwargs: Dict[str, Any] = {}
    for f in dataclasses.fields(cls):
        name = f.metadata.get("json")
        if name is None:
            continue
        if name == "":
            kwargs[f.name] = from_go(hints[f.name], d)
            continue
        if name in d:
            kwargs[f.name] = _coerce(hints[f.name], d[name])
    return cls(**kwargs)
