"""RFC3339 helpers matching Go's ``time.Format(time.RFC3339)`` / ``time.Parse``."""

from __future__ import annotations

import re
import time
from datetime import datetime, timedelta, timezone

_RFC3339 = re.compile(
    r"^(\d{4})-(\d{2})-(\d{2})[Tt](\d{2}):(\d{2}):(\d{2})(\.\d+)?([Zz]|[+-]\d{2}:\d{2})$")


class TimeFormatError(ValueError):
    pass


def parse_rfc3339(s: str) -> datetime:
    """Parse like Go ``time.Parse(time.RFC3339, s)``; raises on bad input
    (the reference service ``log.Fatal``s here — Q5; we raise instead)."""
    m = _RFC3339.match(s.strip()) if isinstance(s, str) else None
    if not m:
        raise TimeFormatError(f"cannot parse {s!r} as RFC3339")
    y, mo, d, hh, mm, ss, frac, tz = m.groups()
    us = 0
    if frac:
        us = int((frac[1:] + "000000")[:6])
    if tz in ("Z", "z"):
        tzinfo = timezone.utc
    else:
        sign = 1 if tz[0] == "+" else -1
        tzinfo = timezone(sign * timedelta(hours=int(tz[1:3]), minutes=int(tz[4:6])))
    return datetime(int(y), int(mo), int(d), int(hh), int(mm), int(ss), us, tzinfo=tzinfo)


def to_unix(s: str) -> float:
    return parse_rfc3339(s).timestamp()


def format_rfc3339(t: float | None = None, local: bool = False) -> str:
    """Go ``time.Now().Format(time.RFC3339)`` (second precision)."""
    if t is None:
        t = time.time()
    dt = datetime.fromtimestamp(int(t), tz=timezone.utc)
    if local:
        dt = dt.astimezone()
    s = dt.isoformat()
    return s.replace("+00:00", "Z")


def format_rfc3339_nano(t: float | None = None) -> str:
    """Go ``time.Time`` JSON encoding (RFC3339Nano, trailing zeros trimmed)."""
    if t is None:
        t = time.time()
    dt = datetime.fromtimestamp(t, tz=timezone.utc)
    base = dt.strftime("%Y-%m-%dT%H:%M:%S")
    if dt.microsecond:
        base += ("." + f"{dt.microsecond:06d}").rstrip("0")
    return base + "Z"
