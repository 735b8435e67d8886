"""Minimal PromQL instant-vector selector parsing and matching.

Foremast only issues plain selectors (``metricsquery.go:56-78``)::

    namespace_pod:<metric>{namespace="ns",pod=~"a|b"}
    namespace_app_per_pod:<metric>{namespace="ns",app="demo"}

Supported matchers: ``=``, ``!=``, ``=~``, ``!~`` (regex anchored as in
Prometheus).
"""

from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Dict, List, Tuple

_SEL = re.compile(r"^\s*([a-zA-Z_:][a-zA-Z0-9_:]*)?\s*(\{(.*)\})?\s*$", re.S)
_MATCH = re.compile(r'\s*([a-zA-Z_][a-zA-Z0-9_]*)\s*(=~|!~|!=|=)\s*"((?:[^"\\]|\\.)*)"\s*,?')


class SelectorError(ValueError):
    pass


@dataclass(frozen=True)
class Selector:
    name: str
    matchers: Tuple[Tuple[str, str, str], ...]

    def matches(self, metric: Dict[str, str]) -> bool:
        if self.name and metric.get("__name__") != self.name:
            return False
        for label, op, val in self.matchers:
            have = metric.get(label, "")
            if op == "=" and have != val:
                return False
            if op == "!=" and have == val:
                return False
            if op == "=~" and not re.fullmatch(val, have):
                return False
            if op == "!~" and re.fullmatch(val, have):
                return False
        return True


def parse_selector(q: str) -> Selector:
    m = _SEL.match(q)
    if not m:
        raise SelectorError(f"unsupported query {q!r}")
    name = m.group(1) or ""
    body = m.group(3) or ""
    matchers: List[Tuple[str, str, str]] = []
    pos = 0
    body = body.strip()
    while pos < len(body):
        mm = _MATCH.match(body, pos)
        if not mm:
            raise SelectorError(f"bad matcher in {q!r} at {body[pos:]!r}")
        matchers.append((mm.group(1), mm.group(2), bytes(mm.group(3), "utf-8").decode("unicode_escape")))
        pos = mm.end()
    if not name and not matchers:
        raise SelectorError("empty selector")
    return Selector(name=name, matchers=tuple(matchers))
