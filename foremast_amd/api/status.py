"""Status-mapping tables.

Two tables exist in the reference and both are part of the contract:

* the service's internal→external map
  (``foremast-service/pkg/converter/converter.go:11-30``);
* barrelman's external→phase map
  (``foremast-barrelman/pkg/client/analyst/analystclient.go:211-230``).

Q4: ``completed_unknown`` maps to ``abort`` in the
service; barrelman's own table would give ``Warning``.  We replicate the
service mapping and also accept ``completed_unknown`` directly on the
barrelman side.
"""

from __future__ import annotations

from . import crd
from . import rest as r

EXT_NEW = "new"
EXT_INPROGRESS = "inprogress"
EXT_SUCCESS = "success"
EXT_ANOMALY = "anomaly"
EXT_ABORT = "abort"
EXT_UNKNOWN = "unknown"

_INTERNAL_TO_EXTERNAL = {
    r.ST_INITIAL: EXT_NEW,
    r.ST_PREPROCESS_INPROGRESS: EXT_INPROGRESS,
    r.ST_POSTPROCESS_INPROGRESS: EXT_INPROGRESS,
    r.ST_PREPROCESS_COMPLETED: EXT_INPROGRESS,
    r.ST_COMPLETED_HEALTH: EXT_SUCCESS,
    r.ST_COMPLETED_UNHEALTH: EXT_ANOMALY,
    r.ST_COMPLETED_UNKNOWN: EXT_ABORT,
    r.ST_PREPROCESS_FAILED: EXT_ABORT,
    r.ST_ABORT: EXT_ABORT,
}


def internal_to_external(status: str) -> str:
    """``ConvertStatusToExternal``: unknown internal states read as in-progress."""
    return _INTERNAL_TO_EXTERNAL.get(status, EXT_INPROGRESS)


_EXTERNAL_TO_PHASE = {
    "created": crd.PHASE_RUNNING,
    "initial": crd.PHASE_RUNNING,
    EXT_NEW: crd.PHASE_RUNNING,
    EXT_INPROGRESS: crd.PHASE_RUNNING,
    EXT_UNKNOWN: crd.PHASE_RUNNING,
    r.ST_COMPLETED_HEALTH: crd.PHASE_HEALTHY,
    EXT_SUCCESS: crd.PHASE_HEALTHY,
    r.ST_COMPLETED_UNHEALTH: crd.PHASE_UNHEALTHY,
    EXT_ANOMALY: crd.PHASE_UNHEALTHY,
    EXT_ABORT: crd.PHASE_ABORT,
    r.ST_COMPLETED_UNKNOWN: crd.PHASE_WARNING,
}


def external_to_phase(status: str) -> str:
    """Barrelman ``GetStatus`` mapping; unmapped strings pass through."""
    return _EXTERNAL_TO_PHASE.get(status, status)
