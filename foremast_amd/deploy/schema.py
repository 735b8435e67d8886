"""OpenAPI v3 structural schemas for the Foremast CRDs, derived from the
Go-tagged dataclasses in :mod:`foremast_amd.api.crd`.

The reference hand-maintains ``deploy/foremast/1_crds/*.yaml`` next to the Go
types (``foremast-barrelman/pkg/apis/deployment/v1alpha1/types.go``).  Here the
schema is computed from the same field table the JSON codec uses: a field
without ``omitempty`` is ``required`` (Go always emits it), ``int`` becomes
``integer``/int64, nested structs become nested ``object`` schemas, free-form
maps (the label selector) keep unknown fields.
"""

from __future__ import annotations

import dataclasses
import typing
from typing import Any, Dict, get_args, get_origin, get_type_hints

from ..api import crd


def _schema_of_type(tp: Any) -> Dict[str, Any]:
    origin = get_origin(tp)
    if origin is typing.Union:  # Optional[X]
        args = [a for a in get_args(tp) if a is not type(None)]
        return _schema_of_type(args[0]) if len(args) == 1 else {"x-kubernetes-preserve-unknown-fields": True}
    if tp is str:
        return {"type": "string"}
    if tp is bool:
        return {"type": "boolean"}
    if tp is int:
        return {"type": "integer", "format": "int64"}
    if tp is float:
        return {"type": "number"}
    if origin in (list, typing.List):
        return {"type": "array", "items": _schema_of_type(get_args(tp)[0])}
    if origin in (dict, typing.Dict):
        k, v = get_args(tp)
        if v is str:
            return {"type": "object", "additionalProperties": {"type": "string"}}
        return {"type": "object", "x-kubernetes-preserve-unknown-fields": True}
    if dataclasses.is_dataclass(tp):
        return schema_of(tp)
    return {"x-kubernetes-preserve-unknown-fields": True}


def schema_of(cls) -> Dict[str, Any]:
    hints = get_type_hints(cls)
    props: Dict[str, Any] = {}
    required = []
    for f in dataclasses.fields(cls):
        name = f.metadata.get("json")
        if not name:
            continue
        props[name] = _schema_of_type(hints[f.name])
        if not f.metadata.get("omitempty", False):
            required.append(name)
    out: Dict[str, Any] = {"type": "object", "properties": props}
    if required:
        out["required"] = required
    return out


def crd_manifest(kind: str, plural: str, spec_cls, status_cls, short_names=(), printer_columns=(),
                 selectable=()) -> Dict[str, Any]:
    group, version = crd.API_VERSION.split("/")
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{plural}.{group}"},
        "spec": {
            "group": group,
            "scope": "Namespaced",
            "names": {"kind": kind, "plural": plural, "singular": kind.lower(), "listKind": kind + "List",
                      "shortNames": list(short_names)},
            "versions": [{
                "name": version, "served": True, "storage": True,
                "subresources": {"status": {}},
                "additionalPrinterColumns": list(printer_columns),
                **({"selectableFields": [{"jsonPath": p} for p in selectable]} if selectable else {}),
                "schema": {"openAPIV3Schema": {
                    "type": "object",
                    "properties": {
                        "apiVersion": {"type": "string"}, "kind": {"type": "string"},
                        "metadata": {"type": "object"},
                        "spec": schema_of(spec_cls),
                        "status": schema_of(status_cls),
                    },
                }},
            }],
        },
    }


def crds(selectable: bool = False):
    """The two CRDs.  ``selectable``: declare the reference's field labels
    (``status.jobId``, ``status.phase``) as ``selectableFields`` — needs
    Kubernetes >= 1.31 (1.30 behind the CustomResourceFieldSelectors gate);
    older API servers reject the unknown field under strict validation, so the
    default bundle leaves it out (``deploy/optional/crds-selectable.yaml`` has it)."""
    return [
        crd_manifest("DeploymentMetadata", "deploymentmetadatas", crd.DeploymentMetadataSpec,
                     crd.DeploymentMetadataStatus, short_names=("dmd",)),
        crd_manifest("DeploymentMonitor", "deploymentmonitors", crd.DeploymentMonitorSpec,
                     crd.DeploymentMonitorStatus, short_names=("dm",),
                     printer_columns=[
                         {"name": "Phase", "type": "string", "jsonPath": ".status.phase"},
                         {"name": "Job", "type": "string", "jsonPath": ".status.jobId"},
                         {"name": "Remediated", "type": "boolean", "jsonPath": ".status.remediationTaken"},
                     ],
                     # the reference's field labels (v1alpha1/register.go:38-53)
                     selectable=(".status.jobId", ".status.phase") if selectable else ()),
    ]


def validate(obj: Any, schema: Dict[str, Any], path: str = "") -> list:
    """Minimal structural validation (types + required), enough to check that
    what the controller writes is accepted by the CRD."""
    errs = []
    if schema.get("x-kubernetes-preserve-unknown-fields") and "type" not in schema:
        return errs
    t = schema.get("type")
    py = {"string": str, "boolean": bool, "integer": int, "number": (int, float), "array": list, "object": dict}
    if t and obj is not None and not isinstance(obj, py[t]):
        return [f"{path or '.'}: expected {t}, got {type(obj).__name__}"]
    if t == "integer" and isinstance(obj, bool):
        return [f"{path}: expected integer, got bool"]
    if t == "object" and isinstance(obj, dict):
        for r in schema.get("required", []):
            if r not in obj:
                errs.append(f"{path}.{r}: required")
        for k, v in obj.items():
            sub = schema.get("properties", {}).get(k)
            if sub is None and isinstance(schema.get("additionalProperties"), dict):
                sub = schema["additionalProperties"]
            if sub is not None:
                errs += validate(v, sub, f"{path}.{k}")
    if t == "array" and isinstance(obj, list):
        for i, v in enumerate(obj):
            errs += validate(v, schema.get("items", {}), f"{path}[{i}]")
    return errs
