"""Deployment bundle: CRDs, RBAC, workloads, recording rules, default
DeploymentMetadata — generated from the code's own type and query tables so
the manifests cannot drift from the wire format (``python -m foremast_amd.deploy``
renders ``deploy/``)."""
