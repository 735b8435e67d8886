"""foremast_amd — an MI355X-native application-health anomaly engine.

Capabilities of Foremast (pzou1974/foremast-1, a fork of intuit/foremast):

* ``api``        — DeploymentMonitor / DeploymentMetadata CRD types and the
                   foremast-service REST wire format (wire-compatible).
* ``store``      — job store with Elasticsearch-document semantics (memory,
                   SQLite, ES-HTTP) and lease-based claims.
* ``service``    — the ``/v1/healthcheck`` REST front end and the Prometheus
                   query proxy.
* ``controller`` — the barrelman equivalent: Deployment watcher, status
                   poller, PromQL query builder, remediation.
* ``k8s``        — KubeAPI protocol, an in-memory fake cluster and an HTTP
                   adapter for a real API server.
* ``promql``     — query_range client, fake Prometheus, synthetic series.
* ``ingest``     — native (C++) Prometheus matrix parser and the HBM ring
                   buffer the scorers read from.
* ``models``     — the brain's scorers as batched models: moving average,
                   (double) exponential smoothing, Holt-Winters, bivariate
                   normal, LSTM autoencoder, Prophet-style regression, and
                   the pairwise rank tests.
* ``ops``        — hand-written HIP kernels for gfx950 (CDNA4) plus their
                   pure-PyTorch references.
* ``parallel``   — one process per GPU over RCCL/xGMI: series sharding, the
                   fused per-tick health collective, LSTM-AE data parallel.
* ``brain``      — the job loop (claim → fetch → fit → pairwise → detect →
                   verdict → export).
* ``utils``      — config (brain env-var names), metrics exporter, logging.
"""

__version__ = "0.1.0"
