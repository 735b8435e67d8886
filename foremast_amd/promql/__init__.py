"""Prometheus access: selectors, query_range client, fake server, synthetic series."""
