"""Barrelman equivalent: Deployment watcher, status poller, query builder,
analyst client and remediation."""
