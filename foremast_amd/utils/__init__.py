"""Config, time helpers, metrics exporter, logging."""
