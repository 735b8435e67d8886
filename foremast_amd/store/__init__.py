"""Job store (ES-document semantics, lease-based claims)."""

from .jobstore import (JobStore, MemoryJobStore, SqliteJobStore, is_claimable,  # noqa: F401
                       job_id_for, new_document, open_store)
