"""``python -m foremast_amd.service`` — serve the job API on :8099.

Environment (same names as ``foremast-service/cmd/manager/main.go:236-244``):
``ELASTIC_URL`` (an ES endpoint, or ``sqlite:///path`` / ``memory://`` via
``FOREMAST_JOB_STORE``) and ``QUERY_SERVICE_ENDPOINT``.
"""

import os

import uvicorn

from .app import create_app


def main() -> None:
    port = int(os.environ.get("FOREMAST_SERVICE_PORT", "8099"))
    uvicorn.run(create_app(), host="0.0.0.0", port=port, log_level="info")


if __name__ == "__main__":
    main()
