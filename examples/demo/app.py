#!/usr/bin/env python
"""Demo service with a built-in fault injector (reference C30:
``examples/spring-boot-demo`` — ``ErrorGenerator`` / ``FileErrorGenerator``).

* ``GET /`` and ``GET /queue/...`` answer 200 (the healthy path);
* ``GET /error5xx`` answers 500, unknown paths 404;
* ``--error-type 5xx|4xx --frequency N`` makes a background task call the
  failing endpoint N times per second (v2 "bad release");
* ``--rate-file FILE`` replays one error rate (calls/s) per line, one line
  per ``--tick`` seconds — e.g. ``data/spike_rates.txt`` holds a quiet
  baseline with two ~40/s bursts.

Metrics (``http_server_requests_seconds_*`` with ``app``/``status`` tags) are
exposed at ``/actuator/prometheus`` by :class:`foremast_amd.instrument.ForemastMetrics`.

    APP_NAME=demo python examples/demo/app.py --error-type 5xx --frequency 5
"""

from __future__ import annotations

import argparse
import asyncio
import os
import sys
from typing import List, Optional

import httpx
from fastapi import FastAPI
from fastapi.responses import JSONResponse

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from foremast_amd.instrument import ForemastMetrics  # noqa: E402


def build_app(app_name: str = "demo"):
    api = FastAPI(title="foremast-demo")
    queue: List[str] = []

    @api.get("/")
    async def root():
        return {"status": "ok"}

    @api.get("/queue/offer/{item}")
    async def offer(item: str):
        queue.append(item)
        return {"size": len(queue)}

    @api.get("/queue/poll")
    async def poll():
        return {"item": queue.pop(0) if queue else None}

    @api.get("/error5xx")
    async def error5xx():
        return JSONResponse(status_code=500, content={"error": "injected"})

    return ForemastMetrics(api, app_name=app_name)


def read_rates(path: str) -> List[float]:
    with open(path) as f:
        return [float(x) for x in (ln.strip() for ln in f) if x and not x.startswith("#")]


class FaultInjector:
    """Calls the failing endpoint at a fixed frequency or a replayed rate."""

    def __init__(self, client: httpx.AsyncClient, error_type: str = "5xx", frequency: float = 0.0,
                 rates: Optional[List[float]] = None, tick: float = 1.0, speed: float = 1.0) -> None:
        self.client = client
        self.url = "/error5xx" if error_type == "5xx" else "/not_existed"
        self.frequency, self.rates, self.tick, self.speed = frequency, rates, tick, speed
        self.sent = 0

    async def _burst(self, rate: float, seconds: float) -> None:
        n = int(round(rate * seconds))
        wall = seconds / self.speed  # `speed` > 1 replays faster than real time (tests, demos)
        gap = wall / max(n, 1)
        for _ in range(n):
            await self.client.get(self.url, params={"t": self.sent})
            self.sent += 1
            await asyncio.sleep(gap)
        if n == 0:
            await asyncio.sleep(wall)

    async def run(self, stop: asyncio.Event) -> None:
        i = 0
        while not stop.is_set():
            if self.rates is not None:
                if i >= len(self.rates):
                    return
                await self._burst(self.rates[i], self.tick)
                i += 1
            elif self.frequency > 0:
                await self._burst(self.frequency, self.tick)
            else:
                return


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--port", type=int, default=8080)
    p.add_argument("--error-type", choices=["5xx", "4xx"], default="5xx")
    p.add_argument("--frequency", type=float, default=0.0)
    p.add_argument("--rate-file", default=None)
    p.add_argument("--tick", type=float, default=1.0)
    args = p.parse_args()
    import uvicorn
    app = build_app(os.environ.get("APP_NAME", "demo"))

    async def serve():
        server = uvicorn.Server(uvicorn.Config(app, host="0.0.0.0", port=args.port))
        stop = asyncio.Event()
        inj = None
        if args.frequency or args.rate_file:
            client = httpx.AsyncClient(base_url=f"http://127.0.0.1:{args.port}")
            inj = FaultInjector(client, args.error_type, args.frequency,
                                read_rates(args.rate_file) if args.rate_file else None, args.tick)
        tasks = [asyncio.create_task(server.serve())]
        if inj:
            tasks.append(asyncio.create_task(inj.run(stop)))
        await asyncio.gather(*tasks)

    asyncio.run(serve())


if __name__ == "__main__":
    main()
