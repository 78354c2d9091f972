"""Resource allocator REST service on :55589 (reference resource_allocator.go:41-74,
pkg/allocator/main.go:13-26): ``POST /allocation`` with an ``AllocationRequest`` JSON body ->
``{"job": n}``; ``GET /metrics``."""
from __future__ import annotations

import argparse
import json
import logging

from ..common.store import open_store
from ..common.types import PORT_ALLOCATOR
from ..utils.http import HttpServer, Router, as_json, text
from .allocator import AllocationRequest, ResourceAllocator


def allocator_router(alloc: ResourceAllocator) -> Router:
    r = Router()

    def allocate(body, _q):
        try:
            req = AllocationRequest.from_dict(json.loads(body))
        except (KeyError, TypeError, ValueError, json.JSONDecodeError) as e:
            return text(400, f"bad allocation request: {e}\n")
        try:
            return as_json(200, alloc.allocate(req))
        except KeyError as e:
            return text(400, f"{e}\n")
        except Exception as e:  # policy invariant violation etc.: the scheduler retries
            return text(500, f"allocation failed: {e}\n")

    r.add("POST", "/allocation", allocate)
    r.add("GET", "/metrics", lambda b, q: (200, "text/plain; version=0.0.4", alloc.metrics.exposition()))
    return r


def main(argv=None):
    ap = argparse.ArgumentParser("vodascheduler-allocator")
    ap.add_argument("--port", type=int, default=PORT_ALLOCATOR)
    ap.add_argument("--store", default="memory://", help="memory:// or sqlite:///path")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    srv = HttpServer(allocator_router(ResourceAllocator(open_store(a.store))), port=a.port, name="allocator")
    logging.info("resource allocator listening on :%d", srv.port)
    srv.serve_forever()


if __name__ == "__main__":
    main()
