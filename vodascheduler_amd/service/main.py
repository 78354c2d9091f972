"""Training-service process (reference pkg/service/main.go:13-26): REST on :55587.

    python -m vodascheduler_amd.service.main --store sqlite:///var/lib/voda/jobs.db \
        --mq sqlite:///var/lib/voda/mq.db
"""
from __future__ import annotations

import argparse
import logging

from ..common.mq import open_queue
from ..common.store import open_store
from ..common.types import PORT_TRAINING_SERVICE
from ..utils.http import HttpServer
from .service import TrainingService


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("vodascheduler-service")
    ap.add_argument("--port", type=int, default=PORT_TRAINING_SERVICE)
    ap.add_argument("--store", default="memory://", help="memory:// or sqlite:///path")
    ap.add_argument("--mq", default="inproc://", help="inproc:// or sqlite:///path (shared with the scheduler)")
    ap.add_argument("--log-level", default="INFO")
    a = ap.parse_args(argv)
    logging.basicConfig(level=a.log_level.upper(), format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    svc = TrainingService(open_store(a.store), open_queue(a.mq))
    srv = HttpServer(svc.router(), port=a.port, name="training-service")
    logging.info("training service listening on :%d", srv.port)
    srv.serve_forever()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
