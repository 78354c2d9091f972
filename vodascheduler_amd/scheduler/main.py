"""Scheduler process (reference pkg/scheduler/main.go:16-60): one per GPU type.

    python -m vodascheduler_amd.scheduler.main --gpu-type amd-instinct-mi355x \
        --store sqlite:///var/lib/voda/jobs.db --mq sqlite:///var/lib/voda/mq.db \
        --backend local --gpus 0,1,2,3,4,5,6,7 [--resume] [--algorithm ElasticFIFO] [--no-placement]

Flags mirror the reference (``-gpu``, ``-resume``, ``-algorithm``, ``-placement``; klog ``-v``
-> ``--log-level``).  ``--allocator URL`` sends allocation requests to a remote allocator
service over HTTP (``POST /allocation``, as the reference does); without it the allocator
runs in-process.  Backends: ``local`` (node agent + warm per-GPU workers, the MI355X-native
path), ``k8s`` (MPIJob CRD + pod tolerations on a Kubernetes cluster, the reference's
deployment model) and ``null`` (record actions only; the virtual-time cluster lives in
``vodascheduler simulate``).  REST on :55588:
``GET /training``, ``PUT /algorithm``, ``PUT /ratelimit``, ``GET /metrics``, ``GET /trace``.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import threading

from ..algorithm import ALGORITHMS, DEFAULT_ALGORITHM
from ..common.mq import open_queue
from ..common.store import open_store
from ..common.types import DEFAULT_GPU_TYPE, PORT_SCHEDULER, RESCHED_RATE_LIMIT_SEC, TIME_METRICS_TICK_SEC
from ..utils.http import HttpServer

log = logging.getLogger("vodascheduler_amd.scheduler")


def parse_gpus(spec: str | None, device_type: str) -> list[int]:
    if spec:
        return [int(x) for x in spec.split(",") if x.strip() != ""]
    if device_type == "cuda":
        import torch

        return list(range(torch.cuda.device_count()))  # counting devices does not initialise HIP
    return [0, 1]


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser("vodascheduler-scheduler")
    ap.add_argument("--gpu-type", "-gpu", default=DEFAULT_GPU_TYPE, help="GPU type this scheduler owns")
    ap.add_argument("--resume", action="store_true", help="reconstruct state from the store on start")
    ap.add_argument("--algorithm", default=DEFAULT_ALGORITHM, choices=sorted(ALGORITHMS))
    ap.add_argument("--no-placement", action="store_true", help="disable the Munkres placement manager")
    ap.add_argument("--rate-limit", type=float, default=RESCHED_RATE_LIMIT_SEC)
    ap.add_argument("--tick", type=float, default=TIME_METRICS_TICK_SEC)
    ap.add_argument("--strict-rate-limit", action="store_true",
                    help="rate-limit reschedules triggered by job completion too (reference behaviour)")
    ap.add_argument("--store", default="memory://", help="memory:// or sqlite:///path")
    ap.add_argument("--mq", default="inproc://", help="inproc:// or sqlite:///path")
    ap.add_argument("--allocator", default=None, help="URL of a remote allocator service")
    ap.add_argument("--backend", default="local", choices=["local", "k8s", "null"])
    ap.add_argument("--k8s-url", default=None, help="API server URL (default: in-cluster service account)")
    ap.add_argument("--k8s-token", default=os.environ.get("VODA_K8S_TOKEN"))
    ap.add_argument("--k8s-insecure", action="store_true", help="skip TLS verification of the API server")
    ap.add_argument("--namespace", default="voda-scheduler")
    ap.add_argument("--no-configmap-opt", action="store_true",
                    help="do not annotate the launcher on resize (reference -configmap_opt=false)")
    ap.add_argument("--node", default=os.environ.get("VODA_NODE", "node0"))
    ap.add_argument("--gpus", default=None, help="comma-separated GPU indices (default: all)")
    ap.add_argument("--device-type", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: workers train on CPU with gloo (simulated cluster)")
    ap.add_argument("--store-port", type=int, default=29400, help="TCPStore port of the worker pool")
    ap.add_argument("--metrics-dir", default=os.environ.get("VODA_METRICS_DIR", "/tmp/voda_metrics"))
    ap.add_argument("--log-dir", default=None, help="per-worker log files")
    ap.add_argument("--port", type=int, default=PORT_SCHEDULER)
    ap.add_argument("--log-level", default="INFO")
    return ap


class SchedulerProcess:
    """Everything the scheduler process owns; also used in-process by ``vodascheduler up``."""

    def __init__(self, a: argparse.Namespace, store=None, mq=None):
        from ..allocator.allocator import HttpAllocatorClient, ResourceAllocator
        from ..backend.base import NullBackend
        from ..scheduler.core import SchedulerCore
        from ..scheduler.runner import SchedulerRunner

        self.args = a
        self.store = store or open_store(a.store)
        self.mq = mq or open_queue(a.mq)
        self.agent = None
        self.tcp_store = None
        self.collector = None
        gpus = parse_gpus(a.gpus, a.device_type) if a.backend != "k8s" else []
        if a.backend == "local":
            from ..agent.node_agent import NodeAgent
            from ..backend.local import LocalBackend
            from ..runtime.rendezvous import connect_store

            self.tcp_store = connect_store("127.0.0.1", a.store_port, is_master=True)
            self.agent = NodeAgent(a.node, gpus, f"127.0.0.1:{a.store_port}", a.device_type, log_dir=a.log_dir,
                                   store=connect_store("127.0.0.1", a.store_port),
                                   backend="rccl" if a.device_type == "cuda" else "gloo")
            self.backend = LocalBackend(self.tcp_store, [self.agent], {"metrics_dir": a.metrics_dir})
        elif a.backend == "k8s":
            from ..backend.k8s import K8sBackend, K8sClient

            self.backend = K8sBackend(K8sClient(a.k8s_url, a.k8s_token, insecure=a.k8s_insecure), a.gpu_type,
                                      a.namespace, configmap_opt=not a.no_configmap_opt)
        else:
            self.backend = NullBackend({a.node: gpus})
        alloc = HttpAllocatorClient(a.allocator) if a.allocator else ResourceAllocator(self.store)
        self.core = SchedulerCore(a.gpu_type, self.store, alloc, self.backend, algorithm=a.algorithm,
                                  rate_limit_sec=a.rate_limit, tick_sec=a.tick, resume=a.resume,
                                  use_placement=not a.no_placement, work_conserving=not a.strict_rate_limit)
        from ..utils.tracing import SchedulerTracer

        self.tracer = SchedulerTracer(self.core)
        self.runner = SchedulerRunner(self.core, self.mq, queue_name=a.gpu_type)
        self.http: HttpServer | None = None
        self._collector_stop = threading.Event()

    def start(self, serve_http: bool = True) -> "SchedulerProcess":
        from .api import scheduler_router

        self.runner.start()
        if self.agent is not None:
            # workers join the inventory as they heartbeat (LocalBackend emits EV_NODES)
            self.agent.start()
        if serve_http:
            self.http = HttpServer(scheduler_router(self.runner, self.tracer), port=self.args.port,
                                   name="scheduler").start()
            log.info("scheduler %s listening on :%d", self.args.gpu_type, self.http.port)
        if self.args.backend == "local" and self.args.metrics_dir:
            from ..collector.collector import MetricsCollector

            self.collector = MetricsCollector(self.store, self.args.metrics_dir)

            def loop():
                while not self._collector_stop.wait(60.0):  # reference cron: every minute
                    try:
                        names = [d["job_name"] for d in self.store.list_metadata(self.args.gpu_type)]
                        self.collector.update_info_all(names)
                    except Exception:
                        log.exception("metrics collector pass failed")

            threading.Thread(target=loop, daemon=True, name="metrics-collector").start()
        return self

    def stop(self) -> None:
        self._collector_stop.set()
        if self.http is not None:
            self.http.stop()
        self.runner.stop()
        self.backend.shutdown()


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    logging.basicConfig(level=a.log_level.upper(), format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    proc = SchedulerProcess(a).start()
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    signal.signal(signal.SIGINT, lambda *_: done.set())
    done.wait()
    proc.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
