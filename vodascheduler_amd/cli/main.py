"""``vodascheduler`` command line (reference cmd/main.go:13-59, cmd/cmd/cmd.go:17-101).

    vodascheduler create -f job.yaml              POST  <service>/training   (raw YAML body)
    vodascheduler delete NAME [NAME ...]          DELETE <service>/training  (JSON string body, per name)
    vodascheduler get jobs                        GET   <scheduler>/training (status table)
    vodascheduler get trace                       GET   <scheduler>/trace    (Chrome-trace JSON timeline)
    vodascheduler set algorithm ElasticTiresias   PUT   <scheduler>/algorithm
    vodascheduler set ratelimit 30                PUT   <scheduler>/ratelimit
    vodascheduler up [--gpus 0,1,...]             all-in-one: service + scheduler + allocator + node agent
    vodascheduler simulate --jobs 32 --gpus 8     discrete-event run of a Philly-style trace (no GPUs)
    vodascheduler gen-manifests --gpu-type T ...  scheduler Deployment + Service per GPU type (k8s)

Fixes of the reference CLI: ``delete`` deletes EVERY name given (the
reference always sends ``Args().Get(0)``) and sends each as a JSON string (the service
expects one); ``get jobs`` asks the scheduler (the reference asked the training service,
which never routed ``GET /training``).  Endpoints default to localhost and can be set with
``--service`` / ``--scheduler`` or ``VODA_SERVICE_URL`` / ``VODA_SCHEDULER_URL``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

from ..common.types import ENTRY_POINT, NAME, PORT_ALLOCATOR, PORT_SCHEDULER, PORT_TRAINING_SERVICE, VERSION
from ..utils.http import http_request


def _service(a) -> str:
    return (a.service or os.environ.get("VODA_SERVICE_URL") or f"http://127.0.0.1:{PORT_TRAINING_SERVICE}").rstrip("/")


def _scheduler(a) -> str:
    return (a.scheduler or os.environ.get("VODA_SCHEDULER_URL") or f"http://127.0.0.1:{PORT_SCHEDULER}").rstrip("/")


def _out(status: int, body: bytes) -> int:
    sys.stdout.write(body.decode(errors="replace"))
    if body and not body.endswith(b"\n"):
        sys.stdout.write("\n")
    return 0 if 200 <= status < 300 else 1


def cmd_create(a) -> int:
    with open(a.filename, "rb") as f:
        data = f.read()
    return _out(*http_request("POST", _service(a) + ENTRY_POINT, data, content_type="application/yaml"))


def cmd_delete(a) -> int:
    rc = 0
    for name in a.names:
        rc |= _out(*http_request("DELETE", _service(a) + ENTRY_POINT, json.dumps(name).encode()))
    return rc


def cmd_get(a) -> int:
    if a.what == "trace":
        return _out(*http_request("GET", _scheduler(a) + "/trace"))
    if a.what not in ("jobs", "job", "training"):
        print(f"unknown resource {a.what!r}; try: get jobs | get trace", file=sys.stderr)
        return 2
    return _out(*http_request("GET", _scheduler(a) + ENTRY_POINT))


def cmd_set(a) -> int:
    if a.what == "algorithm":
        body = json.dumps(a.value)
        return _out(*http_request("PUT", _scheduler(a) + "/algorithm", body.encode()))
    if a.what == "ratelimit":
        v = float(a.value)
        body = json.dumps(int(v) if v.is_integer() else v)
        return _out(*http_request("PUT", _scheduler(a) + "/ratelimit", body.encode()))
    print(f"unknown setting {a.what!r}; expected algorithm | ratelimit", file=sys.stderr)
    return 2


def cmd_up(a) -> int:
    """Service (:55587) + scheduler (:55588) + allocator (:55589) + node agent in one process."""
    import logging
    import signal
    import threading

    from ..allocator.allocator import ResourceAllocator
    from ..allocator.server import allocator_router
    from ..common.mq import open_queue
    from ..common.store import open_store
    from ..scheduler.main import SchedulerProcess, build_parser
    from ..service.service import TrainingService
    from ..utils.http import HttpServer

    logging.basicConfig(level=a.log_level.upper(), format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    store = open_store(a.store)
    mq = open_queue("inproc://")
    sargv = ["--backend", "local", "--device-type", a.device_type, "--algorithm", a.algorithm,
             "--rate-limit", str(a.rate_limit), "--store-port", str(a.store_port), "--port", str(a.scheduler_port),
             "--metrics-dir", a.metrics_dir]
    if a.gpus:
        sargv += ["--gpus", a.gpus]
    if a.resume:
        sargv.append("--resume")
    if a.log_dir:
        sargv += ["--log-dir", a.log_dir]
    sched = SchedulerProcess(build_parser().parse_args(sargv), store=store, mq=mq).start()
    svc = HttpServer(TrainingService(store, mq).router(), port=a.service_port, name="training-service").start()
    alloc = HttpServer(allocator_router(ResourceAllocator(store)), port=a.allocator_port, name="allocator").start()
    print(f"{NAME} {VERSION} up: service :{svc.port}  scheduler :{sched.http.port}  allocator :{alloc.port}",
          flush=True)
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    signal.signal(signal.SIGINT, lambda *_: done.set())
    done.wait()
    svc.stop()
    alloc.stop()
    sched.stop()
    return 0


def cmd_simulate(a) -> int:
    from ..sim.simulator import simulate
    from ..sim.trace import philly_trace

    trace = philly_trace(a.jobs, seed=a.seed, mean_interarrival_s=a.interarrival)
    algos = a.algorithm.split(",")
    for algo in algos:
        tp = a.trace.replace("{algorithm}", algo) if a.trace else None
        r = simulate(trace, algorithm=algo, gpus=a.gpus, rate_limit_sec=a.rate_limit, trace_path=tp)
        print(r.to_json(), flush=True)
    return 0


SCHEDULER_MANIFEST = """apiVersion: apps/v1
kind: Deployment
metadata: {{name: scheduler-{gpu}, namespace: {ns}}}
spec:
  replicas: 1
  selector: {{matchLabels: {{app: scheduler-{gpu}}}}}
  template:
    metadata: {{labels: {{app: scheduler-{gpu}}}}}
    spec:
      serviceAccountName: voda-scheduler
      containers:
        - name: scheduler
          image: {image}
          command: ["vodascheduler-scheduler", "--backend", "k8s", "--gpu-type", "{gpu}",
                    "--algorithm", "{algorithm}", "--resume",
                    "--store", "sqlite:///state/jobs.db", "--mq", "sqlite:///state/mq.db",
                    "--allocator", "http://resource-allocator.{ns}.svc.cluster.local:55589"]
          ports: [{{containerPort: 55588}}]
          volumeMounts: [{{name: state, mountPath: /state}}]
      volumes: [{{name: state, persistentVolumeClaim: {{claimName: voda-state}}}}]
---
apiVersion: v1
kind: Service
metadata: {{name: scheduler-{gpu}, namespace: {ns}}}
spec:
  selector: {{app: scheduler-{gpu}}}
  ports: [{{name: port, port: 55588, targetPort: 55588}}]
"""


def cmd_gen_manifests(a) -> int:
    """One scheduler Deployment + Service per GPU type (reference
    helm/voda-scheduler/gen-scheduler-yaml.sh + scheduler.yaml.base): a heterogeneous cluster
    runs one scheduler per ``vodascheduler/accelerator`` label value."""
    docs = [SCHEDULER_MANIFEST.format(gpu=g, ns=a.namespace, image=a.image, algorithm=a.algorithm)
            for g in a.gpu_type]
    sys.stdout.write("---\n".join(docs))
    return 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(NAME, description=f"{NAME} {VERSION}: elastic DL scheduler for AMD Instinct MI355X")
    ap.add_argument("--service", default=None, help=f"training service URL (default :{PORT_TRAINING_SERVICE})")
    ap.add_argument("--scheduler", default=None, help=f"scheduler URL (default :{PORT_SCHEDULER})")
    sub = ap.add_subparsers(dest="cmd", required=True)

    p = sub.add_parser("create", help="submit a training job (MPIJob YAML)")
    p.add_argument("-f", "--filename", required=True)
    p.set_defaults(fn=cmd_create)

    p = sub.add_parser("delete", help="delete training job(s)")
    p.add_argument("names", nargs="+")
    p.set_defaults(fn=cmd_delete)

    p = sub.add_parser("get", help="show training jobs")
    p.add_argument("what", nargs="?", default="jobs")
    p.set_defaults(fn=cmd_get)

    p = sub.add_parser("set", help="runtime configuration of the scheduler")
    p.add_argument("what", choices=["algorithm", "ratelimit"])
    p.add_argument("value")
    p.set_defaults(fn=cmd_set)

    p = sub.add_parser("up", help="run service + scheduler + allocator + node agent on this node")
    p.add_argument("--gpus", default=None, help="comma-separated GPU indices (default: all)")
    p.add_argument("--device-type", default="cuda", choices=["cuda", "cpu"])
    p.add_argument("--algorithm", default="ElasticFIFO")
    p.add_argument("--rate-limit", type=float, default=30.0)
    p.add_argument("--store", default="memory://")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--store-port", type=int, default=29400)
    p.add_argument("--service-port", type=int, default=PORT_TRAINING_SERVICE)
    p.add_argument("--scheduler-port", type=int, default=PORT_SCHEDULER)
    p.add_argument("--allocator-port", type=int, default=PORT_ALLOCATOR)
    p.add_argument("--metrics-dir", default=os.environ.get("VODA_METRICS_DIR", "/tmp/voda_metrics"))
    p.add_argument("--log-dir", default=None)
    p.add_argument("--log-level", default="INFO")
    p.set_defaults(fn=cmd_up)

    p = sub.add_parser("simulate", help="simulate a Philly-style trace (no GPUs)")
    p.add_argument("--jobs", type=int, default=32)
    p.add_argument("--gpus", type=int, default=8)
    p.add_argument("--algorithm", default="FIFO,ElasticFIFO,Tiresias,ElasticTiresias,FfDLOptimizer,AFS-L")
    p.add_argument("--rate-limit", type=float, default=30.0)
    p.add_argument("--interarrival", type=float, default=30.0)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--trace", default=None, help="Chrome-trace JSON of each run ({algorithm} is substituted)")
    p.set_defaults(fn=cmd_simulate)

    p = sub.add_parser("gen-manifests", help="scheduler Deployment + Service YAML per GPU type (k8s backend)")
    p.add_argument("--gpu-type", action="append", required=True, help="repeat for every GPU type")
    p.add_argument("--namespace", default="voda-scheduler")
    p.add_argument("--image", default="vodascheduler-amd:latest")
    p.add_argument("--algorithm", default="ElasticFIFO")
    p.set_defaults(fn=cmd_gen_manifests)

    p = sub.add_parser("version", help="print the version")
    p.set_defaults(fn=lambda a: print(f"{NAME} {VERSION}") or 0)
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    return int(a.fn(a) or 0)


if __name__ == "__main__":
    raise SystemExit(main())
