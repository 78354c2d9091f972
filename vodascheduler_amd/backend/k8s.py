"""Kubernetes + MPI-Operator backend: drives real clusters with the reference's object shapes.

The MI355X-native path is :class:`~vodascheduler_amd.backend.local.LocalBackend` (warm
per-GPU workers on one node).  For multi-node Kubernetes deployments this backend performs
exactly the API operations of the reference scheduler and placement manager, against the
``kubeflow.org/v1 MPIJob`` CRD:

* start  -> ``POST   .../mpijobs`` with ``Worker.replicas = n``      (scheduler.go:495-518)
* scale  -> ``GET`` + ``PUT .../mpijobs/<job>`` (retry on conflict)   (scheduler.go:542-563)
  plus, with ``configmap_opt``, a random annotation on ``<job>-launcher`` so the kubelet
  re-syncs the discovery ConfigMap sooner                               (scheduler.go:1081-1112)
* halt   -> ``DELETE .../mpijobs/<job>``                              (scheduler.go:576-589)
* migrate-> ``DELETE`` of the moved ``<job>-worker-<i>`` pods          (placement_manager.go:622-633)
* binding-> pending worker pods get the ``vodascheduler/hostname=<node>:NoExecute``
  toleration of their placed node, the launcher an ``Exists`` wildcard (placement_manager.go:174-237)
* nodes  -> ``GET /api/v1/nodes?labelSelector=vodascheduler/accelerator=<gpu>``, capacity
  ``amd.com/gpu`` (``nvidia.com/gpu`` in the reference)              (scheduler.go:689-747)
* done   -> MPIJob ``Succeeded`` / ``Failed`` conditions                (status.go:9-29)

The API client is a small stdlib HTTPS/JSON client (in-cluster service-account token or an
explicit URL + bearer token); nothing is imported from the kubernetes Python package, which
is not in this image.  Change notification follows the informer pattern of the reference
(scheduler.go:170-185,230-242; placement_manager.go:84-134): per resource (MPIJobs, our pods,
GPU nodes) a LIST, then a streaming WATCH from its resourceVersion (re-LIST on 410 Gone or a
dropped stream); events drive completion reports, pod binding and node inventory at once.
A slow periodic resync (default 30 s) re-reads everything, as informers do.
"""
from __future__ import annotations

import json
import logging
import os
import random
import ssl
import string
import threading
import time
import urllib.error
import urllib.request

from ..common import mpijob
from ..common.types import GPU_NAME_LABEL, GPU_RESOURCE, NAMESPACE, TAINT_KEY
from .base import EV_FINISHED, EV_NODES, HALT, MIGRATE, SCALE_IN, SCALE_OUT, START, Backend, JobAction

log = logging.getLogger("vodascheduler_amd.k8s")

MPIJOB_API = "/apis/kubeflow.org/v1"
SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class ApiError(RuntimeError):
    def __init__(self, status: int, body: str):
        super().__init__(f"kubernetes API error {status}: {body[:300]}")
        self.status = status


class K8sClient:
    def __init__(self, base_url: str | None = None, token: str | None = None, ca_file: str | None = None,
                 insecure: bool = False, timeout: float = 30.0):
        if base_url is None:  # in-cluster
            host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            base_url = f"https://{host}:{port}"
            token = token or open(os.path.join(SA_DIR, "token")).read().strip()
            ca_file = ca_file or os.path.join(SA_DIR, "ca.crt")
        self.base = base_url.rstrip("/")
        self.token = token
        self.timeout = timeout
        self.ctx = None
        if self.base.startswith("https"):
            self.ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()
            if insecure:
                self.ctx.check_hostname = False
                self.ctx.verify_mode = ssl.CERT_NONE

    def request(self, method: str, path: str, body=None, content_type: str = "application/json"):
        data = None if body is None else json.dumps(body).encode()
        req = urllib.request.Request(self.base + path, data=data, method=method)
        req.add_header("Accept", "application/json")
        if data is not None:
            req.add_header("Content-Type", content_type)
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout, context=self.ctx) as r:
                raw = r.read()
        except urllib.error.HTTPError as e:
            raise ApiError(e.code, e.read().decode(errors="replace")) from None
        return json.loads(raw) if raw else None

    get = lambda self, p: self.request("GET", p)  # noqa: E731
    post = lambda self, p, b: self.request("POST", p, b)  # noqa: E731
    put = lambda self, p, b: self.request("PUT", p, b)  # noqa: E731
    delete = lambda self, p: self.request("DELETE", p)  # noqa: E731

    def patch(self, path: str, body) -> dict:
        return self.request("PATCH", path, body, content_type="application/merge-patch+json")

    def watch(self, path: str, resource_version: str | None, on_event, stop: threading.Event,
              timeout_s: int = 300) -> str | None:
        """Stream ``?watch=1`` events of a collection until the server closes the stream, the
        timeout passes or ``stop`` is set; returns the last resourceVersion seen.  Raises
        :class:`ApiError` (410 when the version expired: re-LIST and watch again)."""
        sep = "&" if "?" in path else "?"
        url = f"{path}{sep}watch=1&allowWatchBookmarks=true&timeoutSeconds={int(timeout_s)}"
        if resource_version:
            url += f"&resourceVersion={resource_version}"
        req = urllib.request.Request(self.base + url, method="GET")
        req.add_header("Accept", "application/json")
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        rv = resource_version
        try:
            with urllib.request.urlopen(req, timeout=timeout_s + 30, context=self.ctx) as r:
                for line in r:
                    if stop.is_set():
                        break
                    line = line.strip()
                    if not line:
                        continue
                    ev = json.loads(line)
                    typ, obj = ev.get("type"), ev.get("object") or {}
                    if typ == "ERROR":
                        raise ApiError(int(obj.get("code", 500)), json.dumps(obj))
                    rv = (obj.get("metadata") or {}).get("resourceVersion", rv)
                    if typ != "BOOKMARK":
                        on_event(typ, obj)
        except urllib.error.HTTPError as e:
            raise ApiError(e.code, e.read().decode(errors="replace")) from None
        return rv


def _rand(n: int = 5) -> str:
    return "".join(random.choice(string.ascii_lowercase + string.digits) for _ in range(n))


class K8sBackend(Backend):
    def __init__(self, client: K8sClient, gpu_type: str, namespace: str = NAMESPACE, configmap_opt: bool = True,
                 poll_interval: float = 30.0, start_thread: bool = True, watch: bool = True):
        """``poll_interval``: informer resync period; ``watch``: stream change events (off:
        resync polling only)."""
        super().__init__()
        self.c = client
        self.gpu_type = gpu_type
        self.ns = namespace
        self.configmap_opt = configmap_opt
        self.poll_interval = poll_interval
        self.watch_enabled = watch
        self._watchers: list[threading.Thread] = []
        self._lock = threading.Lock()
        self.jobs: dict[str, dict] = {}                # job -> spec as submitted
        self.placement: dict[str, list[tuple[str, int]]] = {}   # job -> worker i -> (node, gpu)
        self._nodes: dict[str, list[int]] = {}
        self._finished: set[str] = set()
        self._watches_down: set[str] = set()   # informer streams currently failing
        self._stop = threading.Event()
        self.refresh_nodes(emit=False)
        self._thread = None
        if start_thread:
            self._thread = threading.Thread(target=self._loop, daemon=True, name="k8s-backend")
            self._thread.start()
            if watch:
                self.start_watches()

    # ------------------------------------------------------------------ paths
    def _mpijobs(self) -> str:
        return f"{MPIJOB_API}/namespaces/{self.ns}/mpijobs"

    def _pods(self) -> str:
        return f"/api/v1/namespaces/{self.ns}/pods"

    # ------------------------------------------------------------------ Backend API
    def apply(self, actions: list[JobAction]) -> None:
        for a in actions:
            name = a.job.name
            if a.workers is not None:
                with self._lock:
                    self.placement[name] = list(a.workers)
            if a.kind == START:
                self._start(a)
            elif a.kind in (SCALE_IN, SCALE_OUT):
                self._scale(name, a.num_workers)
            elif a.kind == HALT:
                self._halt(name)
            elif a.kind == MIGRATE:
                self._migrate(name, a.prev_workers, a.workers or [])

    def _start(self, a: JobAction) -> None:
        spec = mpijob.clone(a.job.spec)
        mpijob.preprocess(spec, self.gpu_type)
        mpijob.set_worker_replicas(spec, a.num_workers)
        spec["metadata"]["namespace"] = self.ns
        spec["metadata"].pop("resourceVersion", None)
        with self._lock:
            self.jobs[a.job.name] = spec
        try:
            self.c.post(self._mpijobs(), spec)
        except ApiError as e:
            if e.status != 409:  # already exists (restart / resume): scale instead
                raise
            self._scale(a.job.name, a.num_workers)

    def _scale(self, name: str, n: int, retries: int = 5) -> None:
        for i in range(retries):
            obj = self.c.get(f"{self._mpijobs()}/{name}")
            mpijob.set_worker_replicas(obj, n)
            try:
                self.c.put(f"{self._mpijobs()}/{name}", obj)
                break
            except ApiError as e:  # RetryOnConflict
                if e.status != 409 or i == retries - 1:
                    raise
        if self.configmap_opt:
            self._touch_launcher(name)

    def _touch_launcher(self, name: str) -> None:
        try:
            self.c.patch(f"{self._pods()}/{name}-launcher",
                         {"metadata": {"annotations": {"vodascheduler/dummy": _rand()}}})
        except ApiError as e:
            if e.status != 404:
                log.warning("configmap_opt annotation on %s-launcher failed: %s", name, e)

    def _halt(self, name: str) -> None:
        try:
            self.c.delete(f"{self._mpijobs()}/{name}")
        except ApiError as e:
            if e.status != 404:
                raise

    def _migrate(self, name: str, old: list, new: list) -> None:
        """Delete the worker pods whose placed node changed; the MPI-Operator recreates them and
        the binding loop gives them their new node's toleration.  If every worker moved, the
        launcher is deleted too (placement_manager.go:603-606)."""
        moved = [i for i, loc in enumerate(new) if i >= len(old) or old[i][0] != loc[0]]
        for i in moved:
            try:
                self.c.delete(f"{self._pods()}/{name}-worker-{i}")
            except ApiError as e:
                if e.status != 404:
                    raise
        if new and len(moved) == len(new):
            try:
                self.c.delete(f"{self._pods()}/{name}-launcher")
            except ApiError as e:
                if e.status != 404:
                    raise

    def delete_job(self, job_name: str) -> None:
        self._halt(job_name)
        with self._lock:
            self.jobs.pop(job_name, None)
            self.placement.pop(job_name, None)

    def nodes(self) -> dict[str, list[int]]:
        with self._lock:
            return {k: list(v) for k, v in self._nodes.items()}

    def list_running(self) -> dict[str, list[tuple[str, int]]]:
        out: dict[str, list[tuple[str, int]]] = {}
        try:
            items = self.c.get(self._mpijobs()).get("items", [])
        except ApiError:
            return out
        for obj in items:
            name = obj["metadata"]["name"]
            n = mpijob.worker_replicas(obj)
            if n > 0 and not mpijob.is_finished(obj.get("status")):
                out[name] = self.placement.get(name) or [("", i) for i in range(n)]
        return out

    def shutdown(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(5)
        for t in self._watchers:
            t.join(2)

    # ------------------------------------------------------------------ watchers
    def refresh_nodes(self, emit: bool = True) -> None:
        sel = urllib.request.quote(f"{GPU_NAME_LABEL}={self.gpu_type}")
        items = self.c.get(f"/api/v1/nodes?labelSelector={sel}").get("items", [])
        nodes = {}
        for n in items:
            cap = int((n.get("status", {}).get("capacity") or {}).get(GPU_RESOURCE, 0))
            if cap > 0 and not n.get("spec", {}).get("unschedulable", False):
                nodes[n["metadata"]["name"]] = list(range(cap))
        with self._lock:
            changed = nodes != self._nodes
            self._nodes = nodes
        if changed and emit:
            self.emit(EV_NODES, self.nodes())

    def poll_jobs(self) -> None:
        items = self.c.get(self._mpijobs()).get("items", [])
        for obj in items:
            name = obj["metadata"]["name"]
            st = obj.get("status")
            self._maybe_finished(name, st)

    def _job_event(self, typ: str, obj: dict) -> None:
        if typ in ("ADDED", "MODIFIED"):
            self._maybe_finished(obj.get("metadata", {}).get("name"), obj.get("status"))

    def _maybe_finished(self, name: str | None, st: dict | None) -> None:
        """Emit a job's completion exactly once: the watch stream and the resync loop both
        see it, and only the thread that records it under the lock emits (the reference's
        informer delivers each completion once)."""
        if not name or not mpijob.is_finished(st):
            return
        with self._lock:
            if name not in self.jobs or name in self._finished:
                return
            self._finished.add(name)
        self.emit(EV_FINISHED, name, mpijob.is_succeeded(st))

    def bind_pods(self) -> None:
        """Give pending pods of our jobs the toleration of their placed node."""
        sel = urllib.request.quote(GPU_NAME_LABEL)
        pods = self.c.get(f"{self._pods()}?labelSelector={sel}").get("items", [])
        for p in pods:
            self._bind_pod(p)

    def _bind_pod(self, p: dict) -> None:
        md = p["metadata"]
        name = md["name"]
        if p.get("status", {}).get("phase") not in (None, "Pending"):
            return
        tols = p.get("spec", {}).get("tolerations") or []
        if any(t.get("key") == TAINT_KEY for t in tols):
            return
        job, _, rest = name.rpartition("-worker-")
        if job and rest.isdigit():
            locs = self.placement.get(job) or []
            i = int(rest)
            if i >= len(locs) or not locs[i][0]:
                return
            tol = {"key": TAINT_KEY, "operator": "Equal", "value": locs[i][0], "effect": "NoExecute"}
        elif name.endswith("-launcher") and name[:-len("-launcher")] in self.jobs:
            tol = {"key": TAINT_KEY, "operator": "Exists", "effect": "NoExecute"}
        else:
            return
        try:
            self.c.patch(f"{self._pods()}/{name}", {"spec": {"tolerations": tols + [tol]}})
        except ApiError as e:
            log.warning("binding %s failed: %s", name, e)

    # ------------------------------------------------------------------ informers
    def start_watches(self) -> None:
        gsel = urllib.request.quote(f"{GPU_NAME_LABEL}={self.gpu_type}")
        psel = urllib.request.quote(GPU_NAME_LABEL)
        specs = [
            ("mpijobs", self._mpijobs(), self._job_event),
            ("pods", f"{self._pods()}?labelSelector={psel}",
             lambda typ, obj: self._bind_pod(obj) if typ in ("ADDED", "MODIFIED") else None),
            ("nodes", f"/api/v1/nodes?labelSelector={gsel}", lambda typ, obj: self.refresh_nodes()),
        ]
        for name, path, handler in specs:
            t = threading.Thread(target=self._informer, args=(path, handler), daemon=True, name=f"k8s-watch-{name}")
            t.start()
            self._watchers.append(t)

    def _informer(self, path: str, handler) -> None:
        """LIST + WATCH loop of one collection (re-LIST when the stream breaks or expires).
        A stream that keeps failing is logged at warning level and marks the watch down, so
        the resync loop polls at ``DEGRADED_POLL_S`` until it is back."""
        fails = 0

        def safe(typ, obj):
            try:
                handler(typ, obj)
            except Exception:  # a bad event must not kill the stream, but must be visible
                log.warning("watch %s: handler failed on %s event", path, typ, exc_info=True)

        while not self._stop.is_set():
            try:
                lst = self.c.get(path)
                for obj in lst.get("items", []):
                    safe("ADDED", obj)
                rv = (lst.get("metadata") or {}).get("resourceVersion")
                if fails:
                    log.info("watch %s re-established after %d failure(s)", path, fails)
                    self._set_watch_down(path, False)
                fails = 0
                while not self._stop.is_set():
                    rv = self.c.watch(path, rv, safe, self._stop)
            except ApiError as e:
                if e.status != 410:  # 410 Gone: resourceVersion expired, a normal re-LIST
                    fails += 1
                    log.warning("watch %s failed (%d in a row): %s", path, fails, e)
                    self._set_watch_down(path, True)
            except Exception as e:  # dropped stream / transient API failure
                fails += 1
                (log.warning if fails >= 2 else log.debug)("watch %s interrupted (%d in a row): %s", path, fails, e)
                if fails >= 2:
                    self._set_watch_down(path, True)
            self._stop.wait(min(30.0, 1.0 * 2 ** min(fails, 5)) if fails else 1.0)

    DEGRADED_POLL_S = 2.0

    def _set_watch_down(self, path: str, down: bool) -> None:
        with self._lock:
            if down:
                self._watches_down.add(path)
            else:
                self._watches_down.discard(path)

    def _loop(self) -> None:
        while not self._stop.wait(self.DEGRADED_POLL_S if self._watches_down else self.poll_interval):
            for fn in (self.refresh_nodes, self.poll_jobs, self.bind_pods):
                try:
                    fn()
                except Exception:
                    log.exception("k8s backend poll %s failed", fn.__name__)
