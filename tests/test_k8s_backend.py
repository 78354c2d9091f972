"""K8sBackend against an in-memory fake Kubernetes API server (MPIJob CRD + pods + nodes)."""
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import unquote, urlparse

import pytest

from vodascheduler_amd.allocator.allocator import ResourceAllocator
from vodascheduler_amd.backend.k8s import K8sBackend, K8sClient
from vodascheduler_amd.common.mq import InProcQueue
from vodascheduler_amd.common.store import MemoryStore
from vodascheduler_amd.common.types import DEFAULT_GPU_TYPE, GPU_RESOURCE, TAINT_KEY, JobStatus
from vodascheduler_amd.scheduler.core import SchedulerCore
from vodascheduler_amd.service.service import TrainingService
from vodascheduler_amd.sim import make_spec
from vodascheduler_amd.utils.clock import ManualClock

NS = "voda-scheduler"


class FakeK8s:
    def __init__(self, nodes):
        self.nodes = nodes  # name -> gpus
        self.mpijobs: dict[str, dict] = {}
        self.pods: dict[str, dict] = {}
        self.log: list[tuple[str, str]] = []
        self.rv = 0
        self.watches = 0
        fake = self

        class H(BaseHTTPRequestHandler):
            def _send(self, code, obj=None):
                body = json.dumps(obj).encode() if obj is not None else b""
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n)) if n else None

            def _watch(self, path, query):
                """Stream ADDED/MODIFIED/DELETED lines by diffing the collection (2 s per stream;
                the first poll re-announces every item, as after a re-LIST)."""
                import time as _t

                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.end_headers()
                prev: dict[str, str] = {}
                t_end = _t.time() + 2.0
                while _t.time() < t_end:
                    code, lst = fake.handle("GET", path, None)
                    cur = {o["metadata"]["name"]: json.dumps(o, sort_keys=True) for o in lst.get("items", [])}
                    lines = []
                    for n, js in cur.items():
                        if prev.get(n) != js:
                            lines.append({"type": "ADDED" if n not in prev else "MODIFIED", "object": json.loads(js)})
                    for n in set(prev) - set(cur):
                        lines.append({"type": "DELETED", "object": json.loads(prev[n])})
                    prev = cur
                    try:
                        for ev in lines:
                            self.wfile.write((json.dumps(ev) + "\n").encode())
                        self.wfile.flush()
                    except OSError:
                        return
                    _t.sleep(0.02)

            def _route(self, method):
                u = urlparse(self.path)
                path = unquote(u.path)
                fake.log.append((method, path))
                if method == "GET" and "watch=1" in u.query:
                    fake.watches += 1
                    return self._watch(path, u.query)
                code, obj = fake.handle(method, path, self._body() if method in ("POST", "PUT", "PATCH") else None)
                self._send(code, obj)

            do_GET = lambda self: self._route("GET")  # noqa: E731
            do_POST = lambda self: self._route("POST")  # noqa: E731
            do_PUT = lambda self: self._route("PUT")  # noqa: E731
            do_PATCH = lambda self: self._route("PATCH")  # noqa: E731
            do_DELETE = lambda self: self._route("DELETE")  # noqa: E731

            def log_message(self, *a):
                pass

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def handle(self, method, path, body):
        mj = f"/apis/kubeflow.org/v1/namespaces/{NS}/mpijobs"
        pods = f"/api/v1/namespaces/{NS}/pods"
        if path == "/api/v1/nodes":
            return 200, {"items": [{"metadata": {"name": n, "labels": {"vodascheduler/accelerator": DEFAULT_GPU_TYPE}},
                                    "status": {"capacity": {GPU_RESOURCE: str(g)}}} for n, g in self.nodes.items()]}
        if path == mj:
            if method == "GET":
                return 200, {"items": list(self.mpijobs.values())}
            name = body["metadata"]["name"]
            if name in self.mpijobs:
                return 409, {"reason": "AlreadyExists"}
            self.rv += 1
            body["metadata"]["resourceVersion"] = str(self.rv)
            self.mpijobs[name] = body
            return 201, body
        if path.startswith(mj + "/"):
            name = path[len(mj) + 1:]
            if name not in self.mpijobs:
                return 404, {"reason": "NotFound"}
            if method == "GET":
                return 200, self.mpijobs[name]
            if method == "PUT":
                self.mpijobs[name] = body
                return 200, body
            if method == "DELETE":
                del self.mpijobs[name]
                return 200, {}
        if path == pods:
            return 200, {"items": list(self.pods.values())}
        if path.startswith(pods + "/"):
            name = path[len(pods) + 1:]
            if name not in self.pods:
                return 404, {"reason": "NotFound"}
            if method == "PATCH":
                p = self.pods[name]
                if "spec" in body:
                    p.setdefault("spec", {}).update(body["spec"])
                if "metadata" in body:
                    p["metadata"].setdefault("annotations", {}).update(body["metadata"].get("annotations", {}))
                return 200, p
            if method == "DELETE":
                del self.pods[name]
                return 200, {}
        return 404, {"reason": f"no route {method} {path}"}

    def stop(self):
        self.srv.shutdown()


@pytest.fixture
def env():
    fake = FakeK8s({"nodeA": 4, "nodeB": 4})
    clock = ManualClock(1000.0)
    store, mq = MemoryStore(), InProcQueue()
    backend = K8sBackend(K8sClient(fake.url), DEFAULT_GPU_TYPE, start_thread=False)
    core = SchedulerCore(DEFAULT_GPU_TYPE, store, ResourceAllocator(store), backend, clock=clock,
                         algorithm="ElasticFIFO", rate_limit_sec=0)
    svc = TrainingService(store, mq, clock)

    def submit(name, np_, mn, mx):
        n = svc.create_training_job(json.dumps(make_spec(name, "resnet50", np_, mn, mx, 2, 10)))
        core.create_training_job(mq.get(DEFAULT_GPU_TYPE).job_name)
        return n

    yield fake, core, backend, submit, clock
    backend.shutdown()
    fake.stop()


def test_nodes_from_labels_and_capacity(env):
    fake, core, backend, submit, clock = env
    assert backend.nodes() == {"nodeA": [0, 1, 2, 3], "nodeB": [0, 1, 2, 3]}
    assert core.total_gpus == 8


def test_start_scale_halt_and_completion(env):
    fake, core, backend, submit, clock = env
    a = submit("a", 2, 1, 8)
    core.poll()
    obj = fake.mpijobs[a]
    w = obj["spec"]["mpiReplicaSpecs"]["Worker"]
    assert w["replicas"] == 8  # elastic: grows to the whole idle cluster
    assert w["template"]["spec"]["containers"][0]["resources"]["limits"][GPU_RESOURCE] == 1
    assert obj["metadata"]["labels"]["vodascheduler/accelerator"] == DEFAULT_GPU_TYPE
    b = submit("b", 4, 4, 4)
    clock.advance(1)
    core.poll()
    assert fake.mpijobs[a]["spec"]["mpiReplicaSpecs"]["Worker"]["replicas"] == 4  # scaled in via PUT
    assert fake.mpijobs[b]["spec"]["mpiReplicaSpecs"]["Worker"]["replicas"] == 4
    assert ("PUT", f"/apis/kubeflow.org/v1/namespaces/{NS}/mpijobs/{a}") in fake.log
    # completion from the MPIJob condition
    fake.mpijobs[b]["status"] = {"conditions": [{"type": "Succeeded", "status": "True"}]}
    backend.poll_jobs()
    core.poll()
    assert core.get_job_status(b) == JobStatus.COMPLETED
    assert fake.mpijobs[a]["spec"]["mpiReplicaSpecs"]["Worker"]["replicas"] == 8
    core.delete_training_job(a)
    assert a not in fake.mpijobs


def test_pod_binding_tolerations_and_migration(env):
    fake, core, backend, submit, clock = env
    a = submit("a", 2, 2, 2)
    core.poll()
    locs = backend.placement[a]
    for i in range(2):
        fake.pods[f"{a}-worker-{i}"] = {"metadata": {"name": f"{a}-worker-{i}", "labels": {}},
                                        "status": {"phase": "Pending"}, "spec": {}}
    fake.pods[f"{a}-launcher"] = {"metadata": {"name": f"{a}-launcher"}, "status": {"phase": "Pending"}, "spec": {}}
    backend.bind_pods()
    for i in range(2):
        tol = fake.pods[f"{a}-worker-{i}"]["spec"]["tolerations"][0]
        assert tol == {"key": TAINT_KEY, "operator": "Equal", "value": locs[i][0], "effect": "NoExecute"}
    assert fake.pods[f"{a}-launcher"]["spec"]["tolerations"][0]["operator"] == "Exists"
    # a node drain moves the workers: their pods are deleted and recreated by the operator
    node = locs[0][0]
    fake.nodes.pop(node)
    backend.refresh_nodes()
    clock.advance(1)
    core.poll()
    assert all(l[0] != node for l in backend.placement[a])
    assert f"{a}-worker-0" not in fake.pods


def test_gen_manifests_one_scheduler_per_gpu_type(capsys):
    """Reference helm/voda-scheduler/gen-scheduler-yaml.sh: one scheduler per GPU type."""
    import yaml

    from vodascheduler_amd.cli.main import main

    assert main(["gen-manifests", "--gpu-type", "amd-instinct-mi355x", "--gpu-type", "amd-instinct-mi300x"]) == 0
    docs = list(yaml.safe_load_all(capsys.readouterr().out))
    kinds = [(d["kind"], d["metadata"]["name"]) for d in docs]
    assert kinds == [("Deployment", "scheduler-amd-instinct-mi355x"), ("Service", "scheduler-amd-instinct-mi355x"),
                     ("Deployment", "scheduler-amd-instinct-mi300x"), ("Service", "scheduler-amd-instinct-mi300x")]
    cmd = docs[2]["spec"]["template"]["spec"]["containers"][0]["command"]
    assert cmd[cmd.index("--gpu-type") + 1] == "amd-instinct-mi300x" and "--resume" in cmd
    assert docs[1]["spec"]["ports"][0]["port"] == 55588


def test_watch_informers_bind_pods_and_report_completion():
    """Informer path: with the resync period effectively off, LIST + WATCH streams alone bind a
    new worker pod to its placed node and report the MPIJob's Succeeded condition."""
    import time

    from vodascheduler_amd.backend.base import EV_FINISHED, START, JobAction
    from vodascheduler_amd.common.trainingjob import TrainingJob

    fake = FakeK8s({"nodeA": 4})
    backend = K8sBackend(K8sClient(fake.url), DEFAULT_GPU_TYPE, poll_interval=3600.0)
    events = []
    backend.set_event_sink(lambda *ev: events.append(ev))
    try:
        store, mq = MemoryStore(), InProcQueue()
        svc = TrainingService(store, mq, ManualClock(0.0))
        name = svc.create_training_job(json.dumps(make_spec("w", "resnet50", 2, 1, 2, 1, 10)))
        job = TrainingJob.from_dict(store.find_metadata(name))
        backend.apply([JobAction(START, job, 2, [("nodeA", 0), ("nodeA", 1)], [])])
        fake.pods[f"{name}-worker-1"] = {"metadata": {"name": f"{name}-worker-1", "labels": {}},
                                         "status": {"phase": "Pending"}, "spec": {}}

        def wait(cond, t=10.0):
            end = time.time() + t
            while time.time() < end:
                if cond():
                    return True
                time.sleep(0.02)
            return False

        assert wait(lambda: fake.pods[f"{name}-worker-1"]["spec"].get("tolerations"))
        tol = fake.pods[f"{name}-worker-1"]["spec"]["tolerations"][0]
        assert tol["key"] == TAINT_KEY and tol["value"] == "nodeA"
        fake.mpijobs[name]["status"] = {"conditions": [{"type": "Succeeded", "status": "True"}]}
        assert wait(lambda: (EV_FINISHED, name, True) in events)
        assert fake.watches >= 3  # mpijobs, pods, nodes
    finally:
        backend.shutdown()
        fake.stop()


def test_completion_emitted_once_when_watch_and_resync_race():
    """the watch thread and the resync loop both see a finished MPIJob;
    the scheduler must get exactly one EV_FINISHED."""

    class NoClient:
        def get(self, path):
            return {"items": []}

    b = K8sBackend(NoClient(), DEFAULT_GPU_TYPE, start_thread=False)
    b.jobs["j"] = {}
    got = []
    b.set_event_sink(lambda ev, *a: got.append((ev, a)))
    st = {"conditions": [{"type": "Succeeded", "status": "True"}]}
    barrier = threading.Barrier(8)

    def hit(i):
        barrier.wait()
        if i % 2:
            b._job_event("MODIFIED", {"metadata": {"name": "j"}, "status": st})
        else:
            b._maybe_finished("j", st)

    ts = [threading.Thread(target=hit, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len([g for g in got if g[0] == "finished"]) == 1, got
