"""Node agent + LocalBackend + CLI end to end on CPU (gloo): real worker processes, the REST
services and the ``vodascheduler`` CLI, plus worker-death fault injection."""
import io
import json
import os
import time
from contextlib import redirect_stdout

import pytest
import yaml

from vodascheduler_amd.cli.main import main as cli
from vodascheduler_amd.common.mq import InProcQueue
from vodascheduler_amd.common.store import MemoryStore
from vodascheduler_amd.runtime.cluster import free_port
from vodascheduler_amd.scheduler.main import SchedulerProcess, build_parser
from vodascheduler_amd.service.service import TrainingService
from vodascheduler_amd.sim.trace import workload_of
from vodascheduler_amd.utils.http import HttpServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cluster(tmp_path, gpus="0,1", algorithm="ElasticFIFO"):
    store, mq = MemoryStore(), InProcQueue()
    a = build_parser().parse_args(["--backend", "local", "--device-type", "cpu", "--gpus", gpus,
                                   "--algorithm", algorithm, "--rate-limit", "0.5", "--tick", "0.5",
                                   "--store-port", str(free_port()), "--port", "0",
                                   "--metrics-dir", str(tmp_path / "metrics"), "--log-dir", str(tmp_path / "logs")])
    sched = SchedulerProcess(a, store=store, mq=mq).start()
    svc = HttpServer(TrainingService(store, mq).router(), port=0).start()
    return sched, svc


def _wait(pred, timeout, what):
    t0 = time.time()
    while time.time() - t0 < timeout:
        v = pred()
        if v:
            return v
        time.sleep(0.1)
    raise TimeoutError(what)


def _job_yaml(tmp_path, name, model, steps, epochs, np_, min_np, max_np):
    spec = yaml.safe_load(open(os.path.join(ROOT, "examples/yaml/pytorch-mnist-elastic.yaml")))
    spec["metadata"]["name"] = name
    env = spec["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]["env"]
    vals = {"JOB_NAME": name, "NP": str(np_), "MIN_NP": str(min_np), "MAX_NP": str(max_np), "EPOCHS": str(epochs)}
    for e in env:
        e["value"] = vals[e["name"]]
    c = spec["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]
    c["args"] = [f"python -m vodascheduler_amd.workloads.train --model {model} --epochs $(EPOCHS) "
                 f"--steps-per-epoch {steps} --batch-size 32"]
    p = tmp_path / f"{name}.yaml"
    p.write_text(yaml.safe_dump(spec))
    return str(p)


def test_reference_and_example_yamls_resolve_to_workloads():
    import glob

    for f in glob.glob(os.path.join(ROOT, "examples/yaml/*.yaml")):
        wl = workload_of(yaml.safe_load(open(f)))
        assert wl["steps_per_epoch"] > 0 and wl["model"]


def test_cli_up_create_get_delete_cpu(tmp_path):
    sched, svc = _cluster(tmp_path)
    try:
        sched.agent.wait_healthy(120)
        _wait(lambda: sched.runner.call(lambda: sched.core.total_gpus) == 2, 30, "inventory")
        surl, kurl = f"http://127.0.0.1:{svc.port}", f"http://127.0.0.1:{sched.http.port}"
        f = _job_yaml(tmp_path, "mnist-a", "mnist-torch", 20, 2, 1, 1, 2)
        buf = io.StringIO()
        with redirect_stdout(buf):
            assert cli(["--service", surl, "create", "-f", f]) == 0
        name = buf.getvalue().strip().split()[-1]
        assert name.startswith("mnist-a-")
        done = _wait(lambda: sched.runner.call(lambda: {n: j.status for n, j in sched.core.done_jobs.items()}),
                     120, "job completion")
        assert done[name] == "Completed"
        buf = io.StringIO()
        with redirect_stdout(buf):
            assert cli(["--scheduler", kurl, "get", "jobs"]) == 0
        assert name in buf.getvalue() and "Completed" in buf.getvalue()
        with redirect_stdout(io.StringIO()):
            assert cli(["--scheduler", kurl, "set", "algorithm", "AFS-L"]) == 0
            assert cli(["--scheduler", kurl, "set", "ratelimit", "2"]) == 0
            assert cli(["--scheduler", kurl, "set", "algorithm", "NoSuch"]) == 1
        assert sched.runner.call(lambda: sched.core.algorithm) == "AFS-L"
        # delete of several names: each is sent (reference bug: only the first)
        f2 = _job_yaml(tmp_path, "mnist-b", "mnist-torch", 5000, 5, 1, 1, 1)
        f3 = _job_yaml(tmp_path, "mnist-c", "mnist-torch", 5000, 5, 1, 1, 1)
        names = []
        for ff in (f2, f3):
            buf = io.StringIO()
            with redirect_stdout(buf):
                assert cli(["--service", surl, "create", "-f", ff]) == 0
            names.append(buf.getvalue().strip().split()[-1])
        _wait(lambda: all(n in sched.runner.call(lambda: dict(sched.core.ready_jobs)) for n in names), 30, "queued")
        with redirect_stdout(io.StringIO()):
            assert cli(["--service", surl, "delete"] + names) == 0
        _wait(lambda: not any(n in sched.runner.call(lambda: dict(sched.core.ready_jobs)) for n in names), 60,
              "deleted jobs leave the scheduler")
    finally:
        svc.stop()
        sched.stop()


def test_worker_death_job_survives_and_worker_rejoins(tmp_path):
    sched, svc = _cluster(tmp_path)
    try:
        agent, backend = sched.agent, sched.backend
        agent.wait_healthy(120)
        _wait(lambda: sched.runner.call(lambda: sched.core.total_gpus) == 2, 30, "inventory")
        spec = yaml.safe_load(open(_job_yaml(tmp_path, "mnist-ft", "mnist-torch", 400, 3, 2, 1, 2)))
        TrainingService(sched.store, sched.mq).create_training_job(json.dumps(spec))
        name = _wait(lambda: next((n for n, m in backend.members.items() if len(m) == 2), None), 60, "2-worker job")
        # let it train a little, then kill one of its workers
        _wait(lambda: backend.resize_latency, 60, "first sync")
        victim = backend.members[name][1]
        agent.kill_worker(victim)
        _wait(lambda: backend.failures, 30, "failure detected")
        assert backend.failures[0]["worker"] == victim and backend.failures[0]["survivors"] == 1
        done = _wait(lambda: sched.runner.call(lambda: {n: j.status for n, j in sched.core.done_jobs.items()}),
                     240, "job completion after failure")
        assert done[name] == "Completed"
        # the killed worker was restarted and is schedulable again
        _wait(lambda: len(agent.healthy_gpus()) == 2, 120, "worker restart")
        assert agent.workers[victim].failures == 1
    finally:
        svc.stop()
        sched.stop()
