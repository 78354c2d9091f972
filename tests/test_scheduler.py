"""Scheduler state machine with an injectable clock, in-memory store, in-proc MQ and a
recording backend; REST contract tests; simulator runs."""
import json

import pytest

from vodascheduler_amd.allocator.allocator import AllocationRequest, ResourceAllocator
from vodascheduler_amd.allocator.server import allocator_router
from vodascheduler_amd.backend.base import HALT, SCALE_IN, SCALE_OUT, START, NullBackend
from vodascheduler_amd.common.mq import InProcQueue, Msg, SqliteQueue
from vodascheduler_amd.common.store import MemoryStore, SqliteStore
from vodascheduler_amd.common.types import DEFAULT_GPU_TYPE, JobStatus
from vodascheduler_amd.scheduler.api import scheduler_router
from vodascheduler_amd.scheduler.core import SchedulerCore
from vodascheduler_amd.scheduler.runner import SchedulerRunner
from vodascheduler_amd.service.service import TrainingService
from vodascheduler_amd.sim import make_spec, philly_trace, simulate
from vodascheduler_amd.utils.clock import ManualClock
from vodascheduler_amd.utils.http import HttpServer, http_request

GPU = DEFAULT_GPU_TYPE


class Env:
    def __init__(self, gpus=8, algorithm="ElasticFIFO", rate=30.0, store=None, backend=None, resume=False,
                 clock=None):
        self.clock = clock or ManualClock(1000.0)
        self.store = store or MemoryStore()
        self.mq = InProcQueue()
        self.svc = TrainingService(self.store, self.mq, self.clock)
        self.backend = backend or NullBackend({"node0": list(range(gpus))})
        self.core = SchedulerCore(GPU, self.store, ResourceAllocator(self.store), self.backend, clock=self.clock,
                                  algorithm=algorithm, rate_limit_sec=rate, resume=resume)

    def submit(self, name, np_=1, mn=1, mx=4, epochs=2, prio=None):
        n = self.svc.create_training_job(json.dumps(make_spec(name, "resnet50", np_, mn, mx, epochs, 10,
                                                              priority=prio)))
        m = self.mq.get(GPU)
        assert m.verb == "create" and m.job_name == n
        self.core.create_training_job(n)
        return n

    def step(self, dt=0.0):
        self.clock.advance(dt)
        self.core.poll()


def test_create_runs_job_and_persists_status():
    e = Env()
    n = e.submit("a", 2, 1, 4)
    assert e.core.get_job_status(n) == JobStatus.WAITING
    e.step()
    assert e.core.get_job_status(n) == JobStatus.RUNNING
    assert e.core.job_num_gpu[n] == 4  # elastic: grows to max on an idle node
    assert e.backend.log[-1].kind == START and len(e.backend.log[-1].workers) == 4
    assert e.store.find_metadata(n)["status"] == "Running"
    assert e.store.find_metadata(n)["spec"]["spec"]["mpiReplicaSpecs"]["Worker"]["replicas"] == 4


def test_rate_limit_coalesces_requests():
    e = Env(rate=30)
    a = e.submit("a", 1, 1, 8)
    e.step()
    assert e.core.resched_count == 1
    b = e.submit("b", 1, 1, 8)
    c = e.submit("c", 1, 1, 8)
    e.step(1)
    assert e.core.resched_count == 1  # blocked by the 30 s rate limit
    e.step(28)
    assert e.core.resched_count == 1  # t = 1029 < 1030
    e.step(1)
    assert e.core.resched_count == 2  # both arrivals handled by ONE reschedule
    assert {e.core.job_num_gpu[x] for x in (a, b, c)} <= {2, 3}
    e.step(100)
    assert e.core.resched_count == 2  # nothing pending, nothing runs


@pytest.mark.parametrize("work_conserving", [True, False])
def test_completion_reschedules_immediately_when_work_conserving(work_conserving):
    e = Env(gpus=2, algorithm="FIFO", rate=30)
    e.core.work_conserving = work_conserving
    a = e.submit("a", 2, 2, 2)
    e.step()
    b = e.submit("b", 2, 2, 2)
    e.step(1)
    assert e.core.job_num_gpu[b] == 0  # queued behind a, arrival rate-limited
    e.core.handle_job_finished(a, True)
    e.step(1)
    # freed GPUs go to the waiting job at once; the reference waits out the rate limit
    assert e.core.job_num_gpu[b] == (2 if work_conserving else 0)
    e.step(30)
    assert e.core.job_num_gpu[b] == 2
    c = e.submit("c", 1, 1, 1)
    e.step(1)
    assert e.core.job_num_gpu[c] == 0  # arrivals on a full cluster are still rate-limited


def test_arrival_on_idle_gpus_starts_immediately():
    e = Env(gpus=4, algorithm="FIFO", rate=30)
    a = e.submit("a", 2, 2, 2)
    e.step()
    b = e.submit("b", 2, 2, 2)
    e.step(1)
    assert e.core.job_num_gpu[b] == 2  # 2 GPUs were idle: no rate-limit wait


def test_finish_and_scale_actions():
    e = Env(rate=0)
    a = e.submit("a", 1, 1, 8)
    e.step()
    b = e.submit("b", 2, 2, 8)
    e.step()
    kinds = [(x.kind, x.job.name) for x in e.backend.log]
    assert (SCALE_IN, a) in kinds and (START, b) in kinds
    e.core.handle_job_finished(a, True)
    e.step()
    assert e.core.get_job_status(a) == JobStatus.COMPLETED
    assert e.core.job_num_gpu[b] == 8
    assert any(x.kind == SCALE_OUT and x.job.name == b for x in e.backend.log)


def test_halt_when_preempted_by_fifo_order():
    e = Env(gpus=4, algorithm="Tiresias", rate=0)
    low = e.submit("low", 4, 4, 4, prio=1)
    e.step()
    assert e.core.job_num_gpu[low] == 4
    hi = e.submit("hi", 4, 4, 4, prio=0)
    e.step()
    assert e.core.job_num_gpu[hi] == 4 and e.core.job_num_gpu[low] == 0
    assert any(x.kind == HALT and x.job.name == low for x in e.backend.log)
    assert e.core.get_job_status(low) == JobStatus.WAITING


def test_tiresias_demotion_and_promotion():
    e = Env(gpus=4, algorithm="Tiresias", rate=0)
    a = e.submit("a", 4, 4, 4)
    e.step()
    # 4 GPUs * 901 s > 3600 GPU-seconds -> demoted to queue 1 at a 5 s tick
    for _ in range(182):
        e.step(5)
    assert e.core.ready_jobs[a].priority == 1
    b = e.submit("b", 4, 4, 4)
    e.step()
    assert e.core.job_num_gpu[b] == 4 and e.core.job_num_gpu[a] == 0  # b (queue 0) preempts a
    # b is demoted after its own 3600 GPU-s, a (earlier first start) wins queue 1 back; b then
    # waits >= 8x its last running time and is promoted to queue 0, preempting a again
    hist = []
    for _ in range(3000):
        e.step(5)
        hist.append((e.core.ready_jobs[b].priority, e.core.job_num_gpu[b]))
    assert (1, 0) in hist
    i = hist.index((1, 0))
    assert (0, 4) in hist[i:]


def test_delete_running_job_tears_down_and_reschedules():
    e = Env(rate=0)
    a = e.submit("a")
    e.step()
    e.svc.delete_training_job(a)
    m = e.mq.get(GPU)
    assert m.verb == "delete"
    e.core.delete_training_job(m.job_name)
    assert a in e.backend.deleted and e.core.get_job_status(a) is None


def test_allocator_failure_retries_after_rate_limit():
    class Flaky(ResourceAllocator):
        fails = 1

        def allocate(self, req):
            if self.fails:
                self.fails -= 1
                raise RuntimeError("down")
            return super().allocate(req)

    e = Env(rate=10)
    e.core.allocator = Flaky(e.store)
    a = e.submit("a")
    e.step()
    assert e.core.job_num_gpu[a] == 0
    e.step(10)
    assert e.core.job_num_gpu[a] == 0  # retry scheduled at +11 s
    e.step(1.5)
    assert e.core.job_num_gpu[a] > 0


def test_resume_reconstructs_state(tmp_path):
    store = SqliteStore(str(tmp_path / "voda.db"))
    e = Env(store=store, rate=0)
    a = e.submit("a", 2, 2, 2)
    b = e.submit("b", 2, 2, 2)
    e.step()
    running = e.backend.list_running()
    e2 = Env(store=SqliteStore(str(tmp_path / "voda.db")), backend=NullBackend({"node0": list(range(8))}),
             resume=False)
    e2.backend.running = running
    e3 = SchedulerCore(GPU, e2.store, ResourceAllocator(e2.store), e2.backend, clock=e2.clock, resume=True,
                       rate_limit_sec=0)
    assert e3.job_num_gpu[a] == 2 and e3.job_num_gpu[b] == 2
    assert e3.ready_jobs[a].status == "Running"
    e3.poll()
    assert not [x for x in e2.backend.log if x.kind != "migrate" or x.workers != running.get(x.job.name)]


def test_status_table_format():
    e = Env()
    e.submit("a")
    e.step()
    lines = e.core.get_all_training_jobs().splitlines()
    assert lines[0].split() == ["NAME", "STATUS", "WORKERS", "SCHEDULER", "WAITING", "RUNNING", "TOTAL"]
    assert "Running" in lines[1] and GPU in lines[1]


def test_gpu_drain_migrates_worker():
    e = Env(rate=0)
    a = e.submit("a", 4, 4, 4)
    b = e.submit("b", 4, 4, 4)
    e.step()
    victim = e.core.job_workers[a][0]
    e.backend._nodes = {"node0": [g for g in range(8) if g != victim[1]]}
    e.core.set_nodes(e.backend.nodes())
    e.step()
    assert e.core.total_gpus == 7
    locs = [l for v in e.core.job_workers.values() for l in v]
    assert victim not in locs


def test_sqlite_queue_cross_instance(tmp_path):
    p = str(tmp_path / "mq.db")
    q1, q2 = SqliteQueue(p), SqliteQueue(p)
    q1.publish("gpu-a", Msg("create", "j1"))
    q1.publish("gpu-b", Msg("create", "j2"))
    assert q2.get("gpu-a").job_name == "j1"
    assert q2.get("gpu-a", timeout=0.05) is None
    assert q2.get("gpu-b").job_name == "j2"


def test_allocation_request_json_shape():
    e = Env()
    e.submit("a")
    req = AllocationRequest(GPU, 8, "FIFO", e.core.make_ready_jobs_list())
    d = json.loads(json.dumps(req.to_dict()))
    assert set(d) == {"SchedulerID", "NumGpu", "AlgorithmName", "ReadyJobs"}
    assert "job_name" in d["ReadyJobs"][0] and "info" not in d["ReadyJobs"][0]
    back = AllocationRequest.from_dict(d)
    assert back.ready_jobs[0].name == req.ready_jobs[0].name


def test_rest_end_to_end():
    store, mq = MemoryStore(), InProcQueue()
    svc = TrainingService(store, mq)
    s_srv = HttpServer(svc.router(), host="127.0.0.1", port=0).start()
    alloc_srv = HttpServer(allocator_router(ResourceAllocator(store)), host="127.0.0.1", port=0).start()
    from vodascheduler_amd.allocator.allocator import HttpAllocatorClient

    core = SchedulerCore(GPU, store, HttpAllocatorClient(f"http://127.0.0.1:{alloc_srv.port}"),
                         NullBackend(), rate_limit_sec=0.0)
    runner = SchedulerRunner(core, mq).start()
    sch_srv = HttpServer(scheduler_router(runner), host="127.0.0.1", port=0).start()
    try:
        spec = make_spec("rest-job", "resnet50", 1, 1, 2, 1, 5)
        import yaml

        st, body = http_request("POST", f"http://127.0.0.1:{s_srv.port}/training", yaml.safe_dump(spec).encode(),
                                content_type="application/yaml")
        assert st == 200 and b"Training job created: rest-job-" in body
        name = body.decode().split(": ")[1].strip()
        import time

        for _ in range(100):
            st, table = http_request("GET", f"http://127.0.0.1:{sch_srv.port}/training")
            if b"Running" in table:
                break
            time.sleep(0.05)
        assert name.encode() in table and b"Running" in table
        assert http_request("PUT", f"http://127.0.0.1:{sch_srv.port}/algorithm", b'"AFS-L"')[0] == 200
        assert core.algorithm == "AFS-L"
        assert http_request("PUT", f"http://127.0.0.1:{sch_srv.port}/algorithm", b'"Bogus"')[0] == 400
        assert http_request("PUT", f"http://127.0.0.1:{sch_srv.port}/ratelimit", b"7")[0] == 200
        assert core.rate_limit_sec == 7
        st, m = http_request("GET", f"http://127.0.0.1:{sch_srv.port}/metrics")
        assert b"voda_scheduler_amd_instinct_mi355x_scheduler_jobs_created_total 1.0" in m
        assert b"voda_scheduler_amd_instinct_mi355x_scheduler_gpus 8.0" in m
        st, m = http_request("GET", f"http://127.0.0.1:{alloc_srv.port}/metrics")
        assert b"voda_scheduler_resource_allocator_labeled_num_gpus_count" in m
        st, m = http_request("GET", f"http://127.0.0.1:{s_srv.port}/metrics")
        assert b"voda_scheduler_training_service_jobs_created_total 1.0" in m
        st, body = http_request("DELETE", f"http://127.0.0.1:{s_srv.port}/training", json.dumps(name).encode())
        assert st == 200, body
        for _ in range(100):
            if core.get_job_status(name) is None:
                break
            time.sleep(0.05)
        assert core.get_job_status(name) is None
        assert http_request("DELETE", f"http://127.0.0.1:{s_srv.port}/training", b"unquoted")[0] == 400
    finally:
        runner.stop()
        for s in (s_srv, alloc_srv, sch_srv):
            s.stop()


def test_service_rejects_spec_without_gpu_type():
    e = Env()
    spec = make_spec("x", "resnet50", 1, 1, 1, 1, 1)
    del spec["spec"]["mpiReplicaSpecs"]["Worker"]["template"]["spec"]["nodeSelector"]
    with pytest.raises(ValueError, match="gpu type not specified"):
        e.svc.create_training_job(json.dumps(spec))
    assert e.store.list_metadata() == []


@pytest.mark.parametrize("algo", ["FIFO", "ElasticFIFO", "SRJF", "ElasticSRJF", "Tiresias", "ElasticTiresias",
                                  "FfDLOptimizer", "AFS-L"])
def test_simulator_completes_trace(algo):
    r = simulate(philly_trace(32, seed=1), algo, gpus=8)
    assert r.n_jobs == 32 and r.avg_jct > 0 and r.makespan > 0 and 0 < r.utilization <= 1.0 + 1e-9


def test_elastic_beats_fifo_on_makespan():
    tr = philly_trace(32, seed=2)
    fifo = simulate(tr, "FIFO", gpus=8)
    efifo = simulate(tr, "ElasticFIFO", gpus=8)
    assert efifo.makespan < fifo.makespan and efifo.avg_jct < fifo.avg_jct


def test_simulated_drain_migrations():
    tr = philly_trace(16, seed=3)
    r = simulate(tr, "ElasticFIFO", gpus=8, drain=[(100.0, "node0", 3), (200.0, "node0", 5)])
    assert r.n_jobs == 16 and r.migrations >= 1


def test_gpu_time_charged_at_allocation_held_during_interval():
    """the interval closed at a halt / scale-out is charged at the OLD allocation."""
    e = Env(gpus=4, algorithm="Tiresias", rate=0)
    low = e.submit("low", 2, 2, 2, prio=1)
    e.step()
    assert e.core.job_num_gpu[low] == 2
    e.clock.advance(10)
    hi = e.submit("hi", 4, 4, 4, prio=0)
    e.step()  # low is halted: its last 10 s ran on 2 GPUs
    assert e.core.job_num_gpu[low] == 0
    m = e.core.ready_jobs[low].time_metrics
    assert m.gpu_time == pytest.approx(20.0)
    assert m.last_gpu_time == pytest.approx(20.0)
    # scale-out: a 1-GPU elastic job grows to 4 once the other finishes
    e2 = Env(gpus=4, algorithm="ElasticFIFO", rate=0)
    a = e2.submit("a", 2, 2, 2)
    b = e2.submit("b", 1, 1, 4)
    e2.step()
    assert e2.core.job_num_gpu[b] == 2
    e2.clock.advance(5)
    e2.core.handle_job_finished(a, True)
    e2.step()
    assert e2.core.job_num_gpu[b] == 4
    assert e2.core.ready_jobs[b].time_metrics.gpu_time == pytest.approx(10.0)


def test_autoscale_node_addition_grows_jobs_in_place():
    """Node addition (reference addNode / updateNode, scheduler.go:689-747;
    placement_manager.go:239-304; README "node addition awareness"): a cluster that starts
    with one GPU and gains GPUs, then a second node.  Elastic jobs grow onto the new
    capacity at once (work-conserving, no rate-limit wait) and placement keeps every
    running worker where it is."""
    e = Env(rate=30.0, backend=NullBackend({"node0": [0]}))
    a = e.submit("a", 1, 1, 4)
    b = e.submit("b", 1, 1, 4)
    e.step()
    assert e.core.total_gpus == 1 and e.core.job_num_gpu == {a: 1, b: 0}
    a_loc = list(e.core.job_workers[a])
    e.backend._nodes = {"node0": [0, 1, 2]}
    e.core.set_nodes(e.backend.nodes())
    e.step()                                  # same instant: the added GPUs are used at once
    assert e.core.total_gpus == 3
    assert e.core.job_num_gpu[a] >= 1 and e.core.job_num_gpu[b] >= 1
    assert sum(e.core.job_num_gpu.values()) == 3
    assert set(a_loc) <= set(e.core.job_workers[a])           # a's worker did not move
    held = {j: list(v) for j, v in e.core.job_workers.items()}
    e.backend._nodes = {"node0": [0, 1, 2, 3], "node1": [0, 1, 2, 3]}
    e.core.set_nodes(e.backend.nodes())
    e.step()
    assert e.core.total_gpus == 8
    assert e.core.job_num_gpu == {a: 4, b: 4}                 # both at MAX_NP
    # node-level best fit consolidates each 4-worker job on one node (the reference's
    # objective); Munkres keeps the job holding most of node0 there, so only the smaller
    # job's workers move to the new node
    for j, locs in e.core.job_workers.items():
        assert len({n for n, _ in locs}) == 1, (j, locs)        # no cross-node job
    big = max(held, key=lambda j: len(held[j]))
    assert set(held[big]) <= set(e.core.job_workers[big])
    moved = sum(len(set(held[j]) - set(e.core.job_workers[j])) for j in held)
    assert moved <= min(len(v) for v in held.values()), (held, e.core.job_workers)


def test_simulated_capacity_ramp_1_to_8():
    """BASELINE config 5 ("autoscale 1->8"): the 32-job trace while capacity ramps 1 -> 2 ->
    4 -> 8 completes; JCT lands between the fixed-8 and fixed-1 clusters."""
    tr = philly_trace(32, seed=5, mean_interarrival_s=30, mean_duration_1gpu_s=300, max_gpus=8)
    ramp = [(0.0, {"node0": [0]}), (600.0, {"node0": [0, 1]}), (1200.0, {"node0": list(range(4))}),
            (1800.0, {"node0": list(range(8))})]
    r = simulate(tr, "FfDLOptimizer", gpus=8, capacity=ramp)
    full = simulate(tr, "FfDLOptimizer", gpus=8)
    one = simulate(tr, "FfDLOptimizer", gpus=1)
    assert r.n_jobs == 32 and full.avg_jct <= r.avg_jct <= one.avg_jct
    assert 0 < r.utilization <= 1.0
    assert r.peak_gpus == 8 and 1 < r.avg_gpus < 8


def test_simulated_drain_survives_later_capacity_snapshot():
    """A GPU drained before a capacity step stays drained: the snapshot is applied
    minus the drained GPUs, so the peak is 7 of the snapshot's 8."""
    tr = philly_trace(8, seed=2, mean_interarrival_s=20, mean_duration_1gpu_s=200, max_gpus=8)
    ramp = [(0.0, {"node0": list(range(4))}), (300.0, {"node0": list(range(8))})]
    r = simulate(tr, "ElasticFIFO", gpus=8, capacity=ramp, drain=[(100.0, "node0", 2)])
    assert r.n_jobs == 8 and r.peak_gpus == 7 and r.gpus == 7
    assert r.avg_gpus <= 7
