"""Elastic runtime on CPU/gloo with real worker processes (BASELINE config 1: Elastic-FIFO,
2 toy MNIST jobs, simulated 2-slot cluster) + runtime unit tests."""
import multiprocessing as mp
import os

import pytest
import torch

from vodascheduler_amd.parallel.comm import GlooCommunicator, LocalCommunicator
from vodascheduler_amd.parallel.ddp import ElasticDDP
from vodascheduler_amd.runtime.cluster import cpu_worker_main, free_port, run_trace
from vodascheduler_amd.runtime.rendezvous import JobRendezvous, connect_store
from vodascheduler_amd.sim.trace import TraceJob, make_spec
from vodascheduler_amd.workloads.metrics_logger import MetricsCSVLogger


def _spawn_workers(port, wids):
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=cpu_worker_main, args=("127.0.0.1", port, w), daemon=True) for w in wids]
    for p in ps:
        p.start()
    return ps


def test_two_mnist_jobs_elastic_fifo_two_slots(tmp_path):
    os.environ["VODA_CKPT_DIR"] = str(tmp_path / "ckpt")
    port = free_port()
    store = connect_store("127.0.0.1", port, is_master=True)
    locs = [("node0", 0), ("node0", 1)]
    procs = _spawn_workers(port, [f"{n}:{g}" for n, g in locs])
    try:
        trace = [TraceJob(0.0, make_spec("mnist-a", "mnist-torch", 2, 1, 2, 2, 40)),
                 TraceJob(1.0, make_spec("mnist-b", "mnist-torch", 1, 1, 2, 2, 40))]
        r = run_trace(store, trace, locs, "ElasticFIFO", rate_limit_sec=0.2, tick_sec=0.5,
                      train_defaults={"commit_every": 1, "metrics_dir": str(tmp_path / "metrics"), "amp": False},
                      timeout=240)
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    assert r["n_jobs"] == 2 and not r["failed"], r
    kinds = [(e["job"].split("-2")[0], e["kind"], e["world"]) for e in r["events"]]
    # job a starts on 2 slots, shrinks to 1 when b arrives, b later grows to 2 when a finishes
    assert ("mnist-a", "start", 2) in kinds
    assert any(k[0] == "mnist-a" and k[1] == "scale_in" and k[2] == 1 for k in kinds), kinds
    assert any(k[0] == "mnist-b" and k[1] == "start" for k in kinds), kinds
    assert r["start_latency_p50_s"] is not None and r["start_latency_p50_s"] < 30
    assert r["n_starts"] >= 2 and r["n_shrinks_to_1"] >= 1  # a: 2 -> 1 (no communicator at world 1)
    csvs = sorted(f for f in os.listdir(tmp_path / "metrics") if f.endswith(".csv"))
    assert len(csvs) == 2
    rows = open(tmp_path / "metrics" / csvs[0]).read().splitlines()
    assert rows[0].startswith("epoch,start_time,epoch_time_sec,step_time_sec,steps,workers")
    assert len(rows) == 3  # header + 2 epochs
    # fast online profiling: rank 0's progress file holds GPU/CPU-timed steps per world size
    import json

    prog = json.load(open(tmp_path / "metrics" / csvs[0].replace(".csv", ".progress.json")))
    assert prog["samples_done"] == prog["samples_total"] > 0
    assert prog["perf"] and all(int(n) > 0 and s > 0 for n, s in prog["perf"].values())


def _ddp_worker(port, rank, world, q):
    torch.set_num_threads(1)
    store = connect_store("127.0.0.1", port)
    comm = GlooCommunicator(store, "t/ddp", rank, world, timeout=60)
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 300), torch.nn.ReLU(), torch.nn.Linear(300, 4))
    ddp = ElasticDDP(m, comm, None, bucket_cap_mb=0.001, first_bucket_mb=0.0005)
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(8, 16, generator=g)
    ddp.zero_grad()
    m(x).square().mean().backward()
    ddp.finalize()
    # numpy payloads pickle by value (torch tensors would be shared by fd and die with us)
    q.put((rank, [p.grad.numpy().copy() for p in m.parameters()], len(ddp.buckets), x.numpy().copy()))


def test_ddp_bucketed_allreduce_matches_full_batch():
    port = free_port()
    store = connect_store("127.0.0.1", port, is_master=True)  # noqa: F841 (keeps the server alive)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ddp_worker, args=(port, r, 2, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, ([torch.from_numpy(a) for a in g], nb, torch.from_numpy(x)))
               for r, g, nb, x in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(30)
    assert res[0][1] > 2  # several buckets
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 300), torch.nn.ReLU(), torch.nn.Linear(300, 4))
    x = torch.cat([res[0][2], res[1][2]])
    # mean of per-rank mean losses == mean over the concatenated batch
    m(x).square().mean().backward()
    for a, b, ref in zip(res[0][0], res[1][0], [p.grad for p in m.parameters()]):
        torch.testing.assert_close(a, b)
        torch.testing.assert_close(a, ref, rtol=1e-5, atol=1e-6)


def test_local_ddp_world_one_noop():
    m = torch.nn.Linear(4, 4)
    ddp = ElasticDDP(m, LocalCommunicator(torch.device("cpu")))
    m(torch.randn(2, 4)).sum().backward()
    ddp.finalize()
    assert m.weight.grad is not None


def test_rendezvous_publish_and_outcome():
    port = free_port()
    store = connect_store("127.0.0.1", port, is_master=True)
    r = JobRendezvous(store, "j")
    assert r.latest_epoch() == 0
    assert r.publish(["a", "b"]) == 1
    assert r.publish(["a"], abort=True) == 2
    assert r.members(1) == ["a", "b"] and r.members(2) == ["a"]
    assert r.aborted(2) and not r.aborted(1)
    assert r.outcome() is None
    r.mark_done()
    assert r.outcome() == "done"


def test_metrics_logger_resume(tmp_path):
    lg = MetricsCSVLogger(str(tmp_path), "job", 5, 32)
    lg.log_epoch(0, 0.0, 2.0, 10, 1.5, workers=2)
    lg.log_epoch(1, 2.0, 1.0, 10, 1.2, workers=4)
    assert MetricsCSVLogger(str(tmp_path), "job", 5, 32).restored_epoch() == 2


def _cache_worker(port, rank, q):
    import torch.distributed  # noqa: F401
    from vodascheduler_amd.parallel.comm import COMM_CACHE, create_communicator
    torch.set_num_threads(1)
    store = connect_store("127.0.0.1", port)
    members = ["w0", "w1"]
    dev = torch.device("cpu")
    out = []
    for epoch in range(4):
        if epoch == 3 and rank == 1:
            COMM_CACHE.clear()      # e.g. a restarted worker: nobody may reuse
        c = create_communicator(store, f"t/cache/{epoch}", rank, 2, dev, "gloo", 60, members=members)
        t = torch.full((4,), float(rank + epoch))
        c.allreduce_(t)
        out.append((c.cid, float(t[0])))
        if epoch == 1:
            # a different member order is a different communicator
            c2 = create_communicator(store, "t/cache/perm", rank, 2, dev, "gloo", 60, members=members[::-1])
            assert c2.cid != c.cid
            COMM_CACHE.put(c2)
        COMM_CACHE.put(c)
    q.put((rank, out, COMM_CACHE.hits, len(COMM_CACHE)))
    COMM_CACHE.clear()


def test_comm_cache_reuses_same_member_list():
    port = free_port()
    store = connect_store("127.0.0.1", port, is_master=True)  # noqa: F841
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_cache_worker, args=(port, r, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (o, h, n)) for r, o, h, n in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(30)
    for r in range(2):
        out, hits, n = res[r]
        cids = [c for c, _ in out]
        assert cids[0] == cids[1] == cids[2]      # epochs 1, 2 reuse epoch 0's communicator
        assert cids[3] != cids[0]                 # rank 1 lost its cache: rebuilt everywhere
        assert [v for _, v in out] == [1.0, 3.0, 5.0, 7.0]
        assert hits == 2 and n == (2 if r == 0 else 1)  # rank 1 dropped the permuted one too
    assert res[0][0] == res[1][0]
