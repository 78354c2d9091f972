"""Multi-GPU data plane on RCCL over xGMI.  Skipped on boxes with fewer
than two GPUs; on an 8 x MI355X node it spawns 2 / 4 / 8 rank processes, one per GPU:

* RcclCommunicator all-reduce (sum / avg / max) / broadcast / all-gather against host sums,
  fp32 and bf16;
* ElasticDDP bucketed fp32 gradients == single-process full-batch gradients;
* a live resize 2 -> 4 -> 2 of one job on RCCL: every member ends with bitwise-identical
  parameters and optimizer slots, equal to a replay of the same trajectory through real
  RCCL communicators of the same world sizes (workloads/replay.py: the replay performs the
  same ring reduction, so only per-rank kernel nondeterminism is left to the tolerance; the
  lock-step digests name the first divergent step on a failure);
* the abort-epoch path: one rank is killed, the survivors restore the last commit and finish.
"""
import multiprocessing as mp
import os

import pytest
import torch

N_DEV = torch.cuda.device_count() if torch.cuda.is_available() else 0
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(N_DEV < 2, reason="needs >= 2 GPUs")]


def _coll_worker(port, rank, world, q):
    torch.cuda.set_device(rank)
    from vodascheduler_amd.parallel.comm import RcclCommunicator
    from vodascheduler_amd.runtime.rendezvous import connect_store

    store = connect_store("127.0.0.1", port)
    dev = torch.device("cuda", rank)
    comm = RcclCommunicator(store, f"t/coll/{world}", rank, world, dev, timeout=120)
    out = {}
    for dt in (torch.float32, torch.bfloat16):
        g = torch.Generator(device="cpu").manual_seed(rank)
        x = torch.randn(3 * (1 << 20) + 7, generator=g).to(dt)   # odd size: no alignment luck
        for op in ("sum", "avg", "max"):
            t = x.to(dev)
            comm.allreduce_(t, op)
            torch.cuda.synchronize()
            out[(str(dt), op)] = t.float().cpu()
        b = x.to(dev)
        comm.broadcast_(b, root=world - 1)
        torch.cuda.synchronize()
        out[(str(dt), "bcast")] = b.float().cpu()
        gat = comm.allgather(x[:4096].to(dev))
        torch.cuda.synchronize()
        out[(str(dt), "gather")] = gat.float().cpu()
    comm.check()
    comm.destroy()
    q.put((rank, {k: v.numpy() for k, v in out.items()}))


from elastic_harness import spawn_ranks as _spawn  # noqa: E402


@pytest.mark.parametrize("world", sorted({2, min(4, N_DEV), min(8, N_DEV)}))
def test_rccl_collectives_match_host(world):
    res = _spawn(_coll_worker, world)
    for dt in (torch.float32, torch.bfloat16):
        xs = [torch.randn(3 * (1 << 20) + 7, generator=torch.Generator().manual_seed(r)).to(dt).float()
              for r in range(world)]
        tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=2e-2, atol=2e-2 * world)
        want = {"sum": sum(xs), "avg": sum(xs) / world, "max": torch.stack(xs).max(0).values,
                "bcast": xs[world - 1], "gather": torch.stack([x[:4096] for x in xs])}
        for r in range(world):
            for k, w in want.items():
                got = torch.from_numpy(res[r][(str(dt), k)])
                torch.testing.assert_close(got, w, **(tol if k in ("sum", "avg") else dict(rtol=0, atol=0)))


def _ddp_worker(port, rank, world, q):
    torch.cuda.set_device(rank)
    from vodascheduler_amd.ops.optim import make_optimizer
    from vodascheduler_amd.parallel.comm import RcclCommunicator
    from vodascheduler_amd.parallel.ddp import ElasticDDP
    from vodascheduler_amd.runtime.rendezvous import connect_store
    from vodascheduler_amd.utils.flat import grad_of

    store = connect_store("127.0.0.1", port)
    dev = torch.device("cuda", rank)
    comm = RcclCommunicator(store, "t/ddp", rank, world, dev, timeout=120)
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(64, 2048), torch.nn.ReLU(), torch.nn.Linear(2048, 2048),
                            torch.nn.ReLU(), torch.nn.Linear(2048, 10)).to(dev)
    opt = make_optimizer("sgd", m.parameters(), lr=0.0)
    ddp = ElasticDDP(m, comm, opt, bucket_cap_mb=4, first_bucket_mb=1)
    x = torch.randn(32, 64, generator=torch.Generator().manual_seed(100 + rank)).to(dev)
    for _ in range(2):  # calibration step, then the overlapped path
        ddp.zero_grad()
        m(x).square().mean().backward()
        ddp.finalize()
    torch.cuda.synchronize()
    q.put((rank, ([grad_of(p).cpu().numpy() for p in m.parameters()], len(ddp.buckets))))
    comm.destroy()


@pytest.mark.parametrize("world", sorted({2, min(8, N_DEV)}))
def test_ddp_bucketed_fp32_grads_match_full_batch(world):
    res = _spawn(_ddp_worker, world)
    assert res[0][1] >= 3
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(64, 2048), torch.nn.ReLU(), torch.nn.Linear(2048, 2048),
                            torch.nn.ReLU(), torch.nn.Linear(2048, 10)).double()
    xs = [torch.randn(32, 64, generator=torch.Generator().manual_seed(100 + r)) for r in range(world)]
    m(torch.cat(xs).double()).square().mean().backward()
    for r in range(world):
        for got, p in zip(res[r][0], m.parameters()):
            torch.testing.assert_close(torch.from_numpy(got).double(), p.grad, rtol=1e-4, atol=1e-6)
    for a, b in zip(res[0][0], res[world - 1][0]):
        assert (a == b).all()  # every rank holds the identical averaged gradient


def _cfg(tmp_path, name, **kw):
    from vodascheduler_amd.workloads.train import TrainConfig

    d = dict(model="mnist-torch", epochs=2, steps_per_epoch=600, per_gpu_batch=64, lr=0.01, commit_every=1,
             amp=False, report_progress=True, final_state_path=str(tmp_path / f"{name}.pt"), graph=False,
             step_digests=True,  # every RCCL run is checked step by step (world + LR exact)
             # deterministic MIOpen solvers: without them the run and its replay drift apart from
             # step 1 on (atomic split-K weight gradients; tests/test_elastic_one_gpu_gpu.py found
             # 3.9e-3 after 400 MNIST steps), so only the ring reduction order is left to the tolerance
             deterministic=True)
    d.update(kw)
    return TrainConfig(**d)


@pytest.fixture
def gpu_pool(tmp_path, monkeypatch):
    from elastic_harness import start_pool, stop_pool

    monkeypatch.setenv("VODA_CKPT_DIR", str(tmp_path / "ckpt"))
    n = min(4, N_DEV)
    wids = [f"node0:{i}" for i in range(n)]
    store, procs, q = start_pool(wids, [f"cuda:{i}" for i in range(n)], "rccl")
    box = {}

    def finish():
        if "results" not in box:
            box["results"] = stop_pool(store, procs, q, timeout=60)
        return box["results"]

    yield store, procs, wids, finish
    finish()


def _digests(results, job):
    return {w: r["result"]["state_digest"] for w, recs in results.items() for r in recs
            if r["job"] == job and isinstance(r["result"], dict) and r["result"].get("state_digest")}


def test_live_resize_2_4_2_on_rccl(gpu_pool, tmp_path):
    from elastic_harness import Controller, assert_matches_replay

    store, procs, wids, finish = gpu_pool
    cfg = _cfg(tmp_path, "resize")
    c = Controller(store, "resize", cfg)
    c.publish(wids[:2])
    c.wait_progress(20)
    if len(wids) >= 4:
        c.publish(wids[:4])
        c.wait_progress(c.progress() + 20)
    c.publish([wids[0], wids[-1]])   # shrink onto a different pair: one member migrates
    assert c.wait_done(timeout=240) == "done"
    ex = assert_matches_replay(cfg, cfg.final_state_path, "cuda:0", exact=False, backend="rccl")
    ws = [ex["world_log"][i + 1] for i in range(0, len(ex["world_log"]), 2)]
    assert ws[0] == 2 and ws[-1] == 2 and (len(wids) < 4 or 4 in ws), ex["world_log"]
    dig = _digests(finish(), "resize")
    assert set(dig) == {wids[0], wids[-1]}, dig      # the final members
    assert len(set(dig.values())) == 1, dig          # bitwise-identical parameters + optimizer slots


def test_abort_epoch_survivors_restore_and_finish(gpu_pool, tmp_path):
    from elastic_harness import Controller, assert_matches_replay

    store, procs, wids, finish = gpu_pool
    cfg = _cfg(tmp_path, "kill", commit_every=4)
    c = Controller(store, "kill", cfg)
    c.publish(wids[:2])
    c.wait_progress(30)
    procs[wids[1]].kill()
    procs[wids[1]].join(10)
    c.publish(wids[:1], abort=True)
    assert c.wait_done(timeout=240) == "done"
    ex = assert_matches_replay(cfg, cfg.final_state_path, "cuda:0", exact=False, backend="rccl")
    assert ex["world_log"][-1] == 1 and ex["world_log"][-2] % 4 == 0
