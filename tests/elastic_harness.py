"""Scripted elastic-job controller + pool-worker processes for the elastic-state equivalence
tests (CPU/gloo here, RCCL on a multi-GPU box).  The controller speaks the PoolBackend
protocol directly (membership epochs + worker mailboxes, runtime/pool.py) so a test can
resize, halt, restart and kill at chosen steps."""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import time
from dataclasses import asdict

import torch

from vodascheduler_amd.runtime.rendezvous import JobRendezvous, connect_store


def worker_proc(port: int, wid: str, device: str, backend: str, q) -> None:
    torch.set_num_threads(1)
    from vodascheduler_amd.runtime.pool import PoolWorker

    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    store = connect_store("127.0.0.1", port)
    watch = connect_store("127.0.0.1", port)
    recs = PoolWorker(store, watch, wid, dev, backend=backend, timeout=120.0).serve()
    q.put((wid, [{k: r[k] for k in ("job", "result")} for r in recs]))


class Controller:
    def __init__(self, store, job: str, cfg):
        self.store = store
        self.job = job
        self.cfg = asdict(cfg)
        self.rdzv = JobRendezvous(store, job)
        self.members: list[str] = []
        self.mail_n: dict[str, int] = {}

    def _mail(self, wid: str, msg: dict) -> None:
        # the pool's mailbox counter, not a per-controller one: several controllers (jobs) may
        # drive one pool one after another
        n = int(self.store.add(f"pool/{wid}/n", 0)) + 1
        self.mail_n[wid] = n
        self.store.set(f"pool/{wid}/msg/{n}", json.dumps(msg))
        self.store.add(f"pool/{wid}/n", 1)

    def publish(self, members: list[str], abort: bool = False, wait_sync: bool = True, timeout: float = 60) -> int:
        e = self.rdzv.publish(members, abort=abort)
        for w in members:
            if w not in self.members:
                self._mail(w, {"job": self.job, "epoch": e, "cfg": self.cfg})
        self.members = list(members)
        if wait_sync and members:
            self.wait(lambda: self.rdzv.get(f"e/{e}/synced") is not None or self.rdzv.outcome() is not None,
                      timeout, f"epoch {e} synced")
        return e

    def progress(self) -> int:
        v = self.rdzv.get("progress")
        return int(v) if v is not None else -1

    def wait_progress(self, step: int, timeout: float = 60) -> None:
        self.wait(lambda: self.progress() >= step or self.rdzv.outcome() is not None, timeout, f"step {step}")

    def wait_state_at_rest(self, timeout: float = 60) -> None:
        self.wait(lambda: (self.rdzv.get_live_epoch() or 0) < 0, timeout, "state at rest")

    def wait_done(self, timeout: float = 120) -> str:
        self.wait(lambda: self.rdzv.outcome() is not None, timeout, "job outcome")
        return self.rdzv.outcome()

    def wait(self, cond, timeout: float, what: str) -> None:
        deadline = time.monotonic() + timeout
        while not cond():
            if time.monotonic() > deadline:
                r = self.rdzv
                raise TimeoutError(f"timed out waiting for {what} (progress={self.progress()} "
                                   f"latest_epoch={r.latest_epoch()} live_epoch={r.get_live_epoch()} "
                                   f"outcome={r.outcome()} ckpt={r.get_ckpt()})")
            time.sleep(0.005)


def start_pool(wids: list[str], devices: list[str], backend: str):
    """Store server (this process) + one spawned PoolWorker per wid."""
    from vodascheduler_amd.runtime.cluster import free_port

    port = free_port()
    store = connect_store("127.0.0.1", port, is_master=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = {w: ctx.Process(target=worker_proc, args=(port, w, d, backend, q), daemon=True)
             for w, d in zip(wids, devices)}
    for p in procs.values():
        p.start()
    return store, procs, q


def stop_pool(store, procs, q, timeout: float = 30) -> dict:
    store.set("pool/shutdown", "1")
    out = {}
    deadline = time.monotonic() + timeout
    alive = [w for w, p in procs.items() if p.is_alive() or p.exitcode == 0]
    while len(out) < len(alive) and time.monotonic() < deadline:
        try:
            w, recs = q.get(timeout=max(0.1, deadline - time.monotonic()))
            out[w] = recs
        except Exception:
            break
    for p in procs.values():
        p.join(5)
        if p.is_alive():
            p.kill()
    return out


def assert_matches_replay(cfg, path: str, device: str, exact: bool = True,
                          tol: tuple[float, float] = (2e-3, 2e-4), backend: str | None = None,
                          devices: list[str] | None = None, inject: dict | None = None) -> dict:
    """The elastic run's final state (rank 0's checkpoint) equals the uninterrupted replay of
    its ``world_log`` (bitwise, or to ``tol`` = (rtol, atol) when ``exact`` is False).

    Runs that trained at a world size >= 3 -- or any run when ``backend`` is given -- are
    replayed through real collectives of that backend (workloads/replay.py): a w-rank ring
    average of identical gradients is not exact, so only a replay that performs the same
    reduction is an oracle.  When the run logged lock-step digests (``step_digests``), a
    mismatch names the first divergent step, and the digests are ASSERTED: every field of
    every common step when ``exact``, the world size and LR of every common step otherwise
    (only the state digest may differ on GPU), so a one-step LR or world error at a resize
    cannot hide inside ``tol``."""
    from vodascheduler_amd.workloads.replay import first_divergence, replay_collective
    from vodascheduler_amd.workloads.train import replay_reference

    payload = torch.load(path, map_location="cpu", weights_only=True)
    ex = payload["extras"]
    wl = list(ex["world_log"])
    if backend is None and max(wl[1::2]) > 2:
        backend = "gloo" if device == "cpu" else "rccl"
    if backend is not None:
        ref, ref_ex = replay_collective(cfg, wl, int(ex["__step__"]), backend, devices, inject=inject)
    else:
        nthreads = torch.get_num_threads()
        torch.set_num_threads(1)
        try:
            ref, ref_ex = replay_reference(cfg, wl, int(ex["__step__"]), torch.device(device))
        finally:
            torch.set_num_threads(nthreads)
    run_log, ref_log = list(ex.get("steplog") or []), list(ref_ex.get("steplog") or [])
    div = first_divergence(run_log, ref_log)
    if run_log or ref_log:  # the run asked for lock-step digests: both logs must hold them
        assert run_log and ref_log, (len(run_log), len(ref_log))
        common = {e.split(":", 1)[0] for e in run_log} & {e.split(":", 1)[0] for e in ref_log}
        assert common, "no common step between the run's and the replay's lock-step logs"
        sched = first_divergence(run_log, ref_log, fields=("world", "lr"))
        assert sched is None, sched
    assert len(ref) == len(payload["tensors"])
    for i, (a, b) in enumerate(zip(payload["tensors"], ref)):
        if exact:
            assert torch.equal(a, b), (i, float((a.float() - b.float()).abs().max()), div, wl)
        else:  # GPU: nondeterministic reductions (atomics) make trajectories differ in the last bits
            torch.testing.assert_close(a.float(), b.float(), rtol=tol[0], atol=tol[1], msg=lambda m: f"{m}\n{div}")
    if exact:
        assert div is None, div
    assert ex["epoch"] == ref_ex["epoch"] and ex["samples"] == ref_ex["samples"]
    return ex


def spawn_ranks(target, world, *args, timeout: float = 180.0):
    """Run ``target(port, rank, world, q, *args)`` in ``world`` daemon processes and collect
    one result per rank.  Never wedges the test session: on a hang, a failure or a bad exit
    code every surviving rank is killed, and the assertion names the ranks that hung."""
    import queue

    from vodascheduler_amd.runtime.cluster import free_port

    port = free_port()
    store = connect_store("127.0.0.1", port, is_master=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(port, r, world, q) + args, daemon=True) for r in range(world)]
    res: dict = {}
    try:
        for p in ps:
            p.start()
        deadline = time.monotonic() + timeout
        while len(res) < world:
            left = deadline - time.monotonic()
            if left <= 0:
                break
            try:
                r, v = q.get(timeout=min(left, 5.0))
                res[r] = v
            except queue.Empty:
                dead = [i for i, p in enumerate(ps) if p.exitcode not in (None, 0) and i not in res]
                if dead:
                    break  # a rank crashed: the others would wait for it forever
        hung = [r for r in range(world) if r not in res]
        assert not hung, (f"ranks {hung} of {world} returned no result within {timeout:.0f}s "
                          f"(exit codes {[p.exitcode for p in ps]})")
        for i, p in enumerate(ps):
            p.join(60)
            assert p.exitcode == 0, f"rank {i} exit code {p.exitcode}"
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
        for p in ps:
            p.join(10)
        del store
    return res
