"""Warm per-GPU worker pool: the MI355X-native replacement of "MPI-Operator creates pods,
kubelet starts containers, horovodrun discovers hosts" (SURVEY.md §3.1-3.2, §5.8 item 3).

* :class:`PoolWorker` -- one long-lived process per GPU (a torchrun rank, or a process the
  node agent started).  It keeps its HIP context, MIOpen/hipBLASLt caches and allocator pool
  across jobs, reads job assignments from its mailbox in the store and runs them with the
  elastic runtime; between jobs it only drops the model.
* :class:`PoolBackend` -- the scheduler-side :class:`Backend`: turns start / scale / halt /
  migrate actions into membership epochs (``JobRendezvous.publish``) + mailbox messages for
  workers that join, watches job outcomes and reports completions, and measures elastic
  resize latency (publish -> new membership synced and training).

A resize therefore costs one communicator rebuild + one state broadcast, not pod creation.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from dataclasses import asdict

import torch

from ..backend.base import EV_FINISHED, HALT, Backend, JobAction
from ..sim.trace import workload_of
from ..workloads.train import TrainConfig, train_elastic
from .elastic import ElasticContext
from .rendezvous import JobRendezvous

log = logging.getLogger("vodascheduler_amd.pool")

Loc = tuple[str, int]


def worker_id(loc: Loc) -> str:
    return f"{loc[0]}:{loc[1]}"


def job_train_config(job, defaults: dict | None = None) -> dict:
    """TrainConfig (as a dict) for a job from its spec's workload annotation + env knobs."""
    wl = workload_of(job.spec)
    d = dict(model=wl["model"], epochs=max(1, job.config.epochs), steps_per_epoch=int(wl["steps_per_epoch"]))
    if "per_gpu_batch" in wl:
        d["per_gpu_batch"] = int(wl["per_gpu_batch"])
    if "lr" in wl:
        d["lr"] = float(wl["lr"])
    d.update(defaults or {})
    for k in ("reduction", "compression"):  # the job's own choice beats the cluster default
        if wl.get(k):
            d[k] = wl[k]
    if wl.get("precision"):  # declared compute precision: fp32 = no autocast (the reference's)
        d["amp"] = wl["precision"] != "fp32"
    return d


class PoolBackend(Backend):
    def __init__(self, store, worker_locs: list[Loc], train_defaults: dict | None = None,
                 poll_interval: float = 0.05, settle_timeout: float = 120.0,
                 initial_nodes: dict[str, list[int]] | None = None):
        super().__init__()
        self.store = store
        self._lock = threading.Lock()
        self._pub_lock = threading.RLock()  # one publisher per job at a time (scheduler vs failure path)
        self.workers = [worker_id(l) for l in worker_locs]
        self.node_gpus_all: dict[str, list[int]] = {}
        for n, g in worker_locs:
            self.node_gpus_all.setdefault(n, []).append(g)
        # the schedulable inventory: every pool GPU, or ``initial_nodes`` (an autoscaled
        # cluster starts small; set_nodes announces the rest)
        self.node_gpus: dict[str, list[int]] = {k: list(v) for k, v in
                                                (initial_nodes or self.node_gpus_all).items()}
        self.train_defaults = dict(train_defaults or {})
        self.members: dict[str, list[str]] = {}    # desired membership (scheduler view)
        self.live: dict[str, tuple[int, list[str]]] = {}  # last published (epoch, members)
        self.pending: dict[str, tuple] = {}           # membership waiting for the live epoch to sync
        # a membership change whose previous epoch has not synced after this long is forced
        # through as an ABORT epoch: members stuck in the stale epoch's collectives abort
        # their communicator instead of blocking (bounds a single resize)
        self.settle_timeout = settle_timeout
        self.active: set[str] = set()
        self.published: dict[tuple[str, int], float] = {}
        self.resize_latency: list[dict] = []
        self.events: list[dict] = []
        self.forced_epochs = 0
        self.forced_log: list[dict] = []  # every forced abort epoch: job, epoch, wait, members without heartbeat
        self._hb_seen: dict[tuple[str, str], list] = {}  # (job, member) -> beat / progress change times
        # mailbox counters continue where an earlier backend on the same warm pool stopped
        # (several traces in a row on one pool: bench.py's control run)
        self._mail_n: dict[str, int] = {w: int(store.add(f"pool/{w}/n", 0)) for w in self.workers}
        self._stop = threading.Event()
        self._poll = poll_interval
        self._mon = threading.Thread(target=self._monitor, daemon=True, name="pool-monitor")
        self._mon.start()

    # ------------------------------------------------------------------ Backend API
    def apply(self, actions: list[JobAction]) -> None:
        for a in actions:
            self._apply_one(a)

    def _apply_one(self, a: JobAction) -> None:
        with self._pub_lock:
            self._apply_locked(a)

    def _apply_locked(self, a: JobAction) -> None:
        name = a.job.name
        if a.kind == HALT:
            new_members: list[str] = []
        else:
            if a.workers is None:
                raise ValueError("PoolBackend needs placement (worker locations) for every action")
            # members in GPU order: the ordered member list keys the per-process communicator
            # cache (parallel/comm.py), so a job that returns to a GPU set it used before --
            # whatever order placement listed it in -- reuses that RCCL communicator.  The
            # state root is chosen by holder (State.sync), so rank order carries no state.
            new_members = [worker_id(l) for l in sorted(a.workers, key=lambda l: (l[0], int(l[1])))]
        old = self.members.get(name, [])
        if new_members == old:
            return
        t = time.time()
        with self._lock:
            self.members[name] = new_members
            if new_members:
                self.active.add(name)
        cfg = job_train_config(a.job, self.train_defaults)
        # One membership change in flight per job: a new epoch is published only after every
        # member of the previous one has joined it (rank 0 writes ``e/<n>/synced`` at the end
        # of the collective state sync).  Publishing earlier lets two members join DIFFERENT
        # epochs (one read the membership before the newer publish, one after) and block
        # forever building two communicators -- reproduced on CPU/gloo with a resize right
        # after a start.  Queued changes coalesce: only the newest membership is published.
        self.pending[name] = (new_members, a.kind, t, cfg)
        self._publish_if_settled(name)

    def _publish_if_settled(self, name: str, force: bool = False) -> None:
        """Publish the job's pending membership if its live epoch has synced (caller holds
        ``_pub_lock``)."""
        if name not in self.pending:
            return
        rdzv = JobRendezvous(self.store, name)
        live_e, live_m = self.live.get(name, (0, []))
        abort = False
        if live_m and not force and rdzv.get(f"e/{live_e}/synced") is None and rdzv.outcome() is None:
            t_req = self.pending[name][2]
            waited = time.time() - t_req
            stale = self._stale_members(rdzv, name, live_m)  # refreshes the beat records every poll
            if waited < self.settle_timeout:
                return  # the monitor retries
            # a slow but healthy epoch (members still training towards the commit that joins
            # it, a state sync in flight) is left alone.  Abort when a member is known to be
            # gone (its beat counter stopped advancing), when NO member made progress (joined
            # epoch / committed step / bootstrap phase) for settle_timeout -- live processes
            # deadlocked in a collective keep beating but stop progressing -- or at the hard
            # limit, which never falls below 2 x settle_timeout
            stuck = not stale and self._no_progress(name, live_m)
            hard = max(2.0 * self.settle_timeout, min(self.STUCK_FACTOR * self.settle_timeout, self.HARD_SETTLE_S))
            if not stale and not stuck and waited < hard:
                return
            why = "stale" if stale else ("no progress" if stuck else "hard limit")
            log.warning("job %s: epoch %d not synced after %.0fs (%s; members without heartbeat: %s); "
                        "publishing an abort epoch", name, live_e, waited, why, stale or "none")
            abort = True
            self.forced_epochs += 1
            self.forced_log.append({"job": name, "epoch": live_e, "waited_s": round(waited, 1), "stale": stale,
                                    "why": why})
        new_members, kind, t, cfg = self.pending.pop(name)
        if new_members == live_m:
            return
        e = rdzv.publish(new_members, abort=abort)
        log.debug("publish %s epoch %d members %s (was %s)", name, e, new_members, live_m)
        with self._lock:
            self.live[name] = (e, list(new_members))
            self.published[(name, e)] = t
            self.events.append({"t": t, "t_publish": time.time(), "job": name, "epoch": e, "kind": kind,
                                "world": len(new_members), "prev_world": len(live_m)})
        for wid in new_members:
            if wid not in live_m:
                self._mail(wid, {"job": name, "epoch": e, "cfg": cfg})

    STUCK_FACTOR = 5.0      # hard limit: abort a never-syncing epoch after this x settle_timeout ...
    HARD_SETTLE_S = 150.0   # ... or this many seconds, whichever is first (bench deadline 540 s),
    #                         but never before 2 x settle_timeout
    HEARTBEAT_STALE_S = 10.0

    def _observe(self, rdzv, job: str, m: str):
        """Track member ``m``'s beat on the backend's own monotonic clock: returns its record
        [count, t_count_changed, progress, t_progress_changed], or None (never beat / left)."""
        hb = rdzv.read_heartbeat(m)
        key = (job, m)
        if hb is None:
            self._hb_seen.pop(key, None)
            return None
        now = time.monotonic()
        n, prog = hb[0], hb[1:]
        rec = self._hb_seen.get(key)
        if rec is None:
            rec = self._hb_seen[key] = [n, now, prog, now]
        if n != rec[0]:
            rec[0], rec[1] = n, now
        if prog != rec[2]:
            rec[2], rec[3] = prog, now
        return rec

    def _stale_members(self, rdzv, job: str, members: list[str]) -> list[str]:
        """Members whose liveness beat (runtime/elastic.py watcher) is missing, tombstoned, or
        has not advanced for HEARTBEAT_STALE_S of this backend's clock."""
        now = time.monotonic()
        out = []
        for m in members:
            rec = self._observe(rdzv, job, m)
            if rec is None or now - rec[1] > self.HEARTBEAT_STALE_S:
                out.append(m)
        return out

    def _no_progress(self, job: str, members: list[str]) -> bool:
        """True when no member's progress (joined epoch, committed step, bootstrap phase) changed during the
        last settle_timeout (records refreshed by the _stale_members call just before)."""
        now = time.monotonic()
        recs = [self._hb_seen.get((job, m)) for m in members]
        return all(r is not None and now - r[3] > self.settle_timeout for r in recs)

    def _mail(self, wid: str, msg: dict) -> None:
        n = self._mail_n.get(wid, 0) + 1
        self._mail_n[wid] = n
        self.store.set(f"pool/{wid}/msg/{n}", json.dumps(msg))
        got = self.store.add(f"pool/{wid}/n", 1)
        if got != n:
            raise RuntimeError(f"mailbox counter mismatch for {wid}: {got} != {n}")

    def delete_job(self, job_name: str) -> None:
        rdzv = JobRendezvous(self.store, job_name)
        with self._pub_lock:
            self.pending.pop(job_name, None)
            if self.live.get(job_name, (0, []))[1]:
                e = rdzv.publish([])
                self.live[job_name] = (e, [])
            rdzv.mark_done(False, "deleted")
            with self._lock:
                self.members.pop(job_name, None)
                self.active.discard(job_name)
            for k in [k for k in self._hb_seen if k[0] == job_name]:
                del self._hb_seen[k]

    def nodes(self):
        return {k: list(v) for k, v in self.node_gpus.items()}

    def set_nodes(self, nodes: dict[str, list[int]]) -> None:
        """Announce a new schedulable inventory (a node / GPUs added by an autoscaler, or
        drained): the scheduler re-plans on the EV_NODES event (reference addNode /
        updateNode / deleteNode, scheduler.go:689-747).  Every announced GPU must have a
        pool worker."""
        known = {worker_id((n, g)) for n, gs in self.node_gpus_all.items() for g in gs}
        for n, gs in nodes.items():
            for g in gs:
                if worker_id((n, g)) not in known:
                    raise ValueError(f"no pool worker for GPU {n}:{g}")
        with self._lock:
            self.node_gpus = {k: sorted(v) for k, v in nodes.items() if v}
        from ..backend.base import EV_NODES

        self.emit(EV_NODES, self.nodes())

    def list_running(self):
        return {j: [(m.rsplit(":", 1)[0], int(m.rsplit(":", 1)[1])) for m in mem]
                for j, mem in self.members.items() if mem}

    def shutdown(self, stop_pool: bool = True) -> None:
        """Stop the monitor; ``stop_pool`` also ends every pool worker's ``serve`` loop (keep
        the pool warm for another trace with ``stop_pool=False``)."""
        self._stop.set()
        if stop_pool:
            self.store.set("pool/shutdown", "1")
        self._mon.join(5)

    # ------------------------------------------------------------------ monitor
    def _monitor(self) -> None:
        while not self._stop.is_set():
            if self.pending:
                with self._pub_lock:
                    for name in list(self.pending):
                        try:
                            self._publish_if_settled(name)
                        except Exception:  # store hiccup: retry next round
                            log.exception("publishing membership of %s failed", name)
            with self._lock:
                jobs = list(self.active)
                pend = [k for k in self.published if k not in {(r["job"], r["epoch"]) for r in self.resize_latency}]
            for name in jobs:
                out = JobRendezvous(self.store, name).outcome()
                if out is not None:
                    with self._pub_lock:
                        self.pending.pop(name, None)
                    with self._lock:
                        self.active.discard(name)
                        self.members.pop(name, None)
                    if out == "done":
                        self.emit(EV_FINISHED, name, True)
                    else:
                        reason = JobRendezvous(self.store, name).get("failed")
                        if reason != "deleted":
                            self.emit(EV_FINISHED, name, False)
            for (name, e) in pend:
                r = JobRendezvous(self.store, name)
                v = r.get(f"e/{e}/synced")
                if v is not None:
                    with self._lock:
                        t0 = self.published[(name, e)]
                        self.resize_latency.append({"job": name, "epoch": e, "latency_s": float(v) - t0})
            self._stop.wait(self._poll)


class PoolWorker:
    """Serve job assignments on one device until ``pool/shutdown`` is set."""

    def __init__(self, store, watch_store, wid: str, device: torch.device, backend: str = "auto",
                 timeout: float = 600.0, idle_poll: float = 0.01):
        self.store = store
        self.watch_store = watch_store
        self.wid = wid
        self.device = device
        self.backend = backend
        self.timeout = timeout
        self.idle_poll = idle_poll
        self.done = 0
        self.results: list[dict] = []

    def serve(self) -> list[dict]:
        # a restarted worker resumes after the last message its predecessor took
        # (at-most-once: a job that was running when the process died is recovered by the
        # backend's abort epoch + migration, never replayed here)
        self.done = int(self.store.add(f"pool/{self.wid}/done", 0))
        while True:
            n = int(self.store.add(f"pool/{self.wid}/n", 0))
            if n > self.done:
                self.done = int(self.store.add(f"pool/{self.wid}/done", 1))
                msg = json.loads(self.store.get(f"pool/{self.wid}/msg/{self.done}"))
                self._run(msg)
                continue
            if self.store.check(["pool/shutdown"]):
                return self.results
            time.sleep(self.idle_poll)

    def _run(self, msg: dict) -> None:
        log.debug("worker %s: mail #%d job %s epoch %s", self.wid, self.done, msg["job"], msg["epoch"])
        ctx = ElasticContext(self.store, msg["job"], self.wid, self.device, self.backend, self.timeout,
                             watch_store=self.watch_store, join_epoch=int(msg["epoch"]))
        cfg = TrainConfig(**msg["cfg"])
        t0 = time.time()
        try:
            out = train_elastic(ctx, cfg)
        except Exception as e:  # a failed job must not take the warm worker down
            log.exception("worker %s: job %s failed", self.wid, msg["job"])
            if ctx.rank == 0 or ctx.rank < 0:
                ctx.rdzv.mark_done(False, f"{type(e).__name__}: {e}")
            out = {"error": repr(e)}
        finally:
            ctx.stop()
        rec = {"job": msg["job"], "wid": self.wid, "t0": t0, "t1": time.time(), "result": out,
               "resize_log": ctx.resize_log}
        self.results.append(rec)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


def train_config_dict(cfg: TrainConfig) -> dict:
    return asdict(cfg)
