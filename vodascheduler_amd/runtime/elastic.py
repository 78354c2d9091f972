"""Elastic training runtime (replaces ``horovod.torch.elastic``: ``hvd.elastic.run``,
``TorchState``, commit / restore / sync, reset callbacks; reference
examples/py/pytorch/pytorch_mnist_elastic.py:125-199 and
examples/py/tensorflow2/tensorflow2_keras_cifar_elastic.py:188-229).

Protocol (see ``rendezvous.py`` for the store layout):
1. A worker *joins* the latest membership epoch that lists it, builds the epoch's
   communicator (RCCL over xGMI on GPU, gloo on CPU) and syncs state: the member holding
   the most recent committed state broadcasts it; if nobody holds state (fresh job, or the
   job was halted / fully migrated) rank 0 loads the checkpoint the previous members left.
2. ``state.commit()`` snapshots the state ON DEVICE (288 GB HBM makes a full copy of
   params + optimizer slots free: ~0.1 ms for ResNet-50), then all members agree -- one
   tiny MAX all-reduce -- on the newest epoch any of them has seen.  If it moved, every
   member raises :class:`HostsUpdatedInterrupt` at the SAME step.
3. On the interrupt, members not in the new epoch leave (the last holders write a checkpoint
   first when no member survives); the rest rebuild the communicator and re-sync.  Reset
   callbacks run (e.g. LR = base_lr * world, sampler re-shard).
4. If a peer dies mid-collective, the backend publishes an *abort* epoch; a watchdog
   thread aborts the communicator, the blocked collective fails, the survivors restore
   the last commit and re-join.
"""
from __future__ import annotations

import contextlib

import io
import logging
import os
import pickle
import threading
import time
from typing import Any, Callable

import torch

from ..parallel.comm import COMM_CACHE, CommError, Communicator, create_communicator
from ..utils.tracing import trace_range
from .rendezvous import JobRendezvous, connect_store

log = logging.getLogger("vodascheduler_amd.elastic")


HEARTBEAT_S = 1.0  # seconds between a member's liveness beats (hb/<worker> in the job's store space)


class HostsUpdatedInterrupt(Exception):
    """Membership changed; raised on every member at the same commit."""

    def __init__(self, skip_sync: bool = False):
        super().__init__("membership changed")
        self.skip_sync = skip_sync


class WorkerRemoved(Exception):
    """This worker is not part of the new membership."""


class JobFinished(Exception):
    pass


# ------------------------------------------------------------------------------------
# context
# ------------------------------------------------------------------------------------
class ElasticContext:
    """Per-process membership + communicator state for one job."""

    def __init__(self, store, job: str, worker_id: str, device: torch.device | str = "cpu",
                 backend: str = "auto", timeout: float = 600.0, ckpt_dir: str | None = None,
                 watch_store=None, poll_interval: float = 0.05, join_epoch: int = 0):
        self.join_epoch = join_epoch  # epoch this worker was started for (0 = unknown)
        self.rdzv = JobRendezvous(store, job)
        self._watch_rdzv = JobRendezvous(watch_store, job) if watch_store is not None else None
        self.job = job
        self.worker_id = worker_id
        self.device = torch.device(device)
        self.backend = backend
        self.timeout = timeout
        self.ckpt_dir = ckpt_dir or os.environ.get("VODA_CKPT_DIR", "/tmp/voda_ckpt")
        self.comm: Communicator | None = None
        self.epoch = 0
        self.members: list[str] = []
        self.rank = -1
        self.size = 0
        self.holds_state = False
        self.committed_step = -1
        self.sync_phase = 0      # bootstrap progress for the heartbeat: bumped by join / comm build / sync
        self._latest_seen = 0
        self._stop = threading.Event()
        self._watcher: threading.Thread | None = None
        self.poll_interval = poll_interval
        self.resize_log: list[dict] = []   # timings of every (re)join, for resize-latency reports
        # after a failed collective only a NEWER epoch can be joined: the failed one still
        # lists the dead peer, and rebuilding its communicator would block until timeout
        self.min_epoch = 0
        self.agreed_epoch = 0   # the epoch a commit's agreement interrupted for (0 = none)
        self.cache_comms = os.environ.get("VODA_COMM_CACHE", "1") != "0"

    # ---------------------------------------------------------------- watcher
    def start_watcher(self) -> None:
        if self._watcher is not None or self._watch_rdzv is None:
            return

        def loop():
            last_hb = 0.0
            while not self._stop.is_set():
                try:
                    now = time.time()
                    if now - last_hb >= HEARTBEAT_S:
                        # liveness + progress for the backend: a dead process stops beating; a
                        # member stuck in a collective keeps beating (the GIL is released there)
                        # but its progress -- joined epoch, committed step -- stops advancing
                        self._watch_rdzv.heartbeat(self.worker_id, self.epoch, self.committed_step,
                                                   self.sync_phase)
                        last_hb = now
                    e = self._watch_rdzv.latest_epoch()
                    if e > self._latest_seen:
                        self._latest_seen = e
                        if self._watch_rdzv.aborted(e) and self.comm is not None:
                            log.warning("%s: abort epoch %d published; aborting communicator", self.job, e)
                            self.comm.abort()
                except Exception:  # store hiccup: keep watching
                    pass
                self._stop.wait(self.poll_interval)

        self._watcher = threading.Thread(target=loop, daemon=True, name=f"voda-watch-{self.job}")
        self._watcher.start()

    def stop(self) -> None:
        self._stop.set()
        if self._watcher is not None:
            self._watcher.join(2)
            self._watcher = None
            try:  # leaving the job: tombstone the beat (a re-listed worker is not "alive" here)
                self._watch_rdzv.clear_heartbeat(self.worker_id)
            except Exception:
                pass

    def latest_seen(self) -> int:
        if self._watcher is None:
            self._latest_seen = max(self._latest_seen, self.rdzv.latest_epoch())
        return self._latest_seen

    # ---------------------------------------------------------------- membership
    def wait_for_membership(self) -> int:
        """Block until an epoch that lists this worker is the latest one; 0 = excluded."""
        deadline = time.monotonic() + self.timeout
        while True:
            e = self.rdzv.latest_epoch()
            if e > 0 and e >= self.min_epoch:
                mem = self.rdzv.members(e)
                if self.worker_id in mem:
                    return e
                if self.rdzv.outcome() is not None:
                    return 0
                if e > self.epoch and self.epoch > 0:
                    return 0  # a newer epoch excludes us
                if self.epoch == 0 and 0 < self.join_epoch <= e:
                    return 0  # superseded before we could join
            if self.rdzv.outcome() is not None:
                return 0
            if time.monotonic() > deadline:
                raise TimeoutError(f"{self.worker_id}: no membership for job {self.job}")
            time.sleep(0.02)

    def join(self, epoch: int) -> None:
        t0 = time.perf_counter()
        self.sync_phase += 1
        self.destroy_comm()
        self.epoch = epoch
        self.members = self.rdzv.members(epoch)
        self.rank = self.members.index(self.worker_id)
        self.size = len(self.members)
        log.debug("%s: %s joins epoch %d as rank %d/%d", self.job, self.worker_id, epoch, self.rank, self.size)
        self._latest_seen = max(self._latest_seen, epoch)
        self._agree_evt = None
        # a newer epoch published before this one's bootstrap finished, or the job ending
        # (finished by the old members before they saw this epoch), means some member will
        # never arrive here: abandon instead of blocking until the timeout
        hits0 = COMM_CACHE.hits
        self.comm = create_communicator(self.rdzv.store, self.rdzv.comm_prefix(epoch), self.rank, self.size,
                                        self.device, self.backend, self.timeout,
                                        cancel=lambda: (self.rdzv.latest_epoch() > epoch
                                                        or self.rdzv.outcome() is not None),
                                        members=self.members if self.cache_comms else None)
        self.sync_phase += 1
        self.resize_log.append({"epoch": epoch, "world": self.size, "comm_init_s": time.perf_counter() - t0,
                                "cached": COMM_CACHE.hits > hits0})

    def destroy_comm(self, abort: bool = False) -> None:
        """Release the epoch's communicator: back into the per-process cache when it is
        healthy (a later epoch or job on the same ordered GPUs reuses it), else abort it."""
        if self.comm is not None:
            try:
                if abort or not self.comm.alive:
                    key = getattr(self.comm, "cache_key", None)
                    self.comm.abort()
                    if key is not None:
                        COMM_CACHE.drop(key)
                elif getattr(self.comm, "cache_key", None) is not None:
                    COMM_CACHE.put(self.comm)
                else:
                    self.comm.destroy()
            except Exception:
                pass
            self.comm = None

    def agree_on_epoch(self) -> int:
        """All members agree (MAX all-reduce) on the newest epoch anyone has seen.

        On GPU the agreement is *lagged by one commit*: the MAX all-reduce of this commit is
        copied to pinned host memory behind an event and read at the next commit, so a
        commit never stalls the host on the step's kernels.  Every member reads the same
        collective's result, so all of them still interrupt at the same commit."""
        seen = self.latest_seen()
        if self.comm is None or self.size == 1:
            return seen
        if self.comm.device.type != "cuda":
            t = torch.tensor([seen], dtype=torch.int64)
            self.comm.allreduce_(t, "max")
            return int(t.item())
        prev = None
        if getattr(self, "_agree_evt", None) is not None:
            self._agree_evt.synchronize()
            self.comm.check()
            prev = int(self._agree_host[0])
        t = torch.tensor([seen], dtype=torch.int64, device=self.comm.device)
        cs = getattr(self.comm, "stream", None)
        cur = torch.cuda.current_stream(self.comm.device)
        if cs is not None:
            cs.wait_stream(cur)  # the H2D copy of ``t`` was enqueued on the current stream
        self.comm.allreduce_(t, "max")
        if cs is not None:
            t.record_stream(cs)
            cur.wait_stream(cs)
        if getattr(self, "_agree_host", None) is None:
            self._agree_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self._agree_host.copy_(t, non_blocking=True)
        self._agree_evt = torch.cuda.Event()
        self._agree_evt.record()
        return prev if prev is not None else self.epoch

    def reset_agreement(self) -> None:
        self._agree_evt = None

    def allreduce_values(self, values, op: str = "avg") -> list[float]:
        """All-reduce a few host/device scalars across the current members and return them on
        the host (Horovod ``metric_average`` = ``hvd.allreduce(tensor)``, reference
        pytorch_mnist_elastic.py:119-122).  Every member must call it at the same point."""
        dev = self.comm.device if self.comm is not None else self.device
        t = torch.as_tensor(values, dtype=torch.float64 if dev.type == "cpu" else torch.float32).to(dev).reshape(-1)
        if self.comm is None or self.size <= 1:
            return [float(v) for v in t.tolist()]
        if dev.type == "cuda":
            cs = getattr(self.comm, "stream", None)
            cur = torch.cuda.current_stream(dev)
            if cs is not None:
                cs.wait_stream(cur)
            self.comm.allreduce_(t, op)
            if cs is not None:
                t.record_stream(cs)
                cur.wait_stream(cs)
        else:
            self.comm.allreduce_(t, op)
        return [float(v) for v in t.tolist()]

    def metric_average(self, value: float) -> float:
        return self.allreduce_values([value], "avg")[0]


# ------------------------------------------------------------------------------------
# state
# ------------------------------------------------------------------------------------
def _pack(obj: Any) -> bytes:
    return pickle.dumps(obj)


def broadcast_object(comm: Communicator, obj: Any, root: int) -> Any:
    """Broadcast a small picklable object from ``root`` through the communicator.
    (Objects produced by this job's own workers -- never external input.)"""
    if comm is None or comm.size == 1:
        return obj
    dev = comm.device
    if comm.rank == root:
        data = torch.frombuffer(bytearray(_pack(obj)), dtype=torch.uint8).to(dev)
        n = torch.tensor([data.numel()], dtype=torch.int64, device=dev)
    else:
        n = torch.zeros(1, dtype=torch.int64, device=dev)
    comm.broadcast_(n, root)
    if comm.rank != root:
        data = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
    comm.broadcast_(data, root)
    if comm.rank == root:
        return obj
    return pickle.loads(data.cpu().numpy().tobytes())


@contextlib.contextmanager
def _collectives_on_current_stream(comm: Communicator | None):
    """Run ``comm``'s collectives on the current stream for the duration (the state sync reads
    their results on the host right away: ``.item()`` / ``.cpu()`` order against the current
    stream only).  After ``ElasticDDP.set_communicator`` an RCCL communicator enqueues on the
    DDP side stream; the current stream first waits for anything still queued there, so the
    collective order every rank issues is kept."""
    s = getattr(comm, "stream", None) if comm is not None else None
    if s is None:
        yield
        return
    torch.cuda.current_stream(comm.device).wait_stream(s)
    comm.stream = None
    try:
        yield
    finally:
        comm.stream = s


class State:
    """Elastic state: tensors (synced by broadcast) + picklable extras (epoch, batch, ...)."""

    def __init__(self, ctx: ElasticContext, **extras):
        self.ctx = ctx
        self._extras = dict(extras)
        self._committed_extras = dict(extras)
        self._reset_callbacks: list[Callable[[], None]] = []
        self.step = 0
        self._snapshot: list[torch.Tensor] | None = None

    # extras behave like attributes (state.epoch, state.batch)
    def __getattr__(self, k):
        ex = self.__dict__.get("_extras")
        if ex is not None and k in ex:
            return ex[k]
        raise AttributeError(k)

    def __setattr__(self, k, v):
        if "_extras" in self.__dict__ and k in self._extras:
            self._extras[k] = v
        else:
            super().__setattr__(k, v)

    # -- to override --
    def tensors(self) -> list[torch.Tensor]:
        return []

    def after_load(self) -> None:
        pass

    # -- callbacks --
    def register_reset_callbacks(self, callbacks: list[Callable[[], None]]) -> None:
        self._reset_callbacks.extend(callbacks)

    def on_reset(self) -> None:
        for cb in self._reset_callbacks:
            cb()

    # -- commit / restore --
    @torch.no_grad()
    def save(self) -> None:
        ts = self.tensors()
        if self._snapshot is None or len(self._snapshot) != len(ts):
            self._snapshot = [t.detach().clone() for t in ts]
        else:
            for s, t in zip(self._snapshot, ts):
                s.copy_(t)
        self._committed_extras = {k: _copy(v) for k, v in self._extras.items()}
        self._committed_extras["__step__"] = self.step
        self.ctx.committed_step = self.step
        self.ctx.holds_state = True

    @torch.no_grad()
    def restore(self) -> None:
        if self._snapshot is None:
            return
        for s, t in zip(self._snapshot, self.tensors()):
            t.copy_(s)
        ex = dict(self._committed_extras)
        self.step = ex.pop("__step__", self.step)
        self._extras = {k: _copy(v) for k, v in ex.items()}
        self.after_load()

    def commit(self) -> None:
        """Snapshot + agree on membership; raises HostsUpdatedInterrupt when it changed."""
        with trace_range("commit", "elastic"):
            self.save()
            self.check_host_updates()

    def check_host_updates(self) -> None:
        e = self.ctx.agree_on_epoch()
        if e > self.ctx.epoch:
            # every member hands off against the AGREED epoch: a member whose own watcher has
            # not polled the store yet would otherwise see the old membership in _transition,
            # skip the at-rest checkpoint of a halt and leave with nobody holding the state
            self.ctx.agreed_epoch = e
            raise HostsUpdatedInterrupt()

    # -- sync on (re)join --
    @torch.no_grad()
    def sync(self) -> None:
        ctx = self.ctx
        comm = ctx.comm
        with _collectives_on_current_stream(comm):
            self._sync_on(comm)

    def _sync_on(self, comm) -> None:
        ctx = self.ctx
        ctx.sync_phase += 1
        held = ctx.committed_step if ctx.holds_state else -1
        if comm is not None and comm.size > 1:
            t = torch.tensor([held], dtype=torch.int64, device=comm.device)
            allh = comm.allgather(t).view(-1).cpu().tolist()
        else:
            allh = [held]
        best = max(allh)
        if best >= 0:
            root = allh.index(best)
            if ctx.rank == root:
                self.restore() if held == best and self._snapshot is not None else None
        else:
            root = 0
            if ctx.rank == 0:
                self._load_from_rest()
        if comm is not None and comm.size > 1:
            from ..parallel.ddp import broadcast_tensors

            broadcast_tensors(comm, self.tensors(), root)  # small tensors coalesced per dtype
            ctx.sync_phase += 1
        extras = dict(self._extras, __step__=self.step)
        extras = broadcast_object(comm, extras, root)
        self.step = extras.pop("__step__")
        self._extras = extras
        self.after_load()
        self.save()
        if ctx.rank == 0:
            ctx.rdzv.set_live_epoch(ctx.epoch)
            ctx.rdzv.set(f"e/{ctx.epoch}/synced", repr(time.time()))  # resize-latency probe

    def _load_from_rest(self) -> None:
        ctx = self.ctx
        if ctx.rdzv.get_live_epoch() is None and ctx.rdzv.get_ckpt() is None:
            return  # fresh job: keep the (seeded) initial state
        ctx.rdzv.wait_state_at_rest(ctx.timeout)
        ck = ctx.rdzv.get_ckpt()
        if ck is None:
            return
        self.load_checkpoint(ck["path"])

    # -- checkpoints --
    def checkpoint_path(self) -> str:
        os.makedirs(os.path.join(self.ctx.ckpt_dir, self.ctx.job), exist_ok=True)
        return os.path.join(self.ctx.ckpt_dir, self.ctx.job, "state.pt")

    @torch.no_grad()
    def save_checkpoint(self, path: str | None = None) -> str:
        path = path or self.checkpoint_path()
        src = self._snapshot if self._snapshot is not None else self.tensors()
        ex = dict(self._committed_extras) if self._snapshot is not None else dict(self._extras, __step__=self.step)
        payload = {"tensors": [t.detach().cpu() for t in src], "extras": _to_plain(ex)}
        tmp = path + f".tmp{os.getpid()}"
        torch.save(payload, tmp)
        os.replace(tmp, path)
        return path

    @torch.no_grad()
    def load_checkpoint(self, path: str) -> None:
        payload = torch.load(path, map_location="cpu", weights_only=True)
        for t, s in zip(self.tensors(), payload["tensors"]):
            t.copy_(s.to(t.device))
        ex = dict(payload["extras"])
        self.step = int(ex.pop("__step__", 0))
        self._extras.update(ex)
        self.after_load()


def _copy(v):
    import copy

    return copy.deepcopy(v)


def _to_plain(d: dict) -> dict:
    out = {}
    for k, v in d.items():
        if isinstance(v, (int, float, str, bool)) or v is None:
            out[k] = v
        elif isinstance(v, (list, tuple)) and all(isinstance(x, (int, float, str, bool)) for x in v):
            out[k] = list(v)
        elif isinstance(v, dict) and all(isinstance(x, (int, float, str, bool)) for x in v.values()):
            out[k] = dict(v)
        elif isinstance(v, dict) and all(isinstance(x, (list, tuple)) and all(isinstance(y, (int, float)) for y in x)
                                         for x in v.values()):
            out[k] = {kk: list(x) for kk, x in v.items()}  # e.g. perf: {world: [steps, seconds]}
    return out


def rng_state(device: torch.device) -> list[int]:
    """The generator state that random layers (dropout) on ``device`` draw from, as plain ints
    (picklable, broadcastable, storable in a weights-only checkpoint)."""
    if device.type == "cuda":
        return torch.cuda.get_rng_state(device).tolist()
    return torch.get_rng_state().tolist()


def set_rng_state(device: torch.device, state: list[int]) -> None:
    t = torch.tensor(state, dtype=torch.uint8)
    if device.type == "cuda":
        torch.cuda.set_rng_state(t, device)
    else:
        torch.set_rng_state(t)


class TorchState(State):
    """Model + (fused flat) optimizer + extras.  Syncs parameters (fp32 masters when the
    optimizer is a fused flat one), every optimizer slot and the model buffers (BN stats).

    The RNG state of the model's device is part of the committed state (extra ``rng``): a
    commit records it, a restore rewinds it and a (re)joining member receives the root's, so
    dropout masks follow one sequence whatever resizes, restores or restarts happen -- every
    member draws the same masks and an elastic run equals an uninterrupted one.  (Horovod's
    TorchState leaves the generators alone; this makes the equivalence testable with dropout.)"""

    def __init__(self, ctx: ElasticContext, model: torch.nn.Module, optimizer=None, **extras):
        self.model = model
        self.optimizer = optimizer
        self._rng_device = ctx.device if isinstance(ctx.device, torch.device) else torch.device(ctx.device)
        super().__init__(ctx, rng=rng_state(self._rng_device), **extras)

    def save(self) -> None:
        self._extras["rng"] = rng_state(self._rng_device)
        super().save()

    def tensors(self):
        ts: list[torch.Tensor] = []
        for m in self.model.modules():  # host-side counters -> buffers before they are synced
            if hasattr(m, "sync_batches_tracked"):
                m.sync_batches_tracked()
        opt = self.optimizer
        if opt is not None and hasattr(opt, "flat_state_tensors"):
            ts += opt.flat_state_tensors()
        else:
            ts += [p.data for p in self.model.parameters()]
            if opt is not None:
                for st in opt.state.values():
                    ts += [v for v in st.values() if torch.is_tensor(v) and v.dim() > 0]
        ts += [b for b in self.model.buffers() if b.dtype.is_floating_point or b.dtype == torch.int64]
        return ts

    def after_load(self):
        if self.optimizer is not None and hasattr(self.optimizer, "after_external_update"):
            self.optimizer.after_external_update()
        rng = self._extras.get("rng")
        if rng:
            set_rng_state(self._rng_device, rng)


# ------------------------------------------------------------------------------------
# run loop
# ------------------------------------------------------------------------------------
def run(func: Callable) -> Callable:
    """Decorator: ``@run def train(state): ...`` (``hvd.elastic.run`` semantics).

    Returns the function's result on members that finish it, or ``None`` on workers that
    were removed from the job.
    """

    def wrapper(state: State, *args, **kwargs):
        ctx = state.ctx
        ctx.start_watcher()
        reset = False
        while True:
            t0 = time.perf_counter()
            e = ctx.wait_for_membership()
            if e == 0:
                _leave(state, e)
                return None
            try:
                with trace_range("comm_bootstrap", "elastic", job=ctx.job, epoch=e):
                    ctx.join(e)
                with trace_range("state_sync", "elastic", job=ctx.job, epoch=e, world=ctx.size):
                    state.sync()
            except CommError as err:  # superseded / peer lost during bootstrap or sync
                log.warning("%s/%s: epoch %d not established (%s); waiting for a newer one", ctx.job,
                            ctx.worker_id, e, err)
                ctx.min_epoch = e + 1
                ctx.destroy_comm(abort=True)
                if ctx.holds_state:
                    state.restore()
                continue
            ctx.resize_log[-1]["sync_s"] = time.perf_counter() - t0
            if reset:
                state.on_reset()
            try:
                out = func(state, *args, **kwargs)
            except HostsUpdatedInterrupt:
                reset = True
                if not _transition(state):
                    return None
                continue
            except CommError as err:
                log.warning("%s/%s: collective failed (%s); restoring last commit", ctx.job, ctx.worker_id, err)
                state.restore()
                ctx.min_epoch = ctx.epoch + 1
                ctx.destroy_comm(abort=True)
                reset = True
                continue
            if ctx.rank == 0:
                ctx.rdzv.mark_done(True)
            ctx.destroy_comm()
            ctx.stop()
            return out

    wrapper.__wrapped__ = func
    return wrapper


def _transition(state: State) -> bool:
    """At an agreed interrupt: hand off the state if nobody survives; False = leave."""
    ctx = state.ctx
    new_e = ctx.agreed_epoch or ctx.latest_seen()
    ctx.agreed_epoch = 0
    new_members = ctx.rdzv.members(new_e) if new_e > 0 else []
    survivors = [m for m in ctx.members if m in new_members]
    if not survivors and ctx.rank == 0:
        path = state.save_checkpoint()
        ctx.rdzv.set_ckpt(path, state.step)
        ctx.rdzv.set_live_epoch(-1)
    ctx.destroy_comm()
    if ctx.worker_id not in new_members:
        _leave(state, new_e)
        return False
    return True


def _leave(state: State, epoch: int) -> None:
    ctx = state.ctx
    ctx.holds_state = False
    ctx.destroy_comm()
    ctx.stop()
