"""Communicators for elastic data parallelism.

* :class:`RcclCommunicator` -- the native engine (csrc/hip/comm.cpp): one RCCL communicator
  per (job, membership epoch) over xGMI, non-blocking init bounded by a timeout, abortable
  from a watchdog thread, collectives enqueued on an explicit HIP stream.
* :class:`GlooCommunicator` -- c10d ProcessGroupGloo built directly on the job's store
  prefix (no global default group, so a process can leave one job and join another):
  the CPU path used by tests and the simulated-cluster config.

Both expose the same surface: ``allreduce_``, ``broadcast_``, ``allgather``, ``barrier``,
``abort``, ``destroy`` and ``rank``/``size``.  The rendezvous (unique-id exchange) goes
through a c10d ``Store`` under a per-epoch key prefix.
"""
from __future__ import annotations

import datetime
import hashlib
import os
import threading
import time
import uuid
from collections import OrderedDict

import torch
import torch.distributed as dist

from ..ops import _native as N

OPS = {"sum": 0, "avg": 1, "max": 2, "min": 3, "prod": 4}
_GLOO_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
             "prod": dist.ReduceOp.PRODUCT, "avg": dist.ReduceOp.SUM}


class CommError(RuntimeError):
    """A collective failed or was aborted (peer died / membership changed)."""


def store_get(store: dist.Store, key: str, timeout: float, cancel=None) -> bytes:
    """Blocking get with an explicit timeout (c10d get blocks up to the store timeout);
    ``cancel()`` returning True abandons the wait (membership epoch superseded)."""
    deadline = time.monotonic() + timeout
    while True:
        try:
            if store.check([key]):
                return store.get(key)
        except RuntimeError:
            pass
        if cancel is not None and cancel():
            raise CommError(f"superseded while waiting for {key!r}")
        if time.monotonic() > deadline:
            raise TimeoutError(f"store key {key!r} not published within {timeout:.0f}s")
        time.sleep(0.01)


def arrival_barrier(store: dist.Store, prefix: str, size: int, timeout: float, cancel=None) -> None:
    """Every member of an epoch announces itself before the collective bootstrap, which can
    then never block on a member that went to a newer epoch (``cancel``) or never came."""
    key = f"{prefix}/arrived"
    store.add(key, 1)
    deadline = time.monotonic() + timeout
    while int(store.add(key, 0)) < size:
        if cancel is not None and cancel():
            raise CommError(f"superseded before all {size} members arrived at {prefix}")
        if time.monotonic() > deadline:
            raise CommError(f"only {int(store.add(key, 0))}/{size} members arrived at {prefix} within {timeout:.0f}s")
        time.sleep(0.005)


class Communicator:
    rank: int
    size: int
    device: torch.device

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor: ...
    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor: ...
    def allgather(self, t: torch.Tensor) -> torch.Tensor: ...
    def barrier(self) -> None: ...
    def abort(self) -> None: ...
    def destroy(self) -> None: ...

    @property
    def alive(self) -> bool:
        return True


class RcclCommunicator(Communicator):
    def __init__(self, store: dist.Store, prefix: str, rank: int, size: int, device: torch.device,
                 timeout: float = 300.0, stream: torch.cuda.Stream | None = None, cancel=None,
                 arrived: bool = False):
        self.rank, self.size, self.device = rank, size, device
        h = N.hip()
        if not arrived:
            arrival_barrier(store, prefix, size, timeout, cancel)
        key = f"{prefix}/rccl_uid"
        if rank == 0:
            uid = h.rccl_unique_id()
            store.set(key, uid)
        else:
            uid = store_get(store, key, timeout, cancel)
        self.cid = hashlib.sha1(bytes(uid)).hexdigest()[:20]
        self.cache_key = None
        with torch.cuda.device(device):
            self._c = h.RcclComm(uid, size, rank, device.index if device.index is not None else
                                 torch.cuda.current_device(), timeout, False)
        deadline = time.monotonic() + timeout
        try:
            while not self._c.poll_ready():  # non-blocking init: abandonable, bounded
                if cancel is not None and cancel():
                    raise CommError("RCCL init superseded by a newer membership epoch")
                if time.monotonic() > deadline:
                    raise CommError(f"RCCL init timed out after {timeout:.0f}s")
                time.sleep(0.001)
        except Exception as e:
            self._c.abort()
            raise e if isinstance(e, CommError) else CommError(str(e)) from e
        self.stream = stream

    def _s(self) -> int:
        s = self.stream if self.stream is not None else torch.cuda.current_stream(self.device)
        return s.cuda_stream

    def _chk(self, t: torch.Tensor) -> None:
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("RCCL collectives need contiguous GPU tensors")

    def allreduce_(self, t, op="sum"):
        self._chk(t)
        try:
            self._c.allreduce(t.data_ptr(), t.data_ptr(), t.numel(), N.comm_dtype_code(t.dtype), OPS[op], self._s())
        except RuntimeError as e:
            raise CommError(str(e)) from e
        return t

    def broadcast_(self, t, root=0):
        self._chk(t)
        try:
            self._c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), N.comm_dtype_code(t.dtype), root, self._s())
        except RuntimeError as e:
            raise CommError(str(e)) from e
        return t

    def allgather(self, t):
        self._chk(t)
        out = torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        try:
            self._c.allgather(t.data_ptr(), out.data_ptr(), t.numel(), N.comm_dtype_code(t.dtype), self._s())
        except RuntimeError as e:
            raise CommError(str(e)) from e
        return out

    def group_start(self):
        self._c.group_start()

    def group_end(self):
        self._c.group_end()

    def barrier(self):
        x = torch.ones(1, device=self.device)
        s = self.stream if self.stream is not None else torch.cuda.current_stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))  # x is written on the current stream
        self.allreduce_(x)
        s.synchronize()  # the stream the collective was enqueued on (the DDP side stream if set)
        self.check()

    def check(self) -> None:
        err = self._c.async_error()
        if err:
            raise CommError(f"RCCL communicator error: {err}")

    def abort(self):
        self._c.abort()

    def destroy(self):
        # ncclCommFinalize completes only when the communicator is GLOBALLY quiescent
        # (rccl.h), i.e. when every peer finalizes too.  Members tear communicators down at
        # different times -- the per-process CommCache evicts by its own LRU, a member that
        # left a job drops its copy later -- so a finalize here could block until the peers
        # reach theirs, or until the timeout.  Abort is local and never waits for peers; an
        # idle communicator has nothing in flight to lose.
        self._c.abort()

    @property
    def alive(self):
        return self._c.alive


class GlooCommunicator(Communicator):
    def __init__(self, store: dist.Store, prefix: str, rank: int, size: int, timeout: float = 300.0,
                 cancel=None, arrived: bool = False):
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        self.rank, self.size, self.device = rank, size, torch.device("cpu")
        if not arrived:
            arrival_barrier(store, prefix, size, timeout, cancel)
        if rank == 0:
            store.set(f"{prefix}/gloo_cid", uuid.uuid4().hex[:20])
        self.cid = store_get(store, f"{prefix}/gloo_cid", timeout, cancel).decode()
        self.cache_key = None
        self._pg = dist.ProcessGroupGloo(dist.PrefixStore(prefix + "/gloo", store), rank, size,
                                         datetime.timedelta(seconds=timeout))
        self._aborted = False

    def _run(self, work):
        try:
            work.wait()
        except RuntimeError as e:
            raise CommError(str(e)) from e

    def allreduce_(self, t, op="sum"):
        if self._aborted:
            raise CommError("communicator aborted")
        opts = dist.AllreduceOptions()
        opts.reduceOp = _GLOO_OPS[op]
        self._run(self._pg.allreduce([t], opts))
        if op == "avg":
            t.div_(self.size)
        return t

    def broadcast_(self, t, root=0):
        if self._aborted:
            raise CommError("communicator aborted")
        opts = dist.BroadcastOptions()
        opts.rootRank = root
        self._run(self._pg.broadcast([t], opts))
        return t

    def allgather(self, t):
        if self._aborted:
            raise CommError("communicator aborted")
        outs = [torch.empty_like(t) for _ in range(self.size)]
        self._run(self._pg.allgather([outs], [t]))
        return torch.stack(outs)

    def barrier(self):
        self.allreduce_(torch.ones(1))

    def check(self):
        pass

    def abort(self):
        self._aborted = True
        try:
            self._pg.abort()
        except Exception:
            pass

    def destroy(self):
        try:
            self._pg.shutdown()
        except Exception:
            pass

    @property
    def alive(self):
        return not self._aborted


class LocalCommunicator(Communicator):
    """World of one: every collective is the identity (1-GPU jobs skip RCCL entirely)."""

    def __init__(self, device: torch.device):
        self.rank, self.size, self.device = 0, 1, device

    def allreduce_(self, t, op="sum"):
        return t

    def broadcast_(self, t, root=0):
        return t

    def allgather(self, t):
        return t.unsqueeze(0).clone()

    def barrier(self):
        pass

    def check(self):
        pass

    def abort(self):
        pass

    def destroy(self):
        pass


def create_communicator(store: dist.Store, prefix: str, rank: int, size: int, device: torch.device,
                        backend: str = "auto", timeout: float = 300.0,
                        stream: torch.cuda.Stream | None = None, cancel=None,
                        members: list[str] | None = None) -> Communicator:
    """New communicator for one membership epoch, or -- when ``members`` is given and every
    member still holds an idle communicator built for exactly this ordered member list --
    that cached one (see :class:`CommCache`)."""
    if size == 1:
        return LocalCommunicator(device)
    if backend == "auto":
        backend = "rccl" if device.type == "cuda" else "gloo"
    if backend not in ("rccl", "gloo"):
        raise ValueError(f"unknown comm backend {backend!r}")
    key = (backend, tuple(members), str(device)) if members is not None else None
    mine = COMM_CACHE.cid(key) if key is not None else ""
    store.set(f"{prefix}/have/{rank}", mine)   # before arriving: peers read it after the barrier
    arrival_barrier(store, prefix, size, timeout, cancel)
    if key is not None and mine:
        theirs = [store_get(store, f"{prefix}/have/{r}", timeout, cancel).decode() for r in range(size)]
        if all(c == mine for c in theirs):
            comm = COMM_CACHE.take(key)
            if comm is not None:
                if hasattr(comm, "stream"):
                    comm.stream = stream
                return comm
    if key is not None:
        COMM_CACHE.drop(key)
    if backend == "rccl":
        comm = RcclCommunicator(store, prefix, rank, size, device, timeout, stream, cancel, arrived=True)
    else:
        comm = GlooCommunicator(store, prefix, rank, size, timeout, cancel, arrived=True)
    comm.cache_key = key
    return comm


class CommCache:
    """Per-process LRU cache of IDLE communicators keyed by (backend, ordered member list,
    device).

    An RCCL communicator binds GPUs, not jobs: when a job shrinks and grows back, or the next
    job lands on the same ordered set of GPUs, the communicator built earlier is reused
    instead of paying another RCCL bootstrap (unique-id exchange, topology detection,
    xGMI connection setup) -- the dominant part of an elastic resize with warm workers.
    Reuse is agreed collectively: every member announces the id of the communicator it
    holds for the member list; only if ALL hold the same id is it reused, otherwise a new
    one is built (a restarted or evicted member therefore forces a rebuild, never a hang).
    Aborted communicators are never cached.

    Capacity: each idle RCCL communicator keeps its channel buffers and proxy thread, so the
    cache is bounded (``VODA_COMM_CACHE_MAX``, default 8 per process -- on an 8-GPU node the
    distinct member lists a GPU takes part in at a time are few; evicted ones are aborted)."""

    def __init__(self, max_entries: int | None = None):
        if max_entries is None:
            max_entries = int(os.environ.get("VODA_COMM_CACHE_MAX", "8"))
        self.max_entries = max_entries
        self._d: "OrderedDict[tuple, Communicator]" = OrderedDict()
        self._lock = threading.Lock()
        self.hits = 0
        self.misses = 0

    def cid(self, key) -> str:
        with self._lock:
            c = self._d.get(key)
            return getattr(c, "cid", "") if c is not None and c.alive else ""

    def take(self, key):
        with self._lock:
            c = self._d.pop(key, None)
            if c is not None:
                self.hits += 1
            return c

    def put(self, comm) -> None:
        key = getattr(comm, "cache_key", None)
        if key is None or not getattr(comm, "cid", "") or not comm.alive:
            _close(comm)
            return
        evicted = []
        with self._lock:
            old = self._d.pop(key, None)
            if old is not None and old is not comm:
                evicted.append(old)
            self._d[key] = comm
            while len(self._d) > self.max_entries:
                evicted.append(self._d.popitem(last=False)[1])
        for c in evicted:
            _close(c)

    def drop(self, key) -> None:
        with self._lock:
            c = self._d.pop(key, None)
            if c is not None:
                self.misses += 1
        if c is not None:
            _close(c)

    def clear(self) -> None:
        with self._lock:
            items = list(self._d.values())
            self._d.clear()
        for c in items:
            _close(c)

    def __len__(self) -> int:
        return len(self._d)


def _close(comm) -> None:
    try:
        comm.destroy() if comm.alive else comm.abort()
    except Exception:
        pass


COMM_CACHE = CommCache()
