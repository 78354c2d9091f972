"""Job rendezvous: membership epochs in a c10d Store.

Replaces Horovod elastic's host-discovery + Gloo rendezvous that the reference drives by
rewriting the MPI-Operator ConfigMap: the scheduler's backend *publishes* a
membership epoch, workers *agree* on it at a commit point and rebuild their communicator.

Key layout under ``job/<name>/`` (all writes are idempotent or counter-based):

    epoch              int counter; bumped AFTER e/<n>/members is written (atomic publish)
    e/<n>/members      JSON list of worker ids; list order = rank order
    e/<n>/abort        "1" if a member died: survivors abort their communicator
    e/<n>/comm/...     communicator bootstrap (RCCL unique id / gloo store)
    live_epoch         epoch whose members hold the live state; "-1" = state at rest on disk
    ckpt               JSON {"path", "step"}: latest checkpoint at rest
    done / failed      job outcome, set by rank 0
"""
from __future__ import annotations

import json
import time

import torch.distributed as dist


def connect_store(host: str, port: int, timeout: float = 300.0, is_master: bool = False) -> dist.TCPStore:
    import datetime

    return dist.TCPStore(host, port, world_size=None, is_master=is_master,
                         timeout=datetime.timedelta(seconds=timeout), wait_for_workers=False,
                         multi_tenant=True)


class JobRendezvous:
    def __init__(self, store: dist.Store, job: str):
        self.store = store
        self.job = job
        self.p = f"job/{job}/"

    # ----------------------------------------------------------- coordinator side
    def publish(self, members: list[str], abort: bool = False) -> int:
        """Publish a new membership (possibly empty = halt).  Returns the new epoch."""
        nxt = self.latest_epoch() + 1
        self.store.set(self.p + f"e/{nxt}/members", json.dumps(list(members)))
        if abort:
            self.store.set(self.p + f"e/{nxt}/abort", "1")
        # publish; concurrent publishers are not supported (one backend owns a job)
        e = self.store.add(self.p + "epoch", 1)
        if e != nxt:
            raise RuntimeError(f"concurrent membership publish on {self.job}: {e} != {nxt}")
        return e

    def mark_done(self, ok: bool = True, reason: str = "") -> None:
        self.store.set(self.p + ("done" if ok else "failed"), reason or "1")

    # ----------------------------------------------------------- shared
    def latest_epoch(self) -> int:
        return int(self.store.add(self.p + "epoch", 0))

    def members(self, epoch: int) -> list[str]:
        if epoch <= 0:
            return []
        return json.loads(self.store.get(self.p + f"e/{epoch}/members"))

    def aborted(self, epoch: int) -> bool:
        return epoch > 0 and bool(self.store.check([self.p + f"e/{epoch}/abort"]))

    def comm_prefix(self, epoch: int) -> str:
        return self.p + f"e/{epoch}/comm"

    def outcome(self) -> str | None:
        if self.store.check([self.p + "done"]):
            return "done"
        if self.store.check([self.p + "failed"]):
            return "failed"
        return None

    def get_live_epoch(self) -> int | None:
        k = self.p + "live_epoch"
        return int(self.store.get(k)) if self.store.check([k]) else None

    def set_live_epoch(self, e: int) -> None:
        self.store.set(self.p + "live_epoch", str(e))

    def set_ckpt(self, path: str, step: int) -> None:
        self.store.set(self.p + "ckpt", json.dumps({"path": path, "step": step}))

    def get_ckpt(self) -> dict | None:
        k = self.p + "ckpt"
        return json.loads(self.store.get(k)) if self.store.check([k]) else None

    def wait_state_at_rest(self, timeout: float) -> None:
        deadline = time.monotonic() + timeout
        while True:
            le = self.get_live_epoch()
            if le is None or le < 0:
                return
            if time.monotonic() > deadline:
                raise TimeoutError(f"{self.job}: previous members never handed the state off (live_epoch={le})")
            time.sleep(0.02)

    # ----------------------------------------------------------- liveness / progress beats
    def heartbeat(self, worker: str, epoch: int, step: int, phase: int = 0) -> None:
        """One beat of ``worker``: a store-side counter (liveness: the backend checks that it
        ADVANCES, on its own clock -- no wall-clock comparison across hosts) and the member's
        progress: the epoch it joined, its last committed step and its bootstrap phase counter
        (bumped by join, communicator build and state broadcast, so a slow first sync of a
        healthy epoch counts as progress)."""
        self.store.set(self.p + f"hb/{worker}/p", f"{int(epoch)}:{int(step)}:{int(phase)}")
        self.store.add(self.p + f"hb/{worker}/n", 1)

    def read_heartbeat(self, worker: str) -> tuple[int, int, int, int] | None:
        """(beat count, joined epoch, committed step, bootstrap phase), or None when the worker
        never beat or left the job (its beat tombstoned by ElasticContext.stop)."""
        kp = self.p + f"hb/{worker}/p"
        if not self.store.check([kp]):
            return None
        v = self.store.get(kp).decode()
        if v == "left":
            return None
        n = int(self.store.add(self.p + f"hb/{worker}/n", 0))
        f = v.split(":")
        return n, int(f[0]), int(f[1]), int(f[2]) if len(f) > 2 else 0

    def clear_heartbeat(self, worker: str) -> None:
        """Tombstone: a worker that left the job no longer counts as a live member, even if
        it is re-listed before its beats would have gone stale."""
        self.store.set(self.p + f"hb/{worker}/p", "left")

    def set(self, key: str, value: str) -> None:
        self.store.set(self.p + key, value)

    def get(self, key: str) -> str | None:
        k = self.p + key
        return self.store.get(k).decode() if self.store.check([k]) else None
