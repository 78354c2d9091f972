"""``vodarun``: the in-launcher elastic driver (replaces ``horovodrun`` elastic mode).

In the reference a job's launcher pod runs ``horovodrun --num-proc $(MIN_NP) --min-num-proc
--max-num-proc --host-discovery-script /etc/mpi/discover_hosts.sh --blacklist-cooldown-range
30 100 python train.py ...`` (examples/yaml/tensorflow2/*.yaml); the scheduler resizes the job
by changing ``Worker.replicas``, the MPI-Operator rewrites ``discover_hosts.sh`` and the
Horovod driver notices, re-rendezvouses and broadcasts state.  ``vodarun``
does the same against this framework's elastic runtime:

* serves the job's rendezvous store (c10d TCPStore) and polls the discovery script
  (``host:slots`` per line, Horovod's format) every ``--discovery-interval`` seconds;
* starts one worker process per slot (locally, or on a remote host over ``ssh`` as
  ``horovodrun`` does), passing ``VODA_STORE`` / ``VODA_WORKER_ID`` / ``VODA_JOIN_EPOCH``;
* publishes a new membership epoch when the host set changes -- one change in flight at a
  time (the previous epoch must have synced), bounded to ``[min-np, max-np]``;
* a worker that exits non-zero is dropped from the membership with an abort epoch and its
  host is blacklisted for a random cooldown in ``--blacklist-cooldown-range``;
* exits 0 when the job reports done, 1 when it failed or dropped below ``min-np`` for good.

    vodarun --min-np 1 --max-np 4 --host-discovery-script ./hosts.sh -- \
        python -m vodascheduler_amd.workloads.train --model resnet50 --name JOB ...
"""
from __future__ import annotations

import argparse
import logging
import os
import random
import shlex
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field

log = logging.getLogger("vodascheduler_amd.vodarun")

LOCAL_HOSTS = {"localhost", "127.0.0.1", socket.gethostname()}


def discover(script: str, timeout: float = 10.0) -> list[tuple[str, int]]:
    """Run the discovery script; ``host:slots`` (or ``host``) per line."""
    out = subprocess.run([script], capture_output=True, text=True, timeout=timeout, check=True).stdout
    hosts = []
    for line in out.splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        host, _, slots = line.partition(":")
        hosts.append((host, int(slots) if slots else 1))
    return hosts


@dataclass
class Worker:
    wid: str
    host: str
    proc: subprocess.Popen
    epoch: int


@dataclass
class Driver:
    cmd: list[str]
    script: str
    min_np: int
    max_np: int
    store_host: str
    store_port: int
    job: str
    cooldown: tuple[float, float] = (30.0, 100.0)
    interval: float = 1.0
    workers: dict[str, Worker] = field(default_factory=dict)
    blacklist: dict[str, float] = field(default_factory=dict)

    def __post_init__(self):
        from .rendezvous import JobRendezvous, connect_store

        self.store = connect_store(self.store_host, self.store_port, is_master=True)
        self.rdzv = JobRendezvous(self.store, self.job)
        self.live: list[str] = []

    # ------------------------------------------------------------------ processes
    def _spawn(self, wid: str, host: str, epoch: int) -> None:
        env = {"VODA_STORE": f"{self.store_host}:{self.store_port}", "VODA_WORKER_ID": wid,
               "VODA_JOIN_EPOCH": str(epoch), "JOB_NAME": self.job,
               "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")}
        slot = wid.rsplit(":", 1)[1]
        env["HIP_VISIBLE_DEVICES"] = os.environ.get("VODA_WORKER_HIP_VISIBLE_DEVICES", slot)
        if host in LOCAL_HOSTS:
            proc = subprocess.Popen(self.cmd, env=dict(os.environ, **env), start_new_session=True)
        else:  # like horovodrun: ssh into the worker pod/host (MPI-Operator sets up the keys)
            remote = " ".join(f"{k}={shlex.quote(v)}" for k, v in env.items()) + " " + shlex.join(self.cmd)
            proc = subprocess.Popen(["ssh", "-o", "StrictHostKeyChecking=no", host,
                                     f"cd {shlex.quote(os.getcwd())} && {remote}"], start_new_session=True)
        self.workers[wid] = Worker(wid, host, proc, epoch)
        log.info("started worker %s on %s (pid %d, epoch %d)", wid, host, proc.pid, epoch)

    def _reap(self) -> list[str]:
        """Workers that exited; returns the ids of the failed ones (non-zero exit)."""
        failed = []
        for wid, w in list(self.workers.items()):
            rc = w.proc.poll()
            if rc is None:
                continue
            del self.workers[wid]
            if rc != 0 and self.rdzv.outcome() is None:
                lo, hi = self.cooldown
                self.blacklist[w.host] = time.time() + random.uniform(lo, hi)
                failed.append(wid)
                log.warning("worker %s exited with %d: host %s blacklisted", wid, rc, w.host)
        return failed

    # ------------------------------------------------------------------ membership
    def desired(self) -> list[str]:
        now = time.time()
        try:
            hosts = discover(self.script)
        except (subprocess.SubprocessError, OSError, ValueError) as e:
            log.warning("host discovery failed: %s", e)
            return list(self.live)
        slots = [f"{h}:{i}" for h, n in hosts if self.blacklist.get(h, 0) <= now for i in range(n)]
        keep = [w for w in self.live if w in slots]  # survivors keep their ranks
        new = keep + [w for w in slots if w not in keep]
        return new[:self.max_np]

    def _settled(self) -> bool:
        e = self.rdzv.latest_epoch()
        return e == 0 or not self.live or self.rdzv.get(f"e/{e}/synced") is not None

    def publish(self, members: list[str], abort: bool = False) -> int:
        e = self.rdzv.publish(members, abort=abort)
        for wid in members:
            if wid not in self.workers:
                self._spawn(wid, wid.rsplit(":", 1)[0], e)
        log.info("epoch %d: %s", e, members)
        self.live = list(members)
        return e

    def run(self, timeout: float | None = None) -> int:
        t0 = time.time()
        below_min_since: float | None = None
        while True:
            out = self.rdzv.outcome()
            if out is not None:
                self._drain()
                return 0 if out == "done" else 1
            failed = self._reap()
            if failed:
                survivors = [w for w in self.live if w not in failed]
                self.publish(survivors, abort=True)
            want = self.desired()
            if len(want) < self.min_np:
                below_min_since = below_min_since or time.time()
                if time.time() - below_min_since > max(self.cooldown[1], 60.0):
                    log.error("fewer than min-np=%d workers available for too long", self.min_np)
                    self.rdzv.mark_done(False, "below min-np")
                    continue
            else:
                below_min_since = None
                if want != self.live and self._settled():
                    self.publish(want)
            if timeout is not None and time.time() - t0 > timeout:
                self.rdzv.mark_done(False, "vodarun timeout")
            time.sleep(self.interval)

    def _drain(self, grace: float = 30.0) -> None:
        deadline = time.time() + grace
        for w in self.workers.values():
            while w.proc.poll() is None and time.time() < deadline:
                time.sleep(0.05)
            if w.proc.poll() is None:
                w.proc.kill()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("vodarun", description=__doc__.split("\n\n")[0])
    ap.add_argument("--num-proc", "-np", type=int, default=None, help="accepted for horovodrun compatibility")
    ap.add_argument("--min-np", "--min-num-proc", type=int, required=True)
    ap.add_argument("--max-np", "--max-num-proc", type=int, required=True)
    ap.add_argument("--host-discovery-script", required=True)
    ap.add_argument("--blacklist-cooldown-range", type=float, nargs=2, default=(30.0, 100.0))
    ap.add_argument("--discovery-interval", type=float, default=1.0)
    ap.add_argument("--store-host", default=os.environ.get("VODA_STORE_HOST", socket.gethostname()))
    ap.add_argument("--store-port", type=int, default=int(os.environ.get("VODA_STORE_PORT", "29400")))
    ap.add_argument("--name", default=os.environ.get("JOB_NAME", "job"))
    ap.add_argument("--network-interface", default=None, help="accepted for horovodrun compatibility")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing the training command")
    logging.basicConfig(level=os.environ.get("VODA_LOG", "INFO"), format="[vodarun] %(levelname)s %(message)s")
    d = Driver(cmd, a.host_discovery_script, a.min_np, a.max_np, a.store_host, a.store_port, a.name,
               tuple(a.blacklist_cooldown_range), a.discovery_interval)
    return d.run()


if __name__ == "__main__":
    sys.exit(main())
