"""Entry point of one warm pool worker process (one per GPU).

    python -m vodascheduler_amd.agent.worker --store 127.0.0.1:29400 --wid node0:3 --device cuda:3

Connects to the cluster store, publishes a heartbeat (``pool/<wid>/hb``, wall-clock seconds)
from a side thread, and serves job assignments from its mailbox with the elastic runtime
until ``pool/shutdown`` is set.  The process keeps its HIP context, MIOpen / hipBLASLt caches,
the caching allocator and the warm workload cache across jobs, so a job start or resize
costs a communicator rebuild + state broadcast, not a process or context creation.
"""
from __future__ import annotations

import argparse
import logging
import os
import threading
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")

HEARTBEAT_SEC = 1.0


def heartbeat_loop(store, wid: str, stop: threading.Event, period: float = HEARTBEAT_SEC) -> None:
    while not stop.is_set():
        try:
            store.set(f"pool/{wid}/hb", repr(time.time()))
        except Exception:  # store gone: the agent is shutting down
            return
        stop.wait(period)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("vodascheduler-worker")
    ap.add_argument("--store", required=True, help="host:port of the cluster TCPStore")
    ap.add_argument("--wid", required=True, help="worker id <node>:<gpu>")
    ap.add_argument("--device", default="cuda:0", help="cuda:<i> or cpu")
    ap.add_argument("--backend", default="auto", help="collective backend: auto | rccl | gloo")
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--threads", type=int, default=1, help="torch CPU threads (cpu device)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("VODA_LOG", "WARNING"),
                        format=f"[worker {a.wid}] %(levelname)s %(name)s: %(message)s")

    import torch

    from ..runtime.pool import PoolWorker
    from ..runtime.rendezvous import connect_store

    dev = torch.device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        from ..ops import _native

        _native.hip()  # a GPU worker without the HIP extension must not start
    else:
        torch.set_num_threads(a.threads)
    host, port = a.store.rsplit(":", 1)
    store = connect_store(host, int(port))
    watch = connect_store(host, int(port))
    hb_store = connect_store(host, int(port))
    stop = threading.Event()
    threading.Thread(target=heartbeat_loop, args=(hb_store, a.wid, stop), daemon=True, name="heartbeat").start()
    try:
        PoolWorker(store, watch, a.wid, dev, backend=a.backend, timeout=a.timeout).serve()
    finally:
        stop.set()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
