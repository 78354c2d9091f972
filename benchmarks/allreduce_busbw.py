"""RCCL all-reduce bus bandwidth vs message size over xGMI (BASELINE.md row "Allreduce busbw
vs bucket size"), through the framework's own communicator (csrc/hip/comm.cpp) -- the path the
DDP buckets take.  One process per GPU:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        benchmarks/allreduce_busbw.py --sizes-mb 1,4,16,64,128,256 --dtype bf16

busbw = 2 (n - 1) / n x bytes / time (the ring all-reduce's per-link traffic), as in
rccl-tests.  Rank 0 prints one JSON line per size.  With ``--device cpu`` it runs over gloo
(orchestration check only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.parallel.comm import create_communicator  # noqa: E402
from vodascheduler_amd.runtime.rendezvous import connect_store  # noqa: E402

DT = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,32,64,128,256")
    ap.add_argument("--dtype", default="bf16", choices=sorted(DT))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    port = [0]
    if rank == 0:
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port[0] = s.getsockname()[1]
    dist.broadcast_object_list(port, src=0)
    store = connect_store("127.0.0.1", port[0], is_master=(rank == 0))
    dev = torch.device("cuda", local) if a.device == "cuda" else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    comm = create_communicator(store, "busbw", rank, world, dev, "auto", timeout=120)
    dt = DT[a.dtype] if dev.type == "cuda" else torch.float32
    esz = torch.tensor([], dtype=dt).element_size()
    for mb in [float(x) for x in a.sizes_mb.split(",")]:
        n = int(mb * 2 ** 20) // esz
        buf = torch.ones(n, dtype=dt, device=dev)
        for _ in range(a.warmup):
            comm.allreduce_(buf, "sum")
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            comm.allreduce_(buf, "sum")
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt_s = (time.perf_counter() - t0) / a.iters
        t = torch.tensor([dt_s], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_s = float(t.item())
        nbytes = n * esz
        if rank == 0:
            print(json.dumps({"ranks": world, "size_mb": mb, "dtype": str(dt).replace("torch.", ""), "time_us": round(dt_s * 1e6, 1),
                              "algbw_GBps": round(nbytes / dt_s / 1e9, 2),
                              "busbw_GBps": round(2 * (world - 1) / world * nbytes / dt_s / 1e9, 2)}), flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
