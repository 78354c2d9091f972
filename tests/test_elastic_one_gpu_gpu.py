"""The elastic runtime on real MI355X hardware with the one GPU a test box has: two pool workers
share cuda:0 and reduce over gloo (RCCL refuses two ranks on one device), so a live resize
1 -> 2 -> 1 with a migration runs the real kernels, the bucketed DDP engine, the membership
epochs, the commit / restore / state broadcast and the lock-step digests end to end.  The
final state must equal a replay of the logged world-size trajectory through real gloo
collectives on the same device (the multi-GPU file repeats this on RCCL when >= 2 GPUs exist).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(tmp_path, name, **kw):
    from vodascheduler_amd.workloads.train import TrainConfig

    d = dict(model="mnist-torch", epochs=2, steps_per_epoch=200, per_gpu_batch=64, lr=0.01, commit_every=1,
             amp=False, report_progress=True, final_state_path=str(tmp_path / f"{name}.pt"), graph=False,
             step_digests=True, deterministic=True)
    d.update(kw)
    return TrainConfig(**d)


def test_live_resize_1_2_1_two_workers_one_gpu_gloo(tmp_path, monkeypatch):
    from elastic_harness import Controller, assert_matches_replay, start_pool, stop_pool

    monkeypatch.setenv("VODA_CKPT_DIR", str(tmp_path / "ckpt"))
    wids = ["node0:0", "node0:1"]
    store, procs, q = start_pool(wids, ["cuda:0", "cuda:0"], "gloo")
    results = None
    try:
        cfg = _cfg(tmp_path, "one_gpu")
        c = Controller(store, "one_gpu", cfg)
        c.publish(wids[:1])
        c.wait_progress(20)
        c.publish(wids)                    # grow: the second worker joins, state is broadcast
        c.wait_progress(c.progress() + 20)
        c.publish(wids[1:])                # shrink onto the OTHER worker: the state migrates
        assert c.wait_done(timeout=240) == "done"
        ex = assert_matches_replay(cfg, cfg.final_state_path, "cuda:0", exact=True, backend="gloo",
                                   devices=["cuda:0", "cuda:0"])
        ws = [ex["world_log"][i + 1] for i in range(0, len(ex["world_log"]), 2)]
        assert ws[0] == 1 and 2 in ws and ws[-1] == 1, ex["world_log"]
    finally:
        results = stop_pool(store, procs, q, timeout=60)
    done = {w for w, recs in results.items() for r in recs if r["job"] == "one_gpu"}
    assert wids[1] in done, results
