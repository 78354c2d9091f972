"""Unit tests of the elastic-equivalence oracle's pieces (workloads/replay.py): world-log
segmentation, lock-step log comparison, and a 3-rank gloo replay against the single-process
replay where both are exact (worlds 1 and 2)."""
import torch

from vodascheduler_amd.workloads.replay import (first_divergence, replay_collective, step_record,
                                                world_segments)
from vodascheduler_amd.workloads.train import TrainConfig, replay_reference


def test_world_segments_last_entry_wins_and_runs_merge():
    assert world_segments([0, 8], 5) == [(0, 5, 8)]
    assert world_segments([0, 8, 3, 4, 6, 8], 9) == [(0, 3, 8), (3, 6, 4), (6, 9, 8)]
    # a restore can log the same start twice: the later entry wins; equal neighbours merge
    assert world_segments([0, 2, 4, 1, 4, 2, 7, 2], 9) == [(0, 9, 2)]
    assert world_segments([0, 2, 5, 1], 5) == [(0, 5, 2)]


def test_first_divergence_names_the_step_and_what_differs():
    t = [torch.zeros(4)]
    a = [step_record(1, 8, 0.08, t), step_record(2, 8, 0.08, t)]
    assert first_divergence(a, list(a)) is None
    b = [step_record(1, 8, 0.08, t), step_record(2, 4, 0.04, [torch.ones(4)])]
    msg = first_divergence(a, b)
    assert msg.startswith("step 2:") and "world" in msg and "lr" in msg and "state" in msg
    # the elastic log holds committed history only: steps missing on one side are skipped
    assert first_divergence(a[1:], a) is None
    assert first_divergence([], a) is None


def test_relaxed_lockstep_check_ignores_state_only():
    """The GPU (exact=False) check compares world and LR of every common step, never the
    state digest: atomics may change the last bits of the state, never the schedule."""
    t, u = [torch.zeros(4)], [torch.ones(4)]
    a = [step_record(1, 8, 0.08, t), step_record(2, 8, 0.08, t)]
    only_state = [step_record(1, 8, 0.08, u), step_record(2, 8, 0.08, u)]
    assert first_divergence(a, only_state) is not None
    assert first_divergence(a, only_state, fields=("world", "lr")) is None
    lr_off = [step_record(1, 8, 0.08, u), step_record(2, 8, 0.16, u)]
    msg = first_divergence(a, lr_off, fields=("world", "lr"))
    assert msg.startswith("step 2:") and "lr" in msg and "state" not in msg
    world_off = [step_record(1, 4, 0.08, t)]
    assert "world" in first_divergence(a, world_off, fields=("world", "lr"))
    import pytest
    with pytest.raises(ValueError):
        first_divergence(a, a, fields=("loss",))


def test_collective_replay_equals_single_process_replay_at_worlds_1_and_2():
    cfg = TrainConfig(model="mnist-torch", epochs=1, steps_per_epoch=40, per_gpu_batch=16, lr=0.01, amp=False,
                      graph=False, step_digests=True)
    wl = [0, 2, 5, 1, 9, 2]
    nt = torch.get_num_threads()
    torch.set_num_threads(1)  # as the replay ranks and the pool workers: CPU kernels block by thread count
    try:
        ref, ref_ex = replay_reference(cfg, wl, 14, torch.device("cpu"))
    finally:
        torch.set_num_threads(nt)
    got, got_ex = replay_collective(cfg, wl, 14, "gloo")
    assert len(ref) == len(got) and all(torch.equal(a, b) for a, b in zip(ref, got))
    assert first_divergence(got_ex["steplog"], ref_ex["steplog"]) is None
    assert got_ex["epoch"] == ref_ex["epoch"] and got_ex["samples"] == ref_ex["samples"]


def test_deterministic_kernels_scoped_to_one_job():
    """cfg.deterministic switches MIOpen's deterministic solvers on for that job only;
    a warm pool worker gets its previous process-global flags back afterwards."""
    from vodascheduler_amd.workloads.train import deterministic_kernels

    prev = (torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = False, True
    try:
        with deterministic_kernels(True):
            assert torch.backends.cudnn.deterministic and not torch.backends.cudnn.benchmark
        assert not torch.backends.cudnn.deterministic and torch.backends.cudnn.benchmark
        with deterministic_kernels(False):
            assert not torch.backends.cudnn.deterministic
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
