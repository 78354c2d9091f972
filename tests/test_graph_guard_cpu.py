"""Replay guard of the trainer (workloads/train.py): a captured step that produces a
non-finite loss rolls the job back to its last commit and continues eagerly, and the job's
final state equals an uninterrupted eager run (docs/kernels.md, hipGraph section).

The graph is simulated on CPU: a stand-in stepper reports a captured graph and poisons the
loss of one replay, which is what a library kernel misbehaving under replay looks like."""
import torch

from elastic_harness import assert_matches_replay
from vodascheduler_amd.runtime.cluster import free_port
from vodascheduler_amd.runtime.elastic import ElasticContext
from vodascheduler_amd.runtime.rendezvous import JobRendezvous, connect_store
from vodascheduler_amd.workloads import train as T


class _PoisonedGraphStepper:
    """Looks like a GraphedStepper holding a captured graph; replay ``bad`` returns NaN."""

    instances = []

    def __init__(self, step_fn, model=None, optimizer=None, warmup=2, enabled=True, graph=None, bad=7):
        self.step_fn = step_fn
        self.enabled = True
        self.graph = object()
        self.n = 0
        self.bad = bad
        self.released = False
        _PoisonedGraphStepper.instances.append(self)

    def __call__(self, batch):
        out = self.step_fn(batch)
        self.n += 1
        if self.graph is not None and self.n == self.bad:
            out = out.clone()
            out[0] = float("nan")
        return out

    def release(self):
        self.graph = None
        self.released = True


def test_nonfinite_replay_restores_last_commit_and_continues_eagerly(tmp_path, monkeypatch):
    monkeypatch.setattr(T, "GraphedStepper", _PoisonedGraphStepper)
    port = free_port()
    store = connect_store("127.0.0.1", port, is_master=True)
    watch = connect_store("127.0.0.1", port)
    JobRendezvous(store, "guard").publish(["node0:0"])
    ctx = ElasticContext(store, "guard", "node0:0", "cpu", watch_store=watch, join_epoch=1)
    cfg = T.TrainConfig(model="mnist-torch", epochs=1, steps_per_epoch=20, per_gpu_batch=16, lr=0.01,
                        commit_every=5, amp=False, final_state_path=str(tmp_path / "guard.pt"), graph=True)
    nthreads = torch.get_num_threads()
    torch.set_num_threads(1)  # as the pool workers and the replay: identical CPU reductions
    try:
        out = T.train_elastic(ctx, cfg, use_cache=False)
    finally:
        torch.set_num_threads(nthreads)
    assert out["graph_fallbacks"] == 1
    st = _PoisonedGraphStepper.instances[-1]
    assert st.released and not st.enabled and st.graph is None
    assert out["final_step"] == 20
    # the poisoned window (steps 6-10) was rolled back and re-run eagerly: the final state is
    # exactly the uninterrupted run's
    assert_matches_replay(cfg, cfg.final_state_path, "cpu")
    assert torch.isfinite(torch.tensor(out["final_loss"]))
