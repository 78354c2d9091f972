"""Interrupt hand-off uses the epoch the members AGREED on (runtime/elastic.py _transition).

A halt publishes an empty epoch; the MAX agreement at a commit interrupts every member, but a
member whose watcher thread has not polled the store yet still "sees" the old epoch.  Deciding
survivors from that stale view skipped the at-rest checkpoint and left the job with nobody
holding its state (found as an intermittent hang of the halt test under load)."""
from vodascheduler_amd.runtime import elastic as E


class _Rdzv:
    def __init__(self, members_by_epoch):
        self.mem = members_by_epoch
        self.ckpt = None
        self.live = None

    def members(self, e):
        return self.mem[e]

    def set_ckpt(self, path, step):
        self.ckpt = (path, step)

    def set_live_epoch(self, e):
        self.live = e


class _Ctx:
    def __init__(self, rdzv, rank, seen, agreed):
        self.rdzv, self.rank, self.worker_id = rdzv, rank, f"w{rank}"
        self.members = ["w0", "w1"]
        self._seen, self.agreed_epoch = seen, agreed
        self.holds_state = True
        self.left = False

    def latest_seen(self):
        return self._seen

    def destroy_comm(self, abort=False):
        pass

    def stop(self):
        self.left = True


class _State:
    def __init__(self, ctx):
        self.ctx, self.step = ctx, 25

    def save_checkpoint(self):
        return "/ckpt/state.pt"


def test_halt_hands_off_on_agreed_epoch_even_if_watcher_lags():
    rdzv = _Rdzv({1: ["w0", "w1"], 2: []})
    ctx = _Ctx(rdzv, rank=0, seen=1, agreed=2)   # rank 1 saw epoch 2, rank 0's watcher did not
    assert E._transition(_State(ctx)) is False  # excluded -> leaves
    assert rdzv.ckpt == ("/ckpt/state.pt", 25) and rdzv.live == -1
    assert ctx.left and ctx.agreed_epoch == 0


def test_resize_keeps_survivor_without_checkpoint():
    rdzv = _Rdzv({1: ["w0", "w1"], 2: ["w0"]})
    ctx = _Ctx(rdzv, rank=0, seen=1, agreed=2)
    assert E._transition(_State(ctx)) is True
    assert rdzv.ckpt is None and rdzv.live is None
