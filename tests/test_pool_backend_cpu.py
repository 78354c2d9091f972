"""PoolBackend membership publication (runtime/pool.py): a resize whose previous epoch has not
synced is forced through as an ABORT epoch only when a member is known to be gone -- its
liveness beat (runtime/elastic.py watcher) stopped advancing -- or when no member made
progress (joined epoch / committed step) for the settle timeout, or at an absolute hard
limit; never merely because the epoch is slow while its members progress.
Beats are store-side counters checked on the backend's own clock (no cross-host wall-clock
comparison), and a member that left the job is tombstoned."""
import time

from vodascheduler_amd.runtime.cluster import free_port
from vodascheduler_amd.runtime.pool import PoolBackend
from vodascheduler_amd.runtime.rendezvous import JobRendezvous, connect_store


def _backend(settle: float):
    store = connect_store("127.0.0.1", free_port(), is_master=True)
    b = PoolBackend(store, [("node0", 0), ("node0", 1)], settle_timeout=settle)
    b._stop.set()                        # drive publication by hand
    b._mon.join(2)
    return store, b


def _start(b, job):
    b.pending[job] = (["node0:0"], "start", time.time(), {})
    b._publish_if_settled(job)
    return b.live[job][0]


def test_settle_timeout_aborts_only_when_a_member_is_gone():
    store, b = _backend(0.2)
    b.HEARTBEAT_STALE_S = 0.5
    b.STUCK_FACTOR = 50.0
    rd = JobRendezvous(store, "j")
    e1 = _start(b, "j")
    assert e1 >= 1 and not rd.aborted(e1)
    # a scale-out requested while epoch e1 is still bootstrapping (not synced), well past the
    # settle timeout, with its member alive and progressing: keep waiting
    b.pending["j"] = (["node0:0", "node0:1"], "scale_out", time.time() - 1.0, {})
    for step in range(3):
        rd.heartbeat("node0:0", e1, step)
        b._publish_if_settled("j")
        time.sleep(0.1)
    assert b.live["j"][0] == e1 and b.forced_epochs == 0 and "j" in b.pending
    # the member's beat counter stops advancing (process died): the change goes out as an abort epoch
    time.sleep(0.7)
    b._publish_if_settled("j")
    e2 = b.live["j"][0]
    assert e2 > e1 and rd.aborted(e2) and b.forced_epochs == 1
    assert b.forced_log[0]["stale"] == ["node0:0"] and b.forced_log[0]["why"] == "stale"


def test_live_member_without_progress_aborts_after_settle_timeout():
    """A member that keeps beating (its watcher thread is alive) but whose joined epoch and
    committed step stop advancing -- deadlocked in a collective -- is aborted after
    settle_timeout, not after STUCK_FACTOR x settle_timeout."""
    store, b = _backend(0.3)
    b.STUCK_FACTOR = 1000.0
    b.HARD_SETTLE_S = 1000.0
    rd = JobRendezvous(store, "s")
    e1 = _start(b, "s")
    b.pending["s"] = (["node0:0", "node0:1"], "scale_out", time.time(), {})
    t0 = time.monotonic()
    while b.live["s"][0] == e1 and time.monotonic() - t0 < 5:
        rd.heartbeat("node0:0", e1, 7)  # alive, same progress
        b._publish_if_settled("s")
        time.sleep(0.05)
    assert b.live["s"][0] > e1 and b.forced_log[0]["why"] == "no progress"
    assert time.monotonic() - t0 < 2.0


def test_settle_timeout_hard_limit_for_live_progressing_members():
    store, b = _backend(0.1)
    b.STUCK_FACTOR = 3.0                 # hard limit 0.3 s
    rd = JobRendezvous(store, "k")
    e1 = _start(b, "k")
    rd.heartbeat("node0:0", e1, 0)
    b.pending["k"] = (["node0:1"], "migrate", time.time() - 0.5, {})   # beyond 3 x 0.1 s
    b._publish_if_settled("k")
    assert b.live["k"][0] > e1 and b.forced_epochs == 1 and b.forced_log[0]["stale"] == []
    assert b.forced_log[0]["why"] == "hard limit"
    # the hard limit is also capped in absolute seconds, but never below 2 x settle_timeout
    store, b = _backend(10.0)
    b.HARD_SETTLE_S = 0.2
    rd = JobRendezvous(store, "h")
    e1 = _start(b, "h")
    rd.heartbeat("node0:0", e1, 0)
    b.pending["h"] = (["node0:1"], "migrate", time.time() - 20.5, {})
    b._publish_if_settled("h")
    assert b.live["h"][0] > e1 and b.forced_log[0]["why"] == "hard limit"


def test_settle_timeout_above_hard_cap_keeps_progressing_member():
    """with settle_timeout >= HARD_SETTLE_S a healthy epoch whose member keeps
    progressing (bootstrap phases: join, communicator build, state broadcast) is not aborted
    the moment settle_timeout expires."""
    store, b = _backend(0.3)
    b.HARD_SETTLE_S = 0.1                # below settle_timeout: hard limit = 2 x 0.3 s
    rd = JobRendezvous(store, "p")
    e1 = _start(b, "p")
    b.pending["p"] = (["node0:0", "node0:1"], "scale_out", time.time(), {})
    t0 = time.monotonic()
    phase = 0
    while time.monotonic() - t0 < 0.5:   # past settle_timeout, below 2 x settle_timeout
        phase += 1
        rd.heartbeat("node0:0", e1, -1, phase)  # no committed step yet: bootstrap progress only
        b._publish_if_settled("p")
        time.sleep(0.02)
    assert b.live["p"][0] == e1 and b.forced_epochs == 0
    # once it stops progressing, the no-progress rule fires
    t1 = time.monotonic()
    while b.live["p"][0] == e1 and time.monotonic() - t1 < 3:
        rd.heartbeat("node0:0", e1, -1, phase)
        b._publish_if_settled("p")
        time.sleep(0.05)
    assert b.live["p"][0] > e1 and b.forced_log[0]["why"] in ("no progress", "hard limit")


def test_left_member_is_tombstoned():
    store, _ = _backend(1.0)
    rd = JobRendezvous(store, "t")
    assert rd.read_heartbeat("node0:0") is None
    rd.heartbeat("node0:0", 3, 11)
    rd.heartbeat("node0:0", 3, 12)
    assert rd.read_heartbeat("node0:0") == (2, 3, 12, 0)
    rd.heartbeat("node0:0", 3, 12, 5)
    assert rd.read_heartbeat("node0:0") == (3, 3, 12, 5)
    rd.clear_heartbeat("node0:0")
    assert rd.read_heartbeat("node0:0") is None
