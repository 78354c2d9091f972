"""PoolBackend membership publication (runtime/pool.py): a resize whose previous epoch has not
synced is forced through as an ABORT epoch only when a member is known to be gone -- its
liveness beat (runtime/elastic.py watcher) stopped -- not merely because the epoch is slow
(a first MIOpen find, an fp32 find-db build, a graph capture)."""
import time

from vodascheduler_amd.runtime.cluster import free_port
from vodascheduler_amd.runtime.pool import PoolBackend
from vodascheduler_amd.runtime.rendezvous import JobRendezvous, connect_store


def test_settle_timeout_aborts_only_when_a_member_is_gone():
    store = connect_store("127.0.0.1", free_port(), is_master=True)
    b = PoolBackend(store, [("node0", 0), ("node0", 1)], settle_timeout=0.2)
    b._stop.set()                        # drive publication by hand
    b._mon.join(2)
    b.HEARTBEAT_STALE_S = 0.5
    b.STUCK_FACTOR = 50.0
    rd = JobRendezvous(store, "j")
    b.pending["j"] = (["node0:0"], "start", time.time(), {})
    b._publish_if_settled("j")
    e1 = b.live["j"][0]
    assert e1 >= 1 and not rd.aborted(e1)
    # a scale-out requested while epoch e1 is still bootstrapping (not synced), well past the
    # settle timeout, with its member alive (fresh heartbeat): keep waiting
    rd.set("hb/node0:0", repr(time.time()))
    b.pending["j"] = (["node0:0", "node0:1"], "scale_out", time.time() - 1.0, {})
    b._publish_if_settled("j")
    assert b.live["j"][0] == e1 and b.forced_epochs == 0 and "j" in b.pending
    # the member's heartbeat stops (process died): the change goes out as an abort epoch
    time.sleep(0.7)
    b._publish_if_settled("j")
    e2 = b.live["j"][0]
    assert e2 > e1 and rd.aborted(e2) and b.forced_epochs == 1
    assert b.forced_log[0]["stale"] == ["node0:0"]


def test_settle_timeout_hard_limit_for_live_but_stuck_members():
    store = connect_store("127.0.0.1", free_port(), is_master=True)
    b = PoolBackend(store, [("node0", 0), ("node0", 1)], settle_timeout=0.1)
    b._stop.set()
    b._mon.join(2)
    b.STUCK_FACTOR = 3.0                 # hard limit 0.3 s
    rd = JobRendezvous(store, "k")
    b.pending["k"] = (["node0:0"], "start", time.time(), {})
    b._publish_if_settled("k")
    e1 = b.live["k"][0]
    rd.set("hb/node0:0", repr(time.time()))
    b.pending["k"] = (["node0:1"], "migrate", time.time() - 0.5, {})   # beyond 3 x 0.1 s
    b._publish_if_settled("k")
    assert b.live["k"][0] > e1 and b.forced_epochs == 1 and b.forced_log[0]["stale"] == []
