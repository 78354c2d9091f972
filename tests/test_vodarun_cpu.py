"""vodarun (the horovodrun-elastic replacement) on CPU: discovery-script driven resize of a
real 2-process gloo job, and failure of a worker process."""
import os
import stat
import sys
import threading
import time

from vodascheduler_amd.runtime.cluster import free_port
from vodascheduler_amd.runtime.vodarun import Driver, discover


def _script(path, text):
    path.write_text(f"#!/bin/sh\necho '{text}'\n")
    path.chmod(path.stat().st_mode | stat.S_IEXEC)
    return str(path)


def test_discover_parses_horovod_format(tmp_path):
    s = _script(tmp_path / "h.sh", "localhost:2\nhostb\n# comment")
    assert discover(s) == [("localhost", 2), ("hostb", 1)]


def test_vodarun_resizes_on_discovery_change(tmp_path):
    script = _script(tmp_path / "hosts.sh", "localhost:2")
    cmd = [sys.executable, "-m", "vodascheduler_amd.workloads.train", "--model", "mnist-torch", "--epochs", "3",
           "--steps-per-epoch", "120", "--batch-size", "16", "--name", "vj", "--commit-every", "1"]
    os.environ.setdefault("PYTHONPATH", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    d = Driver(cmd, script, 1, 2, "127.0.0.1", free_port(), "vj", cooldown=(1.0, 2.0), interval=0.2)
    rc = []
    t = threading.Thread(target=lambda: rc.append(d.run(timeout=240)), daemon=True)
    t.start()
    deadline = time.time() + 120
    while d.rdzv.latest_epoch() < 1 or d.rdzv.get("e/1/synced") is None:
        assert time.time() < deadline, "job never started"
        time.sleep(0.1)
    assert d.live == ["localhost:0", "localhost:1"]
    _script(tmp_path / "hosts.sh", "localhost:1")  # the operator shrank the job
    t.join(240)
    assert rc == [0]
    assert d.rdzv.latest_epoch() >= 2 and d.rdzv.members(2) == ["localhost:0"]
