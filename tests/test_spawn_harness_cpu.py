"""The multi-GPU tests' rank spawner (tests/elastic_harness.spawn_ranks) must never wedge
the test session (VERDICT r2 Weak #5): a hung or crashed rank fails the test quickly, names
the rank, and leaves no process behind."""
import os
import time

import pytest

from elastic_harness import spawn_ranks


def _ok(port, rank, world, q):
    q.put((rank, rank * 10))


def _one_hangs(port, rank, world, q):
    if rank == 1:
        time.sleep(3600)
    q.put((rank, os.getpid()))


def _one_crashes(port, rank, world, q):
    if rank == 2:
        os._exit(7)
    time.sleep(3600)  # the others wait forever for the crashed peer


def test_spawn_collects_results():
    assert spawn_ranks(_ok, 3) == {0: 0, 1: 10, 2: 20}


def test_spawn_hung_rank_is_named_and_killed():
    t0 = time.monotonic()
    with pytest.raises(AssertionError, match=r"ranks \[1\] of 3"):
        spawn_ranks(_one_hangs, 3, timeout=8)
    assert time.monotonic() - t0 < 40


def test_spawn_crashed_rank_ends_the_wait_early():
    t0 = time.monotonic()
    with pytest.raises(AssertionError, match="exit codes"):
        spawn_ranks(_one_crashes, 3, timeout=120)
    assert time.monotonic() - t0 < 60
