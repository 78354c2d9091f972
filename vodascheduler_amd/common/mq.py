"""Message queue between the training service and the per-GPU-type schedulers.

Reference: pkg/common/rabbitmq/rabbitmq.go:13-136 -- ``Msg{verb: create|configure|delete,
job_name}`` JSON, one non-durable queue per GPU type, auto-ack consumer, buffered channel of
200.  Backends: :class:`InProcQueue` (one process) and :class:`SqliteQueue` (cross-process
on one host: the service process publishes, the scheduler process consumes; messages are
deleted on delivery = auto-ack).
"""
from __future__ import annotations

import json
import queue
import sqlite3
import threading
import time
from dataclasses import asdict, dataclass
from typing import Iterator

from .types import MQ_BUFFER

VERB_CREATE = "create"
VERB_CONFIGURE = "configure"
VERB_DELETE = "delete"


@dataclass
class Msg:
    verb: str
    job_name: str

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @classmethod
    def from_json(cls, s: str | bytes) -> "Msg":
        d = json.loads(s)
        if d.get("verb") not in (VERB_CREATE, VERB_CONFIGURE, VERB_DELETE):
            raise ValueError(f"unknown verb {d.get('verb')!r}")
        return cls(verb=d["verb"], job_name=d["job_name"])


class MessageQueue:
    def publish(self, queue_name: str, msg: Msg) -> None:
        raise NotImplementedError

    def get(self, queue_name: str, timeout: float | None = None) -> Msg | None:
        raise NotImplementedError

    def consume(self, queue_name: str, stop: threading.Event, poll: float = 0.1) -> Iterator[Msg]:
        while not stop.is_set():
            m = self.get(queue_name, timeout=poll)
            if m is not None:
                yield m


class InProcQueue(MessageQueue):
    def __init__(self, maxsize: int = MQ_BUFFER):
        self._qs: dict[str, queue.Queue] = {}
        self._lock = threading.Lock()
        self._maxsize = maxsize

    def _q(self, name: str) -> queue.Queue:
        with self._lock:
            return self._qs.setdefault(name, queue.Queue(self._maxsize))

    def publish(self, queue_name, msg):
        self._q(queue_name).put(Msg.from_json(msg.to_json()), timeout=5)

    def get(self, queue_name, timeout=None):
        try:
            return self._q(queue_name).get(timeout=timeout) if timeout else self._q(queue_name).get_nowait()
        except queue.Empty:
            return None


class SqliteQueue(MessageQueue):
    def __init__(self, path: str):
        self.path = path
        self._local = threading.local()
        c = self._conn()
        c.executescript("""PRAGMA journal_mode=WAL;
            CREATE TABLE IF NOT EXISTS mq (id INTEGER PRIMARY KEY AUTOINCREMENT, queue TEXT NOT NULL,
                                           body TEXT NOT NULL);""")

    def _conn(self):
        c = getattr(self._local, "conn", None)
        if c is None:
            c = sqlite3.connect(self.path, timeout=30, isolation_level=None, check_same_thread=False)
            self._local.conn = c
        return c

    def publish(self, queue_name, msg):
        self._conn().execute("INSERT INTO mq (queue, body) VALUES (?, ?)", (queue_name, msg.to_json()))

    def get(self, queue_name, timeout=None):
        deadline = time.monotonic() + (timeout or 0)
        while True:
            c = self._conn()
            c.execute("BEGIN IMMEDIATE")
            row = c.execute("SELECT id, body FROM mq WHERE queue=? ORDER BY id LIMIT 1", (queue_name,)).fetchone()
            if row is not None:
                c.execute("DELETE FROM mq WHERE id=?", (row[0],))
            c.execute("COMMIT")
            if row is not None:
                return Msg.from_json(row[1])
            if time.monotonic() >= deadline:
                return None
            time.sleep(min(0.05, max(0.0, deadline - time.monotonic())))


def open_queue(url: str | None) -> MessageQueue:
    if not url or url == "inproc://":
        return InProcQueue()
    if url.startswith("sqlite://"):
        return SqliteQueue("/" + url[len("sqlite://"):].lstrip("/"))
    raise ValueError(f"unknown mq url {url!r}")
