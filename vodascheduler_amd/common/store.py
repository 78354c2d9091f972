"""Job store: the reference's MongoDB layout behind a small pluggable interface.

Reference layout (pkg/common/mongo/mongo.go, pkg/service/service/handlers.go:23-27,100-116,
pkg/scheduler/scheduler/scheduler.go:49-51,862-863):
* DB ``job_metadata``, collection ``v1beta1``: TrainingJob documents keyed by
  ``{job_name, gpu_type}``;
* DB ``job_info``, one collection per job *category* (the un-timestamped name), documents
  keyed by ``name`` (``TrainingJobInfo`` schema).

Backends: :class:`MemoryStore` (single process, tests/simulator) and :class:`SqliteStore`
(durable, shared by the services of one host; WAL mode, one connection per thread).
"""
from __future__ import annotations

import copy
import json
import sqlite3
import threading
from abc import ABC, abstractmethod
from typing import Any

from .types import COLLECTION_JOB_METADATA, DB_JOB_INFO, DB_JOB_METADATA


class NotFound(KeyError):
    pass


class JobStore(ABC):
    # ---- job_metadata.v1beta1 ----
    @abstractmethod
    def insert_metadata(self, doc: dict[str, Any]) -> None: ...

    @abstractmethod
    def find_metadata(self, job_name: str, gpu_type: str | None = None) -> dict[str, Any]: ...

    @abstractmethod
    def update_metadata(self, job_name: str, gpu_type: str, doc: dict[str, Any]) -> None: ...

    @abstractmethod
    def remove_metadata(self, job_name: str) -> None: ...

    @abstractmethod
    def list_metadata(self, gpu_type: str | None = None) -> list[dict[str, Any]]: ...

    # ---- job_info.<category> ----
    @abstractmethod
    def find_job_info(self, category: str, name: str) -> dict[str, Any]: ...

    @abstractmethod
    def insert_job_info(self, category: str, rec: dict[str, Any]) -> None: ...

    @abstractmethod
    def update_job_info(self, category: str, name: str, fields: dict[str, Any]) -> None:
        """``$set`` semantics; dotted keys (``speedup.4``) update nested maps."""

    @abstractmethod
    def remove_job_info(self, category: str, name: str) -> None: ...

    @abstractmethod
    def list_job_info(self, category: str | None = None) -> list[dict[str, Any]]: ...


def _apply_set(doc: dict[str, Any], fields: dict[str, Any]) -> None:
    for k, v in fields.items():
        cur = doc
        parts = k.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = copy.deepcopy(v)


class MemoryStore(JobStore):
    def __init__(self):
        self._lock = threading.RLock()
        self._meta: dict[tuple[str, str], dict] = {}
        self._info: dict[str, dict[str, dict]] = {}

    def insert_metadata(self, doc):
        with self._lock:
            key = (doc["job_name"], doc["gpu_type"])
            if key in self._meta:
                raise ValueError(f"duplicate job metadata {key}")
            self._meta[key] = copy.deepcopy(doc)

    def find_metadata(self, job_name, gpu_type=None):
        with self._lock:
            for (n, g), d in self._meta.items():
                if n == job_name and (gpu_type is None or g == gpu_type):
                    return copy.deepcopy(d)
        raise NotFound(job_name)

    def update_metadata(self, job_name, gpu_type, doc):
        with self._lock:
            if (job_name, gpu_type) not in self._meta:
                raise NotFound(job_name)
            self._meta[(job_name, gpu_type)] = copy.deepcopy(doc)

    def remove_metadata(self, job_name):
        with self._lock:
            keys = [k for k in self._meta if k[0] == job_name]
            if not keys:
                raise NotFound(job_name)
            for k in keys:
                del self._meta[k]

    def list_metadata(self, gpu_type=None):
        with self._lock:
            return [copy.deepcopy(d) for (n, g), d in self._meta.items() if gpu_type is None or g == gpu_type]

    def find_job_info(self, category, name):
        with self._lock:
            try:
                return copy.deepcopy(self._info[category][name])
            except KeyError:
                raise NotFound(f"{category}/{name}") from None

    def insert_job_info(self, category, rec):
        with self._lock:
            col = self._info.setdefault(category, {})
            if rec["name"] in col:
                raise ValueError(f"duplicate job info {category}/{rec['name']}")
            col[rec["name"]] = copy.deepcopy(rec)

    def update_job_info(self, category, name, fields):
        with self._lock:
            try:
                doc = self._info[category][name]
            except KeyError:
                raise NotFound(f"{category}/{name}") from None
            _apply_set(doc, fields)

    def remove_job_info(self, category, name):
        with self._lock:
            try:
                del self._info[category][name]
            except KeyError:
                raise NotFound(f"{category}/{name}") from None

    def list_job_info(self, category=None):
        with self._lock:
            cats = [category] if category is not None else list(self._info)
            return [copy.deepcopy(d) for c in cats for d in self._info.get(c, {}).values()]


class SqliteStore(JobStore):
    """Durable store; each document is a JSON blob.  Safe across threads and processes."""

    def __init__(self, path: str):
        self.path = path
        self._local = threading.local()
        c = self._conn()
        c.executescript(f"""
            PRAGMA journal_mode=WAL;
            CREATE TABLE IF NOT EXISTS {DB_JOB_METADATA}_{COLLECTION_JOB_METADATA} (
                job_name TEXT NOT NULL, gpu_type TEXT NOT NULL, doc TEXT NOT NULL,
                PRIMARY KEY (job_name, gpu_type));
            CREATE TABLE IF NOT EXISTS {DB_JOB_INFO} (
                category TEXT NOT NULL, name TEXT NOT NULL, doc TEXT NOT NULL,
                PRIMARY KEY (category, name));
        """)
        c.commit()
        self._meta_t = f"{DB_JOB_METADATA}_{COLLECTION_JOB_METADATA}"
        self._lock = threading.RLock()

    def _conn(self) -> sqlite3.Connection:
        c = getattr(self._local, "conn", None)
        if c is None:
            c = sqlite3.connect(self.path, timeout=30, isolation_level=None, check_same_thread=False)
            self._local.conn = c
        return c

    def insert_metadata(self, doc):
        try:
            self._conn().execute(f"INSERT INTO {self._meta_t} VALUES (?,?,?)",
                                 (doc["job_name"], doc["gpu_type"], json.dumps(doc)))
        except sqlite3.IntegrityError as e:
            raise ValueError(f"duplicate job metadata {doc['job_name']}") from e

    def find_metadata(self, job_name, gpu_type=None):
        q = f"SELECT doc FROM {self._meta_t} WHERE job_name=?"
        args: tuple = (job_name,)
        if gpu_type is not None:
            q += " AND gpu_type=?"
            args += (gpu_type,)
        row = self._conn().execute(q, args).fetchone()
        if row is None:
            raise NotFound(job_name)
        return json.loads(row[0])

    def update_metadata(self, job_name, gpu_type, doc):
        cur = self._conn().execute(f"UPDATE {self._meta_t} SET doc=? WHERE job_name=? AND gpu_type=?",
                                   (json.dumps(doc), job_name, gpu_type))
        if cur.rowcount == 0:
            raise NotFound(job_name)

    def remove_metadata(self, job_name):
        cur = self._conn().execute(f"DELETE FROM {self._meta_t} WHERE job_name=?", (job_name,))
        if cur.rowcount == 0:
            raise NotFound(job_name)

    def list_metadata(self, gpu_type=None):
        if gpu_type is None:
            rows = self._conn().execute(f"SELECT doc FROM {self._meta_t}").fetchall()
        else:
            rows = self._conn().execute(f"SELECT doc FROM {self._meta_t} WHERE gpu_type=?", (gpu_type,)).fetchall()
        return [json.loads(r[0]) for r in rows]

    def find_job_info(self, category, name):
        row = self._conn().execute(f"SELECT doc FROM {DB_JOB_INFO} WHERE category=? AND name=?",
                                   (category, name)).fetchone()
        if row is None:
            raise NotFound(f"{category}/{name}")
        return json.loads(row[0])

    def insert_job_info(self, category, rec):
        try:
            self._conn().execute(f"INSERT INTO {DB_JOB_INFO} VALUES (?,?,?)", (category, rec["name"], json.dumps(rec)))
        except sqlite3.IntegrityError as e:
            raise ValueError(f"duplicate job info {category}/{rec['name']}") from e

    def update_job_info(self, category, name, fields):
        with self._lock:
            c = self._conn()
            c.execute("BEGIN IMMEDIATE")
            try:
                row = c.execute(f"SELECT doc FROM {DB_JOB_INFO} WHERE category=? AND name=?",
                                (category, name)).fetchone()
                if row is None:
                    raise NotFound(f"{category}/{name}")
                doc = json.loads(row[0])
                _apply_set(doc, fields)
                c.execute(f"UPDATE {DB_JOB_INFO} SET doc=? WHERE category=? AND name=?",
                          (json.dumps(doc), category, name))
                c.execute("COMMIT")
            except BaseException:
                c.execute("ROLLBACK")
                raise

    def remove_job_info(self, category, name):
        cur = self._conn().execute(f"DELETE FROM {DB_JOB_INFO} WHERE category=? AND name=?", (category, name))
        if cur.rowcount == 0:
            raise NotFound(f"{category}/{name}")

    def list_job_info(self, category=None):
        if category is None:
            rows = self._conn().execute(f"SELECT doc FROM {DB_JOB_INFO}").fetchall()
        else:
            rows = self._conn().execute(f"SELECT doc FROM {DB_JOB_INFO} WHERE category=?", (category,)).fetchall()
        return [json.loads(r[0]) for r in rows]


def open_store(url: str | None) -> JobStore:
    """``memory://`` or ``sqlite:///path/to/db`` (default: memory)."""
    if not url or url == "memory://":
        return MemoryStore()
    if url.startswith("sqlite://"):
        return SqliteStore("/" + url[len("sqlite://"):].lstrip("/"))
    raise ValueError(f"unknown store url {url!r}")
