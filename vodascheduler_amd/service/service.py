"""Training service (reference pkg/service/service/{service.go,handlers.go}, main.go).

``POST /training`` (raw YAML MPIJob body) -> create; ``DELETE /training`` (JSON string job
name) -> delete; ``GET /metrics``; ``GET /``.  Also ``GET /training`` (the reference CLI
calls it but the service never routed it): a status table built from
the job store, so ``vodascheduler get jobs`` works against the service.
"""
from __future__ import annotations

import json
import logging
import time

from ..common import mpijob
from ..common.mq import VERB_CREATE, VERB_DELETE, MessageQueue, Msg
from ..common.store import JobStore, NotFound
from ..common.trainingjob import (TrainingJob, create_base_job_info_record, init_job_info_record,
                                  new_training_job)
from ..common.types import ENTRY_POINT, NAME, VERSION, JobConfigEnv
from ..common.workload import (INFO_MEASURED, INFO_PLACEHOLDER, declared_workload, prior_fields,
                               remaining_from_history)
from ..utils.clock import Clock, RealClock
from ..utils.http import Router, as_json, text
from ..utils.metrics import ServiceMetrics

log = logging.getLogger("vodascheduler_amd.service")


class TrainingService:
    def __init__(self, store: JobStore, mq: MessageQueue, clock: Clock | None = None,
                 metrics: ServiceMetrics | None = None, seed_from_workload: bool = True):
        self.store = store
        self.mq = mq
        self.clock = clock or RealClock()
        self.metrics = metrics or ServiceMetrics()
        # False: the reference's behaviour -- a category without history starts from the
        # CreateBaseJobInfo placeholder (1 s epochs, linear speedup); kept for A/B only
        self.seed_from_workload = seed_from_workload

    # ------------------------------------------------------------ job info history
    def get_or_create_base_job_info(self, category: str) -> dict:
        """Category base record ``job_info.<category>/<category>`` (handlers.go:180-206).
        The metrics collector refreshes this record with each job's measurements, so new
        jobs of a category start from measured speedups (fix for §2.10 #9)."""
        try:
            return self.store.find_job_info(category, category)
        except NotFound:
            info = create_base_job_info_record(category)
            try:
                self.store.insert_job_info(category, info)
            except ValueError:  # raced with another creator
                return self.store.find_job_info(category, category)
            return info

    def initial_job_info(self, base: dict, name: str, epochs: int, spec: dict) -> dict:
        """The new job's job_info record (``initJobInfo``, handlers.go:212-223), with an
        estimate that means something before the job has run a step:

        1. the category has measured history (the collector refreshed its base record):
           measured speedup, remaining = measured 1-GPU step time x the job's own declared
           step count (or the reference's ``epochs x epoch_time(1)``);
        2. else the job declares a workload (annotation or reference launcher flags): the
           MI355X speed model of that model (``common/workload.prior_fields``);
        3. else the reference placeholder (1 s epochs, linear speedup)."""
        info = init_job_info_record(base, name, epochs)
        try:
            wl = declared_workload(spec)
        except Exception:  # an unparsable annotation must not fail the submission
            log.warning("job %s: unreadable workload declaration", name, exc_info=True)
            wl = None
        if base.get("info_source") == INFO_MEASURED:
            info["estimated_remainning_time_sec"] = remaining_from_history(base, wl, epochs)
            info["info_source"] = INFO_MEASURED
        elif wl is not None and self.seed_from_workload:
            info.update(prior_fields(wl, epochs))
        else:
            info["info_source"] = INFO_PLACEHOLDER
        if wl is not None:
            info["per_gpu_batch"] = int(wl.get("per_gpu_batch", 0) or 0)
            info["steps_per_epoch"] = int(wl.get("steps_per_epoch", 0) or 0)
        return info

    # ------------------------------------------------------------ create / delete
    def create_training_job(self, data: bytes | str, submit_time: float | None = None) -> str:
        t0 = time.perf_counter()
        try:
            spec = mpijob.load_spec(data)
            # JOB_CATEGORY knob, else the reference's category = the submitted name
            submitted = spec["metadata"]["name"]
            category = mpijob.get_env(spec, JobConfigEnv.JOB_CATEGORY.value) or submitted
            base = self.get_or_create_base_job_info(category)
            now = self.clock.now() if submit_time is None else submit_time
            name = mpijob.timestamped_name(submitted, now)
            # guarantee uniqueness when several jobs of a name arrive within a second
            k = 1
            while self._exists(name):
                name = f"{mpijob.timestamped_name(submitted, now)}-{k}"
                k += 1
            mpijob.set_name(spec, name)
            job = new_training_job(spec, category, now)
            info = self.initial_job_info(base, name, job.config.epochs, spec)
            self.store.insert_job_info(category, info)
            try:
                self.store.insert_metadata(job.to_dict())
            except Exception:
                self.store.remove_job_info(category, name)
                raise
            try:
                self.mq.publish(job.gpu_type, Msg(VERB_CREATE, name))
            except Exception:
                # keep DB and queue consistent (handlers.go:121-133)
                self.store.remove_job_info(category, name)
                self.store.remove_metadata(name)
                raise
        finally:
            self.metrics.create_duration.observe(time.perf_counter() - t0)
        self.metrics.create_success_duration.observe(time.perf_counter() - t0)
        self.metrics.jobs_created.inc()
        log.info("created training job %s", name)
        return name

    def _exists(self, name: str) -> bool:
        try:
            self.store.find_metadata(name)
            return True
        except NotFound:
            return False

    def delete_training_job(self, name: str) -> None:
        t0 = time.perf_counter()
        try:
            doc = self.store.find_metadata(name)
            self.store.remove_metadata(name)
            self.mq.publish(doc["gpu_type"], Msg(VERB_DELETE, name))
        finally:
            self.metrics.delete_duration.observe(time.perf_counter() - t0)
        self.metrics.delete_success_duration.observe(time.perf_counter() - t0)
        self.metrics.jobs_deleted.inc()

    def status_table(self) -> str:
        fmt = "%-60s %-10s %-10s %-25s %-10s %-10s %-10s\n"
        out = fmt % ("NAME", "STATUS", "WORKERS", "SCHEDULER", "WAITING", "RUNNING", "TOTAL")
        rows = []
        for d in self.store.list_metadata():
            j = TrainingJob.from_dict(d)
            m = j.time_metrics
            workers = 0
            if j.spec is not None:
                try:
                    workers = mpijob.worker_replicas(j.spec) if j.status == "Running" else 0
                except (KeyError, TypeError):
                    workers = 0
            rows.append(fmt % (j.name, j.status, workers, j.gpu_type, f"{round(m.waiting_time)}s",
                               f"{round(m.running_time)}s", f"{round(m.total_time)}s"))
        return out + "".join(sorted(rows))

    # ------------------------------------------------------------ REST
    def router(self) -> Router:
        r = Router()

        def create(body, _q):
            try:
                name = self.create_training_job(body)
            except Exception as e:
                return text(400, f"{e}\n")
            return text(200, f"Training job created: {name}\n")

        def delete(body, _q):
            try:
                name = json.loads(body)
                if not isinstance(name, str):
                    raise ValueError("body must be a JSON string")
            except (ValueError, json.JSONDecodeError) as e:
                return as_json(400, {"error": str(e)})
            try:
                self.delete_training_job(name)
            except NotFound:
                return text(404, f"training job not found: {name}\n")
            return text(200, f"Training job deleted: {name}\n")

        r.add("POST", ENTRY_POINT, create)
        r.add("DELETE", ENTRY_POINT, delete)
        r.add("GET", ENTRY_POINT, lambda b, q: text(200, self.status_table()))
        r.add("GET", "/metrics", lambda b, q: (200, "text/plain; version=0.0.4", self.metrics.exposition()))
        r.add("GET", "/", lambda b, q: text(200, f"{NAME} training service {VERSION}\n"))
        return r
