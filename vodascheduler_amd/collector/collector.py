"""Metrics collector: per-epoch CSV rows -> job_info (reference
python/metrics_collector/metrics_collector.py:15-184, run every minute by a CronJob).

For every job it reads ``<metrics_dir>/<job>.csv`` and updates the job's ``job_info`` record
with ``$set`` semantics: per-worker-count mean step / epoch time, speedup ``t(1)/t(k)``,
efficiency ``speedup/k``, current / remaining epochs and the remaining-time estimate
``epoch_time(1) x remaining_epochs``, plus running / waiting / GPU / elapsed seconds.

Improvements over the reference (documented deviations):
* when no 1-worker epoch was measured, ``t(1)`` is inferred from the smallest measured
  worker count assuming linear scaling below it (the reference divides by the 1-second
  placeholder and produces meaningless speedups);
* unmeasured worker counts are filled by Amdahl interpolation fitted to the measured
  points, so info-driven policies see a monotone, saturating curve;
* the category's base record is refreshed too, so the next job of the same category
  starts from measured history.
"""
from __future__ import annotations

import csv
import logging
import os
import re
import statistics
from datetime import datetime

from ..common.store import JobStore, NotFound
from ..common.types import MAX_NUM_GPU

log = logging.getLogger("vodascheduler_amd.collector")
TS_RE = re.compile(r"-\d{8}-\d{6}(-\d+)?$")
TIME_FMT = "%Y-%m-%d %H:%M:%S.%f"


def category_of(job: str) -> str:
    return TS_RE.sub("", job)


def fit_amdahl(points: dict[int, float]) -> float:
    """Serial fraction ``a`` of speedup(k) = k / (1 + a (k - 1)) fitted to measured points."""
    num = den = 0.0
    for k, s in points.items():
        if k <= 1 or s <= 0:
            continue
        # k/s - 1 = a (k - 1)  -> least squares through the origin
        y, x = k / s - 1.0, k - 1.0
        num += x * y
        den += x * x
    return max(0.0, num / den) if den > 0 else 0.0


def speedup_table(epoch_time: dict[int, float], max_gpu: int = MAX_NUM_GPU) -> dict[str, float]:
    ks = sorted(k for k in epoch_time if k > 0)
    if not ks:
        return {}
    if 1 in epoch_time:
        t1 = epoch_time[1]
    else:
        t1 = epoch_time[ks[0]] * ks[0]  # linear below the smallest measured count
    measured = {k: t1 / epoch_time[k] for k in ks}
    a = fit_amdahl(measured)
    sp = {"0": 0.0}
    for k in range(1, max_gpu + 2):
        sp[str(k)] = measured.get(k, k / (1.0 + a * (k - 1)))
    return sp


class MetricsCollector:
    def __init__(self, store: JobStore, metrics_dir: str, update_category_base: bool = True):
        self.store = store
        self.metrics_dir = metrics_dir
        self.update_category_base = update_category_base

    def jobs(self) -> list[str]:
        if not os.path.isdir(self.metrics_dir):
            return []
        return sorted(f[:-4] for f in os.listdir(self.metrics_dir) if f.endswith(".csv"))

    def update_info_all(self, jobs: list[str] | None = None) -> int:
        n = 0
        for j in jobs if jobs is not None else self.jobs():
            try:
                n += bool(self.parse_csv_and_update_db(j))
            except Exception:
                log.exception("collector: job %s", j)
        return n

    def parse_csv_and_update_db(self, job: str) -> dict | None:
        path = os.path.join(self.metrics_dir, job + ".csv")
        try:
            with open(path) as f:
                rows = list(csv.DictReader(f))
        except OSError:
            return None
        if not rows:
            return None
        cat = category_of(job)
        try:
            post = self.store.find_job_info(cat, job)
        except NotFound:
            return None
        last_epoch = int(rows[-1]["epoch"])
        if int(post.get("current_epoch", -1)) == last_epoch and post.get("_rows") == len(rows):
            return None  # nothing new
        by_w: dict[int, list[dict]] = {}
        for r in rows:
            by_w.setdefault(int(r["workers"]), []).append(r)
        step_t = {k: statistics.fmean(float(r["step_time_sec"]) for r in v) for k, v in by_w.items()}
        epoch_t = {k: statistics.fmean(float(r["epoch_time_sec"]) for r in v) for k, v in by_w.items()}
        sp = speedup_table(epoch_t)
        eff = {k: (v / int(k) if int(k) else 0.0) for k, v in sp.items()}
        total = int(post.get("total_epochs", rows[-1].get("total_epochs", 1)))
        remaining = max(0, total - last_epoch - 1)
        t1 = epoch_t.get(1, epoch_t[min(epoch_t)] * min(epoch_t))
        start = datetime.strptime(rows[0]["start_time"], TIME_FMT)
        end = datetime.strptime(rows[-1]["start_time"], TIME_FMT)
        elapsed = (end - start).total_seconds() + float(rows[-1]["epoch_time_sec"])
        running = sum(float(r["epoch_time_sec"]) for r in rows)
        gpu = sum(float(r["epoch_time_sec"]) * int(r["workers"]) for r in rows)
        fields = {
            "current_epoch": last_epoch,
            "remainning_epochs": remaining,
            "estimated_remainning_time_sec": float(t1 * remaining),
            "running_time_sec": running,
            "waiting_time_sec": max(0.0, elapsed - running),
            "gpu_time_sec": gpu,
            "elasped_time_sec": elapsed,
            "_rows": len(rows),
        }
        for k, v in step_t.items():
            fields[f"step_time_sec.{k}"] = v
        for k, v in epoch_t.items():
            fields[f"epoch_time_sec.{k}"] = v
        for k, v in sp.items():
            fields[f"speedup.{k}"] = v
        for k, v in eff.items():
            fields[f"efficiency.{k}"] = v
        self.store.update_job_info(cat, job, fields)
        if self.update_category_base:
            base = {k: v for k, v in fields.items() if k.split(".")[0] in
                    ("step_time_sec", "epoch_time_sec", "speedup", "efficiency")}
            try:
                self.store.update_job_info(cat, cat, base)
            except NotFound:
                pass
        return fields


def main(argv=None) -> int:
    """One collector pass (the reference runs it as a CronJob every minute,
    helm/voda-scheduler/values.yaml:104) or ``--every SECONDS`` in a loop."""
    import argparse
    import time

    from ..common.store import open_store

    ap = argparse.ArgumentParser("vodascheduler-collector")
    ap.add_argument("--store", required=True, help="sqlite:///path (shared with the services)")
    ap.add_argument("--metrics-dir", default=os.environ.get("VODA_METRICS_DIR", "/metrics"))
    ap.add_argument("--every", type=float, default=0.0, help="repeat every N seconds (0 = one pass)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    c = MetricsCollector(open_store(a.store), a.metrics_dir)
    while True:
        n = c.update_info_all()
        log.info("updated job info of %d job(s)", n)
        if a.every <= 0:
            return 0
        time.sleep(a.every)


if __name__ == "__main__":
    raise SystemExit(main())
