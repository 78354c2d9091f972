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
import json
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


def estimate_tables(step_t: dict[int, float], prior: dict | None = None,
                    max_gpu: int = MAX_NUM_GPU) -> tuple[dict[str, float], dict[str, float]]:
    """Speedup and per-worker-count step-time tables from measured step times.

    ``step_t[k]``: seconds per training step with ``k`` workers (each step processes ``k``
    per-GPU batches), so ``speedup(k) = k t(1) / t(k)`` -- robust to epochs cut short by a
    resize, unlike the epoch-time ratio.  ``t(1)``: measured; else, when only larger counts
    were measured, the smallest measured count's time scaled by the PRIOR CURVE's speedup
    there (``t(1) = t(k) s_prior(k) / k``: the prior -- the workload's MI355X profile or the
    category's history -- supplies the shape of the curve, never an absolute time that may
    be for another precision or batch); else linear below the smallest measured count; with
    nothing measured, the prior's own t(1).  Unmeasured counts: Amdahl fit through the
    measured points when one with k > 1 exists, else the prior's curve, else linear."""
    ks = sorted(k for k, v in step_t.items() if k > 0 and v > 0)
    prior_sp = (prior or {}).get("speedup") or {}
    prior_t1 = float(((prior or {}).get("step_time_sec") or {}).get("1", 0.0) or 0.0)
    if (prior or {}).get("info_source", "placeholder") == "placeholder":
        prior_sp, prior_t1 = {}, 0.0
    if 1 in step_t and step_t[1] > 0:
        t1 = step_t[1]
    elif ks:
        kmin = ks[0]
        s_prior = float(prior_sp.get(str(kmin), 0.0) or 0.0)
        # linear below the smallest measured count unless the prior curve says otherwise
        t1 = step_t[kmin] * min(float(kmin), s_prior) / kmin if s_prior > 0 else step_t[kmin]
    elif prior_t1 > 0:
        t1 = prior_t1
    else:
        return {}, {}
    measured = {k: min(float(k), k * t1 / step_t[k]) for k in ks}
    multi = [k for k in ks if k > 1]
    a = fit_amdahl(measured) if multi else None
    sp = {"0": 0.0}
    st = {"0": 0.0}
    for k in range(1, max_gpu + 2):
        if k in measured:
            v = measured[k]
        elif a is not None:
            v = k / (1.0 + a * (k - 1))
        elif str(k) in prior_sp and float(prior_sp[str(k)]) > 0:
            v = float(prior_sp[str(k)])
        else:
            v = float(k)
        sp[str(k)] = v
        st[str(k)] = step_t[k] if k in measured else k * t1 / v
    return sp, st


class MetricsCollector:
    """``update_info_all`` is one collector pass (the reference's cron job).  Two inputs per
    job, both written by the job's rank 0 into ``metrics_dir``:

    * ``<job>.csv`` -- one row per epoch (the reference's ``MetricsCSVLogger``);
    * ``<job>.progress.json`` -- fast online profiling (extension): rewritten at most every
      second with the samples done / total and the GPU-timed step time per world size, so a
      job's estimate tracks it from its first commits instead of its first epoch row."""

    def __init__(self, store: JobStore, metrics_dir: str, update_category_base: bool = True):
        self.store = store
        self.metrics_dir = metrics_dir
        self.update_category_base = update_category_base

    def jobs(self) -> list[str]:
        if not os.path.isdir(self.metrics_dir):
            return []
        out = set()
        for f in os.listdir(self.metrics_dir):
            if f.endswith(".progress.json"):
                out.add(f[:-len(".progress.json")])
            elif f.endswith(".csv"):
                out.add(f[:-4])
        return sorted(out)

    def update_info_all(self, jobs: list[str] | None = None) -> int:
        n = 0
        for j in jobs if jobs is not None else self.jobs():
            try:
                n += bool(self.parse_csv_and_update_db(j))
            except Exception:
                log.exception("collector: job %s", j)
        return n

    def _category(self, job: str) -> str:
        try:
            return self.store.find_metadata(job).get("job_category") or category_of(job)
        except (NotFound, AttributeError):
            return category_of(job)

    def _read_progress(self, job: str) -> dict | None:
        try:
            with open(os.path.join(self.metrics_dir, job + ".progress.json")) as f:
                return json.load(f)
        except (OSError, ValueError):
            return None

    def parse_csv_and_update_db(self, job: str) -> dict | None:
        path = os.path.join(self.metrics_dir, job + ".csv")
        try:
            with open(path) as f:
                rows = list(csv.DictReader(f))
        except OSError:
            rows = []
        prog = self._read_progress(job)
        if not rows and not prog:
            return None
        cat = self._category(job)
        try:
            post = self.store.find_job_info(cat, job)
        except NotFound:
            return None
        if post.get("_rows") == len(rows) and post.get("_progress_t") == (prog or {}).get("t"):
            return None  # nothing new
        # ---- step times per worker count: GPU-timed progress first, epoch rows second
        step_t: dict[int, float] = {}
        for k, (n, sec) in ((prog or {}).get("perf") or {}).items():
            if int(n) > 0 and float(sec) > 0:
                step_t[int(k)] = float(sec) / int(n)
        by_w: dict[int, list[dict]] = {}
        for r in rows:
            by_w.setdefault(int(r["workers"]), []).append(r)
        for k, v in by_w.items():
            if k not in step_t:
                step_t[k] = statistics.fmean(float(r["step_time_sec"]) for r in v)
        epoch_t = {k: statistics.fmean(float(r["epoch_time_sec"]) for r in v) for k, v in by_w.items()}
        sp, st = estimate_tables(step_t, post)
        if not sp:
            return None
        eff = {k: (v / int(k) if int(k) else 0.0) for k, v in sp.items()}
        t1 = st["1"]
        total = int(post.get("total_epochs", rows[-1].get("total_epochs", 1) if rows else 1))
        fields: dict = {"_rows": len(rows), "_progress_t": (prog or {}).get("t"), "info_source": "measured",
                        "measured_workers": sorted(step_t)}
        if prog and int(prog.get("per_gpu_batch", 0)) > 0:
            # exact progress: remaining single-GPU steps x the single-GPU step time
            bs = int(prog["per_gpu_batch"])
            left = max(0.0, float(prog["samples_total"]) - float(prog["samples_done"]))
            fields["estimated_remainning_time_sec"] = left / bs * t1
            fields["current_epoch"] = int(prog.get("epoch", 0))
            fields["remainning_epochs"] = max(0, int(prog.get("epochs", total)) - int(prog.get("epoch", 0)))
        else:
            last_epoch = int(rows[-1]["epoch"])
            remaining = max(0, total - last_epoch - 1)
            spe = int(post.get("steps_per_epoch", 0) or 0)
            ep1 = spe * t1 if spe > 0 else epoch_t.get(1, epoch_t[min(epoch_t)] * min(epoch_t))
            fields["estimated_remainning_time_sec"] = float(ep1 * remaining)
            fields["current_epoch"] = last_epoch
            fields["remainning_epochs"] = remaining
        if rows:
            start = datetime.strptime(rows[0]["start_time"], TIME_FMT)
            end = datetime.strptime(rows[-1]["start_time"], TIME_FMT)
            elapsed = (end - start).total_seconds() + float(rows[-1]["epoch_time_sec"])
            running = sum(float(r["epoch_time_sec"]) for r in rows)
            fields.update(running_time_sec=running, waiting_time_sec=max(0.0, elapsed - running),
                          gpu_time_sec=sum(float(r["epoch_time_sec"]) * int(r["workers"]) for r in rows),
                          elasped_time_sec=elapsed)
        for k, v in st.items():
            fields[f"step_time_sec.{k}"] = v
        for k, v in epoch_t.items():
            fields[f"epoch_time_sec.{k}"] = v
        for k, v in sp.items():
            fields[f"speedup.{k}"] = v
        for k, v in eff.items():
            fields[f"efficiency.{k}"] = v
        self.store.update_job_info(cat, job, fields)
        if self.update_category_base:
            self._refresh_base(cat, step_t, post, epoch_t)
        return fields

    def _refresh_base(self, cat: str, step_t: dict[int, float], prior: dict,
                      epoch_t: dict[int, float] | None = None) -> None:
        """Fold this job's measured step times into the category's base record, so the next
        job of the category starts from measured history.  Worker
        counts measured by earlier jobs of the category are kept."""
        try:
            base = self.store.find_job_info(cat, cat)
        except NotFound:
            return
        merged = {int(k): float(v) for k, v in (base.get("measured_step_time") or {}).items()}
        merged.update(step_t)
        sp, st = estimate_tables(merged, prior)
        if not sp:
            return
        fields: dict = {"info_source": "measured", "measured_step_time": {str(k): v for k, v in merged.items()}}
        for k, v in st.items():
            fields[f"step_time_sec.{k}"] = v
        for k, v in sp.items():
            fields[f"speedup.{k}"] = v
            fields[f"efficiency.{k}"] = v / int(k) if int(k) else 0.0
        spe = int(prior.get("steps_per_epoch", 0) or 0)
        if spe > 0:
            for k, v in st.items():
                if int(k):
                    fields[f"epoch_time_sec.{k}"] = spe / int(k) * v
        else:  # no declared epoch length: the measured epoch rows (reference semantics)
            ep = dict(epoch_t or {})
            if ep and 1 not in ep:
                k0 = min(ep)
                ep[1] = ep[k0] * float(sp[str(k0)])
            for k, v in ep.items():
                fields[f"epoch_time_sec.{k}"] = v
        self.store.update_job_info(cat, cat, fields)


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
