"""Per-epoch CSV metrics logger (reference examples/py/tensorflow2/callbacks.py:18-158,
``MetricsCSVLogger`` + ``set_logger_params``): rank 0 appends one row per epoch to
``<metrics_dir>/<job>.csv``; the metrics collector turns these rows into per-worker-count
step/epoch times, speedup and remaining-time estimates.  The epoch counter is restored from
an existing CSV so a preempted job resumes where it stopped."""
from __future__ import annotations

import csv
import os
from datetime import datetime

FIELDS = ["epoch", "start_time", "epoch_time_sec", "step_time_sec", "steps", "workers", "local_batch_size",
          "global_batch_size", "total_epochs", "loss", "samples_per_sec", "acc", "val_loss", "val_acc"]
TIME_FMT = "%Y-%m-%d %H:%M:%S.%f"


class MetricsCSVLogger:
    def __init__(self, metrics_dir: str | None, job: str, total_epochs: int, local_batch_size: int):
        self.path = os.path.join(metrics_dir, f"{job}.csv") if metrics_dir else None
        self.total_epochs = total_epochs
        self.local_batch_size = local_batch_size
        self.workers = 1
        if self.path:
            os.makedirs(metrics_dir, exist_ok=True)

    def set_params(self, workers: int) -> None:
        self.workers = workers

    def restored_epoch(self) -> int:
        """Number of epochs already logged (resume point)."""
        if not self.path or not os.path.exists(self.path):
            return 0
        with open(self.path) as f:
            rows = list(csv.DictReader(f))
        return int(rows[-1]["epoch"]) + 1 if rows else 0

    def log_epoch(self, epoch: int, start_time: float, epoch_time: float, steps: int, loss: float | None,
                  workers: int | None = None, acc: float | None = None, val_loss: float | None = None,
                  val_acc: float | None = None) -> dict:
        """One row; ``loss`` / ``acc`` are the epoch's training metrics averaged over the
        workers, ``val_loss`` / ``val_acc`` the eval pass (Keras ``val_*`` names)."""
        w = workers or self.workers
        row = {
            "epoch": epoch,
            "start_time": datetime.fromtimestamp(start_time).strftime(TIME_FMT),
            "epoch_time_sec": round(epoch_time, 6),
            "step_time_sec": round(epoch_time / max(steps, 1), 6),
            "steps": steps,
            "workers": w,
            "local_batch_size": self.local_batch_size,
            "global_batch_size": self.local_batch_size * w,
            "total_epochs": self.total_epochs,
            "loss": "" if loss is None else round(float(loss), 6),
            "samples_per_sec": round(steps * self.local_batch_size * w / max(epoch_time, 1e-9), 3),
            "acc": "" if acc is None else round(float(acc), 6),
            "val_loss": "" if val_loss is None else round(float(val_loss), 6),
            "val_acc": "" if val_acc is None else round(float(val_acc), 6),
        }
        if self.path:
            new = not os.path.exists(self.path)
            with open(self.path, "a", newline="") as f:
                wr = csv.DictWriter(f, fieldnames=FIELDS)
                if new:
                    wr.writeheader()
                wr.writerow(row)
        return row
