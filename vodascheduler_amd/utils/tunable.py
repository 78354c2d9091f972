"""Pre-tuned library GEMM solutions for the reference-precision (fp32) path.

PyTorch-ROCm's TunableOp times every hipBLASLt solution of a GEMM shape and keeps the
fastest; the first use of a shape costs seconds.  The fp32 GEMMs of the bench workloads
(BERT-base, ResNet-50's 1x1 convolutions on the GEMM path) were tuned once on an MI355X and
the results ship in ``var/tunableop/fp32.csv`` (a plain CSV: "op, shape, solution, ms" rows
behind validator rows for the PyTorch / HIP / hipBLASLt versions and the GPU arch -- a file
from another software stack is ignored by PyTorch).  Workers load it with tuning OFF: a
listed shape runs its tuned solution, any other shape the library default; nothing is timed
at run time.  Measured (same box, ``profiles/r4/tunableop_ab.jsonl``): BERT-base fp32 step
39.42 -> 36.88 ms, ResNet-50 fp32 73.89 -> 70.46 ms; the bf16 results (``bf16.csv``) are worth
~1 % on the bf16-amp path.

``VODA_TUNABLEOP=0`` disables it (A/B); ``VODA_TUNABLEOP_TUNE=1`` tunes new shapes and
writes them back (how the file is produced: ``benchmarks/gpu_tunableop.sh``).
"""
from __future__ import annotations

import os

_ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "var", "tunableop")
_DONE: dict[str, bool] = {}


def results_path(precision: str) -> str:
    return os.path.join(os.environ.get("VODA_TUNABLEOP_DIR", _ROOT), f"{precision}.csv")


def configure(precision: str = "fp32") -> bool:
    """Enable TunableOp with the shipped results of ``precision`` (once per process; the
    results of several precisions can be loaded side by side -- entries are keyed by the
    GEMM's dtype and shape).  Returns True when tuned solutions are in use."""
    if precision in _DONE:
        return _DONE[precision]
    ok = False
    path = results_path(precision)
    tune = os.environ.get("VODA_TUNABLEOP_TUNE", "0") == "1"
    if os.environ.get("VODA_TUNABLEOP", "1") != "0" and (os.path.exists(path) or tune):
        import torch

        t = torch.cuda.tunable
        if tune:
            t.set_filename(path, insert_device_ordinal=False)
        else:
            # results written at exit go to a per-process scratch file, never over the shipped one
            t.set_filename(f"/tmp/voda_tunableop_{os.getpid()}.csv", insert_device_ordinal=False)
        t.enable(True)
        t.tuning_enable(tune)
        if os.path.exists(path):
            ok = bool(t.read_file(path))
        ok = ok or tune
    _DONE[precision] = ok
    return ok


def status() -> dict:
    import torch

    t = torch.cuda.tunable
    return {"enabled": bool(t.is_enabled()), "tuning": bool(t.tuning_is_enabled()),
            "entries": len(t.get_results()) if t.is_enabled() else 0}  # ((op, shape, solution, ms), ...)
