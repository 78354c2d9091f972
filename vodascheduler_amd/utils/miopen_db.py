"""Persistent MIOpen tuning state shared by every worker of a node.

Convnets run MIOpen in exhaustive-find mode (``cudnn.benchmark``): the first time a worker
meets a convolution shape MIOpen compiles and times every applicable solver, which for
ResNet-50 at batch 256 costs minutes per fresh process. The results live in two stores:

* the user find-db / perf-db -- small text/sqlite records "shape -> best solver"; and
* the compiled-kernel cache -- code objects of the chosen solvers.

Both default to the user's home, which on a scheduler node is per-container and often
ephemeral. ``configure()`` points them at one directory (``VODA_MIOPEN_DIR``, default
``<install>/var/miopen``) so every pool worker, every restart and every job after the first
reuses them; the node agent and the bench call it before any GPU work. The find-db part is
plain tuning data and can be committed/shipped with a deployment; the kernel cache is
machine code for this exact ROCm build and stays local.
"""
from __future__ import annotations

import os

_ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "var", "miopen")


def miopen_dir() -> str:
    return os.environ.get("VODA_MIOPEN_DIR", _ROOT)


def configure(root: str | None = None) -> str | None:
    """Set ``MIOPEN_USER_DB_PATH`` / ``MIOPEN_CUSTOM_CACHE_DIR`` (unless the user already did).
    Must run before the first convolution of the process. Returns the directory used, or
    None when it is not writable (MIOpen then keeps its defaults)."""
    root = root or miopen_dir()
    try:
        os.makedirs(os.path.join(root, "db"), exist_ok=True)
        os.makedirs(os.path.join(root, "kcache"), exist_ok=True)
        if not os.access(root, os.W_OK):
            return None
    except OSError:
        return None
    os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(root, "db"))
    os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(root, "kcache"))
    return root
