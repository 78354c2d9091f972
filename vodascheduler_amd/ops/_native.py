"""Loader for the native extensions.

GPU tensors are ALWAYS served by the hand-written HIP kernels in ``_vodahip``; if the
extension is missing or fails to load, GPU ops raise instead of silently falling back to
PyTorch.  CPU tensors use the explicit PyTorch reference implementations kept next to
each op (they are the fp32 references the GPU tests compare against).
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

_lock = threading.Lock()
_hip = None
_hip_err: Exception | None = None
_core = None
_core_err: Exception | None = None

DT_F32, DT_BF16, DT_F16 = 0, 1, 2
_DT = {torch.float32: DT_F32, torch.bfloat16: DT_BF16, torch.float16: DT_F16}
# RCCL-only integer codes (see csrc/hip/comm.cpp)
_COMM_DT = {**_DT, torch.int32: 3, torch.int64: 4, torch.uint8: 5}


def dtype_code(dt: torch.dtype) -> int:
    try:
        return _DT[dt]
    except KeyError as e:
        raise TypeError(f"unsupported dtype {dt}; expected float32/bfloat16/float16") from e


def comm_dtype_code(dt: torch.dtype) -> int:
    try:
        return _COMM_DT[dt]
    except KeyError as e:
        raise TypeError(f"unsupported collective dtype {dt}") from e


def _maybe_build(name: str) -> None:
    if os.environ.get("VODA_AUTOBUILD", "0") != "1":
        return
    from .. import _build

    (_build.build_hip if name == "_vodahip" else _build.build_core)()


def hip():
    """Return the loaded ``_vodahip`` module or raise a clear error."""
    global _hip, _hip_err
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None and _hip_err is None:
            try:
                _maybe_build("_vodahip")
                _hip = importlib.import_module("vodascheduler_amd._vodahip")
            except Exception as e:  # pragma: no cover - exercised only when missing
                _hip_err = e
    if _hip is None:
        raise RuntimeError(
            "vodascheduler_amd native HIP extension (_vodahip) is not available: "
            f"{_hip_err!r}. Build it with `python -m vodascheduler_amd._build`."
        )
    return _hip


def hip_available() -> bool:
    try:
        hip()
        return True
    except RuntimeError:
        return False


def core():
    """Return the loaded host-side ``_vodacore`` module (Hungarian, native policies)."""
    global _core, _core_err
    if _core is not None:
        return _core
    with _lock:
        if _core is None and _core_err is None:
            try:
                _maybe_build("_vodacore")
                _core = importlib.import_module("vodascheduler_amd._vodacore")
            except Exception as e:  # pragma: no cover
                _core_err = e
    if _core is None:
        raise RuntimeError(
            "vodascheduler_amd native host extension (_vodacore) is not available: "
            f"{_core_err!r}. Build it with `python -m vodascheduler_amd._build`."
        )
    return _core


def core_available() -> bool:
    try:
        core()
        return True
    except RuntimeError:
        return False


def stream_of(t: torch.Tensor) -> int:
    """Raw hipStream_t of the current stream on ``t``'s device."""
    return torch.cuda.current_stream(t.device).cuda_stream


def check_gpu_tensor(t: torch.Tensor, name: str, *, align: int = 16, contiguous: bool = True) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.data_ptr() % align != 0:
        raise ValueError(f"{name} must be {align}-byte aligned (got ptr % {align} = {t.data_ptr() % align})")


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()
