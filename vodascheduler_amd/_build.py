"""Native build driver for vodascheduler_amd.

Two in-tree extension modules are produced (no setuptools, no hipify step):

* ``_vodacore``  — host-only C++ (g++): Kuhn-Munkres assignment used by the placement
  manager (replaces the external ``github.com/heyfey/munkres`` Go dependency,
  reference ``pkg/placement/placement_manager.go:10,505-507``) and the native
  allocation-policy kernels (FfDL dynamic program).
* ``_vodahip``   — HIP/CDNA4 (hipcc ``--offload-arch=gfx950``): fused optimizers,
  gradient-bucket pack/scale/cast, LayerNorm, masked softmax, MFMA attention and the
  RCCL communicator engine (replaces Horovod core + NCCL used implicitly by the
  reference workloads).

The HIP module links the ``libamdhip64``/``librccl`` that ship inside the torch wheel
(same SONAMEs as /opt/rocm, so one runtime is loaded per process) and is rebuilt only
when a source hash changes.  Run ``python -m vodascheduler_amd._build`` or call
:func:`build_all`.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC = REPO_DIR / "csrc"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
GPU_ARCH = os.environ.get("VODA_GPU_ARCH", "gfx950")


def _python_includes() -> list[str]:
    import pybind11

    incs = [sysconfig.get_paths()["include"], pybind11.get_include()]
    return [f"-I{p}" for p in incs]


def _torch_lib_dir() -> Path:
    # Locate torch/lib without importing torch (importing is slow on a cold image).
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        raise RuntimeError("torch is required to link the HIP extension")
    return Path(spec.origin).parent / "lib"


def _hash_sources(paths: list[Path], extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def _up_to_date(out: Path, digest: str) -> bool:
    stamp = out.with_suffix(out.suffix + ".hash")
    return out.exists() and stamp.exists() and stamp.read_text().strip() == digest


def _write_stamp(out: Path, digest: str) -> None:
    out.with_suffix(out.suffix + ".hash").write_text(digest + "\n")


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError(f"native build failed: {' '.join(cmd[:3])} ... (exit {r.returncode})")
    elif verbose and r.stdout.strip():
        print(r.stdout)


def build_core(verbose: bool = False, force: bool = False) -> Path:
    """Build the host-only C++ module ``_vodacore``."""
    srcs = sorted((CSRC / "host").glob("*.cpp"))
    hdrs = sorted((CSRC / "host").glob("*.h"))
    out = PKG_DIR / f"_vodacore{EXT_SUFFIX}"
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-fvisibility=hidden"]
    digest = _hash_sources(srcs + hdrs, " ".join([cxx] + flags))
    if not force and _up_to_date(out, digest):
        return out
    cmd = [cxx, *flags, *_python_includes(), *map(str, srcs), "-o", str(out)]
    _run(cmd, verbose)
    _write_stamp(out, digest)
    return out


def hip_compile_flags() -> list[str]:
    return [
        f"--offload-arch={GPU_ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-ffp-contract=fast",
        "-munsafe-fp-atomics",
        "-fvisibility=hidden",
        "-Wno-unused-result",
        # extra -D options for A/B builds of a layout constant (e.g. -DSX_KC_PITCH=112)
        *os.environ.get("VODA_HIP_DEFINES", "").split(),
    ]


def build_hip(verbose: bool = False, force: bool = False) -> Path:
    """Build the HIP/CDNA4 module ``_vodahip`` (cross-compiles on a CPU-only host)."""
    hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    srcs = sorted((CSRC / "hip").glob("*.hip")) + sorted((CSRC / "hip").glob("*.cpp"))
    hdrs = sorted((CSRC / "hip").glob("*.h"))
    out = PKG_DIR / f"_vodahip{EXT_SUFFIX}"
    tlib = _torch_lib_dir()
    flags = hip_compile_flags()
    digest = _hash_sources(srcs + hdrs, " ".join([hipcc] + flags + [str(tlib)]))
    if not force and _up_to_date(out, digest):
        return out
    objdir = REPO_DIR / "build" / "hip"
    objdir.mkdir(parents=True, exist_ok=True)
    objs = []
    procs = []
    for s in srcs:
        o = objdir / (s.stem + ".o")
        objs.append(o)
        lang = ["-x", "hip"] if s.suffix in (".hip", ".cpp") else []
        cmd = [hipcc, *flags, *lang, f"-I{ROCM / 'include'}", f"-I{CSRC / 'hip'}",
               *_python_includes(), "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    failed = False
    for cmd, p in procs:
        outp, _ = p.communicate()
        if p.returncode != 0:
            failed = True
            sys.stderr.write(f"$ {' '.join(cmd)}\n{outp}\n")
    if failed:
        raise RuntimeError("HIP extension compile failed")
    # Link against the HIP runtime + RCCL + hipBLASLt bundled with torch (SONAME
    # libamdhip64.so.7 / librccl.so.1 / libhipblaslt.so.1 — the copies torch already loaded
    # are reused).
    link = [hipcc, f"--offload-arch={GPU_ARCH}", "-shared", "-fPIC", *map(str, objs),
            f"-L{tlib}", "-lamdhip64", "-lrccl", "-lhipblaslt", f"-Wl,-rpath,{tlib}", "-o", str(out)]
    _run(link, verbose)
    _write_stamp(out, digest)
    return out


def build_all(verbose: bool = False, force: bool = False) -> list[Path]:
    return [build_core(verbose, force), build_hip(verbose, force)]


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--only", choices=["core", "hip"], default=None)
    a = ap.parse_args()
    if a.only == "core":
        print(build_core(a.verbose, a.force))
    elif a.only == "hip":
        print(build_hip(a.verbose, a.force))
    else:
        for p in build_all(a.verbose, a.force):
            print(p)
