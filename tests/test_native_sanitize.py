"""Host native core under AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer
(SURVEY.md §5.2).

Builds csrc/host/tests/selftest.cpp together with the sources of the ``_vodacore``
extension (Hungarian assignment, FfDL dynamic program) as a standalone executable with
``-fsanitize=address,undefined`` and runs it: random problems checked against brute force,
error paths checked to throw.  Any sanitizer report fails the test (non-recoverable UBSan,
ASan aborts by default)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "csrc", "host")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_core_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "voda_selftest")
    srcs = [os.path.join(HOST, "tests", "selftest.cpp"), os.path.join(HOST, "hungarian.cpp"),
            os.path.join(HOST, "ffdl.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{HOST}", *srcs, "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "selftest OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_core_concurrent_calls_clean_under_tsan(tmp_path):
    """The bindings release the GIL, so placement / allocator threads can run the Hungarian
    solver and the FfDL DP at the same time: 8 threads under ThreadSanitizer must agree with
    the serial answers and produce no race report."""
    exe = str(tmp_path / "voda_selftest_tsan")
    srcs = [os.path.join(HOST, "tests", "selftest.cpp"), os.path.join(HOST, "hungarian.cpp"),
            os.path.join(HOST, "ffdl.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=thread", "-pthread",
           f"-I{HOST}", *srcs, "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([exe, "threads"], capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0 and "unexpected memory mapping" in r.stderr:
        pytest.skip("ThreadSanitizer runtime cannot map its shadow memory on this kernel")
    assert r.returncode == 0 and "selftest OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]


def _build_comm_selftest(tmp_path, san: list[str]) -> str:
    hip_dir = os.path.join(ROOT, "csrc", "hip")
    exe = str(tmp_path / ("comm_selftest_" + "_".join(s.split("=")[-1].replace(",", "_") for s in san)))
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *san, "-pthread",
           f"-I{os.path.join(hip_dir, 'tests', 'mocks')}", f"-I{hip_dir}",
           os.path.join(hip_dir, "tests", "selftest_comm.cpp"), os.path.join(hip_dir, "comm.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    return exe


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_rccl_engine_state_machine_clean_under_asan_ubsan(tmp_path):
    """csrc/hip/comm.cpp (the RCCL communicator engine) against a fake non-blocking RCCL:
    init polling, in-progress enqueues, timeout-abort, and a watchdog abort while other
    threads enqueue / wait -- no use-after-free or UB (the round-1 engine freed the
    communicator under a waiting thread)."""
    exe = _build_comm_selftest(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "selftest OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_rccl_engine_concurrent_abort_clean_under_tsan(tmp_path):
    exe = _build_comm_selftest(tmp_path, ["-fsanitize=thread"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0 and "unexpected memory mapping" in r.stderr:
        pytest.skip("ThreadSanitizer runtime cannot map its shadow memory on this kernel")
    assert r.returncode == 0 and "selftest OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
