"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer.

The render plan (csrc/plan.h) and the NumPy stream primitives (csrc/nprng.h)
run on the host in every batch (msg_render_batch plans on a host thread pool)
and on the device; the render digest's host reference (csrc/digest.h) is the
check of msg_digest.  csrc/host_san.cpp compiles their host entry points
(csrc/host_abi.inc and digest.h, the same sources the product library
includes) with ``g++ -fsanitize=address,undefined -fno-sanitize-recover=undefined``
into a host-only library, and this test runs tests/test_plan_host.py,
tests/test_rng_host.py and the host tests of tests/test_digest.py against it in
a child interpreter with the sanitizer runtimes preloaded.  Any ASan report or
UBSan runtime error fails the run.
"""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "audio-suite_amd", "csrc")


def _runtime(name):
    p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_plan_and_rng_under_asan_ubsan(tmp_path):
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("sanitizer runtimes not installed")
    lib = str(tmp_path / "libmsgpu_hostsan.so")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fPIC", "-shared", "-fno-omit-frame-pointer",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-Wall", "-Werror",
                    "-Wno-unused-function", "-o", lib, os.path.join(CSRC, "host_san.cpp")], check=True)
    env = dict(os.environ, MSGPU_LIB=lib, MSGPU_HOST_ONLY="1", LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_plan_host.py"), os.path.join(REPO, "tests", "test_rng_host.py"),
                        os.path.join(REPO, "tests", "test_digest.py") + "::test_host_digest_matches_definition",
                        os.path.join(REPO, "tests", "test_digest.py") + "::test_digest_sees_bits_and_positions"],
                       capture_output=True, text=True, env=env, cwd=REPO, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert " passed" in out


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_pool_under_tsan(tmp_path):
    """The host pool (csrc/host_pool.h) under ThreadSanitizer: four caller threads
    submit jobs concurrently, as bench.py's per-context enqueue threads do."""
    tsan = _runtime("libtsan.so")
    if not tsan:
        pytest.skip("ThreadSanitizer runtime not installed")
    exe = str(tmp_path / "host_pool_tsan")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-Wall", "-Werror", "-I", CSRC,
                    "-o", exe, os.path.join(REPO, "tests", "host_pool_tsan.cpp"), "-pthread"], check=True)
    env = dict(os.environ, MSGPU_HOST_THREADS="6", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "WARNING: ThreadSanitizer" not in out, out[-4000:]
    assert "bad 0" in out


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_tap_sort_matches_std_sort(tmp_path):
    """The ER merge's stable radix sort of the taps by offset (csrc/tap_sort.h)
    gives std::sort's order of the packed (offset, tap index) keys -- equal
    offsets in tap order, as MS:416-420 adds them -- under ASan + UBSan."""
    exe = str(tmp_path / "tap_sort_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-Wall", "-Werror", "-I", CSRC, "-o", exe, os.path.join(REPO, "tests", "tap_sort_check.cpp")],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "bad 0" in out, out[-4000:]
