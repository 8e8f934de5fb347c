"""The library's host concurrency under the CPU sanitizers ("Build
the C++ shim under ASan/UBSan on CPU"; the reference has no concurrency at all).

tests/native/walk_harness.cpp drives the library's own headers -- WalkPool, Hub
and AbortGate (ambc_sync.h) and the multi-size walk's decisions (ambc_walkcore.h:
parallel walks, the two-phase decide, request-bit claims, per-thread request
buckets, parallel fills, breadth speculation, LZ4 shared across sizes, host-scored
methods) over a synthetic backend, its paths checked against a serial restatement
of the reference's loop -- built with -fsanitize=thread and, separately, with
-fsanitize=address,undefined, each run at 1, 4 and 10 pool threads (the
AMBC_MS_THREADS range the library runs: 1 here, 10 on the GPU box)."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

SRC = os.path.join(REPO, "tests", "native", "walk_harness.cpp")
FLAVOURS = {
    "tsan": ["-fsanitize=thread"],
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
}


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = {}
    d = tmp_path_factory.mktemp("native")
    for name, flags in FLAVOURS.items():
        exe = str(d / f"walk_harness_{name}")
        subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-pthread", "-Wall", "-Werror", *flags, "-o", exe, SRC],
                       check=True, capture_output=True, text=True)
        out[name] = exe
    return out


@pytest.mark.parametrize("flavour", sorted(FLAVOURS))
@pytest.mark.parametrize("threads", [1, 4, 10])
def test_host_concurrency_clean_under_sanitizer(harness, flavour, threads):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness[flavour], str(threads)], capture_output=True, text=True, timeout=300, env=env)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "WARNING: ThreadSanitizer" not in r.stderr, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
    assert f"walk_harness threads={threads}: ok (0 failures)" in r.stdout, tail
