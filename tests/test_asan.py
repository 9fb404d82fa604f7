"""SURVEY §5 (race/memory checking): the library's host C++ under AddressSanitizer.

`make -C leak-det-gnn_amd asan` builds lib/asan/libleakgnn.so with -fsanitize=address on the
host side only (argument and workspace checks, lg_rcm_order, the node-table and reduce-batch
host code; the gfx950 code objects are unchanged and GPU ASan is not available on this pool).
tests/test_host.py then runs against it in a child process with clang's ASan runtime
preloaded.  CPU only."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

from conftest import PKG, REPO

ASAN_LIB = PKG / "lib" / "asan" / "libleakgnn.so"


def _asan_runtime() -> Path | None:
    for p in sorted(Path("/opt/rocm/lib/llvm/lib/clang").glob("*/lib/linux/libclang_rt.asan-x86_64.so")):
        return p
    return None


@pytest.fixture(scope="module")
def asan_lib():
    # make's own dependency check: a no-op when the build is newer than every source
    r = subprocess.run(["make", "-s", "-C", str(PKG), "asan"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("no clang ASan runtime in this image")
    return rt


def test_asan_build_is_instrumented(asan_lib):
    out = subprocess.run(["nm", "-D", "--undefined-only", str(ASAN_LIB)], capture_output=True, text=True).stdout
    assert "__asan_report_load" in out or "__asan_load" in out, "host code is not ASan-instrumented"


def test_host_suite_under_asan(asan_lib):
    env = dict(os.environ, LD_PRELOAD=str(asan_lib), LEAKGNN_LIB=str(ASAN_LIB),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        str(REPO / "tests" / "test_host.py")], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:] + r.stderr[-3000:])
    assert "passed" in r.stdout
