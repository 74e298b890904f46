"""Host code under AddressSanitizer + UBSan (VERDICT r3 hygiene): `make asan`
builds librvx's file/text parsers (api_hnswio.cpp, api_io.cpp, api_gnn.cpp + json.hpp,
runtime.cpp; host side only) and the whole oracle with -fsanitize=address,undefined
against clang's runtime. This test re-runs the CPU tests that drive those paths —
truncated / corrupt hnsw_rs dumps, feature files and layer JSON (test_parsers_fuzz.py),
the formats and golden fixtures, the oracle's known-answer and libm checks — in a child
Python with that runtime preloaded; any sanitizer report fails the child (exit 66)."""
import glob
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "build", "asan", "librvx_asan.so")
ORC = os.path.join(ROOT, "oracle", "_asan", "liboracle_asan.so")
RT = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(ORC) and RT),
                    reason="sanitizer build absent (run `make asan`; __graft_entry__.build() does)")
def test_host_parsers_and_oracle_under_asan_ubsan():
    env = dict(os.environ, LD_PRELOAD=RT[-1], RVX_LIB=LIB, RVX_ORACLE_LIB=ORC,
               ASAN_OPTIONS="detect_leaks=0:exitcode=66:allocator_may_return_null=1:handle_segv=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=66", PYTHONDONTWRITEBYTECODE="1")
    tests = ["tests/test_parsers_fuzz.py", "tests/test_formats.py", "tests/test_golden.py",
             "tests/test_oracle_known_answers.py", "tests/test_libm.py::test_check_counts_wrong_device_outputs"]
    # pytest-timeout is optional: the subprocess timeout below bounds the run either way
    extra = ["--timeout", "600"] if importlib.util.find_spec("pytest_timeout") else []
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider"]
                       + extra + tests, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout[-6000:] + r.stderr[-6000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out
    assert r.returncode == 0, out
