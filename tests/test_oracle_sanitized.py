"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5,
"sanitizers on host code"): oracle/asp_oracle.c built with -fsanitize=address,undefined
(``make -C oracle san``), then the golden-vector checks of the oracle
(tests/test_oracle_golden.py, the cube restatement's tests/test_cube_oracle.py, the
raw-fp64 goldens tests/test_fp64_golden.py) run in a child Python with the sanitizer
runtimes preloaded and that build loaded through ASP_ORACLE_LIB.  Any out-of-bounds
access, use-after-free or undefined behaviour aborts the child (halt on the first
report); the same fixtures must still pass bit for bit."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import REPO

ORACLE = os.path.join(REPO, "oracle")


def _runtime(name):
    cc = shutil.which("gcc")
    if not cc:
        return None
    p = subprocess.run([cc, f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_golden_checks_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not (asan and ubsan):
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.run(["make", "-s", "-C", ORACLE, "san"], check=True)
    lib = os.path.join(ORACLE, "_san", "liboracle_san.so")
    env = dict(os.environ,
               LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               ASP_ORACLE_LIB=lib)
    files = [os.path.join(REPO, "tests", f) for f in
             ("test_oracle_golden.py", "test_cube_oracle.py", "test_fp64_golden.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu",
                        "-p", "no:cacheprovider", *files],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " passed" in out
