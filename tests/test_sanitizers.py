"""ASan + UBSan over the host code (SURVEY §5 "race detection/sanitizers": ASan/UBSan on the CPU
restatement). tests/sanitize/Makefile builds two drivers with -fsanitize=address,undefined
-fno-sanitize-recover=all: the CPU oracle under a driver that calls every entry point over the
parity configurations, and the product's host C++ McClendon restatement (csrc/mz_difficulty.hip)
over oracle-generated perfect, cyclic and degenerate mazes. Any sanitizer report aborts the
driver with a non-zero status. (GPU AddressSanitizer / XNACK runs are not available on the GPU
pool; the device code is covered by the parity tests.)"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "sanitize")


@pytest.fixture(scope="module")
def built():
    if shutil.which("gcc") is None or shutil.which("g++") is None or shutil.which("make") is None:
        pytest.skip("gcc / g++ / make not available")
    r = subprocess.run(["make", "-s", "-C", SAN, "all"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(SAN, "_build")


@pytest.mark.parametrize("driver", ["san_oracle", "san_difficulty"])
def test_host_code_is_sanitizer_clean(built, driver):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(built, driver)], capture_output=True, text=True, env=env,
                       timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
    assert f"{driver} ok" in r.stdout
