"""CPU checks of the drop-in boundary: libmazerl.so builds for gfx950, loads, and exports every
entry point include/mazerl.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mazerl.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(mz_\w+)\s*\(", txt, re.M)))


def test_header_declares_api():
    names = declared()
    for f in ("mz_create", "mz_destroy", "mz_load_mazes", "mz_generate", "mz_reset_all",
              "mz_reset_list", "mz_step", "mz_step_act", "mz_direction_mask", "mz_act",
              "mz_expand_window", "mz_query", "mz_get_grid", "mz_last_error"):
        assert f in names


def test_library_exports_every_declared_symbol():
    from mazerl import _build, _native
    lib = _build.build()
    L = ctypes.CDLL(lib)
    for f in declared():
        assert hasattr(L, f), f
    assert set(_native.EXPORTS) == set(declared())
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", lib],
                         capture_output=True, text=True)
    # the embedded device code object targets gfx950
    blob = open(lib, "rb").read()
    assert b"gfx950" in blob


def test_header_compiles_as_c():
    if subprocess.run(["which", "gcc"], capture_output=True).returncode:
        pytest.skip("no gcc")
    src = '#include "mazerl.h"\nint main(void){mz_config c; (void)c; return 0;}\n'
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-x", "c", "-", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "include")], input=src, text=True,
                       capture_output=True)
    assert r.returncode == 0, r.stderr
