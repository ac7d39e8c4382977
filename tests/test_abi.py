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


def test_difficulty_lds_limits_match_the_header():
    """mz_difficulty_batch's pitch limits as include/mazerl.h states them (odd pitches P > 91,
    toroidal P > 89), derived from the kernel's own LDS plan (the host function
    mz_mcclendon_lds(P, toroidal, &MM) in libmazerl.so; 160 KB of LDS per workgroup)."""
    from mazerl import _build
    L = ctypes.CDLL(_build.build())
    plan = L._Z16mz_mcclendon_ldsibPi
    plan.restype = ctypes.c_size_t
    plan.argtypes = [ctypes.c_int, ctypes.c_bool, ctypes.POINTER(ctypes.c_int)]
    mm = ctypes.c_int()

    def largest_fit(tor):
        fit = [P for P in range(5, 200, 2) if plan(P, tor, ctypes.byref(mm)) <= 160 * 1024]
        # monotone: every pitch up to the largest fitting one fits
        assert fit == list(range(5, fit[-1] + 1, 2))
        return fit[-1]

    txt = open(HEADER).read()
    m = re.search(r"odd pitches: P > (\d+); toroidal P > (\d+)", txt)
    assert m, "the header states the limits"
    assert largest_fit(False) == int(m.group(1))
    assert largest_fit(True) == int(m.group(2))
