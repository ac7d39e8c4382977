"""Build libmazerl.so (HIP, gfx950) in-tree: mazerl/_lib/libmazerl.so.

hipcc cross-compiles for gfx950 without a GPU. -ffp-contract=off keeps every double reward /
score / max_steps expression rounded like CPython (the kernels also use explicit __d*_rn ops).
Each source compiles to its own object (in parallel), so a file can carry extra flags:
mz_qnet.hip (bf16 acting stem, no double / NaN semantics involved) is built with
-ffinite-math-only, which drops the NaN canonicalisation fmaxf puts on every MFMA result;
mz_qact.hip with MFMA results in VGPRs (-amdgpu-mfma-vgpr-form): k_qconv's accumulators then need
no v_accvgpr_read before its VALU epilogue (32 of the 445 VALU instructions of its chunk loop);
the other acting kernels compile to the same registers either way.
"""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIBDIR, "libmazerl.so")
SOURCES = ["mz_env.hip", "mz_api.hip", "mz_difficulty.hip", "mz_qnet.hip", "mz_metrics.hip",
           "mz_stem.hip", "mz_optim.hip", "mz_trainer.hip", "mz_ppo.hip",
           "mz_qact.hip", "mz_mcclendon.hip", "mz_screen.hip"]
EXTRA_FLAGS = {"mz_qnet.hip": ["-ffinite-math-only"],
               "mz_qact.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}
BASE_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall"]
DEPS = SOURCES + ["mz_common.h", "mz_kernels.h", "mz_build.inc.h", "mz_pygen.inc.h",
                  "mz_mcclendon.h", "mz_learner.h", "mz_screen.h"]
HEADER = os.path.join(os.path.dirname(ROOT), "include", "mazerl.h")


def hipcc():
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in DEPS) or os.path.getmtime(HEADER) > t


def build(force=False, verbose=False):
    if not force and not stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(LIBDIR, "obj")
    os.makedirs(objdir, exist_ok=True)

    def compile_one(f):
        obj = os.path.join(objdir, f + ".o")
        cmd = [hipcc()] + BASE_FLAGS + EXTRA_FLAGS.get(f, []) + ["-c", "-o", obj,
                                                                os.path.join(CSRC, f)]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB + ".tmp"
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
