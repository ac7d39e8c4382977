"""The learners' f32 GEMM kernel choices on gfx950 (PyTorch TunableOp, read-only).

The DQN / DDQN / PPO updates run their Linear layers through torch (hipBLASLt by default). For the
fixed shapes of these learners (fc1 1,574 -> 1,024, fc2 1,024 -> 512 at the trainers' batch sizes,
forward and both backward products), timing every hipBLASLt and rocBLAS solution once and keeping
the fastest found faster kernels than the heuristic default: the best-of-6 DDQN training leg
62.1 / 61.7 -> 65.4 / 65.7 M env steps/s (profiles/r06/train_tunableop.jsonl, interleaved). The
choices are the committed results file (tuning/gemm_gfx950.csv, made by profiles/r06j/run.sh); here
it is only read — no tuning at run time, so every run picks the same kernels. The file's validator
lines (PyTorch / HIP / hipBLASLt / rocBLAS versions, the GPU arch) must match, else torch keeps its
defaults. MZ_GEMM_TUNING=0 or a caller-set PYTORCH_TUNABLEOP_* environment leaves torch alone.
"""
import os
import tempfile

import torch

_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "gemm_gfx950.csv")
_state = {"done": False, "active": False}


def enable(device=None):
    """Load the committed GEMM choices once per process (no-op off gfx950 / without the file)."""
    if _state["done"]:
        return _state["active"]
    _state["done"] = True
    if os.environ.get("MZ_GEMM_TUNING", "1") == "0" or any(
            k.startswith("PYTORCH_TUNABLEOP") for k in os.environ):
        return False
    if not torch.version.hip or not torch.cuda.is_available() or not os.path.exists(_FILE):
        return False
    if "gfx950" not in torch.cuda.get_device_properties(device).gcnArchName:
        return False
    import torch.cuda.tunable as T
    try:
        T.enable(True)
        T.tuning_enable(False)
        # (torch writes its in-memory results at exit: to a scratch file, never into the package)
        T.set_filename(os.path.join(tempfile.gettempdir(), f"mazerl_tunableop_{os.getpid()}.csv"))
        ok = bool(T.read_file(_FILE))
    except RuntimeError:  # an unreadable file or a torch without TunableOp: torch's defaults
        ok = False
    if not ok:
        T.enable(False)
    _state["active"] = ok
    return ok
