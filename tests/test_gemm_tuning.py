"""The committed learner GEMM choices (mazerl.gemm_tuning): a well-formed TunableOp results file for
gfx950, read-only and never loaded off a gfx950 GPU."""
import os

import mazerl.gemm_tuning as G


def test_results_file_well_formed():
    assert os.path.exists(G._FILE)
    rows = [l.strip().split(",") for l in open(G._FILE) if l.strip()]
    val = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert val.get("GCN_ARCH_NAME", "").startswith("gfx950")
    gemms = [r for r in rows if r[0] != "Validator"]
    assert gemms and all(len(r) == 4 and float(r[3]) > 0 for r in gemms)
    # the learners' fc1 (1,574 -> 1,024) products are among the tuned shapes
    assert any("1574" in r[1] for r in gemms)


def test_enable_is_noop_without_gfx950(monkeypatch):
    import torch
    if torch.cuda.is_available():
        return
    monkeypatch.setitem(G._state, "done", False)
    assert G.enable() is False
