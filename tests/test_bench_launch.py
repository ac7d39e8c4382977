"""bench.py's own multi-rank launch (`python3 bench.py --gpus N` with no torchrun): the decision is
made from argv + environment before anything touches the GPU, the N child environments carry
torchrun's variables, rank 0's JSON line reaches stdout, and a failing or hung rank stops them
all with a non-zero status. CPU only: the children here are small stand-in scripts."""
import ast
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_decision_from_argv_and_environment():
    assert bench.needs_launch(bench.parse(["--gpus", "8"]), {})
    assert bench.needs_launch(bench.parse(["--gpus", "2", "--steps", "5"]), {"PATH": "/bin"})
    assert not bench.needs_launch(bench.parse(["--gpus", "8"]), {"WORLD_SIZE": "8"})  # torchrun
    assert not bench.needs_launch(bench.parse([]), {})
    assert not bench.needs_launch(bench.parse(["--gpus", "1"]), {})


def test_launch_plan_gives_each_rank_torchruns_variables():
    plan = bench.launch_plan(4, {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 29511)
    assert len(plan) == 4
    for r, e in enumerate(plan):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["PATH"] == "/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert e["MZ_BENCH_LAUNCHER"] == "1"
    assert bench.launch_plan(2, {"MASTER_ADDR": "10.0.0.1"}, 1)[1]["MASTER_ADDR"] == "10.0.0.1"


def test_main_decides_before_importing_torch():
    """main() must start the ranks before `import torch` (nothing may initialise the GPU in the
    supervisor, and it must never exec)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    tree = ast.parse(src)
    main = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main")
    first_import = next(i for i, st in enumerate(main.body)
                        if isinstance(st, (ast.Import, ast.ImportFrom)))
    launch_at = next(i for i, st in enumerate(main.body)
                     if isinstance(st, ast.If) and "needs_launch" in ast.unparse(st.test))
    assert launch_at < first_import
    assert "os.exec" not in src and "execv" not in src


def _run_launcher(tmp_path, body, n, timeout=30.0):
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(body))
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.launch({n}, [], {timeout}, script={str(script)!r}))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=120, env=env)


def test_launch_relays_rank0_json_line(tmp_path):
    p = _run_launcher(tmp_path, """
        import json, os
        r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        print(f"[lib] rank {r} banner on stdout", flush=True)
        print(json.dumps({"rank": r, "world": w, "port": os.environ["MASTER_PORT"]}) if r == 0
              else f"rank {r} stdout", flush=True)
    """, 3)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1  # only rank 0's stdout is stdout
    rec = json.loads(lines[0])
    assert rec["rank"] == 0 and rec["world"] == 3 and int(rec["port"]) > 0
    assert "rank 1 stdout" in p.stderr and "rank 2 stdout" in p.stderr
    assert "[lib] rank 0 banner on stdout" in p.stderr  # rank 0's non-JSON lines go to stderr


def test_launch_stops_every_rank_when_one_fails(tmp_path):
    p = _run_launcher(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "2":
            sys.exit(3)
        time.sleep(60)  # the others would hang: the launcher must kill them
    """, 4)
    assert p.returncode == 3
    assert "a rank exited with 3" in p.stderr


def test_launch_deadline(tmp_path):
    p = _run_launcher(tmp_path, """
        import time
        time.sleep(60)
    """, 2, timeout=2.0)
    assert p.returncode == 124
    assert "deadline" in p.stderr


def test_supervisor_sigterm_stops_the_ranks(tmp_path):
    """An outer `timeout` signals only the supervisor's process group; the ranks run in sessions of
    their own, so the supervisor must kill them on SIGTERM."""
    import signal
    import time
    pidfile = tmp_path / "pids"
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import os, time
        with open({str(pidfile)!r}, "a") as f:
            f.write(str(os.getpid()) + "\\n")
        time.sleep(120)
    """))
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.launch(3, [], 600.0, script={str(script)!r}))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    sup = subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    t0 = time.monotonic()
    while time.monotonic() - t0 < 60:
        if pidfile.exists() and len(pidfile.read_text().split()) == 3:
            break
        time.sleep(0.1)
    pids = [int(x) for x in pidfile.read_text().split()]
    assert len(pids) == 3
    sup.send_signal(signal.SIGTERM)
    out, err = sup.communicate(timeout=60)
    assert sup.returncode == 128 + signal.SIGTERM, err
    assert "got signal" in err

    def alive(pid):
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            return False
        return True
    t0 = time.monotonic()
    while any(alive(p) for p in pids) and time.monotonic() - t0 < 10:
        time.sleep(0.1)
    assert not any(alive(p) for p in pids)
