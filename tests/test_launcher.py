"""bench.py's own launcher (launch_ranks): `python bench.py --gpus N` with no
WORLD_SIZE starts N rank processes itself, before anything touches the GPU.

CPU only: a stub rank stands in for bench.py's rank body.  It reads the
torch.distributed env contract, joins a gloo group (so MASTER_ADDR/PORT and
the ranks' numbering are checked by torch itself), and exits as the test
asks.  Covered: the fan-out, rank 0's line on stdout (and only it), a failing
rank's exit code, the other ranks stopped when one fails (a hung peer too),
and that the launcher's module imports no torch (the parent must not touch
the GPU: it only forks the ranks).
"""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = textwrap.dedent(
    """
    import json, os, sys, time
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    plan = json.loads(os.environ.get("STUB_PLAN", "{}")).get(str(rank), "ok")
    if plan.startswith("fail:"):
        sys.exit(int(plan[5:]))
    if plan == "hang":
        time.sleep(3600)  # never joins the group
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    if plan.startswith("fail_late:"):
        time.sleep(0.5)
        sys.exit(int(plan[10:]))  # inside the group: the others block in the collective below
    t = torch.tensor([rank + 1])
    dist.all_reduce(t)
    dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"world": world, "sum": int(t), "argv": sys.argv[1:],
                          "addr": os.environ["MASTER_ADDR"], "local": os.environ["LOCAL_RANK"]}))
    else:
        print("peer", rank, "stdout")  # must not reach the launcher's stdout
    """
)


def _run(tmp_path, n, plan=None, argv=("--steps", "3")):
    stub = tmp_path / "stub_rank.py"
    stub.write_text(STUB)
    code = textwrap.dedent(
        f"""
        import sys
        sys.path.insert(0, {ROOT!r})
        import bench
        raise SystemExit(bench.launch_ranks({n}, {list(argv)!r}, rank_cmd=[sys.executable, {str(stub)!r}],
                                            grace_s=2.0))
        """
    )
    env = dict(os.environ, STUB_PLAN=json.dumps(plan or {}))
    env.pop("WORLD_SIZE", None)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    return r, time.monotonic() - t0


@pytest.mark.parametrize("n", [2, 3, 8])  # 8: the driver's scaling run (config 4)
def test_fan_out_and_rank0_line(tmp_path, n):
    r, _ = _run(tmp_path, n)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # rank 0's line only; the peers' stdout went to stderr
    d = json.loads(lines[0])
    assert d["world"] == n and d["sum"] == n * (n + 1) // 2  # every rank joined the one gloo group
    assert d["argv"] == ["--steps", "3"] and d["addr"] == "127.0.0.1" and d["local"] == "0"
    assert "peer 1 stdout" in r.stderr


def test_failing_rank_fails_the_job(tmp_path):
    r, _ = _run(tmp_path, 2, {"1": "fail:3"})
    assert r.returncode == 3
    assert "rank 1 exited with 3" in r.stderr


def test_peers_of_a_failed_rank_are_stopped(tmp_path):
    # rank 1 fails inside the group, where rank 0 waits in a collective forever:
    # the launcher ends rank 0 and returns rank 1's code
    r, dt = _run(tmp_path, 2, {"1": "fail_late:5"})
    assert r.returncode == 5, r.stderr[-2000:]
    assert dt < 60


def test_hung_rank_is_killed_when_another_fails(tmp_path):
    # rank 0 sleeps outside the group, rank 1 waits for it in init, rank 2 fails
    r, dt = _run(tmp_path, 3, {"0": "hang", "2": "fail:4"})
    assert r.returncode == 4, r.stderr[-2000:]
    assert dt < 60


def test_launcher_module_does_not_import_torch():
    code = f"import sys; sys.path.insert(0, {ROOT!r}); import bench; print('torch' in sys.modules)"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "False", r.stdout + r.stderr


def test_main_routes_to_the_launcher_without_world_size(monkeypatch):
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", lambda n, argv: calls.append((n, argv)) or 7)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "9"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7 and calls == [(4, ["--gpus", "4", "--steps", "9"])]
