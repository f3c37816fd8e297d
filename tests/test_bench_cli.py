"""bench.py's workload wiring (CPU: no GPU run): each --workload selects its
own step function, so a refactor cannot silently swap the timed path."""
import ast
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _main_body():
    tree = ast.parse(open(os.path.join(ROOT, "bench.py")).read())
    return next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main")


def test_vote_roi_branch_is_guarded_by_full():
    """The vote_roi step (step = None) must only be built when the workload is
    not the full pose step (a dangling `else` once attached it to the linemod
    branch and the default bench timed the vote alone)."""
    for node in ast.walk(_main_body()):
        if isinstance(node, ast.If):
            assigns_none = any(isinstance(s, ast.Assign) and any(getattr(t, "id", None) == "step" for t in s.targets)
                               and isinstance(s.value, ast.Constant) and s.value.value is None
                               for s in node.body + node.orelse)
            if assigns_none:
                src = ast.unparse(node.test)
                assert src == "not full", src
                assert not node.orelse


def test_workload_choices():
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'choices=["full", "vote_roi", "linemod"], default="full"' in src


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_cli_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_local_launch_plan():
    """`bench.py --gpus N` without a launcher starts N rank processes with the
    torch.distributed env: rank r on GPU r, one
    127.0.0.1 rendezvous, the same bench arguments."""
    b = _bench()
    argv = ["--gpus", "4", "--steps", "7", "--global-batch", "64"]
    plan = b.launch_plan(4, argv, {"KEEP": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 29555)
    assert len(plan) == 4
    for r, (cmd, env) in enumerate(plan):
        assert cmd[1].endswith("bench.py") and cmd[2:] == argv
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
        assert env["KEEP"] == "1" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_world_size_must_match_gpus():
    import pytest
    b = _bench()
    assert b.check_world(b.parse(["--gpus", "1"]), {}) is None            # one rank, this process
    assert b.check_world(b.parse([]), {}) is None
    assert b.check_world(b.parse(["--gpus", "8"]), {}) == 8                # start 8 local ranks
    assert b.check_world(b.parse(["--gpus", "8"]), {"WORLD_SIZE": "8"}) is None  # torch.distributed.run
    with pytest.raises(SystemExit):
        b.check_world(b.parse(["--gpus", "8"]), {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        b.check_world(b.parse(["--gpus", "1"]), {"WORLD_SIZE": "4"})


def test_launcher_refuses_missing_gpus():
    """Without enough GPUs the launcher stops before starting any rank."""
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr, r.stderr[-2000:]
