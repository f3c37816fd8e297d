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
