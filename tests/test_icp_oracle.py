"""Oracle checks of the pose-refinement restatement (oracle/orc_icp.cpp, CPU
only): the Eigen LDLT and Sophus SE3 product restatements against numpy, the
live-vertex formula, and df::icp converging on an exact synthetic scene (the
reference holds no fixtures for this path: parity unpinned)."""
import numpy as np
import pytest

from oracle import oracle
from refine_scene import CAMERA, pose_mul, scene


@pytest.fixture(scope="module")
def orc():
    oracle.lib()
    return oracle


def test_ldlt_solve_matches_numpy(orc):
    rng = np.random.default_rng(1)
    for _ in range(20):
        M = rng.normal(size=(6, 6))
        A = (M @ M.T + 0.1 * np.eye(6)).astype(np.float32)
        b = rng.normal(size=6).astype(np.float32)
        x = orc.ldlt_solve6(np.triu(A), b)
        np.testing.assert_allclose(x, np.linalg.solve(A.astype(np.float64), b), rtol=2e-3, atol=1e-4)


def test_ldlt_zero_system_gives_zero(orc):
    assert np.all(orc.ldlt_solve6(np.zeros((6, 6), np.float32), np.ones(6, np.float32)) == 0)


def test_se3_mul_matches_numpy(orc):
    rng = np.random.default_rng(2)
    for _ in range(10):
        a = np.concatenate([rng.normal(size=4), rng.normal(size=3)])
        b = np.concatenate([rng.normal(size=4), rng.normal(size=3)])
        a[:4] /= np.linalg.norm(a[:4])
        b[:4] /= np.linalg.norm(b[:4])
        np.testing.assert_allclose(orc.se3_mul(a, b), pose_mul(a, b), atol=1e-5)


def test_live_vertices_formula(orc):
    sc = scene(0)
    lv = orc.icp_live_vertices(sc["live"]["depth"], sc["live"]["label"], sc["cls"], 10000.0, CAMERA)
    fx, fy, px, py = (np.float32(c) for c in CAMERA)
    ys, xs = np.nonzero(sc["live"]["label"] == sc["cls"])
    d = sc["live"]["depth"][ys, xs].astype(np.float32) / np.float32(10000.0)
    np.testing.assert_array_equal(lv[ys, xs, 2], d)
    np.testing.assert_array_equal(lv[ys, xs, 0], ((xs.astype(np.float32) - px) / fx) * d)
    assert np.all(lv[sc["live"]["label"] != sc["cls"]] == 0)


@pytest.mark.parametrize("seed", [0, 1])
def test_icp_converges_on_exact_scene(orc, seed):
    sc = scene(seed)
    lv = orc.icp_live_vertices(sc["live"]["depth"], sc["live"]["label"], sc["cls"], 10000.0, CAMERA)
    upd, systems = orc.icp(lv, sc["pred"]["pred_v"], sc["pred"]["pred_n"], CAMERA, max_error=0.05, iterations=20)
    assert systems[0, 27] > 1000  # contributing pixels
    refined = pose_mul(upd.astype(np.float64), sc["init"])
    assert np.linalg.norm(refined[4:] - sc["true"][4:]) < 1.5e-3
    dq = abs(float(np.dot(refined[:4] / np.linalg.norm(refined[:4]), sc["true"][:4])))
    assert 2 * np.degrees(np.arccos(min(1.0, dq))) < 0.5
    err0 = np.linalg.norm(sc["init"][4:] - sc["true"][4:])
    assert np.linalg.norm(refined[4:] - sc["true"][4:]) < 0.3 * err0


def test_score_prefers_the_truth(orc):
    sc = scene(4, perturb_deg=2.0, perturb_t=0.006, half=(0.03, 0.025, 0.02))
    lv = orc.icp_live_vertices(sc["live"]["depth"], sc["live"]["label"], sc["cls"], 10000.0, CAMERA)
    hyps = np.stack([sc["init"], sc["true"], sc["init"] + np.array([0, 0, 0, 0, 0, 0, 0.03])]).astype(np.float32)
    # the vertmap from a render at the truth: model points land on the live points exactly at hyps[1]
    from refine_scene import render_box
    vm = render_box(sc["true"], sc["half"], sc["cls"])["vertmap"]
    s, ch = orc.icp_score(lv, sc["live"]["label"], sc["cls"], vm, hyps)
    assert ch == 1 and s[1] > 0.9 and s[2] < s[1]


def test_nelder_mead_bounded_quadratic():
    """The host Nelder-Mead of solve_icp's optEnergy stage: finds a bounded
    quadratic's minimum, never leaves the box, stops at max_eval."""
    from posecnn_amd.synthesize.icp import nelder_mead
    calls = []
    target = np.array([0.05, -0.02, 0.3])

    def f(x):
        calls.append(x.copy())
        return float(np.sum((x - target) ** 2))

    x0 = np.zeros(3)
    lb, ub = np.array([-0.1, -0.1, -0.1]), np.array([0.1, 0.1, 0.1])
    x, fx = nelder_mead(f, x0, lb, ub, 200)
    assert len(calls) <= 200
    assert all(np.all(c >= lb - 1e-12) and np.all(c <= ub + 1e-12) for c in calls)
    np.testing.assert_allclose(x, [0.05, -0.02, 0.1], atol=2e-3)  # z pinned at its bound
    calls.clear()
    nelder_mead(f, x0, lb, ub, 10)
    assert len(calls) <= 10


def test_host_se3_mul_matches_oracle(orc):
    from posecnn_amd.synthesize.icp import _se3_mul
    rng = np.random.default_rng(7)
    for _ in range(10):
        a = np.concatenate([rng.normal(size=4), rng.normal(size=3)])
        b = np.concatenate([rng.normal(size=4), rng.normal(size=3)])
        a[:4] /= np.linalg.norm(a[:4])
        b[:4] /= np.linalg.norm(b[:4])
        np.testing.assert_allclose(_se3_mul(a, b), orc.se3_mul(a, b), atol=1e-5)
