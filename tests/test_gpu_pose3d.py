"""estimatePose3D on the GPU (csrc/pose2d.hip pcnn_pose3d,
posecnn_amd/synthesize/pose3d.py) against the restated reference
(oracle/orc_pose2d.cpp orc_pose3d) on ray-cast box scenes with depth: the
camera coordinates, sampled hypotheses (objects, pixels, 3-point rigid
poses), every round's inlier counts over the hole-skipping subsets, the
survivors, the refit and Nelder-Mead refined poses and their energies --
all bit for bit (the device and the oracle run the same double / float
operations in the same order, sin / cos / acos included); plus the known
answer (the true pose) for exact inputs.  Scenes cover no holes (the parallel
subset scan), scattered and clustered holes (the wave walk), objects small
enough that early rounds take every valid pixel, and an object without
depth."""
import numpy as np
import pytest
import torch

from oracle import oracle
from pose2d_scene import make_scene
from posecnn_amd.synthesize import pose3d

pytestmark = pytest.mark.gpu


def _run(sc, **kw):
    C = sc["C"]
    poses = np.zeros((3, 4, C), np.float32)
    _, d = pose3d.estimate_poses_3d(sc["label"], sc["depth"], sc["vertmap"], sc["extents"], poses, C, *sc["camera"],
                                    sc["depth_factor"], return_diag=True, **kw)
    return poses, {k: v.cpu().numpy() for k, v in d.items()}


def _oracle(sc, **kw):
    return oracle.pose3d(sc["label"], sc["depth"], sc["vertmap"], sc["extents"], *sc["camera"], sc["depth_factor"],
                         **kw)


def _check(sc, poses, d, r):
    np.testing.assert_array_equal(d["eye"], r["eye"])
    np.testing.assert_array_equal(d["hyps"], r["hyps"])        # object, R, t of every hypothesis
    np.testing.assert_array_equal(d["hyp_px"], r["hyp_px"])    # its 3 sampled pixels
    np.testing.assert_array_equal(d["inliers"], r["inliers"])  # every round's counts
    np.testing.assert_array_equal(d["final"], r["final"])      # the survivors
    np.testing.assert_array_equal(d["energy"], r["energy"])    # refined optEnergy3D
    np.testing.assert_array_equal(poses, r["poses"])


def _clustered_holes(sc, seed, n=40, rad=12):
    rng = np.random.default_rng(seed)
    dep = sc["depth"].copy()
    H, W = dep.shape
    yy, xx = np.mgrid[:H, :W]
    for _ in range(n):
        cy, cx = rng.uniform(0, H), rng.uniform(0, W)
        dep[(yy - cy) ** 2 + (xx - cx) ** 2 < rng.uniform(3, rad) ** 2] = 0
    return dict(sc, depth=dep)


@pytest.mark.parametrize("case", ["clean", "holes_noise", "clustered", "dense_holes"])
def test_pose3d_matches_oracle(hip, case):
    if case == "clean":
        sc = make_scene(seed=1)
    elif case == "holes_noise":
        sc = make_scene(seed=2, hole_frac=0.2, depth_noise=0.002, coord_noise=0.01)
    elif case == "clustered":
        sc = _clustered_holes(make_scene(seed=5, coord_noise=0.003), seed=5)
    else:
        sc = make_scene(seed=7, hole_frac=0.6, depth_noise=0.001)
    poses, d = _run(sc)
    r = _oracle(sc)
    _check(sc, poses, d, r)
    for c, p in sc["poses"].items():
        assert d["final"][c][0] >= 0
        if case == "clean":
            np.testing.assert_allclose(poses[:, :3, c], p["R"], atol=1e-4)
            np.testing.assert_allclose(poses[:, 3, c], p["t"], atol=1e-4)
        else:
            np.testing.assert_allclose(poses[:, 3, c], p["t"], atol=1e-2)


def test_pose3d_small_objects(hip):
    """Objects of a few thousand pixels: the early rounds' rate >= 1 takes
    every valid pixel in list order (the compaction path), the later ones
    sample; with holes."""
    sc = make_scene(seed=8, n_obj=4, C=8, extents=None, hole_frac=0.1)
    lab = sc["label"].copy()
    # shrink each object to a band of rows so that it keeps 1500-6000 pixels
    for c in sc["poses"]:
        ys, xs = np.nonzero(lab == c)
        if len(ys) > 6000:
            cut = np.sort(ys)[5000]
            lab[(lab == c) & (np.arange(lab.shape[0])[:, None] > cut)] = 0
    sc = dict(sc, label=lab)
    poses, d = _run(sc, n_hyp=64)
    r = _oracle(sc, n_hyp=64)
    _check(sc, poses, d, r)


@pytest.mark.parametrize("max_iter", [3, 45])
def test_pose3d_attempt_limit_and_missing_depth(hip, max_iter):
    sc = make_scene(seed=4, n_obj=2, coord_noise=0.01)
    c0 = sorted(sc["poses"])[0]
    dep = sc["depth"].copy()
    dep[sc["label"] == c0] = 0  # one object has no depth at all
    sc = dict(sc, depth=dep)
    poses, d = _run(sc, max_iter=max_iter)
    r = _oracle(sc, max_iter=max_iter)
    _check(sc, poses, d, r)
    assert (d["final"][c0] == -1).all()


def test_pose3d_nm_evals_and_seed(hip):
    sc = make_scene(seed=9, coord_noise=0.005, depth_noise=0.001)
    for kw in (dict(nm_evals=7), dict(nm_evals=250), dict(seed=77)):
        poses, d = _run(sc, **kw)
        _check(sc, poses, d, _oracle(sc, **kw))


def test_pose3d_device_inputs_and_errors(hip):
    sc = make_scene(seed=4, n_obj=2)
    dev = torch.device("cuda")
    poses = torch.zeros((3, 4, sc["C"]), device=dev)
    pose3d.estimate_poses_3d(torch.from_numpy(sc["label"]).to(dev), torch.from_numpy(sc["depth"].astype(np.int32)),
                             torch.from_numpy(sc["vertmap"]).to(dev), torch.from_numpy(sc["extents"]).to(dev), poses,
                             sc["C"], *sc["camera"], sc["depth_factor"])
    np.testing.assert_array_equal(poses.cpu().numpy(), _oracle(sc)["poses"])
    lab = np.zeros_like(sc["label"])
    lab[:10, :30] = 1  # below minArea
    p2 = np.full((3, 4, sc["C"]), 7.0, np.float32)
    _, d = pose3d.estimate_poses_3d(lab, sc["depth"], sc["vertmap"], sc["extents"], p2, sc["C"], *sc["camera"],
                                    sc["depth_factor"], return_diag=True)
    assert not p2.any() and (d["final"].cpu().numpy() == -1).all()
    with pytest.raises(ValueError):
        pose3d.estimate_poses_3d(sc["label"], sc["depth"], sc["vertmap"], sc["extents"], p2, sc["C"], *sc["camera"],
                                 sc["depth_factor"], n_hyp=257)
    with pytest.raises(ValueError):
        pose3d.estimate_poses_3d(sc["label"], sc["depth"][:5], sc["vertmap"], sc["extents"], p2, sc["C"],
                                 *sc["camera"], sc["depth_factor"])
    # depth must be raw integer units (a float map in metres used
    # to truncate silently), within 0..65535; nm_evals must cover the simplex
    for bad in (sc["depth"].astype(np.float32) / sc["depth_factor"],
                torch.from_numpy(sc["depth"].astype(np.float32)),
                np.where(np.arange(sc["depth"].size).reshape(sc["depth"].shape) == 0, -1,
                         sc["depth"].astype(np.int32)),
                sc["depth"].astype(np.int32) + 70000):
        with pytest.raises(ValueError):
            pose3d.estimate_poses_3d(sc["label"], bad, sc["vertmap"], sc["extents"], p2, sc["C"], *sc["camera"],
                                     sc["depth_factor"])
    with pytest.raises(ValueError):
        pose3d.estimate_poses_3d(sc["label"], sc["depth"], sc["vertmap"], sc["extents"], p2, sc["C"], *sc["camera"],
                                 sc["depth_factor"], nm_evals=6)


def _mat2quat(R):
    """(w, x, y, z) of a rotation matrix (the role of test.py's mat2quat)."""
    m = np.asarray(R, np.float64)
    tr = np.trace(m)
    if tr > 0:
        s = 2.0 * np.sqrt(tr + 1.0)
        q = [0.25 * s, (m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s]
    else:
        i = int(np.argmax(np.diag(m)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = 2.0 * np.sqrt(1.0 + m[i, i] - m[j, j] - m[k, k])
        q = [0.0] * 4
        q[0] = (m[k, j] - m[j, k]) / s
        q[1 + i] = 0.25 * s
        q[1 + j] = (m[j, i] + m[i, j]) / s
        q[1 + k] = (m[k, i] + m[i, k]) / s
    q = np.asarray(q)
    return q / np.linalg.norm(q) * (1 if q[0] >= 0 else -1)


def test_pose3d_then_refine_poses(hip):
    """test.py:1383-1416 under VERTEX_REG_3D + POSE_REFINE: estimate_poses_3d,
    the found classes turned into (rois, poses) rows, then refine_poses
    (solve_icp, the box ray-caster as the renderer): every object found, the
    refined translation within 5 mm of the truth on a noisy frame."""
    from posecnn_amd.synthesize import icp as R
    from refine_scene import render_box
    sc = make_scene(seed=12, n_obj=3, hole_frac=0.05, depth_noise=0.001, coord_noise=0.005)
    C = sc["C"]
    poses_tmp = np.zeros((3, 4, C), np.float32)
    pose3d.estimate_poses_3d(sc["label"], sc["depth"], sc["vertmap"], sc["extents"], poses_tmp, C, *sc["camera"],
                             sc["depth_factor"])
    found = [j for j in range(C) if poses_tmp[2, 3, j] > 0]
    assert sorted(found) == sorted(sc["poses"])
    rois = np.zeros((len(found), 6), np.float32)
    poses = np.zeros((len(found), 7), np.float32)
    for i, j in enumerate(found):
        rois[i, 1] = j
        poses[i, :4] = _mat2quat(poses_tmp[:3, :3, j])
        poses[i, 4:] = poses_tmp[:, 3, j]

    def render(obj, pose):
        m = render_box(np.asarray(pose, np.float64), sc["extents"][obj] / 2.0, obj)
        dev = torch.device("cuda")
        return (torch.from_numpy(m["vertmap"]).to(dev), torch.from_numpy(m["pred_v"]).to(dev),
                torch.from_numpy(m["pred_n"]).to(dev))

    params = list(sc["camera"]) + [0.25, 6.0, sc["depth_factor"]]
    dev = torch.device("cuda")
    depth = torch.from_numpy(sc["depth"].astype(np.int32)).to(dev).to(torch.uint16)
    pnew, picp = R.solve_icp(torch.from_numpy(sc["label"]).to(dev), depth, params, rois, poses, render,
                             max_error=0.02, nm_evals=20)
    for i, j in enumerate(found):
        assert np.linalg.norm(picp[i, 4:] - sc["poses"][j]["t"]) < 5e-3
        assert abs(np.linalg.norm(picp[i, :4]) - 1) < 1e-4


@pytest.mark.parametrize("H,W,C,n_hyp,factor", [(240, 321, 16, 7, 1000.0), (480, 640, 22, 1, 10000.0),
                                                 (240, 300, 4, 64, 5000.0)])
def test_pose3d_shapes(hip, H, W, C, n_hyp, factor):
    """Odd and small frames, LINEMOD's C = 16 with its depth factor 1000,
    one hypothesis, and a 4-class frame: every output against the oracle."""
    sc = make_scene(seed=13, n_obj=min(3, C - 1), C=C, H=H, W=W, hole_frac=0.05, depth_noise=0.001,
                    coord_noise=0.003, depth_factor=factor)
    poses, d = _run(sc, n_hyp=n_hyp)
    _check(sc, poses, d, _oracle(sc, n_hyp=n_hyp))


@pytest.mark.parametrize("H,W,e,seed", [(480, 640, 0.30, 21), (720, 960, 0.55, 22)])
def test_pose3d_long_class_lists(hip, H, W, e, seed):
    """One object filling most of the frame with 10 % holes: its class list
    (243 k / 449 k positions) is past the skip bytes' 64 k (the bit walk from
    LDS) and, in the second frame, past the 327 k positions of the LDS bit
    copy (the walk reads the bits from HBM)."""
    C = 4
    ext = np.zeros((C, 3), np.float32)
    ext[1:] = e
    sc = make_scene(seed=seed, n_obj=1, C=C, H=H, W=W, extents=ext, hole_frac=0.1, depth_noise=0.001,
                    coord_noise=0.003)
    c = list(sc["poses"])[0]
    assert (sc["label"] == c).sum() > (65536 if H == 480 else 327680)
    poses, d = _run(sc, n_hyp=32)
    _check(sc, poses, d, _oracle(sc, n_hyp=32))
