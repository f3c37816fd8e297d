"""Pose refinement on the GPU (csrc/icp.hip through the C-ABI) against the
oracle restatement (oracle/orc_icp.cpp) of df::icp and solveICP's pieces
 on the synthetic box scene of refine_scene.py.

Bars: the live vertex map is bit-exact (same float operations); the ICP
systems, updates, centres and energies are float reductions whose order
differs (GPU: fixed per-lane / wave / workgroup tree; oracle: double in raster
order), so they are compared with tolerances written below."""
import numpy as np
import pytest
import torch

from refine_scene import CAMERA, pose_mul, scene

pytestmark = pytest.mark.gpu
D = torch.device("cuda")
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(D)


def _live(sc, orc):
    from posecnn_amd.synthesize import icp as R
    lv = R.live_vertices(t(sc["live"]["depth"].astype(np.int32)).to(torch.uint16), t(sc["live"]["label"]),
                         torch.tensor([sc["cls"]], dtype=torch.int32), 10000.0, CAMERA)
    ref = orc.icp_live_vertices(sc["live"]["depth"], sc["live"]["label"], sc["cls"], 10000.0, CAMERA)
    return lv, ref


def test_live_vertices_bit_exact(hip, orc):
    sc = scene(0)
    lv, ref = _live(sc, orc)
    np.testing.assert_array_equal(lv[0].cpu().numpy(), ref)


@pytest.mark.parametrize("iters", [1, 8, 20])
def test_icp_matches_oracle(hip, orc, iters):
    from posecnn_amd.synthesize import icp as R
    sc = scene(1)
    lv, ref_lv = _live(sc, orc)
    pv, pn = t(sc["pred"]["pred_v"])[None], t(sc["pred"]["pred_n"])[None]
    upd, pout, systems = R.icp(lv, pv, pn, CAMERA, max_error=0.05, iterations=iters,
                               pose_in=t(sc["init"].astype(np.float32))[None], return_systems=True)
    oupd, osys = orc.icp(ref_lv, sc["pred"]["pred_v"], sc["pred"]["pred_n"], CAMERA, max_error=0.05,
                         iterations=iters)
    s = systems[0].cpu().numpy()
    # iteration 0 sees identical inputs: same pixel set, sums within float
    # accumulation error (|sum| scale 1e-5 relative)
    assert s[0, 27] == osys[0, 27]
    scale = np.abs(osys[0, :27]).max()
    np.testing.assert_allclose(s[0, :27], osys[0, :27], rtol=1e-4, atol=1e-5 * scale)
    u = upd[0].cpu().numpy()
    np.testing.assert_allclose(u, oupd, atol=2e-5 * max(1, iters))
    np.testing.assert_allclose(pout[0].cpu().numpy(), pose_mul(u.astype(np.float64), sc["init"]), atol=1e-5)
    if iters == 20:  # converged onto the truth
        refined = pose_mul(u.astype(np.float64), sc["init"])
        assert np.linalg.norm(refined[4:] - sc["true"][4:]) < 1.5e-3


def test_icp_batched_problems_and_live_index(hip, orc):
    """N = 3 problems sharing one live map (the 8-hypothesis batch of
    solveICP:2255-2286 in miniature), one of them with no usable pixel."""
    from posecnn_amd.synthesize import icp as R
    scs = [scene(s) for s in (0, 2)]
    lv, ref_lv = _live(scs[0], orc)
    far = scs[0]["pred"]["pred_v"].copy()
    far[..., 2] = 100.0  # every rendered depth outside (znear, zfar): no pixel contributes
    pv = t(np.stack([scs[0]["pred"]["pred_v"], scs[1]["pred"]["pred_v"], far]))
    pn = t(np.stack([scs[0]["pred"]["pred_n"], scs[1]["pred"]["pred_n"], scs[0]["pred"]["pred_n"]]))
    upd, _ = R.icp(lv, pv, pn, CAMERA, max_error=0.05, iterations=8, live_index=torch.zeros(3, dtype=torch.int32))
    u = upd.cpu().numpy()
    for k, sc in enumerate(scs):
        o, _ = orc.icp(ref_lv, sc["pred"]["pred_v"], sc["pred"]["pred_n"], CAMERA, max_error=0.05, iterations=8)
        np.testing.assert_allclose(u[k], o, atol=2e-4)
    np.testing.assert_array_equal(u[2], np.array([1, 0, 0, 0, 0, 0, 0], np.float32))
    # a device-side live index is not checked on the host: out of range, the problem contributes nothing
    bad = torch.tensor([0, 5, -1], dtype=torch.int32, device=D)
    u2, _ = R.icp(lv, pv, pn, CAMERA, max_error=0.05, iterations=8, live_index=bad)
    u2 = u2.cpu().numpy()
    np.testing.assert_array_equal(u2[0], u[0])
    np.testing.assert_array_equal(u2[1:], np.tile(np.array([1, 0, 0, 0, 0, 0, 0], np.float32), (2, 1)))


def test_icp_center_and_energy(hip, orc):
    from posecnn_amd.synthesize import icp as R
    sc = scene(3, perturb_deg=1.0, perturb_t=0.004)
    lv, ref_lv = _live(sc, orc)
    p = sc["pred"]
    lab = t(sc["live"]["label"])
    init = sc["init"].astype(np.float32)
    out, pout = R.icp_center(lv, lab, torch.tensor([sc["cls"]]), t(p["vertmap"])[None], t(p["pred_v"])[None],
                             t(p["pred_n"])[None], max_error=0.02, pose_in=t(init)[None])
    ref = orc.icp_center(ref_lv, sc["live"]["label"], sc["cls"], p["vertmap"], p["pred_v"], p["pred_n"],
                         max_error=0.02)
    o = out[0].cpu().numpy()
    assert o[3] == ref[3] and ref[3] > 500
    np.testing.assert_allclose(o[:3], ref[:3], rtol=1e-5, atol=1e-6)
    po = pout[0].cpu().numpy()
    np.testing.assert_array_equal(po[:4], init[:4])
    np.testing.assert_allclose(po[4:], [init[4] / init[6] * o[2], init[5] / init[6] * o[2], o[2]], rtol=1e-6)
    poses = np.stack([init, sc["true"].astype(np.float32), np.array([1, 0, 0, 0, 0, 0, 0.5], np.float32)])
    e = R.pose_energy(lv[0], lab, sc["cls"], t(p["pred_v"]), t(poses)).cpu().numpy()
    eo = orc.pose_energy(ref_lv, sc["live"]["label"], sc["cls"], p["pred_v"], poses)
    np.testing.assert_allclose(e, eo, rtol=2e-5)


def test_icp_score_matches_oracle(hip, orc):
    """SegICP hypothesis scores: same candidate sets, same float distance
    arithmetic and tie rule -> identical scores and choice."""
    from posecnn_amd.synthesize import icp as R
    sc = scene(4, perturb_deg=2.0, perturb_t=0.006, half=(0.03, 0.025, 0.02))
    lv, ref_lv = _live(sc, orc)
    hyps = np.repeat(sc["init"].astype(np.float32)[None], 8, 0)
    hyps[1:, 6] += np.array([-0.02, -0.01, 0.01, 0.02, 0.03, 0.04, 0.05], np.float32)
    hyps[3] = sc["true"].astype(np.float32)
    s, ch = R.icp_score(lv[0], t(sc["live"]["label"]), sc["cls"], t(sc["pred"]["vertmap"]), t(hyps))
    so, cho = orc.icp_score(ref_lv, sc["live"]["label"], sc["cls"], sc["pred"]["vertmap"], hyps)
    np.testing.assert_array_equal(s.cpu().numpy(), so)
    assert int(ch[0]) == cho


@pytest.mark.parametrize("radius", [0.005, 0.01, 0.03])
def test_icp_score_grid_ties_and_far_points(hip, orc, radius):
    """The grid-bucketed nearest-point search against the oracle's brute force
    on a dense lattice cloud: depth and model points on a 4 mm lattice (many
    candidates per 1 cm radius, exact distance ties -> the lowest index wins),
    duplicated depth points, points far from the camera (60 m) and a
    hypothesis that moves the model onto them, and one that misses all."""
    from posecnn_amd.synthesize import icp as R
    H, W, obj = 48, 64, 3
    rng = np.random.default_rng(7)
    lat = rng.integers(-6, 7, size=(H * W, 3)).astype(np.float32) * 0.004
    live = (lat + np.array([0.0, 0.0, 0.8], np.float32)).astype(np.float32)
    live[100:140] = live[60:100]                          # exact duplicates: ties by index
    live[-50:] += np.array([0.0, 0.0, 60.0], np.float32)  # far points
    model = rng.integers(-6, 7, size=(H * W, 3)).astype(np.float32) * 0.004
    vm = model.copy()
    vm[:, 0] += obj                                        # the class offset in x's integer part
    label = np.full((H, W), obj, np.int32)
    label[0, :5] = 0                                       # not the object
    hyps = np.zeros((4, 7), np.float32)
    hyps[:, 0] = 1.0
    hyps[0, 6] = 0.8                                       # onto the lattice: exact ties
    hyps[1, 4:] = (0.001, -0.002, 0.803)
    hyps[2, 6] = 60.8                                      # onto the far points
    hyps[3, 6] = 5.0                                       # misses everything
    hyps[1, :4] = (0.9995, 0.02, -0.01, 0.0)
    s, ch = R.icp_score(t(live.reshape(H, W, 3)), t(label), obj, t(vm.reshape(H, W, 3)), t(hyps), radius=radius)
    so, cho = orc.icp_score(live.reshape(H, W, 3), label, obj, vm.reshape(H, W, 3), hyps, radius=radius)
    np.testing.assert_array_equal(s.cpu().numpy(), so)
    assert int(ch[0]) == cho
    assert so[0] > 0 and so[2] > 0 and so[3] == 0


def test_icp_score_no_object_points(hip, orc):
    """An object with no pixel in the label map (M = 0, the count every score
    launch reads from the device): every score 0 and the choice hyps[0]
    (synthesize.cpp:2333-2334), as the oracle."""
    from posecnn_amd.synthesize import icp as R
    H, W, obj = 32, 48, 2
    rng = np.random.default_rng(3)
    live = (rng.uniform(-0.05, 0.05, (H, W, 3)) + np.array([0, 0, 0.9])).astype(np.float32)
    vm = rng.uniform(-0.05, 0.05, (H, W, 3)).astype(np.float32)
    label = np.ones((H, W), np.int32)  # another class everywhere
    hyps = np.zeros((5, 7), np.float32)
    hyps[:, 0] = 1.0
    hyps[:, 6] = 0.9
    s, ch = R.icp_score(t(live), t(label), obj, t(vm), t(hyps))
    so, cho = orc.icp_score(live, label, obj, vm, hyps)
    np.testing.assert_array_equal(s.cpu().numpy(), so)
    assert int(ch[0]) == cho == 0 and not so.any()


def test_solve_icp_end_to_end(hip, orc):
    """The solveICP flow (synthesize.cpp:2052-2395) with the box ray-caster as
    the renderer: poses_new is the re-centred pose (no Nelder-Mead stage here),
    poses_icp the SegICP-chosen ICP hypothesis, closer to the truth than the
    initial pose; a RoI of class 0 and one without enough pixels stay zero."""
    from posecnn_amd.synthesize import icp as R
    from refine_scene import render_box
    sc = scene(5, perturb_deg=2.0, perturb_t=0.01)

    def render(obj, pose):
        m = render_box(np.asarray(pose, np.float64), sc["half"], obj)
        return t(m["vertmap"]), t(m["pred_v"]), t(m["pred_n"])

    params = list(CAMERA) + [0.25, 6.0, 10000.0]
    rois = np.array([[0, sc["cls"], 0, 0, 1, 1], [0, 0, 0, 0, 1, 1], [0, 7, 0, 0, 1, 1]], np.float32)
    poses = np.stack([sc["init"], sc["init"], sc["init"]]).astype(np.float32)
    depth = t(sc["live"]["depth"].astype(np.int32)).to(torch.uint16)
    pnew, picp = R.solve_icp(t(sc["live"]["label"]), depth, params, rois, poses, render, max_error=0.02, nm_evals=0)
    assert np.all(pnew[1:] == 0) and np.all(picp[1:] == 0)
    # re-centring step against the oracle
    ref_lv = orc.icp_live_vertices(sc["live"]["depth"], sc["live"]["label"], sc["cls"], 10000.0, CAMERA)
    c = orc.icp_center(ref_lv, sc["live"]["label"], sc["cls"], sc["pred"]["vertmap"], sc["pred"]["pred_v"],
                       sc["pred"]["pred_n"], max_error=0.02)
    init = sc["init"].astype(np.float32)
    np.testing.assert_allclose(pnew[0, 4:], [init[4] / init[6] * c[2], init[5] / init[6] * c[2], c[2]], rtol=1e-5)
    e_icp = np.linalg.norm(picp[0, 4:] - sc["true"][4:])
    assert e_icp < np.linalg.norm(init[4:] - sc["true"][4:]) and e_icp < 3e-3
    # with the Nelder-Mead stage the result stays a unit-quaternion pose near the truth
    pnew2, picp2 = R.solve_icp(t(sc["live"]["label"]), depth, params, rois[:1], poses[:1], render, max_error=0.02,
                               nm_evals=50)
    assert abs(np.linalg.norm(picp2[0, :4]) - 1) < 1e-4
    assert np.linalg.norm(picp2[0, 4:] - sc["true"][4:]) < 5e-3


def test_icp_edges(hip, orc):
    """iterations = 0 is the identity update (pose_out = pose_in normalised);
    argument errors come back as ValueError (PCNN_EINVAL), never a crash."""
    from posecnn_amd.synthesize import icp as R
    sc = scene(0)
    lv, _ = _live(sc, orc)
    pv, pn = t(sc["pred"]["pred_v"])[None], t(sc["pred"]["pred_n"])[None]
    pin = np.array([[2.0, 0, 0, 0, 0.1, 0.2, 0.7]], np.float32)
    upd, pout = R.icp(lv, pv, pn, CAMERA, iterations=0, pose_in=t(pin))
    np.testing.assert_array_equal(upd.cpu().numpy(), [[1, 0, 0, 0, 0, 0, 0]])
    np.testing.assert_allclose(pout.cpu().numpy(), [[1, 0, 0, 0, 0.1, 0.2, 0.7]], atol=1e-7)
    with pytest.raises(ValueError):  # H * W % 4 != 0 for the float4 live-vertex stores
        R.live_vertices(torch.zeros((3, 3), dtype=torch.uint16, device=D), torch.zeros((3, 3), dtype=torch.int32,
                                                                                      device=D), [1], 1.0, CAMERA)
    with pytest.raises(ValueError):  # more than 64 hypotheses
        R.icp_score(lv[0], t(sc["live"]["label"]), sc["cls"], t(sc["pred"]["vertmap"]),
                    torch.zeros((65, 7), device=D))


def test_solve_icp_batched_over_rois(hip):
    """Two boxes of different classes in one frame plus a repeated RoI: the
    batched solve_icp (one launch per step for all RoIs, Nelder-Mead in lock
    step) gives each RoI what a call with that RoI alone gives (ICP's
    workgroup count depends on the batch, so the refined poses agree to float
    rounding), and both objects land near their true poses."""
    from posecnn_amd.synthesize import icp as R
    from refine_scene import axis_angle_quat, quat_mul, render_box
    rng = np.random.default_rng(11)
    halves = {3: (0.06, 0.045, 0.035), 5: (0.05, 0.05, 0.03)}
    trues = {3: np.concatenate([axis_angle_quat([1, 1, 0.3], 0.6), [0.08, -0.02, 0.8]]),
             5: np.concatenate([axis_angle_quat([0.2, 1, 0.5], 1.1), [-0.1, 0.05, 0.9]])}
    live = {c: render_box(trues[c], halves[c], c) for c in trues}
    zs = {c: np.where(live[c]["hit"], live[c]["pred_v"][..., 2], np.inf) for c in trues}
    front3 = zs[3] <= zs[5]
    label = np.where(live[3]["hit"] & front3, 3, np.where(live[5]["hit"], 5, 0)).astype(np.int32)
    depth = np.where(label == 3, live[3]["depth"], np.where(label == 5, live[5]["depth"], 0)).astype(np.uint16)

    def render(obj, pose):
        m = render_box(np.asarray(pose, np.float64), halves[obj], obj)
        return t(m["vertmap"]), t(m["pred_v"]), t(m["pred_n"])

    inits = {}
    for c in trues:
        dq = axis_angle_quat(rng.normal(size=3), np.deg2rad(2.0))
        inits[c] = np.concatenate([quat_mul(dq, trues[c][:4]), trues[c][4:] + rng.normal(size=3) * 0.005])
    rois = np.array([[0, 3, 0, 0, 1, 1], [0, 5, 0, 0, 1, 1], [0, 3, 0, 0, 1, 1]], np.float32)
    poses = np.stack([inits[3], inits[5], inits[3]]).astype(np.float32)
    params = list(CAMERA) + [0.25, 6.0, 10000.0]
    lab_d = t(label)
    dep_d = t(depth.astype(np.int32)).to(torch.uint16)
    pnew, picp = R.solve_icp(lab_d, dep_d, params, rois, poses, render, max_error=0.02, nm_evals=20)
    for i in range(3):
        a, b = R.solve_icp(lab_d, dep_d, params, rois[i:i + 1], poses[i:i + 1], render, max_error=0.02, nm_evals=20)
        np.testing.assert_allclose(pnew[i], a[0], atol=1e-6)
        np.testing.assert_allclose(picp[i], b[0], atol=2e-4)
    np.testing.assert_array_equal(pnew[0], pnew[2])
    for i, c in enumerate((3, 5)):
        assert np.linalg.norm(picp[i, 4:] - trues[c][4:]) < 5e-3


@pytest.mark.parametrize("max_eval", [8, 12, 50])
def test_nelder_mead_device_matches_host(hip, orc, max_eval):
    """refinePose's Nelder-Mead (poseWithOpt, synthesize.cpp:2529-2573) run
    wholly on the device, one workgroup per problem (pcnn_nelder_mead_energy),
    against the host search (icp.py nelder_mead) over the same record-based
    optEnergy (pcnn_energy_rec): the same points, values and evaluation counts,
    bit for bit, for max_eval equal to the initial simplex (8), with shrinks
    (12) and at solveICP's 50 (budgets below the simplex are refused: NLopt's
    maxeval counts it, test_nelder_mead_device_refuses_small_budget).  The record energy is optEnergy over the pixels of
    the full-frame kernel (pcnn_pose_energy, parity-tested against the
    oracle), summed in another fixed order."""
    from posecnn_amd.synthesize import icp as R
    scs = [scene(s, perturb_deg=3.0, perturb_t=0.01) for s in (7, 8)]
    lvs = [_live(sc, orc)[0] for sc in scs]
    live = torch.cat(lvs)
    lab = t(scs[0]["live"]["label"])
    # problems: the two scenes' objects (live maps 0 / 1) and scene 0 again with a shifted start
    pv = torch.stack([t(scs[0]["pred"]["pred_v"]), t(scs[1]["pred"]["pred_v"]), t(scs[0]["pred"]["pred_v"])])
    objs = [scs[0]["cls"], scs[1]["cls"], scs[0]["cls"]]
    labs = [scs[0]["live"]["label"], scs[1]["live"]["label"]]
    if not np.array_equal(labs[0], labs[1]):  # one label map for all problems: use scene 0's
        live = torch.cat([lvs[0], lvs[0]])
    rec, cnt = R.energy_records(live, lab, objs, [0, 1, 0], pv, (0.25, 6.0))
    assert int(cnt.min()) > 1000
    x0 = np.array([[1, 0, 0, 0, 0, 0, 0], [1, 0, 0, 0, 0, 0, 0], [0.99, 0.02, -0.01, 0.0, 0.002, -0.001, 0.01]],
                  np.float64)
    r = np.array([0.1, 0.1, 0.1, 0.1, 0.01, 0.01, 0.1])
    x, f, nev = R.nelder_mead_device(rec, cnt, x0, x0 - r, x0 + r, max_eval)
    x, f, nev = x.cpu().numpy(), f.cpu().numpy(), nev.cpu().numpy()
    for i in range(3):
        def fn(p, i=i):
            e = R.pose_energy_records(rec, cnt, torch.from_numpy(np.asarray(p, np.float32)[None]).to(D),
                                      torch.tensor([i], dtype=torch.int32))
            return float(e.cpu().numpy()[0])
        hx, hf = R.nelder_mead(fn, x0[i], x0[i] - r, x0[i] + r, max_eval)
        np.testing.assert_array_equal(x[i], hx)
        assert f[i] == hf
        assert nev[i] == max(8, max_eval)
    # the record energy against the full-frame optEnergy kernel (oracle-pinned) on the same poses
    P = torch.from_numpy(np.concatenate([x0[:1], x[:1]]).astype(np.float32)).to(D)
    e_rec = R.pose_energy_records(rec, cnt, P, torch.zeros(2, dtype=torch.int32)).cpu().numpy()
    e_ff = R.pose_energy(live[0], lab, objs[0], pv[0], P).cpu().numpy()
    np.testing.assert_allclose(e_rec, e_ff, rtol=2e-5)
    if max_eval == 50:
        assert f[0] < e_rec[0]  # the search lowered the energy


def test_nelder_mead_device_launch_paths_agree(hip, orc):
    """The three device searches behind nelder_mead_device -- speculative
    rounds (N <= 32: reflection, expansion and both contractions evaluated in
    one cross-workgroup round), one evaluation per round (N <= 128), one
    workgroup per problem (larger N) -- give the same points, values and
    evaluation counts on the same problems."""
    from posecnn_amd.synthesize import icp as R
    sc = scene(7, perturb_deg=3.0, perturb_t=0.01)
    lv = _live(sc, orc)[0]
    lab = t(sc["live"]["label"])
    pv = t(sc["pred"]["pred_v"])[None].expand(3, -1, -1, -1).contiguous()
    rec, cnt = R.energy_records(lv, lab, [sc["cls"]] * 3, [0, 0, 0], pv, (0.25, 6.0))
    x0 = np.array([[1, 0, 0, 0, 0, 0, 0], [0.99, 0.02, -0.01, 0.0, 0.002, -0.001, 0.01],
                   [0.98, -0.03, 0.02, 0.01, -0.004, 0.003, -0.02]], np.float64)
    r = np.array([0.1, 0.1, 0.1, 0.1, 0.01, 0.01, 0.1])
    out = {}
    ran = {}
    for N, force in ((3, 0), (40, 0), (130, 0), (3, 2), (3, 3), (40, 3)):
        sel = torch.arange(N, device=D) % 3
        recN, cntN = rec.index_select(0, sel).contiguous(), cnt.index_select(0, sel).contiguous()
        xN = x0[np.arange(N) % 3]
        x, f, nev, path = R.nelder_mead_device(recN, cntN, xN, xN - r, xN + r, 30, force_path=force,
                                               return_path=True)
        out[(N, force)] = (x.cpu().numpy()[:3], f.cpu().numpy()[:3], nev.cpu().numpy()[:3])
        ran[(N, force)] = path
        del recN
    # the comparison must not be one kernel against itself -- the
    # speculative and cooperative paths (and their barriers) really ran
    assert ran[(3, 0)] == 1 and ran[(40, 0)] == 2 and ran[(130, 0)] == 3, ran
    assert ran[(3, 2)] == 2 and ran[(3, 3)] == 3 and ran[(40, 3)] == 3, ran
    for key in out:
        for a, b in zip(out[key], out[(3, 0)]):
            np.testing.assert_array_equal(a, b)
    assert (out[(3, 0)][2] == 30).all()


def test_nelder_mead_device_refuses_small_budget(hip):
    """max_eval below the 7-D initial simplex is refused (the
    device search used to evaluate all 8 points and report nev 8 anyway)."""
    from posecnn_amd.synthesize import icp as R
    rec = torch.zeros((1, 16, 6), device=D)
    cnt = torch.ones((1,), dtype=torch.int32, device=D)
    x0 = np.array([[1, 0, 0, 0, 0, 0, 0]], np.float64)
    with pytest.raises(ValueError):
        R.nelder_mead_device(rec, cnt, x0, x0 - 0.1, x0 + 0.1, 5)
    with pytest.raises(ValueError):
        R.solve_icp(None, None, None, None, None, None, nm_evals=5)


def test_solve_icp_device_search_matches_host_driver(hip):
    """solve_icp with the Nelder-Mead searches on the device (the default)
    against the host-driven lock-step searches (nm_device=False): identical
    poses_new and poses_icp."""
    from posecnn_amd.synthesize import icp as R
    from refine_scene import render_box
    sc = scene(9, perturb_deg=2.0, perturb_t=0.01)

    def render(obj, pose):
        m = render_box(np.asarray(pose, np.float64), sc["half"], obj)
        return t(m["vertmap"]), t(m["pred_v"]), t(m["pred_n"])

    params = list(CAMERA) + [0.25, 6.0, 10000.0]
    rois = np.array([[0, sc["cls"], 0, 0, 1, 1], [0, sc["cls"], 0, 0, 1, 1]], np.float32)
    poses = np.stack([sc["init"], sc["init"] * np.array([1, 1, 1, 1, 1.0, 1.0, 1.01])]).astype(np.float32)
    depth = t(sc["live"]["depth"].astype(np.int32)).to(torch.uint16)
    a = R.solve_icp(t(sc["live"]["label"]), depth, params, rois, poses, render, max_error=0.02, nm_evals=50)
    b = R.solve_icp(t(sc["live"]["label"]), depth, params, rois, poses, render, max_error=0.02, nm_evals=50,
                    nm_device=False)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    assert np.linalg.norm(a[1][0, 4:] - sc["true"][4:]) < 5e-3


def test_solve_icp_batched_renderer_matches(hip):
    """A renderer with render_many is called once per stage (three calls per
    solve) instead of once per pose; the maps are the same, so poses_new and
    poses_icp are identical to the per-pose calls (2 RoIs, Nelder-Mead on)."""
    from posecnn_amd.synthesize import icp as R
    from refine_scene import GraphBoxRenderer
    sc = scene(5, perturb_deg=2.0, perturb_t=0.01)
    rnd = GraphBoxRenderer(lambda o: sc["half"])
    calls = {"many": 0}

    class Counting:
        def render_many(self, objs, poses):
            calls["many"] += 1
            return rnd.render_many(objs, poses)

    params = list(CAMERA) + [0.25, 6.0, 10000.0]
    rois = np.array([[0, sc["cls"], 0, 0, 1, 1], [0, sc["cls"], 0, 0, 1, 1]], np.float32)
    poses = np.stack([sc["init"], sc["init"]]).astype(np.float32)
    depth = t(sc["live"]["depth"].astype(np.int32)).to(torch.uint16)
    lab = t(sc["live"]["label"])
    a = R.solve_icp(lab, depth, params, rois, poses, lambda o, p: rnd(o, p), max_error=0.02, nm_evals=20)
    b = R.solve_icp(lab, depth, params, rois, poses, Counting(), max_error=0.02, nm_evals=20)
    assert calls["many"] == 3
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    assert np.linalg.norm(b[1][0, 4:] - sc["true"][4:]) < 5e-3
