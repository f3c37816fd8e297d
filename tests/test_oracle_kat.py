"""Known-answer tests pinning the oracle (oracle/*.cpp) — CPU only.

The reference ships no golden vectors for this path, so
the oracle is pinned here by (a) hand-derived known answers (SURVEY §8(c)
(i)-(v)) and (b) an independent numpy re-derivation of the reference's
per-cell vote (compute_hough_kernel, hough_voting_gpu_op.cu.cc:253-294, with
angle_distance :32-42 and project_box :84-120) evaluated by brute force over
every cell.  numpy float32 scalar/array ops round every operation, like the
oracle's -ffp-contract=off build, so counts and distance sums must match
bit for bit.
"""
import math

import numpy as np
import pytest

from posecnn_amd import synth

F = np.float32


# ---------------------------------------------------------------------------
# (b) independent brute-force restatement of the reference vote
def np_project_box(cls, extents, meta, d, factor=F(0.6)):
    """project_box (cu.cc:84-120) in float32."""
    xh, yh, zh = (F(np.float64(extents[cls, i]) * 0.5) for i in range(3))
    fx, fy, px, py = F(meta[0]), F(meta[4]), F(meta[2]), F(meta[5])
    zf, zb = F(zh + d), F(-zh + d)
    xs, ys = [], []
    for i in range(8):
        X = -xh if i & 1 else xh
        Y = -yh if i & 2 else yh
        Z = zb if i & 4 else zf
        xs.append(F(fx * F(X / Z)) + px)
        ys.append(F(fy * F(Y / Z)) + py)
    w = F(F(max(xs) - min(xs)) + F(1))
    h = F(F(max(ys) - min(ys)) + F(1))
    return F(max(w, h) * factor)


def np_vote(label, vertex, extents, meta, cls, skip, thr=F(0.9)):
    H, W = label.shape
    ys, xs = np.nonzero(label == cls)  # C order = ascending y*W + x (the canonical list order)
    cy, cx = np.mgrid[0:H, 0:W]
    counts = np.zeros((H, W), F)
    dsum = np.zeros((H, W), F)
    with np.errstate(invalid="ignore", divide="ignore"):
        for i in range(0, len(xs), skip):  # list positions 0, skip, 2 skip (cu.cc:269)
            x, y = int(xs[i]), int(ys[i])
            u, v, z = (F(vertex[y, x, 3 * cls + k]) for k in range(3))
            d = F(math.exp(float(z)))  # (float)exp((double)z)
            T = np_project_box(cls, extents, meta, d)
            dx = (cx - x).astype(F)
            dy = (cy - y).astype(F)
            n1 = F(np.sqrt(F(u * u) + F(v * v)))
            n2 = np.sqrt(dx * dx + dy * dy)
            cos = (u * dx + v * dy) / (n1 * n2)
            vote = (cos > thr) & (np.abs((x - cx).astype(F)) < T) & (np.abs((y - cy).astype(F)) < T)
            counts[vote] += F(1)
            dsum[vote] += d
    return counts, dsum, (len(xs) + skip - 1) // skip


@pytest.mark.parametrize("skip", [1, 4])
def test_vote_counts_match_bruteforce(orc, skip):
    fr = synth.make_frames(1, H=36, W=48, num_classes=4, objects_per_image=2, seed=21)
    lab, vert, ext, meta = fr["label"][0], fr["vertex"][0], fr["extents"], fr["meta"][0].reshape(-1)
    present = [c for c in range(1, 4) if (lab == c).sum() > 0]
    assert present
    for c in present:
        oc, od, onv = orc.hough_class_counts(lab, vert, ext, meta, c, skip)
        nc, nd, nnv = np_vote(lab, vert, ext, meta, c, skip)
        assert onv == nnv
        np.testing.assert_array_equal(oc, nc)
        np.testing.assert_array_equal(od, nd)
        assert oc.max() > 0


# ---------------------------------------------------------------------------
# (i) a disc with exact radial vectors peaks at its centre
def _disc(H=64, W=80, cx=40, cy=30, rad=14):
    label = np.zeros((1, H, W), np.int32)
    vertex = np.zeros((1, H, W, 6), np.float32)
    yy, xx = np.mgrid[0:H, 0:W]
    inside = (xx - cx) ** 2 + (yy - cy) ** 2 <= rad * rad
    label[0][inside] = 1
    dxv, dyv = (cx - xx).astype(np.float64), (cy - yy).astype(np.float64)
    n = np.hypot(dxv, dyv)
    n[n == 0] = 1.0
    vertex[0, :, :, 3] = np.where(inside, dxv / n, 0).astype(np.float32)
    vertex[0, :, :, 4] = np.where(inside, dyv / n, 0).astype(np.float32)
    vertex[0, :, :, 5] = 0.0  # log z = 0 -> d = 1 exactly
    extents = np.array([[0, 0, 0], [0.5, 0.5, 0.5]], np.float32)
    K = np.array([[100, 0, 40], [0, 100, 32], [0, 0, 1]], np.float64)
    meta = synth.make_meta(K, 1)
    return label, vertex, extents, meta, int(inside.sum())


@pytest.mark.parametrize("skip", [1, 3])
def test_disc_peaks_at_centre(orc, skip):
    label, vertex, extents, meta, npx = _disc()
    assert npx > 500  # present (label threshold, cu.cc:656)
    counts, dsum, nv = orc.hough_class_counts(label[0], vertex[0], extents, meta[0].reshape(-1), 1, skip)
    assert nv == (npx + skip - 1) // skip
    # the centre pixel (40, 30) is voter #k of the raster-ordered list; its own
    # direction is (0,0) -> NaN cosine -> it votes nowhere
    order = np.flatnonzero(label[0].reshape(-1) == 1)
    k = int(np.flatnonzero(order == 30 * 80 + 40)[0])
    expected = nv - (1 if k % skip == 0 else 0)
    assert counts[30, 40] == expected
    assert counts.max() == expected and (counts == expected).sum() == 1
    assert dsum[30, 40] == float(expected)  # d = 1 per vote, exact

    # whole op, test mode: one RoI at the centre, bb = 2 * radius, d = 1
    box, pose, tgt, wgt, dom, n = orc.hough_voting(label, vertex, extents, meta, np.zeros((0, 13), np.float32),
                                                   0, -1.0, 0.02, skip)
    assert n == 1
    # bb = 2 * max |dx|, |dy| over the sampled voters (all in the cone at the
    # centre and inside T(1) ~ 40.6 px), i.e. 28 at skip 1
    samp = order[::skip]
    sx, sy = samp % 80, samp // 80
    bw, bh = 2.0 * np.abs(sx - 40).max(), 2.0 * np.abs(sy - 30).max()
    if skip == 1:
        assert bw == bh == 28.0
    np.testing.assert_allclose(box[0], [0, 1, 40 - 0.55 * bw, 30 - 0.55 * bh, 40 + 0.55 * bw, 30 + 0.55 * bh,
                                        expected], rtol=0, atol=1e-5)
    np.testing.assert_allclose(pose[0], [1, 0, 0, 0, 0.0, (30 - 32) / 100.0, 1.0], rtol=0, atol=1e-7)
    # test mode writes no domain/target/weight (cu.cc:556-575): zeroed temps
    assert dom[0] == 0 and not tgt.any() and not wgt.any()


def test_disc_train_mode_targets(orc):
    """Train mode: 9 rows per max; GT of the same class/image with IoU > 0.2
    sets targets/weights on all 9 rows (cu.cc:440-466); domain = 0 with GT."""
    label, vertex, extents, meta, _ = _disc(rad=24)  # RoI ~53 px vs the ~70 px projected GT box
    q = np.array([0.95, 0.1, -0.2, 0.2]); q /= np.linalg.norm(q)
    gt = np.array([[0, 1, 0, 0, 0, 0, *q, 0.0, -0.02, 1.0]], np.float32)
    box, pose, tgt, wgt, dom, n = orc.hough_voting(label, vertex, extents, meta, gt, 1, -1.0, 0.02, 1)
    assert n == 9
    np.testing.assert_array_equal(tgt[:, 4:8], np.tile(q.astype(np.float32), (9, 1)))
    np.testing.assert_array_equal(wgt[:, 4:8], np.ones((9, 4), np.float32))
    assert not tgt[:, :4].any() and not tgt[:, 8:].any()
    assert (dom == 0).all()
    # jitter rows keep the class/batch columns and the score
    assert (box[:, 0] == 0).all() and (box[:, 1] == 1).all() and (box[:, 6] == box[0, 6]).all()
    # wrong class in GT -> no targets, still domain 0 (GT present)
    gt2 = gt.copy(); gt2[0, 1] = 2
    _, _, tgt2, wgt2, dom2, _ = orc.hough_voting(label, vertex, extents, meta, gt2, 1, -1.0, 0.02, 1)
    assert not tgt2.any() and not wgt2.any() and (dom2 == 0).all()


def test_no_objects_dummy_row(orc):
    """No class above the label threshold -> a single all-zero row
    (hough_voting_gpu_op.cc:382-383)."""
    label = np.zeros((2, 20, 30), np.int32)
    label[0, :5, :5] = 1  # 25 px < 500
    vertex = np.zeros((2, 20, 30, 6), np.float32)
    extents = np.ones((2, 3), np.float32)
    meta = synth.make_meta(np.eye(3) * 50 + np.array([[0, 0, 15], [0, 0, 10], [0, 0, -49]]), 2)
    box, pose, tgt, wgt, dom, n = orc.hough_voting(label, vertex, extents, meta, np.zeros((0, 13), np.float32),
                                                   1, -1.0, 0.02, 1)
    assert n == 0 and box.shape == (1, 7) and not box.any() and not pose.any() and dom[0] == 0


# ---------------------------------------------------------------------------
# (ii) RoI pooling on iota features: known bins / argmax / gradient routing
def test_roi_pool_iota(orc):
    H = W = 16
    C = 2
    data = np.zeros((1, H, W, C), np.float32)
    hh, ww = np.mgrid[0:H, 0:W]
    for c in range(C):
        data[0, :, :, c] = hh * W + ww + 1000 * c
    rois = np.array([[0, 3, 0, 0, 13, 13]], np.float32)  # 14 x 14 px at scale 1 -> 2 x 2 bins
    top, arg = orc.roi_pool_fwd(data, rois, 7, 7, 1.0)
    for ph in range(7):
        for pw in range(7):
            h, w = 2 * ph + 1, 2 * pw + 1  # bottom-right of each bin holds the max
            for c in range(C):
                assert top[0, ph, pw, c] == h * W + w + 1000 * c
                assert arg[0, ph, pw, c] == (h * W + w) * C + c  # flat NHWC index within the image
    g = orc.roi_pool_bwd(np.ones_like(top), arg, data.shape, rois, 7, 7, 1.0)
    expect = np.zeros_like(data)
    expect[0, 1::2, 1::2, :] = 1.0
    expect[0, 14:, :, :] = 0
    expect[0, :, 14:, :] = 0
    np.testing.assert_array_equal(g, expect)
    # pool_channel = 1 pools only channel `cls` (rois[:,1]) -> one output channel
    top1, arg1 = orc.roi_pool_fwd(data, np.array([[0, 1, 0, 0, 13, 13]], np.float32), 7, 7, 1.0, pool_channel=1)
    assert top1.shape == (1, 7, 7, 1) and top1[0, 0, 0, 0] == 1 * W + 1 + 1000


def test_roi_pool_round_half_away(orc):
    """roi start/end = round(coord * scale), half away from zero
    (roi_pooling_op_gpu.cu.cc:48-51): x1 = 2.5 -> 3, y1 = -0.5 -> -1."""
    H = W = 16
    data = np.zeros((1, H, W, 1), np.float32)
    hh, ww = np.mgrid[0:H, 0:W]
    data[0, :, :, 0] = hh * W + ww
    top, arg = orc.roi_pool_fwd(data, np.array([[0, 0, 2.5, -0.5, 9.5, 6.5]], np.float32), 7, 7, 1.0)
    # bin (0,0): rows [max(-1 + 0, 0), -1 + ceil(9/7)) = [0, 1), cols [3, 3 + ceil(8/7)) = [3, 5)
    assert top[0, 0, 0, 0] == 0 * W + 4 and arg[0, 0, 0, 0] == 4
    # an RoI fully outside the map -> empty bins: 0 / -1
    top2, arg2 = orc.roi_pool_fwd(data, np.array([[0, 0, 40, 40, 50, 50]], np.float32), 7, 7, 1.0)
    assert not top2.any() and (arg2 == -1).all()


# ---------------------------------------------------------------------------
# (iii)/(iv) ADD loss: zero at the target, closed form for a 90 degree z turn
def _add_case(pred_q, tgt_q, pts, sym):
    C = 2
    pred = np.zeros((1, 4 * C), np.float32)
    tgt = np.zeros((1, 4 * C), np.float32)
    wgt = np.zeros((1, 4 * C), np.float32)
    pred[0, 4:8], tgt[0, 4:8], wgt[0, 4:8] = pred_q, tgt_q, 1
    points = np.zeros((C, len(pts), 3), np.float32)
    points[1] = pts
    return pred, tgt, wgt, points, np.array([0, sym], np.float32)


def test_add_zero_at_target(orc):
    rng = np.random.default_rng(3)
    q = rng.normal(size=4).astype(np.float32)
    q /= np.linalg.norm(q)
    pts = rng.normal(size=(50, 3)).astype(np.float32)
    for sym in (0, 1):
        loss, diff, rows = orc.average_distance_loss(*_add_case(q, q, pts, sym), 0.01)
        assert loss[0] == 0 and not diff.any()


def test_add_closed_form_quarter_turn(orc):
    s = np.float32(np.sqrt(0.5))
    pts = np.eye(3, dtype=np.float32)
    ident = np.array([1, 0, 0, 0], np.float32)
    rz90 = np.array([s, 0, 0, s], np.float32)  # 90 deg about z
    # ADD: |X - Rz X|^2 = 2 (x^2 + y^2) -> 2, 2, 0 ; loss = sum(d - m) / (2 R P), d >= m
    loss, diff, _ = orc.average_distance_loss(*_add_case(ident, rz90, pts, 0), 0.01)
    np.testing.assert_allclose(loss[0], (2 - 0.01) * 2 / 6, rtol=1e-6)
    # ADD-S: nearest target point: (1,0,0) -> min(2, 4, 2) = 2, (0,1,0) -> 0, (0,0,1) -> 0
    loss_s, _, _ = orc.average_distance_loss(*_add_case(ident, rz90, pts, 1), 0.01)
    np.testing.assert_allclose(loss_s[0], (2 - 0.01) / 6, rtol=1e-6)


def test_add_gradient_finite_difference(orc):
    """bottom_diff is the gradient of the loss w.r.t. the (unnormalised)
    predicted quaternion (cu.cc:97-139, 183-203)."""
    rng = np.random.default_rng(4)
    pts = rng.normal(size=(40, 3)).astype(np.float32)
    tq = rng.normal(size=4); tq /= np.linalg.norm(tq)
    pq = tq + rng.normal(scale=0.3, size=4)
    case = _add_case(pq.astype(np.float32), tq.astype(np.float32), pts, 0)
    loss, diff, _ = orc.average_distance_loss(*case, 0.0)
    h = 1e-3
    for k in range(4):
        p1, p2 = case[0].copy(), case[0].copy()
        p1[0, 4 + k] += h
        p2[0, 4 + k] -= h
        l1 = orc.average_distance_loss(p1, *case[1:], 0.0)[0][0]
        l2 = orc.average_distance_loss(p2, *case[1:], 0.0)[0][0]
        np.testing.assert_allclose(diff[0, 4 + k], (l1 - l2) / (2 * h), rtol=2e-2, atol=1e-4)


def test_add_first_weighted_class_wins(orc):
    """Only the first class with weight > 0 in a row is used (cu.cc:48-92)."""
    rng = np.random.default_rng(5)
    C = 3
    pred = rng.normal(size=(1, 4 * C)).astype(np.float32)
    tgt = rng.normal(size=(1, 4 * C)).astype(np.float32)
    wgt = np.zeros((1, 4 * C), np.float32)
    wgt[0, 4:12] = 1
    pts = rng.normal(size=(C, 10, 3)).astype(np.float32)
    loss, diff, _ = orc.average_distance_loss(pred, tgt, wgt, pts, np.zeros(C, np.float32), 0.0)
    assert diff[0, 4:8].any() and not diff[0, 8:].any() and not diff[0, :4].any()


# ---------------------------------------------------------------------------
# (v) backprojection with an identity pose: known pixel hits
def test_backproject_identity(orc):
    B, H, W, Ch, NC, G = 1, 6, 3, 2, 2, 4
    rng = np.random.default_rng(6)
    data = rng.normal(size=(B, H, W, Ch)).astype(np.float32)
    label = rng.normal(size=(B, H, W, NC)).astype(np.float32)
    depth = np.full((B, H, W, 1), 10.0, np.float32)
    depth[0, 2, 1, 0] = 11.0  # fails |depth - Z| < threshold
    K = np.diag([10.0, 10.0, 1.0])
    # voxel (d, h, w) -> X = d, Y = h, Z = 10 (step_z 0) -> pixel (x, y) = (d, h)
    meta = synth.make_meta(K, B, voxel=((1, 1, 0), (0, 0, 10)))
    label3d = rng.normal(size=(B, G, G, G, NC)).astype(np.float32)
    td, tl, tf = orc.backproject_fwd(data, label, depth, meta, label3d, G, 0, 0.5)
    for d in range(G):
        for h in range(G):
            for w in range(G):
                hit = d < W and h < H and not (d == 1 and h == 2)
                if hit:
                    np.testing.assert_array_equal(td[0, d, h, w], data[0, h, d])
                    np.testing.assert_array_equal(tl[0, d, h, w], label[0, h, d])
                    assert (tf[0, d, h, w] == 1).all()
                else:
                    assert not td[0, d, h, w].any() and not tf[0, d, h, w].any()
                    np.testing.assert_array_equal(tl[0, d, h, w], label3d[0, d, h, w])
    # backward: pixel (w, h) at depth 10 -> voxel (w, h, 0) when inside the grid
    meta_b = synth.make_meta(K, B, voxel=((1, 1, 1), (0, 0, 10)))
    top = rng.normal(size=(B, G, G, G, Ch)).astype(np.float32)
    gb = orc.backproject_bwd(top, np.full((B, H, W, 1), 10.0, np.float32), meta_b, H, W, G)
    for h in range(H):
        for w in range(W):
            if w < G and h < G:
                np.testing.assert_allclose(gb[0, h, w], top[0, w, h, 0], rtol=0, atol=0)
            else:
                assert not gb[0, h, w].any()
