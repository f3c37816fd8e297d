"""GPU parity for RoI pooling, ADD loss, backprojection and the pose-head GEMM
against the oracle (or an fp64 numpy reference for the GEMM)."""
import os

import numpy as np
import pytest
import torch

from posecnn_amd import synth
from posecnn_amd.roi_pooling_layer import roi_pooling_op as rp
from posecnn_amd.average_distance_loss import average_distance_loss_op as adl
from posecnn_amd.backprojecting_layer import backprojecting_op as bp
from posecnn_amd import pose_head as ph

pytestmark = pytest.mark.gpu
D = torch.device("cuda")


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(D)


def _rois(rng, R, B, H, W, scale_img):
    x1 = rng.uniform(-20, W * scale_img - 10, R)
    y1 = rng.uniform(-20, H * scale_img - 10, R)
    w = rng.uniform(1, 200, R)
    h = rng.uniform(1, 200, R)
    b = np.sort(rng.integers(0, B, R))
    cls = rng.integers(0, 8, R)
    return np.stack([b, cls, x1, y1, x1 + w, y1 + h, np.zeros(R)], 1).astype(np.float32)


@pytest.mark.parametrize("pool_channel", [0, 1])
def test_roi_pool_fwd_bwd(hip, orc, pool_channel):
    rng = np.random.default_rng(0)
    B, H, W, C = 3, 30, 40, 64 if not pool_channel else 8
    data = rng.normal(size=(B, H, W, C)).astype(np.float32)
    data[0, :4, :4] = 1.0  # ties -> first max
    rois = _rois(rng, 37, B, H, W, 16)
    top, arg = rp.roi_pool(T(data), T(rois), 7, 7, 1.0 / 16, pool_channel)
    ot, oa = orc.roi_pool_fwd(data, rois, 7, 7, 1.0 / 16, pool_channel)
    np.testing.assert_array_equal(top.cpu().numpy(), ot)
    np.testing.assert_array_equal(arg.cpu().numpy(), oa)
    g = rng.normal(size=ot.shape).astype(np.float32)
    dd = rp.roi_pool_grad(T(data), T(rois), arg, T(g), 7, 7, 1.0 / 16, pool_channel)
    od = orc.roi_pool_bwd(g, oa, data.shape, rois, 7, 7, 1.0 / 16, pool_channel)
    np.testing.assert_array_equal(dd.cpu().numpy(), od)


@pytest.mark.parametrize("C,B,H,W,scale", [(512, 2, 60, 80, 1 / 8), (68, 3, 30, 40, 1 / 16), (260, 2, 13, 21, 1 / 4),
                                            (96, 2, 7, 9, 1 / 2), (66, 2, 30, 40, 1 / 16), (3, 2, 30, 40, 1 / 16)])
def test_roi_pool_bwd_overlap(hip, orc, C, B, H, W, scale):
    """Heavily overlapping RoIs (jittered copies, as the train-mode Hough op
    emits), tiny and huge bins, RoIs past the map edges, ragged tiles and
    channel chunks; then arbitrary (malformed) argmax values — the backward
    must follow the reference's own membership tests, not the forward's."""
    rng = np.random.default_rng(int(C) * 7 + H)
    data = rng.normal(size=(B, H, W, C)).astype(np.float32)
    data[:, 2:6, 3:9] = 0.5  # plateaus -> first-max ties
    s = 1.0 / scale
    base = _rois(rng, 12, B, H, W, s)
    rows = []
    for r in base:
        for dx in (-0.05, 0.0, 0.05):
            for dy in (-0.05, 0.0):
                q = r.copy()
                w, h = q[4] - q[2], q[5] - q[3]
                q[2] += dx * w; q[4] += dx * w; q[3] += dy * h; q[5] += dy * h
                rows.append(q)
    rois = np.array(rows, np.float32)
    rois = rois[np.argsort(rois[:, 0], kind="stable")]
    top, arg = rp.roi_pool(T(data), T(rois), 7, 7, scale, 0)
    ot, oa = orc.roi_pool_fwd(data, rois, 7, 7, scale, 0)
    np.testing.assert_array_equal(arg.cpu().numpy(), oa)
    g = rng.normal(size=ot.shape).astype(np.float32)
    dd = rp.roi_pool_grad(T(data), T(rois), arg, T(g), 7, 7, scale, 0)
    od = orc.roi_pool_bwd(g, oa, data.shape, rois, 7, 7, scale, 0)
    np.testing.assert_array_equal(dd.cpu().numpy(), od)
    bad = oa.copy()
    sel = rng.random(bad.shape) < 0.3
    bad[sel] = rng.integers(-1, H * W * C, int(sel.sum()))
    dd = rp.roi_pool_grad(T(data), T(rois), T(bad), T(g), 7, 7, scale, 0)
    od = orc.roi_pool_bwd(g, bad, data.shape, rois, 7, 7, scale, 0)
    np.testing.assert_array_equal(dd.cpu().numpy(), od)


def test_roi_pool_device_count(hip, orc):
    rng = np.random.default_rng(1)
    B, H, W, C = 2, 60, 80, 512
    data = rng.normal(size=(B, H, W, C)).astype(np.float32)
    rois = _rois(rng, 20, B, H, W, 8)
    n = torch.tensor([13], dtype=torch.int32, device=D)
    top, arg = rp.roi_pool(T(data), T(rois), 7, 7, 1.0 / 8, 0, num_rois=n)
    ot, oa = orc.roi_pool_fwd(data, rois[:13], 7, 7, 1.0 / 8, 0)
    np.testing.assert_array_equal(top[:13].cpu().numpy(), ot)
    g = rng.normal(size=(20,) + ot.shape[1:]).astype(np.float32)
    dd = rp.roi_pool_grad(T(data), T(rois), arg, T(g), 7, 7, 1.0 / 8, 0, num_rois=n)
    od = orc.roi_pool_bwd(g[:13], oa, data.shape, rois[:13], 7, 7, 1.0 / 8, 0)
    np.testing.assert_array_equal(dd.cpu().numpy(), od)


def test_roi_pool_pair(hip, orc):
    """pool5 + pool4 in one pass == the two oracle pools added in fp32, argmax of
    both maps bit-exact, device row count honoured (rows past it untouched)."""
    rng = np.random.default_rng(9)
    B, C = 2, 64
    d5 = rng.normal(size=(B, 30, 40, C)).astype(np.float32)
    d4 = rng.normal(size=(B, 60, 80, C)).astype(np.float32)
    d4[0, 10:20, 10:30] = 0.25  # plateaus -> first-max ties
    rois = _rois(rng, 29, B, 480, 640, 1)
    nr = torch.tensor([23], dtype=torch.int32, device=D)
    top = torch.full((29, 7, 7, C), 7.0, device=D)
    a5 = torch.full((29, 7, 7, C), -7, dtype=torch.int32, device=D)
    a4 = torch.full((29, 7, 7, C), -7, dtype=torch.int32, device=D)
    rp.roi_pool_pair(T(d5), 1.0 / 16, T(d4), 1.0 / 8, T(rois), 7, 7, num_rois=nr, out=(top, a5, a4))
    o5, oa5 = orc.roi_pool_fwd(d5, rois, 7, 7, 1.0 / 16, 0)
    o4, oa4 = orc.roi_pool_fwd(d4, rois, 7, 7, 1.0 / 8, 0)
    np.testing.assert_array_equal(top[:23].cpu().numpy(), (o5 + o4)[:23])
    np.testing.assert_array_equal(a5[:23].cpu().numpy(), oa5[:23])
    np.testing.assert_array_equal(a4[:23].cpu().numpy(), oa4[:23])
    assert (top[23:] == 7.0).all() and (a5[23:] == -7).all()


def test_roi_pool_pair_pixel_argmax(hip, orc):
    """Compact argmax of the fused step (uint16 pixel index, 0xFFFF = empty
    bin): the oracle's flat argmax // C, pooled sums unchanged, and both pool
    backwards on it bit-equal to the oracle's (jittered overlapping RoIs, RoIs
    past the map edges, empty bins, a device row count)."""
    rng = np.random.default_rng(13)
    B, C = 2, 64
    d5 = rng.normal(size=(B, 30, 40, C)).astype(np.float32)
    d4 = rng.normal(size=(B, 60, 80, C)).astype(np.float32)
    d4[1, 10:20, 10:30] = 0.25  # plateaus -> first-max ties
    base = _rois(rng, 9, B, 480, 640, 1)
    rows = []
    for r in base:
        for dx in (-0.05, 0.0, 0.05):
            q = r.copy()
            w = q[4] - q[2]
            q[2] += dx * w; q[4] += dx * w
            rows.append(q)
    rois = np.array(rows, np.float32)
    rois = rois[np.argsort(rois[:, 0], kind="stable")]
    rois[0, 2:6] = [700.0, 500.0, 760.0, 560.0]  # entirely past the map: empty bins
    R, live = len(rois), len(rois) - 2
    nr = torch.tensor([live], dtype=torch.int32, device=D)
    top = torch.full((R, 7, 7, C), 7.0, device=D)
    a5 = torch.full((R, 7, 7, C), -7, dtype=torch.int16, device=D)
    a4 = torch.full((R, 7, 7, C), -7, dtype=torch.int16, device=D)
    rp.roi_pool_pair(T(d5), 1.0 / 16, T(d4), 1.0 / 8, T(rois), 7, 7, num_rois=nr, out=(top, a5, a4))
    o5, oa5 = orc.roi_pool_fwd(d5, rois, 7, 7, 1.0 / 16, 0)
    o4, oa4 = orc.roi_pool_fwd(d4, rois, 7, 7, 1.0 / 8, 0)
    np.testing.assert_array_equal(top[:live].cpu().numpy(), (o5 + o4)[:live])
    px = lambda oa: np.where(oa < 0, 0xFFFF, oa // C).astype(np.int64)
    assert (oa5[:live] < 0).any()
    np.testing.assert_array_equal(a5[:live].cpu().numpy().astype(np.int64) & 0xFFFF, px(oa5[:live]))
    np.testing.assert_array_equal(a4[:live].cpu().numpy().astype(np.int64) & 0xFFFF, px(oa4[:live]))
    assert (a5[live:] == -7).all()
    g = rng.normal(size=(R, 7, 7, C)).astype(np.float32)
    for data, arg, oa, s in ((d5, a5, oa5, 1.0 / 16), (d4, a4, oa4, 1.0 / 8)):
        dd = rp.roi_pool_grad(T(data), T(rois), arg, T(g), 7, 7, s, 0, num_rois=nr)
        od = orc.roi_pool_bwd(g[:live], oa[:live], data.shape, rois[:live], 7, 7, s, 0)
        np.testing.assert_array_equal(dd.cpu().numpy(), od)


def _add_inputs(rng, R, C=22, sym_rows=True):
    pts, sym = synth.rescaled_points(C)
    pred = rng.normal(size=(R, 4 * C)).astype(np.float32) * 0.5
    target = np.zeros((R, 4 * C), np.float32)
    weight = np.zeros((R, 4 * C), np.float32)
    for r in range(R):
        c = [16, 21, 3, 7][r % 4] if sym_rows else int(rng.integers(1, C))
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        if r % 5 != 4:  # some rows without weight
            target[r, 4 * c:4 * c + 4] = q
            weight[r, 4 * c:4 * c + 4] = 1
        p = pred[r, 4 * c:4 * c + 4]
        pred[r, 4 * c:4 * c + 4] = p / np.linalg.norm(p)
    return pred, target, weight, pts, sym


def test_add_loss(hip, orc):
    rng = np.random.default_rng(2)
    pred, target, weight, pts, sym = _add_inputs(rng, 23)
    loss, diff = adl.average_distance_loss(T(pred), T(target), T(weight), T(pts), T(sym), 0.01)
    ol, od, _ = orc.average_distance_loss(pred, target, weight, pts, sym, 0.01)
    np.testing.assert_allclose(loss.cpu().numpy(), ol, rtol=1e-4)
    np.testing.assert_allclose(diff.cpu().numpy(), od, rtol=1e-4, atol=1e-7)
    g = np.array([0.7], np.float32)
    out = adl.average_distance_loss_grad(diff, T(g))
    np.testing.assert_allclose(out.cpu().numpy(), 0.7 * diff.cpu().numpy(), rtol=0, atol=0)


def test_add_loss_prepared_on_side_stream(hip, orc):
    """pcnn_add_loss_prep on another stream + pcnn_add_loss_fwd_prepared ==
    pcnn_add_loss_fwd, bit for bit (device row count, symmetric rows)."""
    rng = np.random.default_rng(21)
    pred, target, weight, pts, sym = _add_inputs(rng, 40)
    nr = torch.tensor([31], dtype=torch.int32, device=D)
    args = (T(pred), T(target), T(weight), T(pts), T(sym), 0.01)
    loss0, diff0 = adl.average_distance_loss(*args, num_rois=nr)
    ws = torch.empty(adl.workspace_bytes(40, 22, pts.shape[1]), dtype=torch.uint8, device=D)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        adl.average_distance_loss_prep(args[2], args[4], pts.shape[1], ws, num_rois=nr)
    torch.cuda.current_stream().wait_stream(side)
    loss1, diff1 = adl.average_distance_loss(*args, num_rois=nr, workspace=ws, prepared=True)
    np.testing.assert_array_equal(loss1.cpu().numpy(), loss0.cpu().numpy())
    np.testing.assert_array_equal(diff1[:31].cpu().numpy(), diff0[:31].cpu().numpy())


def test_add_loss_identity_zero(hip, orc):
    rng = np.random.default_rng(3)
    pred, target, weight, pts, sym = _add_inputs(rng, 8, sym_rows=False)
    pred = target.copy()
    loss, diff = adl.average_distance_loss(T(pred), T(target), T(weight), T(pts), T(sym), 0.01)
    assert float(loss.item()) == 0.0 and not diff.cpu().numpy().any()


def test_add_loss_symmetric_ties(hip, orc):
    """ADD-S first-minimum tie-breaking: lattice model points with pred = identity
    and target = the unnormalised quaternion (1, 0, 0, 1) (exactly 2 x Rot90z in
    float) make exact distance ties between different candidates everywhere —
    across blocks of 4 and across the candidate ranges the lane groups split.
    The gradient of a row depends on which tied candidate wins, so bitwise
    agreement with the sequential strict-< scan of the oracle checks it."""
    rng = np.random.default_rng(11)
    C, P, R = 3, 1500, 6
    pts = np.zeros((C, P, 3), np.float32)
    pts[1] = rng.integers(-3, 4, size=(P, 3)).astype(np.float32)
    pts[2] = rng.integers(-2, 3, size=(P, 3)).astype(np.float32)
    sym = np.array([0, 1, 1], np.float32)
    pred = np.zeros((R, 4 * C), np.float32)
    target = np.zeros((R, 4 * C), np.float32)
    weight = np.zeros((R, 4 * C), np.float32)
    for r in range(R):
        c = 1 + r % 2
        pred[r, 4 * c:4 * c + 4] = [1, 0, 0, 0] if r < 4 else [0, 1, 0, 0]
        target[r, 4 * c:4 * c + 4] = [1, 0, 0, 1] if r % 3 else [0, 0, 1, 1]
        weight[r, 4 * c:4 * c + 4] = 1
    loss, diff = adl.average_distance_loss(T(pred), T(target), T(weight), T(pts), T(sym), 0.01)
    ol, od, _ = orc.average_distance_loss(pred, target, weight, pts, sym, 0.01)
    # the loss does not depend on which tied candidate wins (equal distances):
    # its tolerance covers summation order only; a wrong pick moves a row's
    # gradient by O(1) relative
    np.testing.assert_allclose(loss.cpu().numpy(), ol, rtol=1e-5)
    np.testing.assert_allclose(diff.cpu().numpy(), od, rtol=1e-4, atol=1e-6 * np.abs(od).max())


@pytest.mark.parametrize("P,near", [(4096, True), (4096, False), (2620, True), (4200, False), (700, True),
                                    (100, True), (300, False), (512, True)])
def test_add_loss_symmetric_large(hip, orc, P, near):
    """ADD-S at up to 4200 model points: predictions near the target and
    arbitrary ones, duplicated model points and lattice coordinates (exact
    distance ties), against the oracle's sequential first-minimum scan.  P
    covers whole 256-point chunks only (4096, 512), a short last chunk of <= 128
    points (the one-pair scan: 2620, 4200, 300, 100) and of > 128 (700)."""
    rng = np.random.default_rng(P + int(near))
    C, R = 3, 7
    pts = rng.normal(size=(C, P, 3)).astype(np.float32)
    pts[1, P // 2:P // 2 + 40] = pts[1, 10:50]          # duplicate points -> tied candidates
    pts[2] = np.round(pts[2] * 4) / 4                    # lattice-like coordinates -> equal x values
    sym = np.array([0, 1, 1], np.float32)
    pred = np.zeros((R, 4 * C), np.float32)
    target = np.zeros((R, 4 * C), np.float32)
    weight = np.zeros((R, 4 * C), np.float32)
    for r in range(R):
        c = 1 + r % 2
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        dq = q + (rng.normal(size=4) * 0.02 if near else rng.normal(size=4))
        target[r, 4 * c:4 * c + 4] = q
        pred[r, 4 * c:4 * c + 4] = dq / np.linalg.norm(dq)
        weight[r, 4 * c:4 * c + 4] = 1
    loss, diff = adl.average_distance_loss(T(pred), T(target), T(weight), T(pts), T(sym), 0.01)
    ol, od, _ = orc.average_distance_loss(pred, target, weight, pts, sym, 0.01)
    np.testing.assert_allclose(loss.cpu().numpy(), ol, rtol=1e-5)
    np.testing.assert_allclose(diff.cpu().numpy(), od, rtol=1e-4, atol=1e-6 * np.abs(od).max())


def _add_s_f64(pred, target, weight, pts, margin):
    """ADD-S loss and bottom_diff in float64 from fp32 first-minimum picks: the
    nearest GT-rotated point by the reference's fp32 expression (numpy does not
    contract, so these are the oracle's picks), then the per-point terms of
    cu.cc:174-203 summed in float64 -- a reference free of the fp32 sums'
    order, so a single different pick shows up far above its tolerance."""
    R, PC = pred.shape
    P = pts.shape[1]
    loss = 0.0
    diff = np.zeros((R, PC))

    def rot(q):
        s, u, v, w = q
        return np.array([[s * s + u * u - v * v - w * w, 2 * (u * v - s * w), 2 * (u * w + s * v)],
                         [2 * (u * v + s * w), s * s - u * u + v * v - w * w, 2 * (v * w - s * u)],
                         [2 * (u * w - s * v), 2 * (v * w + s * u), s * s - u * u - v * v + w * w]], np.float32)
    for r in range(R):
        cls = np.flatnonzero(weight[r, 0::4] > 0)
        if len(cls) == 0:
            continue
        c = cls[0]
        s, u, v, w = (float(x) for x in pred[r, 4 * c:4 * c + 4])
        X = pts[c]
        Rp, Rg = rot(pred[r, 4 * c:4 * c + 4]), rot(target[r, 4 * c:4 * c + 4])
        q = np.stack([Rp[i, 0] * X[:, 0] + Rp[i, 1] * X[:, 1] + Rp[i, 2] * X[:, 2] for i in range(3)], 1)
        g = np.stack([Rg[i, 0] * X[:, 0] + Rg[i, 1] * X[:, 1] + Rg[i, 2] * X[:, 2] for i in range(3)], 1)
        e = [q[:, None, i] - g[None, :, i] for i in range(3)]
        d = e[0] * e[0] + e[1] * e[1] + e[2] * e[2]
        j = np.argmin(d, 1)
        dist = d[np.arange(P), j]
        on = ~(dist < margin)
        loss += np.sum((dist[on].astype(np.float64) - margin) / (2.0 * R * P))
        df = (q - g[j]).astype(np.float64)[on]
        Xo = X.astype(np.float64)[on]
        D = [np.array(m, np.float64).reshape(3, 3) for m in (
            [2 * s, -2 * w, 2 * v, 2 * w, 2 * s, -2 * u, -2 * v, 2 * u, 2 * s],
            [2 * u, 2 * v, 2 * w, 2 * v, -2 * u, -2 * s, 2 * w, 2 * s, -2 * u],
            [-2 * v, 2 * u, 2 * s, 2 * u, 2 * v, 2 * w, -2 * s, 2 * w, -2 * v],
            [-2 * w, -2 * s, 2 * u, 2 * s, -2 * w, 2 * v, 2 * u, 2 * v, 2 * w])]
        for i in range(4):
            diff[r, 4 * c + i] = np.einsum("na,ab,nb->", df, D[i], Xo) / (R * P)
    return loss, diff


@pytest.mark.parametrize("scale", [1e-3, 0.05, 3.0])
def test_add_loss_symmetric_unnormalised(hip, orc, scale):
    """ADD-S on unnormalised predicted quaternions -- the random-init head's outputs: query
    points shrunk towards the origin (|q|^2 = 1e-6 .. 2.5e-3) or spread past
    the candidates (|q|^2 ~ 9) -- and on the LOV models of the two symmetric
    classes.  Against the oracle (whose sequential fp32 sums of R P nearly
    equal terms drift by ~1e-5 when the queries collapse: rtol 1e-4) and
    against a float64 evaluation of the oracle's picks (rtol 2e-6)."""
    rng = np.random.default_rng(int(scale * 1000) + 5)
    pts, sym = synth.rescaled_points(22)
    R, C = 24, 22
    pred = (rng.normal(size=(R, 4 * C)) * scale).astype(np.float32)
    target = np.zeros((R, 4 * C), np.float32)
    weight = np.zeros((R, 4 * C), np.float32)
    for r in range(R):
        c = (16, 21)[r % 2]
        q = rng.normal(size=4)
        target[r, 4 * c:4 * c + 4] = q / np.linalg.norm(q)
        weight[r, 4 * c:4 * c + 4] = 1
    loss, diff = adl.average_distance_loss(T(pred), T(target), T(weight), T(pts), T(sym), 0.01)
    loss, diff = loss.cpu().numpy(), diff.cpu().numpy()
    ol, od, _ = orc.average_distance_loss(pred, target, weight, pts, sym, 0.01)
    np.testing.assert_allclose(loss, ol, rtol=1e-4)
    np.testing.assert_allclose(diff, od, rtol=1e-4, atol=1e-6 * np.abs(od).max())
    l64, d64 = _add_s_f64(pred, target, weight, pts, 0.01)
    np.testing.assert_allclose(loss[0], l64, rtol=2e-6)
    np.testing.assert_allclose(diff, d64, rtol=2e-5, atol=1e-6 * np.abs(d64).max())


@pytest.mark.parametrize("Ch,NC,ks", [(16, 5, 1), (12, 8, 1), (64, 16, 2), (20, 4, 0), (8, 8, 3)])
def test_backproject(hip, orc, Ch, NC, ks):
    """Scalar kernels (NC = 5) and the float4 vector forms (lanes per row 4 /
    16 / 8 / 2), kernel sizes 0-2 (compile-time) and 3 (runtime), bit-exact
    against the restated op."""
    rng = np.random.default_rng(4)
    B, H, W, G = 2, 48, 64, 12
    K = np.array([[80.0, 0, 32], [0, 80.0, 24], [0, 0, 1]])
    meta = synth.make_meta(K, B, voxel=([0.1, 0.08, 0.1], [-0.6, -0.48, 0.5]))
    depth = rng.uniform(0.5, 1.7, size=(B, H, W, 1)).astype(np.float32)
    data = rng.normal(size=(B, H, W, Ch)).astype(np.float32)
    label = rng.uniform(size=(B, H, W, NC)).astype(np.float32)
    l3 = rng.uniform(size=(B, G, G, G, NC)).astype(np.float32)
    td, tl, tf = bp.backproject(T(data), T(label), T(depth), T(meta), T(l3), G, ks, 0.3)
    od, ol, of = orc.backproject_fwd(data, label, depth, meta, l3, G, ks, 0.3)
    np.testing.assert_array_equal(td.cpu().numpy(), od)
    np.testing.assert_array_equal(tl.cpu().numpy(), ol)
    np.testing.assert_array_equal(tf.cpu().numpy(), of)
    assert of.any() and not of.all()
    g = rng.normal(size=od.shape).astype(np.float32)
    gd = bp.backproject_grad(T(data), T(depth), T(meta), T(g), G, 1, 0.3)
    np.testing.assert_array_equal(gd.cpu().numpy(), orc.backproject_bwd(g, depth, meta, H, W, G))


@pytest.mark.parametrize("background", [None, (1.0, 2.0)])
def test_backproject_linemod_config(hip, orc, background):
    """configs[4] sizes for one image: 640x480 LINEMOD frame (15 objects' extents,
    4 objects, rendered depth; with a floor plane behind them, the bench's
    workload, or depth holes around them), G = 64, Ch = 64, NC = 16,
    kernel_size 1, threshold 0.02, forward and backward
    bit-exact."""
    rng = np.random.default_rng(45)
    mdl = synth.models()
    G, Ch, NC = 64, 64, 16
    voxel = ([1.2 / G, 0.9 / G, 1.2 / G], [-0.6, -0.45, 0.9])  # the camera frustum at 0.9-2.1 m (bench.py)
    fr = synth.make_frames(1, 480, 640, num_classes=16, objects_per_image=4, seed=5,
                           extents=mdl["linemod_extents"], with_depth=True, voxel=voxel,
                           depth_background=background)
    depth = fr["depth"]
    data = rng.normal(size=(1, 480, 640, Ch)).astype(np.float32)
    label = rng.uniform(size=(1, 480, 640, NC)).astype(np.float32)
    l3 = rng.uniform(size=(1, G, G, G, NC)).astype(np.float32)
    td, tl, tf = bp.backproject(T(data), T(label), T(depth), T(fr["meta"]), T(l3), G, 1, 0.02)
    od, ol, of = orc.backproject_fwd(data, label, depth, fr["meta"], l3, G, 1, 0.02)
    np.testing.assert_array_equal(td.cpu().numpy(), od)
    np.testing.assert_array_equal(tl.cpu().numpy(), ol)
    np.testing.assert_array_equal(tf.cpu().numpy(), of)
    assert of.any() and not of.all()
    if background is not None:  # the scene's surfaces cross the grid: percent-level hits
        assert (of[..., 0] > 0).mean() > 0.01
    g = rng.normal(size=od.shape).astype(np.float32)
    gd = bp.backproject_grad(T(data), T(depth), T(fr["meta"]), T(g), G, 1, 0.02)
    np.testing.assert_array_equal(gd.cpu().numpy(), orc.backproject_bwd(g, depth, fr["meta"], 480, 640, G))


# Tolerances: precision 0 is fp32 MFMA (fp32 products, fp32 accumulation);
# precision 2 is the exact three-way split-bf16 x6 MFMA (products to within
# 2^-24 |a||b|, fp32 accumulation) and is held to the same fp32 bound;
# precision 1 is the split-bf16 x3 MFMA (hi*hi + hi*lo + lo*hi, fp32
# accumulation): per-product relative error <= ~2^-16, so the error of a
# K-term dot product of O(1) values is ~2^-16 * sqrt(K) -- held to the
# north-star 1e-4 relative bound, with atol scaled by sqrt(K).
def _gemm_tol(prec, K):
    return dict(rtol=2e-5, atol=2e-4) if prec != 1 else dict(rtol=1e-4, atol=1e-4 * np.sqrt(K))


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize("at,bt", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_layouts(hip, at, bt, prec):
    rng = np.random.default_rng(5)
    M, N, K = 200, 300, 1000
    A = rng.normal(size=(M, K)).astype(np.float32)
    A2 = rng.normal(size=(M, K)).astype(np.float32)
    B = rng.normal(size=(K, N)).astype(np.float32)
    bias = rng.normal(size=N).astype(np.float32)
    As = A.T.copy() if at else A
    A2s = A2.T.copy() if at else A2
    Bs = B.T.copy() if bt else B
    C = torch.empty((M, N), dtype=torch.float32, device=D)
    ph.gemm(T(As), T(Bs), C, a_trans=at, b_trans=bt, A2=T(A2s), bias=T(bias), act=1, precision=prec)
    ref = np.maximum((A.astype(np.float64) + A2) @ B + bias, 0)
    np.testing.assert_allclose(C.cpu().numpy(), ref, **_gemm_tol(prec, 2 * K))


@pytest.mark.parametrize("prec", [0, 1, 2])
def test_gemm_device_dims_split(hip, prec):
    rng = np.random.default_rng(6)
    M, N, K = 1152, 256, 8192
    A = rng.normal(size=(M, K)).astype(np.float32)
    B = rng.normal(size=(K, N)).astype(np.float32)
    mask = rng.normal(size=(M, N)).astype(np.float32)
    Mdev = torch.tensor([333], dtype=torch.int32, device=D)
    C = torch.zeros((M, N), dtype=torch.float32, device=D)
    ph.gemm(T(A), T(B), C, mask=T(mask), M_dev=Mdev, precision=prec)
    ref = (A[:333].astype(np.float64) @ B) * (mask[:333] > 0)
    np.testing.assert_allclose(C[:333].cpu().numpy(), ref, **(dict(rtol=2e-5, atol=5e-4) if prec != 1 else _gemm_tol(1, K)))
    assert not C[333:].cpu().numpy().any()
    # K on device (weight-gradient form: C = A^T B over the first 77 rows)
    Kdev = torch.tensor([77], dtype=torch.int32, device=D)
    C2 = torch.empty((K, N), dtype=torch.float32, device=D)
    ph.gemm(T(A), T(B[:M].copy()), C2, a_trans=1, K_dev=Kdev, M=K, N=N, K=M, precision=prec)
    ref2 = A[:77].T.astype(np.float64) @ B[:77]
    np.testing.assert_allclose(C2.cpu().numpy(), ref2, **(dict(rtol=2e-5, atol=5e-4) if prec != 1 else _gemm_tol(1, 77)))


@pytest.mark.parametrize("prec", [1, 2])
def test_gemm_weight_grad_unsplit(hip, prec):
    """Unsplit persistent grid in the fc6 / fc7 dW form: C = A^T B over a
    device-side row count, 16 x 8 tiles of 256, K = 405 rows of 1152."""
    rng = np.random.default_rng(9)
    R, M, N = 1152, 4096, 2048
    A = rng.normal(size=(R, M)).astype(np.float32)
    B = rng.normal(size=(R, N)).astype(np.float32)
    Kdev = torch.tensor([405], dtype=torch.int32, device=D)
    C = torch.empty((M, N), dtype=torch.float32, device=D)
    ph.gemm(T(A), T(B), C, a_trans=1, K_dev=Kdev, M=M, N=N, K=R, precision=prec)
    ref = A[:405].T.astype(np.float64) @ B[:405]
    np.testing.assert_allclose(C.cpu().numpy(), ref, **_gemm_tol(prec, 405))


@pytest.mark.parametrize("prec", [1, 2])
@pytest.mark.parametrize("bt", [0, 1])
def test_gemm_live_row_blocks(hip, bt, prec):
    """Device-side row counts that leave every number (0-4) of live 32-row
    accumulator blocks in a wave's half of a 256-row tile (the K loop is
    specialised on that count): fc7-like capacity shape, bias + relu + mask."""
    rng = np.random.default_rng(11)
    M, N, K = 1152, 512, 640
    A = rng.normal(size=(M, K)).astype(np.float32)
    B = rng.normal(size=(K, N)).astype(np.float32)
    bias = rng.normal(size=N).astype(np.float32)
    mask = rng.normal(size=(M, N)).astype(np.float32)
    tA, tB = T(A), T(B.T.copy() if bt else B)
    for live in (1, 31, 33, 70, 100, 128, 129, 200, 257, 290, 333, 405, 449, 511, 512, 700, 1152):
        Mdev = torch.tensor([live], dtype=torch.int32, device=D)
        C = torch.zeros((M, N), dtype=torch.float32, device=D)
        ph.gemm(tA, tB, C, b_trans=bt, bias=T(bias), act=1, mask=T(mask), M_dev=Mdev, precision=prec)
        ref = np.maximum(A[:live].astype(np.float64) @ B + bias, 0) * (mask[:live] > 0)
        np.testing.assert_allclose(C[:live].cpu().numpy(), ref, err_msg=f"live={live}", **_gemm_tol(prec, K))
        assert not C[live:].cpu().numpy().any(), live


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize("at,bt", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_ragged_padded(hip, at, bt, prec):
    """Ragged M/N/K (no multiple of 4 or of the tile) through padded leading dims."""
    rng = np.random.default_rng(8)
    M, N, K = 203, 301, 999
    A = rng.normal(size=(M, K)).astype(np.float32)
    B = rng.normal(size=(K, N)).astype(np.float32)

    def padded(X, trans):
        X = X.T if trans else X
        buf = torch.zeros((X.shape[0], (X.shape[1] + 7) // 4 * 4), dtype=torch.float32, device=D)
        buf[:, :X.shape[1]] = T(X)
        return buf[:, :X.shape[1]]
    C = torch.empty((M, N), dtype=torch.float32, device=D)
    ph.gemm(padded(A, at), padded(B, bt), C, a_trans=at, b_trans=bt, M=M, N=N, K=K, precision=prec)
    ref = A.astype(np.float64) @ B
    np.testing.assert_allclose(C.cpu().numpy(), ref, **_gemm_tol(prec, K))


@pytest.mark.parametrize("prec", [1, 2])
@pytest.mark.parametrize("shape", [(332, 88, 1000), (204, 300, 100), (88, 500, 404), (1152, 4096, 88)])
@pytest.mark.parametrize("at,bt", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_small_tile(hip, shape, at, bt, prec):
    """Shapes with an edge <= 128 (the fc8 GEMMs) run the 128 x 128 x3 tile:
    A + A2, bias, relu, mask and a device-side M (333 live rows)."""
    rng = np.random.default_rng(10)
    M, N, K = shape
    A = rng.normal(size=(M, K)).astype(np.float32)
    A2 = rng.normal(size=(M, K)).astype(np.float32)
    B = rng.normal(size=(K, N)).astype(np.float32)
    bias = rng.normal(size=N).astype(np.float32)
    mask = rng.normal(size=(M, N)).astype(np.float32)
    live = min(M, 333)
    Mdev = torch.tensor([live], dtype=torch.int32, device=D)
    C = torch.zeros((M, N), dtype=torch.float32, device=D)
    ph.gemm(T(A.T.copy() if at else A), T(B.T.copy() if bt else B), C, a_trans=at, b_trans=bt,
            A2=T(A2.T.copy() if at else A2), bias=T(bias), act=1, mask=T(mask), M_dev=Mdev, precision=prec)
    ref = np.maximum((A[:live].astype(np.float64) + A2[:live]) @ B + bias, 0) * (mask[:live] > 0)
    np.testing.assert_allclose(C[:live].cpu().numpy(), ref, **_gemm_tol(prec, 2 * K))
    assert not C[live:].cpu().numpy().any()


def test_roi_pool_accumulate(hip, orc):
    """pool5 + pool4 produced in place by the second pool (both argmaxes kept)."""
    rng = np.random.default_rng(9)
    B = 2
    c5 = rng.normal(size=(B, 30, 40, 64)).astype(np.float32)
    c4 = rng.normal(size=(B, 60, 80, 64)).astype(np.float32)
    rois = _rois(rng, 17, B, 30, 40, 16)
    top = torch.empty((17, 7, 7, 64), dtype=torch.float32, device=D)
    a5 = torch.empty((17, 7, 7, 64), dtype=torch.int32, device=D)
    a4 = torch.empty_like(a5)
    rp.roi_pool(T(c5), T(rois), 7, 7, 1 / 16, 0, out=(top, a5))
    rp.roi_pool(T(c4), T(rois), 7, 7, 1 / 8, 0, out=(top, a4), accumulate=True)
    o5, oa5 = orc.roi_pool_fwd(c5, rois, 7, 7, 1 / 16)
    o4, oa4 = orc.roi_pool_fwd(c4, rois, 7, 7, 1 / 8)
    np.testing.assert_array_equal(top.cpu().numpy(), o5 + o4)
    np.testing.assert_array_equal(a5.cpu().numpy(), oa5)
    np.testing.assert_array_equal(a4.cpu().numpy(), oa4)


@pytest.mark.parametrize("dbl", [0, 1])
def test_add_loss_division_correctly_rounded(hip, dbl):
    """The ADD loss divides every per-point term by the launch's normaliser
    b = (2) R P (cu.cc:181,196-202) through r = RN(1/b) and two fma
    corrections (average_distance.hip div_rn).  Against IEEE division over
    random x in many binades and quotients with their mantissa near 1 and
    near 2 (where one correction alone is not enough), for the normalisers
    of R = 1..1152 rows of P = 2620 points: bit-exact."""
    import ctypes
    rng = np.random.default_rng(21 + dbl)
    lib = hip
    for R in (1, 3, 9, 405, 1152, 777):
        b = np.float32((2 if dbl else 1) * R * 2620)
        x = (rng.uniform(-1, 1, 200000) * np.exp2(rng.integers(-30, 10, 200000))).astype(np.float32)
        # quotients with mantissa just above 1 and just below 2 (x = b * q)
        q = np.concatenate([1 + rng.uniform(0, 1e-3, 20000), 2 - rng.uniform(0, 1e-3, 20000)])
        q = q * np.exp2(rng.integers(-20, 5, q.size))
        x = np.concatenate([x, (b * q).astype(np.float32), np.nextafter((b * q).astype(np.float32), np.float32(3))])
        xd = torch.from_numpy(x).to(D)
        out = torch.empty_like(xd)
        rc = lib.pcnn_div_rn_check(ctypes.c_void_p(xd.data_ptr()), ctypes.c_float(b), x.size, dbl,
                                   ctypes.c_void_p(out.data_ptr()), None)
        assert rc == 0
        ref = (x.astype(np.float64) / np.float64(b)).astype(np.float32) if dbl else x / b
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"R={R}")


def _add_modes(args, **kw):
    """The loss with the pruned ADD-S search (PCNN_ADD_SEARCH=pruned) and the
    full scan (the default), on the same inputs."""
    out = []
    for mode in ("pruned", "full"):
        os.environ["PCNN_ADD_SEARCH"] = mode
        try:
            loss, diff = adl.average_distance_loss(*args, **kw)
            torch.cuda.synchronize()
            out.append((loss.cpu().numpy(), diff.cpu().numpy()))
        finally:
            os.environ.pop("PCNN_ADD_SEARCH", None)
    return out


@pytest.mark.parametrize("case", ["random", "near", "ties", "small_p", "p4096", "p4100", "nonfinite", "scaled"])
def test_add_s_pruned_search_matches_full_scan(hip, case):
    """The pruned nearest-point search (PCNN_ADD_SEARCH=pruned: Morton-ordered
    blocks with bounding spheres, wave-uniform skips; k_add_search) against
    the reference's full O(P^2) scan (the default): loss and bottom_diff bit for bit -- random and near-correct
    predictions, exact distance ties on a lattice, P below one block row and
    at / past the pruned path's 4096 limit, non-finite rows and points, and
    unnormalised quaternions."""
    rng = np.random.default_rng({"random": 1, "near": 2, "ties": 3, "small_p": 4, "p4096": 5, "p4100": 6,
                                 "nonfinite": 7, "scaled": 8}[case])
    C, R = 4, 37
    P = {"small_p": 13, "p4096": 4096, "p4100": 4100}.get(case, 2620)
    if case == "ties":
        pts = rng.integers(-3, 4, size=(C, P, 3)).astype(np.float32)
    else:
        pts = (rng.normal(size=(C, P, 3)) * np.array([1.0, 2.0, 0.5])).astype(np.float32)
    sym = np.array([0, 1, 1, 0], np.float32)
    pred = np.zeros((R, 4 * C), np.float32)
    target = np.zeros((R, 4 * C), np.float32)
    weight = np.zeros((R, 4 * C), np.float32)
    for r in range(R):
        c = 1 + r % 3
        qt = rng.normal(size=4)
        qt /= np.linalg.norm(qt)
        qp = rng.normal(size=4)
        qp /= np.linalg.norm(qp)
        if case == "near":
            qp = qt + rng.normal(size=4) * 0.02
            qp /= np.linalg.norm(qp)
        if case == "ties":
            qt = np.array([1, 0, 0, 1.0]) if r % 2 else np.array([0, 0, 1, 1.0])
            qp = np.array([1, 0, 0, 0.0]) if r % 3 else np.array([0, 1, 0, 0.0])
        if case == "scaled":
            qp *= 1.0 + r * 0.3
            qt *= 0.7
        pred[r, 4 * c:4 * c + 4] = qp
        target[r, 4 * c:4 * c + 4] = qt
        weight[r, 4 * c:4 * c + 4] = 1
    if case == "nonfinite":
        pred[4, 4 * 2] = np.nan       # symmetric rows (class 1 + r % 3) with a non-finite prediction
        pred[6, 4 * 1 + 2] = np.inf
        pts[2, 17] = np.nan
        pts[1, 100] = np.inf
    args = (T(pred), T(target), T(weight), T(pts), T(sym), 0.01)
    (lp, dp), (lf, df) = _add_modes(args)
    np.testing.assert_array_equal(lp, lf)
    np.testing.assert_array_equal(dp, df)
    # and through the prepared path (prep with the points on another stream)
    ws = torch.empty(adl.workspace_bytes(R, C, P), dtype=torch.uint8, device=D)
    side = torch.cuda.Stream()
    os.environ["PCNN_ADD_SEARCH"] = "pruned"
    try:
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            adl.average_distance_loss_prep(args[2], args[4], P, ws, points=args[3])
        torch.cuda.current_stream().wait_stream(side)
        l2, d2 = adl.average_distance_loss(*args, workspace=ws, prepared=True)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("PCNN_ADD_SEARCH", None)
    np.testing.assert_array_equal(l2.cpu().numpy(), lf)
    np.testing.assert_array_equal(d2.cpu().numpy(), df)


def _morton_np(X):
    """numpy restatement of k_add_order: 10-bit per-axis cell of the class's
    bounding box, interleaved x0 y0 z0 x1 ..., ties by point index."""
    lo, hi = X.min(0), X.max(0)
    ext = (hi - lo).astype(np.float32)
    f = np.where(ext > 0, (X - lo) / np.where(ext > 0, ext, 1) * np.float32(1023), 0).astype(np.float32)
    q = np.where(f > 0, np.where(f < 1023, f.astype(np.int64), 1023), 0)
    code = np.zeros(len(X), np.int64)
    for b in range(10):
        for a in range(3):
            code |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return np.argsort(code * 8192 + np.arange(len(X)), kind="stable").astype(np.int32)


def test_add_s_search_order_and_pruning(hip):
    """The symmetric classes' Morton orders match the numpy restatement, and
    on the bench's model points (YCB rescaled, random unit predictions) the
    search scans a small part of the blocks -- the pruning is real."""
    rng = np.random.default_rng(31)
    C = 22
    pts, sym = synth.rescaled_points(C)
    P = pts.shape[1]
    R = 40
    pred = np.zeros((R, 4 * C), np.float32)
    target = np.zeros((R, 4 * C), np.float32)
    weight = np.zeros((R, 4 * C), np.float32)
    scls = np.nonzero(sym)[0]
    for r in range(R):
        c = int(scls[r % len(scls)])
        for arr in (pred, target):
            q = rng.normal(size=4)
            arr[r, 4 * c:4 * c + 4] = q / np.linalg.norm(q)
        weight[r, 4 * c:4 * c + 4] = 1
    args = (T(pred), T(target), T(weight), T(pts), T(sym), 0.01)
    ws = torch.empty(adl.workspace_bytes(R, C, P), dtype=torch.uint8, device=D)
    os.environ["PCNN_ADD_SEARCH"] = "pruned"
    try:
        adl.average_distance_loss_prep(args[2], args[4], P, ws, points=args[3])
        adl.average_distance_loss(*args, workspace=ws, prepared=True)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("PCNN_ADD_SEARCH", None)
    perm, stat = adl.search_diagnostics(ws, R, C, P)
    for c in scls:
        np.testing.assert_array_equal(perm[c].cpu().numpy(), _morton_np(pts[c]))
    scanned, held = (int(v) for v in stat.cpu().numpy())
    assert held == R * ((P + 63) // 64) * ((P + 7) // 8)
    assert scanned < 0.35 * held, (scanned, held)
