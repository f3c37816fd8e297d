"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes bindings of oracle/build/liborc.so, the CPU C++ restatement of the
reference ops (see orc_common.h for the parity status: UNPINNED — no reference
golden vectors exist and the reference cannot be built here; pinned by the
hand-derived KATs in tests/test_oracle_kat.py).

May be imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, and only as the checker / CPU baseline.
"""
import ctypes
import os
import subprocess
import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liborc.so")
_lib = None

F32P = ctypes.POINTER(ctypes.c_float)
I32P = ctypes.POINTER(ctypes.c_int)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_hough_voting.restype = ctypes.c_int
        _lib.orc_hough_class_counts.restype = ctypes.c_int
        _lib.orc_roi_pool_fwd.restype = ctypes.c_int
        _lib.orc_roi_pool_bwd.restype = ctypes.c_int
        _lib.orc_ransac_hough.restype = ctypes.c_int
    return _lib


def _f(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a, a.ctypes.data_as(F32P)


def _i(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(I32P)


MAX_ROI = 128


def hough_voting(label, vertex, extents, meta, gt, is_train, threshold_vote, threshold_percentage, skip_pixels,
                 inlier_threshold=0.9, label_threshold=500, batch_base=0, global_batch=None, exact_rows=True):
    """Reference semantics of hough_voting_gpu (canonical order).  Returns
    (box, pose, target, weight, domain, num_rois) with exact-size outputs
    (one zero dummy row when num_rois == 0) when exact_rows."""
    label, lp = _i(label)
    vertex, vp = _f(vertex)
    extents, ep = _f(extents)
    B, H, W = label.shape
    C = vertex.shape[3] // 3
    meta2 = np.ascontiguousarray(np.asarray(meta, np.float32).reshape(B, -1))
    num_meta = meta2.shape[1]
    meta2, mp = _f(meta2)
    gt2 = np.ascontiguousarray(np.asarray(gt, np.float32).reshape(-1, 13))
    gt2, gp = _f(gt2)
    cap = MAX_ROI * 9
    box = np.zeros((cap, 7), np.float32)
    pose = np.zeros((cap, 7), np.float32)
    target = np.zeros((cap, 4 * C), np.float32)
    weight = np.zeros((cap, 4 * C), np.float32)
    domain = np.zeros((cap,), np.int32)
    n = lib().orc_hough_voting(lp, vp, ep, mp, num_meta, gp, gt2.shape[0], B, H, W, C, batch_base,
                               global_batch or B, int(is_train), ctypes.c_float(inlier_threshold), label_threshold,
                               ctypes.c_float(threshold_vote), ctypes.c_float(threshold_percentage), skip_pixels,
                               box.ctypes.data_as(F32P), pose.ctypes.data_as(F32P), target.ctypes.data_as(F32P),
                               weight.ctypes.data_as(F32P), domain.ctypes.data_as(I32P), cap)
    if n < 0:
        raise RuntimeError("oracle hough: capacity exceeded")
    if exact_rows:
        k = max(n, 1)
        return box[:k], pose[:k], target[:k], weight[:k], domain[:k], n
    return box, pose, target, weight, domain, n


def hough_class_counts(label_img, vertex_img, extents, meta_row, cls, skip, inlier_threshold=0.9):
    label_img, lp = _i(label_img)
    vertex_img, vp = _f(vertex_img)
    extents, ep = _f(extents)
    meta_row, mp = _f(np.asarray(meta_row, np.float32).reshape(-1))
    H, W = label_img.shape
    C = vertex_img.shape[2] // 3
    counts = np.zeros((H, W), np.float32)
    dsum = np.zeros((H, W), np.float32)
    nv = lib().orc_hough_class_counts(lp, vp, ep, mp, H, W, C, cls, ctypes.c_float(inlier_threshold), skip,
                                      counts.ctypes.data_as(F32P), dsum.ctypes.data_as(F32P))
    return counts, dsum, nv


def hough_data_at(label_img, vertex_img, extents, meta_row, cls, skip, cx, cy, count, dsum, inlier_threshold=0.9):
    label_img, lp = _i(label_img)
    vertex_img, vp = _f(vertex_img)
    extents, ep = _f(extents)
    meta_row, mp = _f(np.asarray(meta_row, np.float32).reshape(-1))
    H, W = label_img.shape
    C = vertex_img.shape[2] // 3
    out = np.zeros(3, np.float32)
    lib().orc_hough_data_at(lp, vp, ep, mp, H, W, C, cls, ctypes.c_float(inlier_threshold), skip, cx, cy,
                            ctypes.c_float(count), ctypes.c_float(dsum), out.ctypes.data_as(F32P))
    return out


def roi_pool_fwd(data, rois, pooled_h, pooled_w, spatial_scale, pool_channel=0):
    data, dp = _f(data)
    rois, rp = _f(np.asarray(rois, np.float32).reshape(np.asarray(rois).shape[0], -1))
    B, H, W, C = data.shape
    R, rs = rois.shape
    Co = 1 if pool_channel else C
    top = np.zeros((R, pooled_h, pooled_w, Co), np.float32)
    arg = np.zeros((R, pooled_h, pooled_w, Co), np.int32)
    rc = lib().orc_roi_pool_fwd(dp, B, H, W, C, rp, R, rs, ctypes.c_float(spatial_scale), pooled_h, pooled_w,
                                int(pool_channel), top.ctypes.data_as(F32P), arg.ctypes.data_as(I32P))
    if rc != 0:
        raise ValueError("roi batch index out of range")
    return top, arg


def roi_pool_bwd(top_diff, argmax, data_shape, rois, pooled_h, pooled_w, spatial_scale, pool_channel=0):
    top_diff, tp = _f(top_diff)
    argmax, ap = _i(argmax)
    rois, rp = _f(np.asarray(rois, np.float32).reshape(np.asarray(rois).shape[0], -1))
    B, H, W, C = data_shape
    R, rs = rois.shape
    out = np.zeros((B, H, W, C), np.float32)
    lib().orc_roi_pool_bwd(tp, ap, B, H, W, C, rp, R, rs, ctypes.c_float(spatial_scale), pooled_h, pooled_w,
                           int(pool_channel), out.ctypes.data_as(F32P))
    return out


def average_distance_loss(pred, target, weight, points, symmetry, margin):
    pred, pp = _f(pred)
    target, tp = _f(target)
    weight, wp = _f(weight)
    points, ptp = _f(points)
    symmetry, sp = _f(symmetry)
    R, PC = pred.shape
    C = PC // 4
    P = points.shape[1]
    loss = np.zeros(1, np.float32)
    diff = np.zeros((R, PC), np.float32)
    rows = np.zeros(R, np.float32)
    lib().orc_add_loss_fwd(pp, tp, wp, ptp, sp, R, C, P, ctypes.c_float(margin), loss.ctypes.data_as(F32P),
                           diff.ctypes.data_as(F32P), rows.ctypes.data_as(F32P))
    return loss, diff, rows


def backproject_fwd(data, label, depth, meta, label_3d, grid_size, kernel_size, threshold):
    data, dp = _f(data)
    label, lp = _f(label)
    depth, zp = _f(depth)
    B, H, W, Ch = data.shape
    NC = label.shape[3]
    meta2 = np.ascontiguousarray(np.asarray(meta, np.float32).reshape(B, -1))
    meta2, mp = _f(meta2)
    label_3d, l3p = _f(label_3d)
    G = grid_size
    td = np.zeros((B, G, G, G, Ch), np.float32)
    tl = np.zeros((B, G, G, G, NC), np.float32)
    tf = np.zeros((B, G, G, G, Ch), np.float32)
    lib().orc_backproject_fwd(dp, lp, zp, mp, meta2.shape[1], l3p, B, H, W, Ch, NC, G, kernel_size,
                              ctypes.c_float(threshold), td.ctypes.data_as(F32P), tl.ctypes.data_as(F32P),
                              tf.ctypes.data_as(F32P))
    return td, tl, tf


def backproject_bwd(top_diff, depth, meta, H, W, grid_size):
    top_diff, tp = _f(top_diff)
    depth, zp = _f(depth)
    B = top_diff.shape[0]
    Ch = top_diff.shape[-1]
    meta2 = np.ascontiguousarray(np.asarray(meta, np.float32).reshape(B, -1))
    meta2, mp = _f(meta2)
    out = np.zeros((B, H, W, Ch), np.float32)
    lib().orc_backproject_bwd(tp, zp, mp, meta2.shape[1], B, H, W, Ch, grid_size, out.ctypes.data_as(F32P))
    return out


def ransac_hough(label, vertex, extents, meta, is_train=0, num_threads=0):
    """CPU baseline (reference Houghvoting op restatement); rows of 13 floats."""
    label, lp = _i(label)
    vertex, vp = _f(vertex)
    extents, ep = _f(extents)
    B, H, W = label.shape
    C = vertex.shape[3] // 3
    meta2 = np.ascontiguousarray(np.asarray(meta, np.float32).reshape(B, -1))
    meta2, mp = _f(meta2)
    cap = 4096
    rows = np.zeros((cap, 13), np.float32)
    n = lib().orc_ransac_hough(lp, vp, ep, mp, meta2.shape[1], B, H, W, C, int(is_train), int(num_threads),
                               rows.ctypes.data_as(F32P), cap)
    return rows[:min(n, cap)]


def ransac_hough_op(label, vertex, extents, meta, is_train=0, num_threads=0):
    """The reference CPU op's outputs (hough_voting_op.cc:161-225): top_box
    (R, 6) [b, cls, x1, y1, x2, y2] and top_pose (R, 7); with no detection in
    the batch, the one dummy row box [0, -1, 0, 0, 1, 1], pose [1, 0, ...]
    (:163-177; cv::Vec zero-initialises the rest)."""
    rows = ransac_hough(label, vertex, extents, meta, is_train, num_threads)
    if rows.shape[0] == 0:
        rows = np.zeros((1, 13), np.float32)
        rows[0, [1, 4, 5, 6]] = (-1, 1, 1, 1)
    return np.ascontiguousarray(rows[:, :6]), np.ascontiguousarray(rows[:, 6:])


def box_nms(dets, thresh):
    """lib/utils/nms.py:3-32 (canonical tie order): kept row indices, score descending."""
    d, dp = _f(dets)
    keep = np.zeros((max(d.shape[0], 1),), np.int32)
    n = lib().orc_box_nms(dp, d.shape[0], d.shape[1], ctypes.c_float(thresh), keep.ctypes.data_as(I32P))
    return keep[:n]


def nms_combine(rois, poses_init, poses_pred, keep):
    """lib/fcn/test.py:199-211: kept rows and combined poses."""
    r, rp = _f(rois)
    pi, pip = _f(poses_init)
    pp, ppp = _f(poses_pred)
    k, kp = _i(keep)
    ro = np.zeros((len(k), 7), np.float32)
    po = np.zeros((len(k), 7), np.float32)
    lib().orc_nms_combine(rp, r.shape[1], pip, ppp, pp.shape[1], kp, len(k), ro.ctypes.data_as(F32P),
                          po.ctypes.data_as(F32P))
    return ro, po


def argmax_2d(prob):
    """lib/networks/network.py:433-434 `tf.to_int32(tf.argmax(input, 3))`:
    numpy argmax over the class axis (first maximum; first NaN wins)."""
    return np.argmax(np.asarray(prob, np.float32), axis=3).astype(np.int32)


def hard_label(prob, gt, threshold):
    """Hardlabel forward, restated from the CPU op (hard_label_op.cc:94-106) and
    HardlabelForward (hard_label_op_gpu.cu.cc:17-29): per pixel a zero row, then
    1 at gt if gt != -1 and (gt > 0 or prob[gt] < threshold).  gt outside
    [-1, C) stores past the pixel row in the reference (undefined): zero row."""
    prob = np.asarray(prob, np.float32)
    gt = np.asarray(gt, np.int32)
    B, H, W, C = prob.shape
    top = np.zeros((B, H, W, C), np.float32)
    for b in range(B):
        for y in range(H):
            for x in range(W):
                g = int(gt[b, y, x])
                if g == -1 or g < -1 or g >= C:
                    continue
                if g > 0 or prob[b, y, x, g] < np.float32(threshold):
                    top[b, y, x, g] = 1.0
    return top


def vertex_pred_compact(feat, weights, biases, label):
    """vertex_pred (vgg16_convs.py:152-163: conv2d 1x1 K -> 3C, then bias_add,
    network.py:168-185) at each pixel's own class channels 3l..3l+2: the dot
    product summed in k order in float32 (each product and sum rounded), then
    the bias; labels outside [0, C) give zeros."""
    feat = np.asarray(feat, np.float32)
    B, H, W, K = feat.shape
    w = np.asarray(weights, np.float32).reshape(K, -1)
    b = np.asarray(biases, np.float32).reshape(-1)
    C = w.shape[1] // 3
    lab = np.asarray(label).reshape(-1).astype(np.int64)
    x = feat.reshape(-1, K)
    ok = (lab >= 0) & (lab < C)
    cols = 3 * np.where(ok, lab, 0)[:, None] + np.arange(3)[None, :]
    acc = np.zeros((x.shape[0], 3), np.float32)
    for k in range(K):
        acc = acc + x[:, k:k + 1] * w[k][cols]
    acc = acc + b[cols]
    acc[~ok] = 0.0
    return acc.reshape(B, H, W, 3)


# --- test-time pose refinement (orc_icp.cpp) --------------------------------
def icp_live_vertices(depth_u16, label, obj, factor, camera):
    H, W = label.shape
    d = np.ascontiguousarray(depth_u16, dtype=np.uint16)
    lab, lp = _i(label)
    out = np.empty((H, W, 3), np.float32)
    fx, fy, px, py = (float(c) for c in camera)
    lib().orc_icp_live_vertices(d.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), lp, H, W, int(obj),
                                ctypes.c_float(factor), ctypes.c_float(fx), ctypes.c_float(fy), ctypes.c_float(px),
                                ctypes.c_float(py), out.ctypes.data_as(F32P))
    return out


def icp(live, pred_v, pred_n, camera, depth_range=(0.25, 6.0), max_error=0.01, iterations=8):
    """df::icp restated: returns (update (7,), systems (iterations, 28))."""
    H, W = live.shape[:2]
    lv, lp = _f(live)
    pv, pvp = _f(pred_v)
    pn, pnp = _f(pred_n)
    upd = np.empty(7, np.float32)
    sysm = np.empty((max(iterations, 1), 28), np.float32)
    fx, fy, px, py = (float(c) for c in camera)
    c = ctypes.c_float
    lib().orc_icp(lp, pvp, pnp, H, W, c(fx), c(fy), c(px), c(py), c(depth_range[0]), c(depth_range[1]),
                  c(max_error), int(iterations), upd.ctypes.data_as(F32P), sysm.ctypes.data_as(F32P))
    return upd, sysm[:iterations]


def icp_center(live, label, obj, vertmap, pred_v, pred_n, max_error=0.01):
    H, W = label.shape
    lv, lp = _f(live)
    lab, labp = _i(label)
    vm, vmp = _f(vertmap)
    pv, pvp = _f(pred_v)
    pn, pnp = _f(pred_n)
    out = np.empty(4, np.float32)
    lib().orc_icp_center(lp, labp, int(obj), vmp, pvp, pnp, H, W, ctypes.c_float(max_error), out.ctypes.data_as(F32P))
    return out


def pose_energy(live, label, obj, pred_v, poses, depth_range=(0.25, 6.0)):
    H, W = label.shape
    lv, lp = _f(live)
    lab, labp = _i(label)
    pv, pvp = _f(pred_v)
    P, Pp = _f(np.asarray(poses).reshape(-1, 7))
    e = np.empty(P.shape[0], np.float32)
    lib().orc_pose_energy(lp, labp, int(obj), pvp, H, W, ctypes.c_float(depth_range[0]),
                          ctypes.c_float(depth_range[1]), Pp, P.shape[0], e.ctypes.data_as(F32P))
    return e


def se3_mul(a, b):
    A, ap = _f(a)
    B, bp = _f(b)
    c = np.empty(7, np.float32)
    lib().orc_se3_mul(ap, bp, c.ctypes.data_as(F32P))
    return c


def ldlt_solve6(A, b):
    A_, ap = _f(A)
    b_, bp = _f(b)
    x = np.empty(6, np.float32)
    lib().orc_ldlt_solve6(ap, bp, x.ctypes.data_as(F32P))
    return x


def icp_score(live, label, obj, vertmap, hyps, radius=0.01):
    H, W = label.shape
    lv, lp = _f(live)
    lab, labp = _i(label)
    vm, vmp = _f(vertmap)
    P, Pp = _f(np.asarray(hyps).reshape(-1, 7))
    sc = np.empty(P.shape[0], np.float32)
    ch = np.zeros(1, np.int32)
    lib().orc_icp_score(lp, labp, int(obj), vmp, H, W, Pp, P.shape[0], ctypes.c_float(radius),
                        sc.ctypes.data_as(F32P), ch.ctypes.data_as(I32P))
    return sc, int(ch[0])


def pose2d(label, vertmap, extents, fx, fy, px, py, seed=1305, n_hyp=256, max_iter=100000):
    """Synthesizer::estimatePose2D restated (orc_pose2d.cpp).  Returns dict:
    poses (3, 4, C) in the reference's output layout, hyps (n_hyp, 13)
    [objID | R | t], hyp_px (n_hyp, 4) sampled pixels, inliers (n_hyp, 8)
    per preemptive round, final (C, 3) [h, inliers, hypotheses], n_obj."""
    label, lp = _i(label)
    vertmap, vp = _f(vertmap)
    extents, ep = _f(extents)
    H, W = label.shape
    C = extents.shape[0]
    poses = np.zeros((3, 4, C), np.float32)
    hyps = np.zeros((n_hyp, 13), np.float32)
    hpx = np.zeros((n_hyp, 4), np.int32)
    inl = np.zeros((n_hyp, 8), np.int32)
    fin = np.zeros((C, 3), np.int32)
    lib().orc_pose2d.restype = ctypes.c_int
    n = lib().orc_pose2d(lp, vp, ep, H, W, C, ctypes.c_float(fx), ctypes.c_float(fy), ctypes.c_float(px),
                         ctypes.c_float(py), ctypes.c_uint64(seed), n_hyp, max_iter, poses.ctypes.data_as(F32P),
                         hyps.ctypes.data_as(F32P), hpx.ctypes.data_as(I32P), inl.ctypes.data_as(I32P),
                         fin.ctypes.data_as(I32P))
    return dict(poses=poses, hyps=hyps, hyp_px=hpx, inliers=inl, final=fin, n_obj=n)


def pose3d(label, depth, vertmap, extents, fx, fy, px, py, depth_factor, seed=1305, n_hyp=256, max_iter=100000,
           nm_evals=100):
    """Synthesizer::estimatePose3D restated (orc_pose2d.cpp, orc_pose3d).
    depth (H, W) uint16 raw depth.  Returns dict: poses (3, 4, C) in the
    reference's output layout, eye (H, W, 3) camera coordinates, hyps
    (n_hyp, 13) [objID | R | t], hyp_px (n_hyp, 3), inliers (n_hyp, 8) per
    preemptive round, final (C, 3) [h, inliers, hypotheses], energy (C)
    optEnergy3D at the refined pose, n_obj."""
    label, lp = _i(label)
    depth = np.ascontiguousarray(depth, np.uint16)
    vertmap, vp = _f(vertmap)
    extents, ep = _f(extents)
    H, W = label.shape
    assert depth.shape == (H, W)
    C = extents.shape[0]
    poses = np.zeros((3, 4, C), np.float32)
    eye = np.zeros((H, W, 3), np.float32)
    hyps = np.zeros((n_hyp, 13), np.float32)
    hpx = np.zeros((n_hyp, 3), np.int32)
    inl = np.zeros((n_hyp, 8), np.int32)
    fin = np.zeros((C, 3), np.int32)
    en = np.zeros(C, np.float32)
    lib().orc_pose3d.restype = ctypes.c_int
    n = lib().orc_pose3d(lp, depth.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), vp, ep, H, W, C,
                         ctypes.c_float(fx), ctypes.c_float(fy), ctypes.c_float(px), ctypes.c_float(py),
                         ctypes.c_float(depth_factor), ctypes.c_uint64(seed), n_hyp, max_iter, nm_evals,
                         poses.ctypes.data_as(F32P), eye.ctypes.data_as(F32P), hyps.ctypes.data_as(F32P),
                         hpx.ctypes.data_as(I32P), inl.ctypes.data_as(I32P), fin.ctypes.data_as(I32P),
                         en.ctypes.data_as(F32P))
    return dict(poses=poses, eye=eye, hyps=hyps, hyp_px=hpx, inliers=inl, final=fin, energy=en, n_obj=n)
