"""Synthetic PoseCNN frames: label map, vertex (centre-direction + log-depth)
map, meta data, GT poses, depth.

Follows the reference's target generator `_generate_vertex_targets`
(lib/gt_synthesize_layer/minibatch.py:517-575: unit vector from the pixel to
the projected object centre, log z in channel 3c+2) and its meta/pose layouts
(minibatch.py:412-425 pose rows [b, cls, 0,0,0,0, qw,qx,qy,qz, tx,ty,tz];
minibatch.py:440-482 meta [K | Kinv | world2live | live2world | voxel step |
voxel min]).  Objects are the class 3-D boxes (data/LOV/extents.txt) at a
random rotation, depth z ~ U[0.5, 2.0] (lib/fcn/config.py:85-86), painted
far-to-near.  Seeded per global image index, so a sharded run sees exactly
the frames of the equivalent single-device run.
"""
import os
import numpy as np

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "models.npz")
_MODELS = None


def models():
    """Dataset constants packed by data/make_model_fixtures.py."""
    global _MODELS
    if _MODELS is None:
        with np.load(_DATA, allow_pickle=False) as z:
            _MODELS = {k: z[k] for k in z.files}
    return _MODELS


def quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], np.float64)


def _hull(pts):
    """Monotone-chain convex hull, counter-clockwise."""
    pts = sorted(map(tuple, pts))
    if len(pts) <= 2:
        return np.array(pts)

    def cross(o, a, b):
        return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0])
    lower, upper = [], []
    for p in pts:
        while len(lower) >= 2 and cross(lower[-2], lower[-1], p) <= 0:
            lower.pop()
        lower.append(p)
    for p in reversed(pts):
        while len(upper) >= 2 and cross(upper[-2], upper[-1], p) <= 0:
            upper.pop()
        upper.append(p)
    return np.array(lower[:-1] + upper[:-1])


def _fill_convex(mask, hull, value):
    H, W = mask.shape
    x0 = max(int(np.floor(hull[:, 0].min())), 0)
    x1 = min(int(np.ceil(hull[:, 0].max())), W - 1)
    y0 = max(int(np.floor(hull[:, 1].min())), 0)
    y1 = min(int(np.ceil(hull[:, 1].max())), H - 1)
    if x1 < x0 or y1 < y0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    ys, xs = np.mgrid[y0:y1 + 1, x0:x1 + 1]
    inside = np.ones(xs.shape, bool)
    n = len(hull)
    for i in range(n):
        a, b = hull[i], hull[(i + 1) % n]
        inside &= (b[0] - a[0]) * (ys - a[1]) - (b[1] - a[1]) * (xs - a[0]) >= 0
    yy, xx = ys[inside], xs[inside]
    mask[yy, xx] = value
    return yy, xx


def make_meta(K, B, voxel=None):
    """(B,1,1,48) meta rows.  voxel = (step[3], vmin[3]) for backprojection;
    world2live / live2world default to the identity pose."""
    K = np.asarray(K, np.float64)
    Kinv = np.linalg.pinv(K)
    m = np.zeros(48, np.float32)
    m[0:9] = K.flatten()
    m[9:18] = Kinv.flatten()
    eye = np.hstack([np.eye(3), np.zeros((3, 1))])
    m[18:30] = eye.flatten()
    m[30:42] = eye.flatten()
    if voxel is not None:
        m[42:45], m[45:48] = voxel[0], voxel[1]
    return np.tile(m, (B, 1)).reshape(B, 1, 1, 48).astype(np.float32)


def make_frames(B, H=480, W=640, num_classes=22, objects_per_image=6, seed=0, image_offset=0,
                extents=None, K=None, dir_noise=0.05, depth_noise=0.01, with_depth=False, voxel=None,
                depth_background=None):
    """Generate B synthetic frames; image i uses rng seed (seed*1000 + image_offset + i).
    depth_background = (z_top, z_bottom): with_depth frames also get a scene
    behind the objects -- a plane whose depth runs linearly from z_top at the
    top image row to z_bottom at the bottom one (a floor / table seen at an
    angle), as an RGB-D sensor reports depth at every pixel; None leaves the
    pixels outside the objects at depth 0 (holes)."""
    mdl = models()
    if extents is None:
        extents = mdl["lov_extents"][:num_classes]
    extents = np.asarray(extents, np.float32)
    if K is None:
        K = mdl["K"].astype(np.float64)
        if (H, W) != (480, 640):  # scaled camera for reduced test frames (im_scale, minibatch.py:448-450)
            s = W / 640.0
            K = K.copy()
            K[:2] *= s
    K = np.asarray(K, np.float64)
    C = num_classes
    fx, fy, px, py = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    label = np.zeros((B, H, W), np.int32)
    vertex = np.empty((B, H, W, 3 * C), np.float32)
    depth = np.zeros((B, H, W, 1), np.float32) if with_depth else None
    if depth is not None and depth_background is not None:
        zt, zb = depth_background
        depth[:] = (zt + (zb - zt) * np.arange(H, dtype=np.float64) / max(H - 1, 1)).astype(np.float32)[None, :, None, None]
    gts = []
    margin = max(4, int(round(40 * W / 640)))
    for i in range(B):
        gi = image_offset + i
        rng = np.random.default_rng(seed * 1000 + gi)
        vertex[i] = rng.uniform(-1.0, 1.0, size=(H, W, 3 * C)).astype(np.float32)
        nobj = min(objects_per_image, C - 1)
        classes = rng.choice(np.arange(1, C), size=nobj, replace=False)
        objs = []
        for cls in classes:
            z = rng.uniform(0.5, 2.0)
            cx = rng.uniform(margin, W - margin)
            cy = rng.uniform(margin, H - margin)
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            if q[0] < 0:
                q = -q
            t = np.array([(cx - px) / fx * z, (cy - py) / fy * z, z])
            objs.append((int(cls), z, cx, cy, q, t))
        for (cls, z, cx, cy, q, t) in sorted(objs, key=lambda o: -o[1]):  # far to near
            e = extents[cls] / 2.0
            corners = np.array([[sx * e[0], sy * e[1], sz * e[2]] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
            P = corners @ quat2mat(q).T + t
            uv = np.stack([fx * P[:, 0] / P[:, 2] + px, fy * P[:, 1] / P[:, 2] + py], 1)
            yy, xx = _fill_convex(label[i], _hull(uv), cls)
            if len(yy) == 0:
                continue
            R = np.stack([cx - xx, cy - yy], 0).astype(np.float64)
            N = np.linalg.norm(R, axis=0) + 1e-10
            R = R / N
            vertex[i, yy, xx, 3 * cls + 0] = (R[0] + rng.normal(0, dir_noise, len(xx))).astype(np.float32)
            vertex[i, yy, xx, 3 * cls + 1] = (R[1] + rng.normal(0, dir_noise, len(xx))).astype(np.float32)
            vertex[i, yy, xx, 3 * cls + 2] = (np.log(z) + rng.normal(0, depth_noise, len(xx))).astype(np.float32)
            if depth is not None:
                depth[i, yy, xx, 0] = np.float32(z)
        for (cls, z, cx, cy, q, t) in objs:
            gts.append([gi, cls, 0, 0, 0, 0, q[0], q[1], q[2], q[3], t[0], t[1], t[2]])
    gt = np.array(gts, np.float32).reshape(-1, 13)
    meta = make_meta(K, B, voxel)
    out = dict(label=label, vertex=vertex, meta=meta, gt=gt, extents=extents, K=K.astype(np.float32))
    if depth is not None:
        out["depth"] = depth
    return out


def cpu_vertex(vertex):
    """The vertex map in the convention of the reference CPU op `Houghvoting`:
    channel 3c+2 is the raw distance (TransHyp::compute_distance,
    ransac.h:108-119; hypotheses with a negative one are skipped,
    hough_voting_op.cc:583-599), where the GPU op reads log-depth and takes
    exp (hough_voting_gpu_op.cu.cc:280).  The CPU baseline is timed on this
    form of the same frames."""
    v = vertex.copy()
    v[..., 2::3] = np.exp(v[..., 2::3])
    return v


def rescaled_points(num_classes=22, symmetric=True):
    """Model points rescaled as minibatch.py:50-60 does, plus the symmetry vector."""
    mdl = models()
    ext = mdl["lov_extents"][:num_classes]
    pts = mdl["lov_points"][:num_classes].copy()
    sym = mdl["lov_symmetry"][:num_classes].copy()
    for i in range(1, num_classes):
        w = 2.0 / np.amax(ext[i])
        if w < 10:
            w = 10
        if sym[i] > 0 and symmetric:
            pts[i] = 4 * w * pts[i]
        else:
            pts[i] = w * pts[i]
    if not symmetric:
        sym = np.zeros_like(sym)
    return pts.astype(np.float32), sym.astype(np.float32)


def box_points(extents, P=2620, seed=0):
    """(C, P, 3) model points for datasets whose meshes are not in the
    reference (LINEMOD: only data/LINEMOD/extents.txt ships): P points spread
    uniformly over each class's 3-D box surface (class 0, background, zero)."""
    ext = np.asarray(extents, np.float64)
    rng = np.random.default_rng(seed)
    out = np.zeros((len(ext), P, 3), np.float32)
    for c in range(1, len(ext)):
        e = ext[c] / 2.0
        areas = np.array([e[1] * e[2], e[0] * e[2], e[0] * e[1]])
        face = rng.choice(3, size=P, p=areas / areas.sum())
        pts = rng.uniform(-1.0, 1.0, size=(P, 3)) * e
        side = np.where(rng.uniform(size=P) < 0.5, -1.0, 1.0)
        pts[np.arange(P), face] = side * e[face]
        out[c] = pts.astype(np.float32)
    return out


def linemod_points(P=2620, symmetric=True):
    """LINEMOD (C = 16) model points on the class boxes, rescaled as
    minibatch.py:50-60 does, and the symmetry vector (linemod.py:44)."""
    mdl = models()
    ext = mdl["linemod_extents"]
    pts = box_points(ext, P, seed=16)
    sym = mdl["linemod_symmetry"].copy()
    for i in range(1, len(ext)):
        w = max(2.0 / np.amax(ext[i]), 10.0)
        pts[i] = (4 * w if sym[i] > 0 and symmetric else w) * pts[i]
    if not symmetric:
        sym = np.zeros_like(sym)
    return pts.astype(np.float32), sym.astype(np.float32)
