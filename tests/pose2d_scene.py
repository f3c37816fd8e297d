"""Test-only scenes for the RGB-only pose estimator (estimatePose2D,
synthesize.cpp:1571): oriented boxes ray-cast through a pinhole camera
(refine_scene.render_box), composited by depth into a label map and the
object-coordinate vertex map the cfg.TEST.VERTEX_REG_3D network regresses --
each pixel of class c carries its box-frame point normalised by the class
extents, (X + e / 2) / e, the inverse of getMode3D (synthesize.cpp:1052-1071),
in channels 3c .. 3c + 2; other channels hold uniform noise."""
import numpy as np

from refine_scene import CAMERA, axis_angle_quat, quat_to_R, render_box


def make_scene(seed=0, n_obj=3, C=6, H=480, W=640, coord_noise=0.0, extents=None, depth_factor=10000.0,
               hole_frac=0.0, depth_noise=0.0):
    rng = np.random.default_rng(seed)
    if extents is None:
        extents = np.zeros((C, 3), np.float32)
        extents[1:] = rng.uniform(0.08, 0.2, size=(C - 1, 3))
    classes = rng.choice(np.arange(1, C), size=n_obj, replace=False)
    fx, fy, px, py = CAMERA
    label = np.zeros((H, W), np.int32)
    zbuf = np.full((H, W), np.inf)
    vertmap = rng.uniform(0, 1, size=(H, W, 3 * C)).astype(np.float32)
    poses = {}
    for i, c in enumerate(classes):
        z = rng.uniform(0.6, 1.1)
        u = rng.uniform(140, W - 140)
        v = rng.uniform(110, H - 110)
        t = np.array([(u - px) / fx * z, (v - py) / fy * z, z])
        q = axis_angle_quat(rng.normal(size=3), rng.uniform(0.3, 2.5))
        pose = np.concatenate([q, t])
        r = render_box(pose, extents[c] / 2.0, cls=int(c), H=H, W=W)
        depth = np.where(r["hit"], r["pred_v"][..., 2], np.inf)
        front = depth < zbuf
        zbuf = np.where(front, depth, zbuf)
        label[front] = c
        canon = r["vertmap"].astype(np.float64)
        canon[..., 0] -= c                                  # render_box puts the class in x's integer part
        norm = canon / extents[c] + 0.5                     # getMode3D inverse: (X - vmin) / (vmax - vmin)
        if coord_noise:
            norm = norm + rng.normal(0, coord_noise, size=norm.shape)
        vertmap[front, 3 * c:3 * c + 3] = norm[front].astype(np.float32)
        poses[int(c)] = dict(R=quat_to_R(q), t=t, uv=(u, v))
    # raw depth for estimatePose3D (getEye, synthesize.cpp:1393): the
    # z-buffer in depth_factor units, optional noise (m) and holes (0)
    z = np.where(np.isfinite(zbuf), zbuf, 1.5)
    if depth_noise:
        z = z + rng.normal(0, depth_noise, size=z.shape)
    depth = np.clip(np.rint(z * depth_factor), 1, 65535).astype(np.uint16)
    if hole_frac:
        depth[rng.uniform(size=depth.shape) < hole_frac] = 0
    return dict(label=label, vertmap=vertmap, extents=extents.astype(np.float32), poses=poses, camera=CAMERA, C=C,
                depth=depth, depth_factor=float(depth_factor))
