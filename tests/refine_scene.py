"""Test-only synthetic scene for the pose-refinement tests: an oriented box
ray-cast through a pinhole camera, giving the maps the reference takes from
its OpenGL pass (synthesize.cpp:2106-2137): rendered vertices / normals
(H,W,4), canonical model coordinates with the class in the integer part of x
(H,W,3, NaN off the model), and a uint16 depth image with its label map."""
import numpy as np

CAMERA = (1066.778, 1067.487, 312.9869, 241.3109)  # YCB K (my_tools/model2.py:226)


def quat_to_R(q):
    w, x, y, z = (float(v) for v in q)
    n = np.sqrt(w * w + x * x + y * y + z * z)
    w, x, y, z = w / n, x / n, y / n, z / n
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def axis_angle_quat(axis, ang):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    return np.concatenate([[np.cos(ang / 2)], np.sin(ang / 2) * a])


def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2, w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2])


def pose_mul(a, b):
    """(q, t) composition a * b of 7-vectors (float64)."""
    Ra = quat_to_R(a[:4])
    return np.concatenate([quat_mul(a[:4], b[:4]), Ra @ np.asarray(b[4:7]) + np.asarray(a[4:7])])


def render_box(pose, half, cls=1, H=480, W=640, camera=CAMERA, factor=10000.0):
    fx, fy, px, py = camera
    R = quat_to_R(pose[:4])
    t = np.asarray(pose[4:7], np.float64)
    h = np.asarray(half, np.float64)
    xs, ys = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    d = np.stack([(xs - px) / fx, (ys - py) / fy, np.ones_like(xs)], -1)       # camera ray, z = 1
    o = R.T @ (-t)                                                              # camera centre in the box frame
    dd = d @ R                                                                  # R^T d per pixel
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = (-h - o) / dd
        t2 = (h - o) / dd
    tn = np.minimum(t1, t2)
    tf = np.maximum(t1, t2)
    tmin = tn.max(-1)
    tmax = tf.min(-1)
    hit = (tmax >= tmin) & (tmin > 0)
    axis = tn.argmax(-1)
    nobj = np.zeros(d.shape)
    sgn = -np.sign(np.take_along_axis(dd, axis[..., None], -1)[..., 0])
    np.put_along_axis(nobj, axis[..., None], sgn[..., None], -1)
    P = d * tmin[..., None]
    N = nobj @ R.T
    canon = o + dd * tmin[..., None]
    pv = np.zeros((H, W, 4), np.float32)
    pn = np.zeros((H, W, 4), np.float32)
    pv[hit, :3] = P[hit]
    pv[hit, 3] = 1
    pn[hit, :3] = N[hit]
    vm = np.full((H, W, 3), np.nan, np.float32)
    vm[hit] = canon[hit]
    vm[hit, 0] += cls
    depth = np.zeros((H, W), np.uint16)
    depth[hit] = np.round(P[hit, 2] * factor).astype(np.uint16)
    label = np.where(hit, cls, 0).astype(np.int32)
    return dict(pred_v=pv, pred_n=pn, vertmap=vm, depth=depth, label=label, hit=hit)


def scene(seed=0, perturb_deg=3.0, perturb_t=0.01, half=(0.06, 0.045, 0.035), cls=3):
    """Ground-truth box pose, a perturbed initial pose, the live depth at the
    truth and the rendered maps at the initial pose."""
    rng = np.random.default_rng(seed)
    q_true = axis_angle_quat([1.0, 1.0, 0.3], np.deg2rad(35.0))
    t_true = np.array([0.03, -0.02, 0.75])
    true = np.concatenate([q_true, t_true])
    dq = axis_angle_quat(rng.normal(size=3), np.deg2rad(perturb_deg))
    init = np.concatenate([quat_mul(dq, q_true), t_true + rng.normal(size=3) * perturb_t / np.sqrt(3)])
    live = render_box(true, half, cls)
    pred = render_box(init, half, cls)
    return dict(true=true, init=init, live=live, pred=pred, cls=cls, half=half)


def render_box_torch(pose, half, cls, H=480, W=640, camera=CAMERA, device="cuda"):
    """render_box on the GPU (torch), returning the (vertmap, pred_vertices,
    pred_normals) device maps solve_icp's renderer hands back."""
    import torch
    rt = torch.tensor(_rt_of(pose)[None], dtype=torch.float64, device=device)
    h = torch.tensor(np.asarray(half, np.float64)[None], device=device)
    c = torch.tensor([float(cls)], dtype=torch.float64, device=device)
    return tuple(m[0] for m in _render_boxes(rt, h, c, H, W, camera, device))


def _rt_of(pose):
    p = np.asarray(pose, np.float64)
    return np.concatenate([quat_to_R(p[:4]).reshape(-1), p[4:7]])


class GraphBoxRenderer:
    """The torch box ray-caster replayed from captured HIP graphs: the poses,
    boxes and classes enter through static device tensors, so a call is one
    small H2D copy, one graph launch and clones of the maps (solve_icp keeps
    several renders alive at once).  __call__ renders one pose; render_many
    renders K (object, pose) pairs in one pass (one graph per K), which
    solve_icp uses once per stage.  The test harness's stand-in for the
    reference's OpenGL pass."""

    def __init__(self, half_of, H=480, W=640, camera=CAMERA, device="cuda", dtype=None):
        import torch
        self.half_of, self.H, self.W, self.camera, self.device = half_of, H, W, camera, device
        self.dtype = dtype or torch.float32  # the ray-box arithmetic (the maps are float32 either way)
        self.graphs = {}

    def _graph(self, K):
        import torch
        if K not in self.graphs:
            rt = torch.zeros((K, 12), dtype=self.dtype, device=self.device)
            rt[:, 0] = rt[:, 4] = rt[:, 8] = 1.0
            rt[:, 11] = 1.0
            h = torch.full((K, 3), 0.05, dtype=self.dtype, device=self.device)
            c = torch.ones(K, dtype=self.dtype, device=self.device)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):  # warm-up outside the capture
                _render_boxes(rt, h, c, self.H, self.W, self.camera, self.device)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = _render_boxes(rt, h, c, self.H, self.W, self.camera, self.device)
            self.graphs[K] = (g, out, rt, h, c)
        return self.graphs[K]

    def render_many(self, objs, poses):
        import torch
        K = len(objs)
        g, out, rt, h, c = self._graph(K)
        rt.copy_(torch.from_numpy(np.stack([_rt_of(p) for p in poses])).to(self.dtype))
        h.copy_(torch.from_numpy(np.stack([np.asarray(self.half_of(o), np.float64) for o in objs])).to(self.dtype))
        c.copy_(torch.tensor([float(o) for o in objs], dtype=self.dtype))
        g.replay()
        return tuple(o.clone() for o in out)

    def __call__(self, obj, pose):
        return tuple(m[0] for m in self.render_many([obj], [pose]))


def _render_boxes(rt, h, cls, H, W, camera, device):
    """K boxes at once: rt (K, 12) [R | t], h (K, 3) half extents, cls (K)
    -> vertmap (K,H,W,3), pred_vertices (K,H,W,4), pred_normals (K,H,W,4);
    elementwise arithmetic only, so a pose renders the same in any batch."""
    import torch
    fx, fy, px, py = camera
    K = rt.shape[0]
    R = rt[:, :9].reshape(K, 3, 3)
    tt = rt[:, 9:12]
    ys, xs = torch.meshgrid(torch.arange(H, dtype=rt.dtype, device=device),
                            torch.arange(W, dtype=rt.dtype, device=device), indexing="ij")
    d = torch.stack([(xs - px) / fx, (ys - py) / fy, torch.ones_like(xs)], -1)[None]      # (1,H,W,3)
    o = -(R[:, 0, :] * tt[:, 0:1] + R[:, 1, :] * tt[:, 1:2] + R[:, 2, :] * tt[:, 2:3])  # R^T (-t), (K,3)
    Rb = R[:, None, None]                                                                 # (K,1,1,3,3)
    dd = d[..., 0:1] * Rb[..., 0, :] + d[..., 1:2] * Rb[..., 1, :] + d[..., 2:3] * Rb[..., 2, :]  # d @ R
    hb = h[:, None, None, :]
    ob = o[:, None, None, :]
    t1 = (-hb - ob) / dd
    t2 = (hb - ob) / dd
    tn = torch.minimum(t1, t2)
    tf = torch.maximum(t1, t2)
    tmin = tn.max(-1).values
    tmax = tf.min(-1).values
    hit = (tmax >= tmin) & (tmin > 0)
    axis = tn.argmax(-1)
    sgn = -torch.sign(torch.gather(dd, -1, axis[..., None])[..., 0])
    nobj = torch.zeros_like(dd).scatter_(-1, axis[..., None], sgn[..., None])
    P = d * tmin[..., None]
    N = nobj[..., 0:1] * Rb[..., :, 0] + nobj[..., 1:2] * Rb[..., :, 1] + nobj[..., 2:3] * Rb[..., :, 2]  # nobj @ R^T
    canon = ob + dd * tmin[..., None]
    pv = torch.zeros((K, H, W, 4), dtype=torch.float32, device=device)
    pn = torch.zeros((K, H, W, 4), dtype=torch.float32, device=device)
    pv[..., :3] = torch.where(hit[..., None], P, torch.zeros_like(P)).float()
    pv[..., 3] = hit.float()
    pn[..., :3] = torch.where(hit[..., None], N, torch.zeros_like(N)).float()
    vm = torch.where(hit[..., None], canon, torch.full_like(canon, float("nan"))).float()
    vm[..., 0] = torch.where(hit, vm[..., 0] + cls[:, None, None].float(), vm[..., 0])
    return vm, pv, pn
