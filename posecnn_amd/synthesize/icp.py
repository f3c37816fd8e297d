"""Test-time pose refinement, backed by
libposecnn_hip.so (csrc/icp.hip).

Mirrors the numerical pieces of lib/synthesize (Synthesizer::solveICP,
synthesize.cpp:2052-2395, exposed as synthesizer.icp_python,
synthesizer.pyx:60-75) and of lib/kinect_fusion's df::icp
(src/optimization/icp.cpp:20-106):

live_vertices(depth, label, obj_ids, factor, camera)      -> (L,H,W,3)
icp(live, pred_vertices, pred_normals, camera, ...)        -> (update (N,7), pose_out (N,7) | None)
icp_center(live, label, obj_ids, vertmap, pred_v, pred_n)  -> (out (L,4), pose_out (L,7) | None)
pose_energy(live, label, obj, pred_vertices, poses, ...)   -> (K,)

Poses are (qw, qx, qy, qz, tx, ty, tz) float32 rows; camera = (fx, fy, px, py).
The rendered maps (the reference's OpenGL pass) are inputs.
"""
import torch

from .. import _lib


def _f(t):
    return t.contiguous().float()


def live_vertices(depth, label, obj_ids, factor, camera, stream=None):
    """df::backproject of the depth masked to each object (synthesize.cpp:2140-2160)."""
    _lib.require_gpu(depth, label)
    H, W = depth.shape[-2:]
    obj = torch.as_tensor(obj_ids).to(device=depth.device, dtype=torch.int32).contiguous()
    L = obj.numel()
    out = torch.empty((L, H, W, 3), dtype=torch.float32, device=depth.device)
    fx, fy, px, py = (float(c) for c in camera)
    rc = _lib.load().pcnn_icp_live_vertices(_lib.ptr(depth.contiguous().to(torch.uint16)),
                                            _lib.ptr(label.contiguous().to(torch.int32)), H, W, _lib.ptr(obj), L,
                                            float(factor), fx, fy, px, py, _lib.ptr(out), _lib.stream_ptr(stream))
    _lib.check(rc, "icp_live_vertices")
    return out


def icp(live, pred_vertices, pred_normals, camera, depth_range=(0.25, 6.0), max_error=0.01, iterations=8,
        live_index=None, pose_in=None, return_systems=False, stream=None):
    """df::icp for N problems (one per row of pred_vertices (N,H,W,4)).
    Returns (update (N,7), pose_out (N,7) = update * pose_in or None[, systems (N,it,28)])."""
    _lib.require_gpu(live, pred_vertices, pred_normals)
    pv, pn, lv = _f(pred_vertices), _f(pred_normals), _f(live)
    N, H, W = pv.shape[0], pv.shape[1], pv.shape[2]
    if pv.shape != (N, H, W, 4) or pn.shape != (N, H, W, 4) or lv.shape[1:] != (H, W, 3):
        raise ValueError("icp: pred maps (N,H,W,4), live (L,H,W,3)")
    li = None
    if live_index is not None:
        if not live_index.is_cuda:  # validated here; a device index out of range contributes no pixel (no sync)
            if live_index.numel() != N or int(live_index.min()) < 0 or int(live_index.max()) >= lv.shape[0]:
                raise ValueError("icp: live_index must map each problem to a live map")
        elif live_index.numel() != N:
            raise ValueError("icp: live_index must map each problem to a live map")
        li = live_index.to(device=pv.device, dtype=torch.int32).contiguous()
    elif lv.shape[0] != N:
        raise ValueError("icp: one live map per problem, or a live_index")
    dev = pv.device
    update = torch.empty((N, 7), dtype=torch.float32, device=dev)
    pin = _f(pose_in) if pose_in is not None else None
    if pin is not None and pin.shape != (N, 7):
        raise ValueError("icp: pose_in must be (N,7)")
    pout = torch.empty((N, 7), dtype=torch.float32, device=dev) if pin is not None else None
    systems = torch.empty((N, iterations, 28), dtype=torch.float32, device=dev) if return_systems else None
    L = _lib.load()
    nbytes = L.pcnn_icp_workspace_size(N, H, W)
    ws = _lib.workspace(nbytes, dev, "icp", stream)
    fx, fy, px, py = (float(c) for c in camera)
    rc = L.pcnn_icp(_lib.ptr(lv), lv.shape[0], _lib.ptr(li), _lib.ptr(pv), _lib.ptr(pn), N, H, W, fx, fy, px, py,
                    float(depth_range[0]), float(depth_range[1]), float(max_error), int(iterations), _lib.ptr(pin),
                    _lib.ptr(update), _lib.ptr(pout), _lib.ptr(systems), _lib.ptr(ws), ws.numel(),
                    _lib.stream_ptr(stream))
    _lib.check(rc, "icp")
    return (update, pout, systems) if return_systems else (update, pout)


def icp_center(live, label, obj_ids, vertmap, pred_vertices, pred_normals, max_error=0.01, pose_in=None,
               stream=None):
    """Translation re-centring of solveICP (synthesize.cpp:2163-2219) for L objects."""
    _lib.require_gpu(live, label, vertmap, pred_vertices, pred_normals)
    lv, vm, pv, pn = _f(live), _f(vertmap), _f(pred_vertices), _f(pred_normals)
    L_, H, W = lv.shape[0], lv.shape[1], lv.shape[2]
    obj = torch.as_tensor(obj_ids).to(device=lv.device, dtype=torch.int32).contiguous()
    if obj.numel() != L_ or vm.shape != (L_, H, W, 3) or pv.shape != (L_, H, W, 4) or pn.shape != (L_, H, W, 4):
        raise ValueError("icp_center: live (L,H,W,3), vertmap (L,H,W,3), pred maps (L,H,W,4), obj_ids (L)")
    dev = lv.device
    out = torch.empty((L_, 4), dtype=torch.float32, device=dev)
    pin = _f(pose_in) if pose_in is not None else None
    if pin is not None and pin.shape != (L_, 7):
        raise ValueError("icp_center: pose_in must be (L,7)")
    pout = torch.empty((L_, 7), dtype=torch.float32, device=dev) if pin is not None else None
    lib = _lib.load()
    ws = _lib.workspace(lib.pcnn_icp_reduce_workspace_size(L_, H, W), dev, "icp_red", stream)
    rc = lib.pcnn_icp_center(_lib.ptr(lv), _lib.ptr(label.contiguous().to(torch.int32)), _lib.ptr(obj), L_,
                             _lib.ptr(vm), _lib.ptr(pv), _lib.ptr(pn), H, W, float(max_error), _lib.ptr(pin),
                             _lib.ptr(out), _lib.ptr(pout), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "icp_center")
    return out, pout


def pose_energy(live, label, obj, pred_vertices, poses, depth_range=(0.25, 6.0), stream=None):
    """optEnergy (synthesize.cpp:2474-2526) of K candidate poses (K,7)."""
    _lib.require_gpu(live, label, pred_vertices, poses)
    lv, pv, P = _f(live), _f(pred_vertices), _f(poses)
    H, W = lv.shape[-3], lv.shape[-2]
    if P.dim() != 2 or P.shape[1] != 7 or pv.shape != (H, W, 4) or label.shape[-2:] != (H, W):
        raise ValueError("pose_energy: poses (K,7), pred_vertices (H,W,4), label (H,W)")
    K = P.shape[0]
    dev = lv.device
    energy = torch.empty((K,), dtype=torch.float32, device=dev)
    lib = _lib.load()
    ws = _lib.workspace(lib.pcnn_icp_reduce_workspace_size(K, H, W), dev, "icp_energy", stream)
    rc = lib.pcnn_pose_energy(_lib.ptr(lv), _lib.ptr(label.contiguous().to(torch.int32)), int(obj), _lib.ptr(pv),
                              H, W, float(depth_range[0]), float(depth_range[1]), _lib.ptr(P), K, _lib.ptr(energy),
                              _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "pose_energy")
    return energy


def icp_score(live, label, obj, vertmap, hyps, radius=0.01, stream=None):
    """SegICP score of J hypotheses (synthesize.cpp:2288-2330) -> (score (J,), choose (1,) int32)."""
    _lib.require_gpu(live, label, vertmap, hyps)
    lv, vm, P = _f(live), _f(vertmap), _f(hyps)
    H, W = lv.shape[-3], lv.shape[-2]
    if P.dim() != 2 or P.shape[1] != 7 or vm.shape[-3:] != (H, W, 3) or label.shape[-2:] != (H, W):
        raise ValueError("icp_score: hyps (J,7), vertmap (H,W,3), label (H,W)")
    J = P.shape[0]
    dev = lv.device
    score = torch.empty((J,), dtype=torch.float32, device=dev)
    choose = torch.empty((1,), dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws = _lib.workspace(lib.pcnn_icp_score_workspace_size(J, H, W), dev, "icp_score", stream)
    rc = lib.pcnn_icp_score(_lib.ptr(lv), _lib.ptr(label.contiguous().to(torch.int32)), int(obj), _lib.ptr(vm), H, W,
                            _lib.ptr(P), J, float(radius), _lib.ptr(score), _lib.ptr(choose), _lib.ptr(ws),
                            ws.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "icp_score")
    return score, choose


def _se3_mul(a, b):
    """Sophus SE3 a * b of (qw,qx,qy,qz,tx,ty,tz) float rows (host side, float64)."""
    import numpy as np
    w1, x1, y1, z1 = a[:4]
    w2, x2, y2, z2 = b[:4]
    q = np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                  w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2, w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2])
    v = np.asarray(b[4:7], np.float64)
    u = np.array([x1, y1, z1])
    uv = 2 * np.cross(u, v)
    t = v + w1 * uv + np.cross(u, uv) + np.asarray(a[4:7], np.float64)
    return np.concatenate([q / np.linalg.norm(q), t])


def nelder_mead(f, x0, lb, ub, max_eval):
    """Bounded Nelder-Mead (NLopt LN_NELDERMEAD's role in poseWithOpt,
    synthesize.cpp:2529-2573): initial steps NLopt's default (a quarter of the
    bound range, 0.75 of the distance to a nearer bound), reflection 1,
    expansion 2, contraction 1/2, shrink 1/2, trial points clamped to the
    bounds, at most max_eval evaluations of f.  NLopt is absent here: the
    search's exact trajectory is unpinned."""
    import numpy as np
    x0 = np.asarray(x0, np.float64)
    n = x0.size
    lb, ub = np.asarray(lb, np.float64), np.asarray(ub, np.float64)
    step = np.minimum(0.25 * (ub - lb), np.minimum(0.75 * (ub - x0), 0.75 * (x0 - lb)))
    pts = [x0] + [x0 + step[i] * np.eye(n)[i] for i in range(n)]
    vals = [f(p) for p in pts]
    nev = len(pts)
    clamp = lambda p: np.minimum(np.maximum(p, lb), ub)
    while nev < max_eval:
        order = np.argsort(vals, kind="stable")
        pts = [pts[i] for i in order]
        vals = [vals[i] for i in order]
        c = np.mean(pts[:-1], axis=0)
        xr = clamp(c + (c - pts[-1]))
        fr = f(xr)
        nev += 1
        if fr < vals[0] and nev < max_eval:
            xe = clamp(c + 2 * (c - pts[-1]))
            fe = f(xe)
            nev += 1
            pts[-1], vals[-1] = (xe, fe) if fe < fr else (xr, fr)
        elif fr < vals[-2]:
            pts[-1], vals[-1] = xr, fr
        elif nev < max_eval:
            xc = clamp(c + 0.5 * (pts[-1] - c)) if fr >= vals[-1] else clamp(c + 0.5 * (xr - c))
            fc = f(xc)
            nev += 1
            if fc < min(fr, vals[-1]):
                pts[-1], vals[-1] = xc, fc
            else:
                for i in range(1, n + 1):
                    if nev >= max_eval:
                        break
                    pts[i] = clamp(pts[0] + 0.5 * (pts[i] - pts[0]))
                    vals[i] = f(pts[i])
                    nev += 1
    i = int(np.argmin(vals))
    return pts[i], vals[i]


def solve_icp(labelmap, depth, parameters, rois, poses, render, max_error=0.01, nm_evals=50, icp_iterations=8,
              min_pixels=400, stream=None):
    """Synthesizer::solveICP (synthesize.cpp:2052-2395) on the GPU ops above.

    labelmap (H,W) int32, depth (H,W) uint16, parameters = (fx, fy, px, py,
    znear, zfar, factor) (icp_python's meta, synthesize.cpp:2031-2049), rois
    (R, >= 2) with the class at column 1, poses (R,7).  render(obj_id, pose7)
    -> (vertmap (H,W,3), pred_vertices (H,W,4), pred_normals (H,W,4)) device
    tensors stands in for the reference's OpenGL pass.  Returns (poses_new,
    poses_icp) (R,7) as the reference fills `outputs` / `outputs_icp`: rows of
    skipped RoIs stay zero.  Per RoI: live vertices, translation re-centring,
    the Nelder-Mead search on optEnergy (nm_evals evaluations; 0 skips it),
    eight depth hypotheses refined by one batched 8-iteration ICP launch, and
    the SegICP score picks one."""
    import numpy as np
    fx, fy, px, py, znear, zfar, factor = (float(v) for v in parameters)
    cam = (fx, fy, px, py)
    dev = labelmap.device
    R_ = rois.shape[0]
    poses_new = np.zeros((R_, 7), np.float32)
    poses_icp = np.zeros((R_, 7), np.float32)
    rois_h = rois.detach().cpu().numpy() if torch.is_tensor(rois) else np.asarray(rois)
    poses_h = poses.detach().cpu().numpy() if torch.is_tensor(poses) else np.asarray(poses, np.float32)
    dz = [0.0, -0.02, -0.01, 0.01, 0.02, 0.03, 0.04, 0.05]  # synthesize.cpp:2255-2280
    for i in range(R_):
        obj = int(rois_h[i, 1])
        if obj <= 0:
            continue
        p = poses_h[i].astype(np.float64)
        T = np.concatenate([p[:4] / np.linalg.norm(p[:4]), p[4:7]]).astype(np.float32)
        vm, pv, pn = render(obj, T)
        objt = torch.tensor([obj], dtype=torch.int32, device=dev)
        live = live_vertices(depth, labelmap, objt, factor, cam, stream)
        if int((labelmap == obj).sum()) < min_pixels:
            continue
        out, Tc = icp_center(live, labelmap, objt, vm[None], pv[None], pn[None], max_error,
                             pose_in=torch.from_numpy(T).to(dev)[None], stream=stream)
        c = float(out[0, 3])
        if c > 0:
            T = Tc[0].cpu().numpy()
            if nm_evals > 0:  # refinePose(..., 0): optEnergy over a correction of the re-rendered pose
                _, pv0, _ = render(obj, T)

                def energy(x):
                    return float(pose_energy(live[0], labelmap, obj, pv0,
                                             torch.tensor(x, dtype=torch.float32, device=dev)[None], (znear, zfar),
                                             stream)[0])

                x0 = np.array([1, 0, 0, 0, 0, 0, 0], np.float64)
                r = np.array([0.1, 0.1, 0.1, 0.1, 0.01, 0.01, 0.1])
                x, _ = nelder_mead(energy, x0, x0 - r, x0 + r, nm_evals)
                T = _se3_mul(np.concatenate([x[:4] / np.linalg.norm(x[:4]), x[4:]]), T).astype(np.float32)
        Tz = float(T[6])
        poses_new[i] = T
        hyps = np.repeat(T[None], len(dz), 0)
        hyps[1:, 6] = [Tz + d for d in dz[1:]]
        maps = [render(obj, h) for h in hyps]
        pvs = torch.stack([m[1] for m in maps])
        pns = torch.stack([m[2] for m in maps])
        _, refined = icp(live, pvs, pns, cam, (znear, zfar), max_error, icp_iterations,
                         live_index=torch.zeros(len(dz), dtype=torch.int32, device=dev),
                         pose_in=torch.from_numpy(hyps).to(dev), stream=stream)
        _, choose = icp_score(live[0], labelmap, obj, vm, refined, 0.01, stream)
        poses_icp[i] = refined[int(choose[0])].cpu().numpy()
    return poses_new, poses_icp
