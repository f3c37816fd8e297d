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
import ctypes
import os

import numpy as np
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


def pose_energy_batch(live, label, pose_obj, pose_live, pred_vertices, pose_pv, poses, depth_range=(0.25, 6.0),
                      stream=None):
    """optEnergy of K poses in one launch: pose k (poses (K,7)) is scored for
    object pose_obj[k] against live[pose_live[k]] (live (L,H,W,3)) and
    pred_vertices[pose_pv[k]] (pred_vertices (P,H,W,4)).  Index arrays are
    device int32 (K,), validated here on the host side when given as CPU data."""
    _lib.require_gpu(live, label, pred_vertices, poses)
    lv, pv, P = _f(live), _f(pred_vertices), _f(poses)
    if lv.dim() != 4 or pv.dim() != 4 or P.dim() != 2 or P.shape[1] != 7:
        raise ValueError("pose_energy_batch: live (L,H,W,3), pred_vertices (P,H,W,4), poses (K,7)")
    L_, H, W = lv.shape[0], lv.shape[1], lv.shape[2]
    K = P.shape[0]
    if pv.shape[1:] != (H, W, 4) or lv.shape[3] != 3 or label.shape[-2:] != (H, W):
        raise ValueError("pose_energy_batch: map shapes disagree")
    idx = []
    for a, n in ((pose_obj, None), (pose_live, L_), (pose_pv, pv.shape[0])):
        t = torch.as_tensor(a)
        if t.numel() != K:
            raise ValueError("pose_energy_batch: one index per pose")
        if not t.is_cuda and n is not None and K and (int(t.min()) < 0 or int(t.max()) >= n):
            raise ValueError("pose_energy_batch: index out of range")
        idx.append(t.to(device=lv.device, dtype=torch.int32).contiguous())
    energy = torch.empty((K,), dtype=torch.float32, device=lv.device)
    lib = _lib.load()
    ws = _lib.workspace(lib.pcnn_icp_reduce_workspace_size(K, H, W), lv.device, "icp_energy", stream)
    rc = lib.pcnn_pose_energy_batch(_lib.ptr(lv), L_, _lib.ptr(label.contiguous().to(torch.int32)), _lib.ptr(pv),
                                    pv.shape[0], H, W, float(depth_range[0]), float(depth_range[1]), _lib.ptr(P), K,
                                    _lib.ptr(idx[0]), _lib.ptr(idx[1]), _lib.ptr(idx[2]), _lib.ptr(energy),
                                    _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "pose_energy_batch")
    return energy


def energy_records(live, label, prob_obj, prob_live, pred_vertices, depth_range=(0.25, 6.0), stream=None):
    """optEnergy's inputs of N problems compacted on the device: problem i's
    object pixels (label == prob_obj[i]) whose live vertex (live
    (L,H,W,3)[prob_live[i]]) lies inside depth_range, in raster order, as
    (rendered vertex (pred_vertices (N,H,W,4)[i]), live vertex) records.
    Returns (records (N, H*W, 6), counts (N,) int32)."""
    _lib.require_gpu(live, label, pred_vertices)
    lv, pv = _f(live), _f(pred_vertices)
    if lv.dim() != 4 or pv.dim() != 4 or lv.shape[3] != 3 or pv.shape[3] != 4 or pv.shape[1:3] != lv.shape[1:3]:
        raise ValueError("energy_records: live (L,H,W,3), pred_vertices (N,H,W,4)")
    N, H, W = pv.shape[0], pv.shape[1], pv.shape[2]
    dev = lv.device
    po = torch.as_tensor(prob_obj).to(device=dev, dtype=torch.int32).contiguous()
    pl = torch.as_tensor(prob_live).to(device=dev, dtype=torch.int32).contiguous()
    if po.numel() != N or pl.numel() != N:
        raise ValueError("energy_records: one object id and live index per problem")
    rec = torch.empty((N, H * W, 6), dtype=torch.float32, device=dev)
    cnt = torch.empty((N,), dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws = _lib.workspace(lib.pcnn_energy_records_workspace_size(N, H, W), dev, "icp_records", stream)
    rc = lib.pcnn_energy_records(_lib.ptr(lv), lv.shape[0], _lib.ptr(label.contiguous().to(torch.int32)), _lib.ptr(pv),
                                 H, W, float(depth_range[0]), float(depth_range[1]), N, _lib.ptr(po), _lib.ptr(pl),
                                 _lib.ptr(rec), _lib.ptr(cnt), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "energy_records")
    return rec, cnt


def pose_energy_records(records, counts, poses, pose_prob, depth_range=(0.25, 6.0), stream=None):
    """optEnergy of K poses (K,7), pose k over problem pose_prob[k]'s records
    (energy_records): one 1024-thread workgroup per pose, the same summation
    as nelder_mead_device's evaluations."""
    _lib.require_gpu(records, counts, poses)
    P = _f(poses)
    K = P.shape[0]
    pp = torch.as_tensor(pose_prob).to(device=records.device, dtype=torch.int32).contiguous()
    if P.dim() != 2 or P.shape[1] != 7 or pp.numel() != K:
        raise ValueError("pose_energy_records: poses (K,7), one problem index per pose")
    energy = torch.empty((K,), dtype=torch.float32, device=records.device)
    rc = _lib.load().pcnn_energy_rec(_lib.ptr(records), _lib.ptr(counts), records.shape[1], _lib.ptr(P), _lib.ptr(pp),
                                     K, float(depth_range[0]), float(depth_range[1]), _lib.ptr(energy),
                                     _lib.stream_ptr(stream))
    _lib.check(rc, "pose_energy_records")
    return energy


NM_PATHS = {0: "auto", 1: "k_nm_spec (speculative rounds, cooperative)", 2: "k_nm<8> (cooperative)",
            3: "k_nm<1> (one workgroup per problem)"}


def nelder_mead_device(records, counts, x0, lb, ub, max_eval, depth_range=(0.25, 6.0), stream=None, force_path=None,
                       return_path=False):
    """The bounded Nelder-Mead of nelder_mead_steps on optEnergy, for N
    problems at once on the device (eight cooperating workgroups per
    evaluated point, up to four points of a step per round while N <= 32; no
    host read until the end): x0 / lb / ub (N,7) float64.  Returns (x (N,7), f (N,), nev (N,))
    as device tensors; the same bits as nelder_mead over pose_energy_records.
    nev[i] = -1: a cross-workgroup wait of problem i gave up (results invalid).
    max_eval must cover the initial simplex (>= 8; NLopt's maxeval counts it).
    force_path (or env PCNN_NM_PATH) pins the kernel (NM_PATHS: 1 speculative,
    2 cooperative, 3 one workgroup); return_path adds the path that ran."""
    _lib.require_gpu(records, counts)
    if int(max_eval) < 8:
        raise ValueError("nelder_mead_device: max_eval must be >= 8 (the 7-D initial simplex)")
    if force_path is None:
        force_path = int(os.environ.get("PCNN_NM_PATH", "0") or 0)
    if force_path not in NM_PATHS:
        raise ValueError(f"nelder_mead_device: force_path in {sorted(NM_PATHS)}")
    dev = records.device
    d64 = dict(dtype=torch.float64, device=dev)
    x0_, lb_, ub_ = (torch.as_tensor(a).to(**d64).contiguous() for a in (x0, lb, ub))
    N = records.shape[0]
    if x0_.shape != (N, 7) or lb_.shape != (N, 7) or ub_.shape != (N, 7):
        raise ValueError("nelder_mead_device: x0, lb, ub (N,7), one row per problem")
    x = torch.empty((N, 7), **d64)
    f = torch.empty((N,), **d64)
    nev = torch.empty((N,), dtype=torch.int32, device=dev)
    L = _lib.load()
    path = ctypes.c_int32(0)
    if N <= 128:  # kNmCoop workgroups per problem, launched cooperatively (same bits as one workgroup)
        ws = _lib.workspace(L.pcnn_nelder_mead_energy_workspace_size(N), dev, "nelder_mead", stream)
        rc = L.pcnn_nelder_mead_energy_coop_path(_lib.ptr(records), _lib.ptr(counts), records.shape[1], N,
                                                 _lib.ptr(x0_), _lib.ptr(lb_), _lib.ptr(ub_), int(max_eval),
                                                 float(depth_range[0]), float(depth_range[1]), _lib.ptr(x),
                                                 _lib.ptr(f), _lib.ptr(nev), _lib.ptr(ws), ws.numel(), int(force_path),
                                                 ctypes.byref(path), _lib.stream_ptr(stream))
    else:
        if force_path not in (0, 3):
            raise ValueError("nelder_mead_device: more than 128 problems run on the one-workgroup path only")
        rc = L.pcnn_nelder_mead_energy(_lib.ptr(records), _lib.ptr(counts), records.shape[1], N, _lib.ptr(x0_),
                                       _lib.ptr(lb_), _lib.ptr(ub_), int(max_eval), float(depth_range[0]),
                                       float(depth_range[1]), _lib.ptr(x), _lib.ptr(f), _lib.ptr(nev),
                                       _lib.stream_ptr(stream))
        path.value = 3
    _lib.check(rc, "nelder_mead_device")
    return (x, f, nev, int(path.value)) if return_path else (x, f, nev)


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


def nelder_mead_steps(x0, lb, ub, max_eval):
    """Bounded Nelder-Mead (NLopt LN_NELDERMEAD's role in poseWithOpt,
    synthesize.cpp:2529-2573) as a generator: it yields (m, n) arrays of points
    to evaluate and receives their m values (send), and returns (x, f).  The
    initial simplex and a shrink step are asked for as one batch; otherwise one
    point at a time, in the same order and count as the sequential search.
    Initial steps NLopt's default (a quarter of the bound range, 0.75 of the
    distance to a nearer bound), reflection 1, expansion 2, contraction 1/2,
    shrink 1/2, trial points clamped to the bounds, at most max_eval
    evaluations.  NLopt is absent here: the search's exact trajectory is
    unpinned."""
    import numpy as np
    x0 = np.asarray(x0, np.float64)
    n = x0.size
    lb, ub = np.asarray(lb, np.float64), np.asarray(ub, np.float64)
    step = np.minimum(0.25 * (ub - lb), np.minimum(0.75 * (ub - x0), 0.75 * (x0 - lb)))
    pts = [x0] + [x0 + step[i] * np.eye(n)[i] for i in range(n)]
    vals = list((yield np.stack(pts)))
    nev = len(pts)
    clamp = lambda p: np.minimum(np.maximum(p, lb), ub)
    one = lambda p: float((yield p[None])[0])  # noqa: E731 (a one-point request)
    while nev < max_eval:
        order = np.argsort(vals, kind="stable")
        pts = [pts[i] for i in order]
        vals = [vals[i] for i in order]
        c = np.mean(pts[:-1], axis=0)
        xr = clamp(c + (c - pts[-1]))
        fr = yield from one(xr)
        nev += 1
        if fr < vals[0] and nev < max_eval:
            xe = clamp(c + 2 * (c - pts[-1]))
            fe = yield from one(xe)
            nev += 1
            pts[-1], vals[-1] = (xe, fe) if fe < fr else (xr, fr)
        elif fr < vals[-2]:
            pts[-1], vals[-1] = xr, fr
        elif nev < max_eval:
            xc = clamp(c + 0.5 * (pts[-1] - c)) if fr >= vals[-1] else clamp(c + 0.5 * (xr - c))
            fc = yield from one(xc)
            nev += 1
            if fc < min(fr, vals[-1]):
                pts[-1], vals[-1] = xc, fc
            else:
                m = min(n, max_eval - nev)
                if m > 0:
                    new = [clamp(pts[0] + 0.5 * (pts[i] - pts[0])) for i in range(1, m + 1)]
                    fv = list((yield np.stack(new)))
                    for i in range(1, m + 1):
                        pts[i], vals[i] = new[i - 1], fv[i - 1]
                    nev += m
    i = int(np.argmin(vals))
    return pts[i], vals[i]


def nelder_mead(f, x0, lb, ub, max_eval):
    """The search of nelder_mead_steps driven by a scalar function f."""
    import numpy as np
    gen = nelder_mead_steps(x0, lb, ub, max_eval)
    try:
        req = next(gen)
        while True:
            req = gen.send(np.array([f(p) for p in req]))
    except StopIteration as e:
        return e.value


def nelder_mead_batch(fbatch, starts, lb, ub, max_eval):
    """Lock-step Nelder-Mead searches, one per start: every round collects the
    pending requests of all live searches and evaluates them with ONE call
    fbatch(list of (search, points)) -> list of value arrays (solve_icp: one
    batched optEnergy launch for every RoI's simplex)."""
    gens = [nelder_mead_steps(x0, l, u, max_eval) for x0, l, u in zip(starts, lb, ub)]
    res = [None] * len(gens)
    reqs = {}
    for i, g in enumerate(gens):
        reqs[i] = next(g)
    while reqs:
        items = sorted(reqs.items())
        vals = fbatch(items)
        reqs = {}
        for (i, _), v in zip(items, vals):
            try:
                reqs[i] = gens[i].send(v)
            except StopIteration as e:
                res[i] = e.value
    return res


def _render_many(render, objs, poses):
    """(vertmap, pred_vertices, pred_normals) stacked over K (object, pose)
    pairs: one call of render.render_many(objs, poses) when the renderer
    offers a batched pass, else K calls of render(obj, pose)."""
    many = getattr(render, "render_many", None)
    if many is not None:
        return many(list(objs), np.stack([np.asarray(p, np.float32) for p in poses]))
    maps = [render(o, p) for o, p in zip(objs, poses)]
    return tuple(torch.stack([m[i] for m in maps]) for i in range(3))


def solve_icp(labelmap, depth, parameters, rois, poses, render, max_error=0.01, nm_evals=50, icp_iterations=8,
              min_pixels=400, nm_device=True, stream=None):
    """Synthesizer::solveICP (synthesize.cpp:2052-2395) on the GPU ops above,
    batched over the RoIs (the reference refines them one after another; no
    state passes between RoIs, :2090-2392).

    labelmap (H,W) int32, depth (H,W) uint16, parameters = (fx, fy, px, py,
    znear, zfar, factor) (icp_python's meta, synthesize.cpp:2031-2049), rois
    (R, >= 2) with the class at column 1, poses (R,7).  render(obj_id, pose7)
    -> (vertmap (H,W,3), pred_vertices (H,W,4), pred_normals (H,W,4)) device
    tensors stands in for the reference's OpenGL pass (a renderer with a
    render_many(objs, poses (K,7)) method is called once per stage with every
    pose of the stage instead: three calls per solve).  Returns (poses_new,
    poses_icp) (R,7) as the reference fills `outputs` / `outputs_icp`: rows of
    skipped RoIs stay zero.  The steps, each one launch for all RoIs: live
    vertices of every RoI's object; the >= min_pixels test (one host read);
    the translation re-centring (one host read); the Nelder-Mead search on
    optEnergy (nm_evals evaluations each, 0 skips it): every RoI's search in
    one launch on the device, one host read at its end (nm_device=False: the
    same searches driven from the host, one energy launch and one host read
    per lock-step round -- the reference driver its tests compare against,
    bit for bit); the eight
    depth hypotheses of every RoI refined by one 8-iteration ICP launch; the
    SegICP score per RoI, its choice read once at the end."""
    if nm_evals and int(nm_evals) < 8:
        raise ValueError("solve_icp: nm_evals must be 0 (no search) or >= 8 (the 7-D initial simplex)")
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
    lab = labelmap.contiguous().to(torch.int32)
    cand = [i for i in range(R_) if int(rois_h[i, 1]) > 0]
    if not cand:
        return poses_new, poses_icp
    objs = [int(rois_h[i, 1]) for i in cand]
    # the object's pixel count (:2152-2160, >= 400 to go on): one histogram, one host read
    counts = torch.bincount(lab.reshape(-1).long(), minlength=max(objs) + 1).cpu().numpy()
    keep = [k for k, o in enumerate(objs) if counts[o] >= min_pixels]
    if not keep:
        return poses_new, poses_icp
    rows = [cand[k] for k in keep]
    objs = [objs[k] for k in keep]
    n = len(rows)
    objt = torch.tensor(objs, dtype=torch.int32, device=dev)
    live = live_vertices(depth, lab, objt, factor, cam, stream)          # (n, H, W, 3)
    T = []
    for i in rows:
        p = poses_h[i].astype(np.float64)
        T.append(np.concatenate([p[:4] / np.linalg.norm(p[:4]), p[4:7]]).astype(np.float32))
    vm, pv_c, pn_c = _render_many(render, objs, T)
    out, Tc = icp_center(live, lab, objt, vm, pv_c, pn_c, max_error, pose_in=torch.from_numpy(np.stack(T)).to(dev),
                         stream=stream)
    cT = torch.cat([out[:, 3:4].float(), Tc.float()], 1).cpu().numpy()  # one host read
    c_h, Tc_h = cT[:, 0], cT[:, 1:].astype(np.float32)
    for k in range(n):
        if c_h[k] > 0:
            T[k] = Tc_h[k]
    nm = [k for k in range(n) if c_h[k] > 0] if nm_evals > 0 else []
    if nm:  # refinePose(..., 0): optEnergy over a correction of each re-rendered pose (:2221-2250)
        pv0 = _render_many(render, [objs[k] for k in nm], [T[k] for k in nm])[1]
        x0 = np.array([1, 0, 0, 0, 0, 0, 0], np.float64)
        r = np.array([0.1, 0.1, 0.1, 0.1, 0.01, 0.01, 0.1])  # poseWithOpt's bounds (:2535-2558)
        rec, cnt = energy_records(live, lab, [objs[k] for k in nm], nm, pv0, (znear, zfar), stream)
        X0 = np.repeat(x0[None], len(nm), 0)
        res = None
        if nm_device:
            xs, _, nev = nelder_mead_device(rec, cnt, X0, X0 - r, X0 + r, nm_evals, (znear, zfar), stream)
            xn = torch.cat([xs, nev.view(-1, 1).double()], 1).cpu().numpy()  # one host read
            if (xn[:, -1] >= 0).all():
                res = [(x, None) for x in xn[:, :-1]]
            # else: a cross-workgroup wait gave up (nev -1): the host-driven
            # search below, which gives the same bits when the device one works
        if res is None:
            def energies(items):  # every search's pending points: one launch, one host read
                P = np.concatenate([pts for _, pts in items]).astype(np.float32)
                who = np.concatenate([np.full(len(pts), j, np.int32) for j, pts in items])
                e = pose_energy_records(rec, cnt, torch.from_numpy(P).to(dev), torch.from_numpy(who), (znear, zfar),
                                        stream).cpu().numpy()
                out_, o = [], 0
                for _, pts in items:
                    out_.append(e[o:o + len(pts)].astype(np.float64))
                    o += len(pts)
                return out_
            res = nelder_mead_batch(energies, [x0] * len(nm), [x0 - r] * len(nm), [x0 + r] * len(nm), nm_evals)
        for j, k in enumerate(nm):
            x = res[j][0]
            T[k] = _se3_mul(np.concatenate([x[:4] / np.linalg.norm(x[:4]), x[4:]]), T[k]).astype(np.float32)
    # eight depth hypotheses per RoI (:2255-2280), all refined by one ICP launch
    hyps = np.repeat(np.stack(T)[:, None], len(dz), 1)                    # (n, 8, 7)
    hyps[:, 1:, 6] = np.stack(T)[:, 6:7] + np.array(dz[1:])[None]
    _, pvs, pns = _render_many(render, [objs[k] for k in range(n) for _ in dz], list(hyps.reshape(-1, 7)))
    li = torch.arange(n, dtype=torch.int32, device=dev).repeat_interleave(len(dz))
    _, refined = icp(live, pvs, pns, cam, (znear, zfar), max_error, icp_iterations, live_index=li,
                     pose_in=torch.from_numpy(hyps.reshape(-1, 7)).to(dev), stream=stream)
    refined = refined.view(n, len(dz), 7)
    chosen = [icp_score(live[k], lab, objs[k], vm[k], refined[k], 0.01, stream)[1] for k in range(n)]
    chr_ = torch.cat([torch.cat(chosen).float()[:, None], refined.reshape(n, -1).float()], 1).cpu().numpy()
    ch, ref_h = chr_[:, 0].astype(np.int64), chr_[:, 1:].reshape(n, len(dz), 7).astype(np.float32)  # one host read
    for k, i in enumerate(rows):
        poses_new[i] = T[k]
        poses_icp[i] = ref_h[k, int(ch[k])]
    return poses_new, poses_icp
