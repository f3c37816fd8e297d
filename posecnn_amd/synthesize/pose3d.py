"""Depth-based pose estimation (the
cfg.TEST.VERTEX_REG_3D branch), backed by libposecnn_hip.so
(csrc/pose2d.hip, pcnn_pose3d).

Mirrors Synthesizer.estimate_poses_3d (lib/synthesize/synthesizer.pyx:86-95)
over Synthesizer::estimatePose3D (synthesize.cpp:1769-1965), as
lib/fcn/test.py:1385 calls it:

    estimate_poses_3d(labels, depth, vertmap, extents, poses, num_classes, fx, fy, px, py, factor)

labels (H,W) int32, depth (H,W) uint16 raw depth (metres = depth / factor),
vertmap (H,W,3C) object coordinates scaled to [0,1] by the class extents,
extents (C,3), poses (3,4,C) float32 filled in place with [R | t] per class
found; test.py:1386-1416 then hands them to refine_poses (solveICP,
posecnn_amd.synthesize.icp.solve_icp).  Inputs may be numpy arrays or device
tensors; the compute runs on the GPU only."""
import numpy as np
import torch

from .. import _lib
from .pose2d import _dev_tensor


def estimate_poses_3d(labels, depth, vertmap, extents, poses, num_classes, fx, fy, px, py, factor, seed=1305,
                      n_hyp=256, max_iter=100000, nm_evals=100, return_diag=False, stream=None):
    """Fills poses (3, 4, num_classes) in place; returns it (and a diagnostics
    dict -- hypotheses, sampled pixels, per-round inliers, survivors, refined
    energies, camera coordinates -- when return_diag)."""
    if not torch.cuda.is_available():
        raise _lib.PcnnError("posecnn_amd ops run only on an AMD GPU (HIP); none is visible")
    dev = vertmap.device if torch.is_tensor(vertmap) and vertmap.is_cuda else torch.device("cuda")
    lab = _dev_tensor(labels, torch.int32, dev)
    # the raw uint16 depth travels as int16 of the same bits (the kernel reads
    # uint16).  Only integer raw units are accepted: a float map (e.g. depth
    # already in metres) would truncate to holes / single units,
    # and values outside 0..65535 would wrap
    if torch.is_tensor(depth):
        d = depth
        if d.dtype.is_floating_point or d.dtype.is_complex or d.dtype == torch.bool:
            raise ValueError("estimate_poses_3d: depth must hold raw integer sensor units (uint16 / int16 / "
                             "int32), not %s; convert metres with round(depth * factor) first" % d.dtype)
        if d.dtype == torch.uint16:
            d = d.view(torch.int16)
        elif d.dtype == torch.int16:
            if bool((d < 0).any()):
                raise ValueError("estimate_poses_3d: negative raw depth (int16 is read as uint16 bits only for "
                                 "torch.uint16 inputs)")
        else:
            d = d.to(torch.int64)
            if bool(((d < 0) | (d > 65535)).any()):
                raise ValueError("estimate_poses_3d: raw depth outside 0..65535")
            d = torch.where(d > 32767, d - 65536, d).to(torch.int16)
        dep = d.to(dev).contiguous()
    else:
        a = np.asarray(depth)
        if a.dtype.kind not in "ui":
            raise ValueError("estimate_poses_3d: depth must hold raw integer sensor units (uint16 / int16 / int32), "
                             "not %s; convert metres with round(depth * factor) first" % a.dtype)
        if a.size and (int(a.min()) < 0 or int(a.max()) > 65535):
            raise ValueError("estimate_poses_3d: raw depth outside 0..65535")
        dep = torch.from_numpy(np.ascontiguousarray(a, np.uint16).view(np.int16)).to(dev)
    vm = _dev_tensor(vertmap, torch.float32, dev)
    ext = _dev_tensor(extents, torch.float32, dev)
    C = int(num_classes)
    if lab.dim() != 2:
        raise ValueError("estimate_poses_3d: labels must be (H, W)")
    H, W = lab.shape
    if tuple(dep.shape) != (H, W):
        raise ValueError("estimate_poses_3d: depth must be (H, W) like labels")
    if vm.shape != (H, W, 3 * C) or ext.shape != (C, 3):
        raise ValueError("estimate_poses_3d: vertmap (H, W, 3 num_classes), extents (num_classes, 3)")
    if tuple(poses.shape) != (3, 4, C):
        raise ValueError("estimate_poses_3d: poses must be (3, 4, num_classes)")
    if not 0 < n_hyp <= 256:  # ransacIterations (synthesize.cpp:1794): 8 rounds halve to one
        raise ValueError("estimate_poses_3d: n_hyp in 1..256")
    if not float(factor) > 0:
        raise ValueError("estimate_poses_3d: factor must be positive")
    if int(nm_evals) < 7:  # the 6-D search's initial simplex; NLopt's maxeval counts it too
        raise ValueError("estimate_poses_3d: nm_evals must be >= 7 (the initial simplex)")
    f32 = dict(dtype=torch.float32, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    out = torch.zeros((3, 4, C), **f32)
    hyps = torch.empty((n_hyp, 13), **f32)
    hpx = torch.empty((n_hyp, 3), **i32)
    inl = torch.empty((n_hyp, 8), **i32)
    fin = torch.empty((C, 3), **i32)
    en = torch.empty((C,), **f32)
    eye = torch.empty((H, W, 3), **f32) if return_diag else None
    L = _lib.load()
    ws = _lib.workspace(L.pcnn_pose3d_workspace_size(H, W, C, n_hyp), dev, "pose3d", stream)
    rc = L.pcnn_pose3d(_lib.ptr(lab), _lib.ptr(dep), _lib.ptr(vm), _lib.ptr(ext), H, W, C, float(fx), float(fy),
                       float(px), float(py), float(factor), int(seed) & ((1 << 64) - 1), int(n_hyp), int(max_iter),
                       int(nm_evals), _lib.ptr(out), _lib.ptr(hyps), _lib.ptr(hpx), _lib.ptr(inl), _lib.ptr(fin),
                       _lib.ptr(en), _lib.ptr(eye) if eye is not None else None, _lib.ptr(ws), ws.numel(),
                       _lib.stream_ptr(stream))
    _lib.check(rc, "pose3d")
    if torch.is_tensor(poses):
        poses.copy_(out.to(poses.device))
    else:
        poses[...] = out.cpu().numpy()
    if return_diag:
        return poses, dict(hyps=hyps, hyp_px=hpx, inliers=inl, final=fin, energy=en, eye=eye)
    return poses
