"""RGB-only pose estimation (the RANSAC half), backed
by libposecnn_hip.so (csrc/pose2d.hip).

Mirrors Synthesizer.estimate_poses_2d (lib/synthesize/synthesizer.pyx:74-82)
over Synthesizer::estimatePose2D (synthesize.cpp:1571-1766), as
lib/fcn/test.py:1364 calls it:

    estimate_poses_2d(labels, vertmap, extents, poses, num_classes, fx, fy, px, py)

labels (H,W) int32, vertmap (H,W,3C) object coordinates scaled to [0,1] by the
class extents, extents (C,3), poses (3,4,C) float32 filled in place with
[R | t] per class found (test.py:1365-1376 then reads poses[2,3,j] > 0).
Inputs may be numpy arrays (as the reference passes them) or device tensors;
the compute runs on the GPU only."""
import numpy as np
import torch

from .. import _lib


def _dev_tensor(x, dtype, device):
    if torch.is_tensor(x):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(x)).to(device=device, dtype=dtype)


def estimate_poses_2d(labels, vertmap, extents, poses, num_classes, fx, fy, px, py, seed=1305, n_hyp=256,
                      max_iter=100000, return_diag=False, stream=None):
    """Fills poses (3, 4, num_classes) in place; returns it (and a diagnostics
    dict -- hypotheses, sampled pixels, per-round inliers, survivors -- when
    return_diag)."""
    if not torch.cuda.is_available():
        raise _lib.PcnnError("posecnn_amd ops run only on an AMD GPU (HIP); none is visible")
    dev = vertmap.device if torch.is_tensor(vertmap) and vertmap.is_cuda else torch.device("cuda")
    lab = _dev_tensor(labels, torch.int32, dev)
    vm = _dev_tensor(vertmap, torch.float32, dev)
    ext = _dev_tensor(extents, torch.float32, dev)
    C = int(num_classes)
    if lab.dim() != 2:
        raise ValueError("estimate_poses_2d: labels must be (H, W)")
    H, W = lab.shape
    if vm.shape != (H, W, 3 * C) or ext.shape != (C, 3):
        raise ValueError("estimate_poses_2d: vertmap (H, W, 3 num_classes), extents (num_classes, 3)")
    if tuple(poses.shape) != (3, 4, C):
        raise ValueError("estimate_poses_2d: poses must be (3, 4, num_classes)")
    if not 0 < n_hyp <= 256:  # the reference's ransacIterations (synthesize.cpp:1601): 8 rounds halve to one
        raise ValueError("estimate_poses_2d: n_hyp in 1..256")
    f32 = dict(dtype=torch.float32, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    out = torch.zeros((3, 4, C), **f32)
    hyps = torch.empty((n_hyp, 13), **f32)
    hpx = torch.empty((n_hyp, 4), **i32)
    inl = torch.empty((n_hyp, 8), **i32)
    fin = torch.empty((C, 3), **i32)
    L = _lib.load()
    ws = _lib.workspace(L.pcnn_pose2d_workspace_size(H, W, C, n_hyp), dev, "pose2d", stream)
    rc = L.pcnn_pose2d(_lib.ptr(lab), _lib.ptr(vm), _lib.ptr(ext), H, W, C, float(fx), float(fy), float(px),
                       float(py), int(seed) & ((1 << 64) - 1), int(n_hyp), int(max_iter), _lib.ptr(out),
                       _lib.ptr(hyps), _lib.ptr(hpx), _lib.ptr(inl), _lib.ptr(fin), _lib.ptr(ws), ws.numel(),
                       _lib.stream_ptr(stream))
    _lib.check(rc, "pose2d")
    if torch.is_tensor(poses):
        poses.copy_(out.to(poses.device))
    else:
        poses[...] = out.cpu().numpy()
    if return_diag:
        return poses, dict(hyps=hyps, hyp_px=hpx, inliers=inl, final=fin)
    return poses
