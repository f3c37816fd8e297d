"""Drop-in for lib/hard_label_layer/hard_label_op.py (:4-7): `hard_label` /
`hard_label_grad`, backed by libposecnn_hip.so (pcnn_hard_label_fwd/bwd).

REGISTER_OP("Hardlabel") (hard_label_op.cc:30-44): bottom_prob (B,H,W,C)
float, bottom_gt (B,H,W) int32, attr threshold > 0 -> top_data (B,H,W,C): the
one-hot of gt where gt != -1 and (gt > 0 or prob[gt] < threshold)
(hard_label_op_gpu.cu.cc:17-29).  The gradient (hard_label_op_grad.py:12-24,
cu.cc:56-64) is zero for both inputs.
"""
import torch

from .. import _lib


def hard_label(bottom_prob, bottom_gt, threshold, name=None):
    _lib.require_gpu(bottom_prob, bottom_gt)
    if float(threshold) <= 0:
        raise ValueError(f"Need threshold > 0, got {threshold}")  # hard_label_op.cc:50-52
    if bottom_prob.dim() != 4:
        raise ValueError("prob must be 4-dimensional")  # hard_label_op.cc:68-69
    if bottom_gt.dim() != 3:
        raise ValueError("gt label must be 3-dimensional")  # :70-71
    B, H, W, C = bottom_prob.shape
    if tuple(bottom_gt.shape) != (B, H, W):
        raise ValueError(f"gt shape {tuple(bottom_gt.shape)} does not match prob {tuple(bottom_prob.shape)}")
    prob = bottom_prob.contiguous().float()
    gt = bottom_gt.contiguous().to(torch.int32)
    top = torch.empty((B, H, W, C), dtype=torch.float32, device=prob.device)
    rc = _lib.load().pcnn_hard_label_fwd(_lib.ptr(prob), _lib.ptr(gt), B, H, W, C, float(threshold), _lib.ptr(top),
                                         _lib.stream_ptr())
    _lib.check(rc, "hard_label")
    return top


def hard_label_grad(bottom_prob, bottom_gt, grad, threshold, name=None):
    """HardlabelGrad: (zeros like prob, zeros (B,H,W) float for gt)."""
    _lib.require_gpu(bottom_prob, bottom_gt, grad)
    B, H, W, C = bottom_prob.shape
    gp = torch.empty((B, H, W, C), dtype=torch.float32, device=bottom_prob.device)
    gg = torch.empty((B, H, W), dtype=torch.float32, device=bottom_prob.device)
    rc = _lib.load().pcnn_hard_label_bwd(_lib.ptr(gp), _lib.ptr(gg), B, H, W, C, _lib.stream_ptr())
    _lib.check(rc, "hard_label_grad")
    return gp, gg
