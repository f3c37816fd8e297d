"""Drop-in for lib/average_distance_loss/average_distance_loss_op.py (:4-7):
`average_distance_loss` / `average_distance_loss_grad` (REGISTER_OP
"Averagedistance" / "AveragedistanceGrad", average_distance_loss_op.cc:38-54),
backed by libposecnn_hip.so.

average_distance_loss(pred (R,4C), target, weight, points (C,P,3), symmetry (C), margin)
    -> (loss (1,), bottom_diff (R,4C))   [ADD, or ADD-S for symmetric classes]
average_distance_loss_grad(bottom_diff, grad, margin) -> grad[0] * bottom_diff
"""
import torch

from .. import _lib


def workspace_bytes(R, num_classes, num_points):
    return _lib.load().pcnn_add_loss_workspace_size(R, num_classes, num_points)


def average_distance_loss_prep(bottom_weight, bottom_symmetry, num_points, workspace, num_rois=None):
    """Row classification of the loss (pcnn_add_loss_prep) into `workspace`
    (uint8, >= workspace_bytes); may run on another stream as soon as the
    weights exist.  Follow with average_distance_loss(..., prepared=True,
    workspace=workspace) ordered after it."""
    _lib.require_gpu(bottom_weight, bottom_symmetry, workspace)
    w = bottom_weight.contiguous().float()
    R, PC = w.shape
    rc = _lib.load().pcnn_add_loss_prep(_lib.ptr(w), _lib.ptr(bottom_symmetry.contiguous().float()), R,
                                        _lib.ptr(num_rois), PC // 4, int(num_points), _lib.ptr(workspace),
                                        workspace.numel(), _lib.stream_ptr())
    _lib.check(rc, "average_distance_loss_prep")


def average_distance_loss(bottom_prediction, bottom_target, bottom_weight, bottom_point, bottom_symmetry, margin,
                          name=None, num_rois=None, loss_norm_rows=0, loss_norm_rows_dev=None, out=None,
                          workspace=None, prepared=False):
    _lib.require_gpu(bottom_prediction, bottom_target, bottom_weight, bottom_point, bottom_symmetry)
    if margin < 0:
        raise ValueError(f"Need margin >= 0, got {margin}")  # average_distance_loss_op.cc:64-65
    pred = bottom_prediction.contiguous().float()
    R, PC = pred.shape
    C = PC // 4
    P = bottom_point.shape[1]
    lib = _lib.load()
    if prepared and workspace is None:
        raise ValueError("prepared=True needs the workspace average_distance_loss_prep wrote")
    ws = workspace if workspace is not None else _lib.workspace(lib.pcnn_add_loss_workspace_size(R, C, P),
                                                                pred.device, "add_loss")
    if out is None:
        loss = torch.empty((1,), dtype=torch.float32, device=pred.device)
        diff = torch.empty((R, PC), dtype=torch.float32, device=pred.device)
    else:
        loss, diff = out
    fn = lib.pcnn_add_loss_fwd_prepared if prepared else lib.pcnn_add_loss_fwd
    rc = fn(_lib.ptr(pred), _lib.ptr(bottom_target.contiguous().float()), _lib.ptr(bottom_weight.contiguous().float()),
            _lib.ptr(bottom_point.contiguous().float()), _lib.ptr(bottom_symmetry.contiguous().float()), R,
            _lib.ptr(num_rois), C, P, float(margin), int(loss_norm_rows), _lib.ptr(loss_norm_rows_dev), _lib.ptr(loss),
            _lib.ptr(diff), _lib.ptr(ws), ws.numel(), _lib.stream_ptr())
    _lib.check(rc, "average_distance_loss")
    return loss, diff


def average_distance_loss_grad(bottom_diff, grad, margin=0.01, name=None, num_rois=None, out=None):
    _lib.require_gpu(bottom_diff, grad)
    bd = bottom_diff.contiguous()
    o = out if out is not None else torch.empty_like(bd)
    rc = _lib.load().pcnn_add_loss_bwd(_lib.ptr(grad.contiguous().float()), _lib.ptr(bd), bd.numel(),
                                       _lib.ptr(num_rois), bd.shape[-1], _lib.ptr(o), _lib.stream_ptr())
    _lib.check(rc, "average_distance_loss_grad")
    return o


class AverageDistanceFunction(torch.autograd.Function):
    """autograd binding (average_distance_loss_op_grad.py:5-14)."""

    @staticmethod
    def forward(ctx, pred, target, weight, points, symmetry, margin):
        loss, diff = average_distance_loss(pred, target, weight, points, symmetry, margin)
        ctx.save_for_backward(diff)
        ctx.margin = margin
        return loss

    @staticmethod
    def backward(ctx, grad):
        (diff,) = ctx.saved_tensors
        return average_distance_loss_grad(diff, grad.reshape(1), ctx.margin), None, None, None, None, None
