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


def average_distance_loss_prep(bottom_weight, bottom_symmetry, num_points, workspace, num_rois=None, points=None):
    """Row classification of the loss (pcnn_add_loss_prep) into `workspace`
    (uint8, >= workspace_bytes); may run on another stream as soon as the
    weights exist.  Follow with average_distance_loss(..., prepared=True,
    workspace=workspace) ordered after it.  With the model `points` (C, P, 3)
    it also orders the symmetric classes' points for the pruned ADD-S search
    (pcnn_add_loss_prep_points); without them the loss scans in full (the
    same bits)."""
    _lib.require_gpu(bottom_weight, bottom_symmetry, workspace)
    w = bottom_weight.contiguous().float()
    R, PC = w.shape
    lib = _lib.load()
    if points is not None:
        if points.shape[1] != num_points:
            raise ValueError("average_distance_loss_prep: points (C, num_points, 3)")
        rc = lib.pcnn_add_loss_prep_points(_lib.ptr(w), _lib.ptr(bottom_symmetry.contiguous().float()),
                                           _lib.ptr(points.contiguous().float()), R, _lib.ptr(num_rois), PC // 4,
                                           int(num_points), _lib.ptr(workspace), workspace.numel(),
                                           _lib.stream_ptr())
    else:
        rc = lib.pcnn_add_loss_prep(_lib.ptr(w), _lib.ptr(bottom_symmetry.contiguous().float()), R,
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


def average_distance_loss_head_bwd(pred, target, weight, points, symmetry, margin, tanh_out, d_pred_scale, diff, dy8,
                                   workspace, num_rois=None, loss_norm_rows_dev=None):
    """The pose step's fused loss tail (pcnn_add_loss_fwd_head_bwd, prepared
    rows): bottom_diff into `diff` and the pose head's backward of it into
    `dy8`; the scalar loss follows with average_distance_loss_total."""
    _lib.require_gpu(pred, target, weight, points, symmetry, tanh_out, diff, dy8, workspace)
    R, PC = pred.shape
    rc = _lib.load().pcnn_add_loss_fwd_head_bwd(
        _lib.ptr(pred), _lib.ptr(target), _lib.ptr(weight), _lib.ptr(points), _lib.ptr(symmetry), R,
        _lib.ptr(num_rois), PC // 4, points.shape[1], float(margin), 0, _lib.ptr(loss_norm_rows_dev), _lib.ptr(diff),
        _lib.ptr(workspace), workspace.numel(), _lib.ptr(tanh_out), _lib.ptr(d_pred_scale), _lib.ptr(dy8),
        _lib.stream_ptr())
    _lib.check(rc, "average_distance_loss_head_bwd")


def average_distance_loss_total(R, num_classes, num_points, workspace, loss, num_rois=None):
    """The scalar loss of an average_distance_loss_head_bwd call (its row losses in `workspace`)."""
    _lib.require_gpu(workspace, loss)
    rc = _lib.load().pcnn_add_loss_total(R, _lib.ptr(num_rois), num_classes, num_points, _lib.ptr(workspace),
                                         workspace.numel(), _lib.ptr(loss), _lib.stream_ptr())
    _lib.check(rc, "average_distance_loss_total")


def search_diagnostics(workspace, R, num_classes, num_points):
    """(Morton orders (C, P) int32, [blocks scanned, blocks held]) that the
    pruned ADD-S search left in `workspace` (None when it is off)."""
    lib = _lib.load()
    o_perm = lib.pcnn_add_loss_ws_offset(R, num_classes, num_points, 0)
    o_stat = lib.pcnn_add_loss_ws_offset(R, num_classes, num_points, 1)
    if o_perm < 0:
        return None
    n = num_classes * num_points * 4
    perm = workspace[o_perm:o_perm + n].view(torch.int32).view(num_classes, num_points)
    stat = workspace[o_stat:o_stat + 8].view(torch.int32)
    return perm, stat


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
