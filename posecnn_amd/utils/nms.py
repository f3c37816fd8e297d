"""Device box NMS with the surface of lib/utils/nms.py (the reference's numpy
NMS over the Hough op's RoI rows) plus the pose combination of
lib/fcn/test.py:197-211, both on the HIP kernel pcnn_box_nms.

    keep = nms(rois, 0.5)                      # list of kept row indices (nms.py:3)
    keep_dev, n = nms_device(rois, 0.5)        # device tensors, no host sync
    rois_k, poses_k, n = nms_combine(rois, poses_init, poses_pred, 0.5)

Order of equal scores: numpy's argsort()[::-1] leaves it unspecified; here the
lower row index goes first.
"""
import torch

from .. import _lib

MAX_ROWS = 1152  # MAX_ROI * 9, the Hough op's row capacity


def _run(dets, thresh, num_rois=None, poses_init=None, poses_pred=None, keep=None, out=None):
    _lib.require_gpu(dets)
    d = dets.contiguous().float()
    R, stride = d.shape
    if R > MAX_ROWS:
        raise ValueError(f"nms: at most {MAX_ROWS} rows (got {R})")
    if stride < 7:
        raise ValueError("nms: rows are [b, cls, x1, y1, x2, y2, score]")
    dev = d.device
    keep = keep if keep is not None else torch.empty((max(R, 1),), dtype=torch.int32, device=dev)
    num_keep = torch.zeros((1,), dtype=torch.int32, device=dev)
    rois_out = poses_out = None
    pi = pp = None
    pred_dim = 0
    if poses_init is not None:
        pi = poses_init.contiguous().float()
        pp = poses_pred.contiguous().float() if poses_pred is not None else None
        pred_dim = pp.shape[1] if pp is not None else 0
        rois_out, poses_out = out if out is not None else (torch.zeros((max(R, 1), 7), device=dev),
                                                            torch.zeros((max(R, 1), 7), device=dev))
    rc = _lib.load().pcnn_box_nms(_lib.ptr(d), R, stride, _lib.ptr(num_rois), float(thresh), _lib.ptr(keep),
                                  _lib.ptr(num_keep), _lib.ptr(pi), _lib.ptr(pp), pred_dim, _lib.ptr(rois_out),
                                  _lib.ptr(poses_out), _lib.stream_ptr())
    _lib.check(rc, "nms")
    return keep, num_keep, rois_out, poses_out


def nms(dets, thresh):
    """lib/utils/nms.py:3 — indices of the kept rows, highest score first (one D2H)."""
    keep, n, _, _ = _run(dets, thresh)
    return keep[: int(n.item())].tolist()


def nms_device(dets, thresh, num_rois=None):
    """Kept row indices (capacity-sized int32) and their count, on the device."""
    keep, n, _, _ = _run(dets, thresh, num_rois=num_rois)
    return keep, n


def nms_combine(rois, poses_init, poses_pred, thresh, num_rois=None, out=None):
    """test.py:197-211 on the device: kept rows, their initial poses with the
    quaternion replaced by the class's predicted one, and the kept count."""
    _, n, r, p = _run(rois, thresh, num_rois=num_rois, poses_init=poses_init, poses_pred=poses_pred, out=out)
    return r, p, n
