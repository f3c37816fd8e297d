"""Drop-in for lib/hough_voting_gpu_layer/hough_voting_gpu_op.py (:4-7):
`hough_voting_gpu` / `hough_voting_gpu_grad`, backed by libposecnn_hip.so.

Same positional signature as the TF op wrapper and the same five outputs
(REGISTER_OP("Houghvotinggpu"), hough_voting_gpu_op.cc:37-52):
  top_box (R,7) [b,cls,x1,y1,x2,y2,score], top_pose (R,7), top_target (R,4C),
  top_weight (R,4C), top_domain (R,) int32
with R >= 1 (one all-zero dummy row when nothing is detected,
hough_voting_gpu_op.cc:382-383).  The hard-coded inlier (0.9) and label
(500) thresholds of the reference Compute (:356-357) are keyword arguments
with those defaults.  Row order is canonical: image-major, ascending class
(default path) or ascending Hough cell (threshold_vote > 0).

`hough_voting_gpu_capacity` is the sync-free form used by the fused pose step:
capacity-sized outputs plus a device-side row count.
"""
import torch

from .. import _lib

MAX_ROI = 128
CAPACITY = MAX_ROI * 9


def _as_meta2d(meta, B):
    return meta.reshape(B, -1).contiguous()


def hough_voting_gpu_capacity(label, vertex, extents, meta_data, gt, is_train, threshold_vote,
                              threshold_percentage, skip_pixels, inlier_threshold=0.9, label_threshold=500,
                              batch_base=0, global_batch=None, out=None, debug_counts=None, stream=None, prob=None,
                              vertex_compact=False):
    """Launch without host sync.  Returns dict of capacity-sized tensors and
    `num_rois` (int32[2] on device: rows, max(rows, 1)).

    With `prob` (B,H,W,C) given instead of `label` (pass label=None), the
    label producer runs fused into the op (pcnn_hough_voting_prob): label_2d =
    argmax over the class axis (network.py:433-434) is computed inside the
    compaction pass and returned as out["label"].

    vertex_compact=True: `vertex` is the class-compact (B,H,W,3) map of
    vertex_pred.vertex_pred_compact (each pixel's own class channels; SURVEY
    8(f) row 3); the class count then comes from `extents` (C,3)."""
    _lib.require_gpu(label, prob, vertex, extents, meta_data, gt)
    lib = _lib.load()
    if (label is None) == (prob is None):
        raise ValueError("pass exactly one of label / prob")
    if label is not None and label.dim() != 3:
        raise ValueError("label must be 3-dimensional")  # hough_voting_gpu_op.cc:328-329
    if prob is not None and prob.dim() != 4:
        raise ValueError("prob must be 4-dimensional")
    if vertex.dim() != 4:
        raise ValueError("vertex must be 4-dimensional")  # :331-332
    B, H, W = (label.shape if label is not None else prob.shape[:3])
    if vertex_compact:
        if label is None or vertex.shape[3] != 3:
            raise ValueError("vertex_compact takes label and a (B,H,W,3) vertex map")
        C = extents.shape[0]
    else:
        C = vertex.shape[3] // 3
    if prob is not None and prob.shape[3] != C:
        raise ValueError(f"prob has {prob.shape[3]} classes, vertex has {C}")
    dev = vertex.device
    if label is not None:
        label = label.contiguous().to(torch.int32)
    else:
        prob = prob.contiguous().float()
    vertex = vertex.contiguous().float()
    extents = extents.contiguous().float()
    meta = _as_meta2d(meta_data.float(), B)
    gt = gt.reshape(-1, 13).contiguous().float() if gt.numel() else gt.reshape(0, 13).float()
    if out is None:
        out = dict(
            box=torch.empty((CAPACITY, 7), dtype=torch.float32, device=dev),
            pose=torch.empty((CAPACITY, 7), dtype=torch.float32, device=dev),
            target=torch.empty((CAPACITY, 4 * C), dtype=torch.float32, device=dev),
            weight=torch.empty((CAPACITY, 4 * C), dtype=torch.float32, device=dev),
            domain=torch.empty((CAPACITY,), dtype=torch.int32, device=dev),
            num_rois=torch.empty((2,), dtype=torch.int32, device=dev),
        )
    if prob is not None and out.get("label") is None:
        out["label"] = torch.empty((B, H, W), dtype=torch.int32, device=dev)
    nbytes = lib.pcnn_hough_voting_workspace_size(B, H, W, C, int(skip_pixels), float(threshold_vote))
    ws = _lib.workspace(nbytes, dev, "hough", stream)
    if prob is not None:
        head = (lib.pcnn_hough_voting_prob, _lib.ptr(prob), _lib.ptr(out["label"]))
    elif vertex_compact:
        head = (lib.pcnn_hough_voting_compact, _lib.ptr(label))
    else:
        head = (lib.pcnn_hough_voting, _lib.ptr(label))
    rc = head[0](
        *head[1:], _lib.ptr(vertex), _lib.ptr(extents), _lib.ptr(meta), meta.shape[1],
        _lib.ptr(gt) if gt.numel() else None, gt.shape[0], B, H, W, C, int(batch_base),
        int(global_batch or B), int(is_train), float(inlier_threshold), int(label_threshold),
        float(threshold_vote), float(threshold_percentage), int(skip_pixels),
        _lib.ptr(out["box"]), _lib.ptr(out["pose"]), _lib.ptr(out["target"]), _lib.ptr(out["weight"]),
        _lib.ptr(out["domain"]), _lib.ptr(out["num_rois"]), out["box"].shape[0], _lib.ptr(debug_counts),
        _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "hough_voting_gpu")
    out["_ws"] = ws
    out["_dims"] = (B, H, W, C, int(skip_pixels), float(threshold_vote))
    return out


def hough_voting_diag(out):
    """Self-check counters of the last call (see pcnn_hough_voting_diag)."""
    import numpy as np
    B, H, W, C, skip, thr = out["_dims"]
    d = np.zeros(4, np.int32)
    rc = _lib.load().pcnn_hough_voting_diag(_lib.ptr(out["_ws"]), B, H, W, C, skip, thr,
                                            d.ctypes.data_as(_lib.c_void_p), _lib.stream_ptr())
    _lib.check(rc, "hough_voting_diag")
    return d


def hough_voting_gpu(bottom_label, bottom_vertex, bottom_extents, bottom_meta_data, bottom_gt, is_train,
                     threshold_vote, threshold_percentage, skip_pixels, name=None, inlier_threshold=0.9,
                     label_threshold=500, batch_base=0, global_batch=None):
    """Reference-shaped op: exact-size outputs (one device->host read of the row count)."""
    o = hough_voting_gpu_capacity(bottom_label, bottom_vertex, bottom_extents, bottom_meta_data, bottom_gt,
                                  is_train, threshold_vote, threshold_percentage, skip_pixels,
                                  inlier_threshold=inlier_threshold, label_threshold=label_threshold,
                                  batch_base=batch_base, global_batch=global_batch)
    n = int(o["num_rois"][1].item())
    return (o["box"][:n].clone(), o["pose"][:n].clone(), o["target"][:n].clone(), o["weight"][:n].clone(),
            o["domain"][:n].clone())


def hough_voting_gpu_from_prob(bottom_prob, bottom_vertex, bottom_extents, bottom_meta_data, bottom_gt, is_train,
                               threshold_vote, threshold_percentage, skip_pixels, name=None, inlier_threshold=0.9,
                               label_threshold=500, batch_base=0, global_batch=None):
    """argmax_2d(prob) -> hough_voting_gpu fused (vgg16_convs.py:144-146 feeding
    :167-170): returns (label_2d, top_box, top_pose, top_target, top_weight,
    top_domain), the outputs equal to argmax_2d + hough_voting_gpu."""
    o = hough_voting_gpu_capacity(None, bottom_vertex, bottom_extents, bottom_meta_data, bottom_gt, is_train,
                                  threshold_vote, threshold_percentage, skip_pixels,
                                  inlier_threshold=inlier_threshold, label_threshold=label_threshold,
                                  batch_base=batch_base, global_batch=global_batch, prob=bottom_prob)
    n = int(o["num_rois"][1].item())
    return (o["label"], o["box"][:n].clone(), o["pose"][:n].clone(), o["target"][:n].clone(),
            o["weight"][:n].clone(), o["domain"][:n].clone())


def hough_voting_gpu_grad(bottom_label, bottom_vertex, grad, name=None):
    """HoughvotinggpuGrad (hough_voting_gpu_op.cc:440-484): zero gradients."""
    _lib.require_gpu(bottom_label, bottom_vertex)
    B, H, W = bottom_label.shape
    C = bottom_vertex.shape[3] // 3
    gl = torch.empty((B, H, W), dtype=torch.float32, device=bottom_label.device)
    gv = torch.empty(bottom_vertex.shape, dtype=torch.float32, device=bottom_vertex.device)
    rc = _lib.load().pcnn_hough_voting_grad(_lib.ptr(gl), _lib.ptr(gv), B, H, W, C, _lib.stream_ptr())
    _lib.check(rc, "hough_voting_gpu_grad")
    return gl, gv
