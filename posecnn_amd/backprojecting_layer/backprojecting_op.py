"""Drop-in for lib/backprojecting_layer/backprojecting_op.py (:4-7):
`backproject` / `backproject_grad` (REGISTER_OP("Backproject") /
"BackprojectGrad", backprojecting_op.cc:30-53), backed by libposecnn_hip.so.

backproject(data (B,H,W,Ch), label (B,H,W,NC), depth (B,H,W,1), meta (B,1,1,48),
            label_3d (B,G,G,G,NC), grid_size, kernel_size, threshold)
    -> (top_data (B,G,G,G,Ch), top_label (B,G,G,G,NC), top_flag (B,G,G,G,Ch))
backproject_grad(data, depth, meta, grad, grid_size, kernel_size, threshold) -> (B,H,W,Ch)
"""
import torch

from .. import _lib


def backproject(bottom_data, bottom_label, bottom_depth, bottom_meta_data, bottom_label_3d, grid_size, kernel_size,
                threshold, name=None):
    _lib.require_gpu(bottom_data, bottom_label, bottom_depth, bottom_meta_data, bottom_label_3d)
    data = bottom_data.contiguous().float()
    B, H, W, Ch = data.shape
    NC = bottom_label.shape[3]
    G = int(grid_size)
    meta = bottom_meta_data.reshape(B, -1).contiguous().float()
    dev = data.device
    td = torch.empty((B, G, G, G, Ch), dtype=torch.float32, device=dev)
    tl = torch.empty((B, G, G, G, NC), dtype=torch.float32, device=dev)
    tf = torch.empty((B, G, G, G, Ch), dtype=torch.float32, device=dev)
    rc = _lib.load().pcnn_backproject_fwd(_lib.ptr(data), _lib.ptr(bottom_label.contiguous().float()),
                                          _lib.ptr(bottom_depth.contiguous().float()), _lib.ptr(meta), meta.shape[1],
                                          _lib.ptr(bottom_label_3d.contiguous().float()), B, H, W, Ch, NC, G,
                                          int(kernel_size), float(threshold), _lib.ptr(td), _lib.ptr(tl),
                                          _lib.ptr(tf), _lib.stream_ptr())
    _lib.check(rc, "backproject")
    return td, tl, tf


def backproject_grad(bottom_data, bottom_depth, bottom_meta_data, grad, grid_size, kernel_size, threshold,
                     name=None):
    _lib.require_gpu(bottom_data, bottom_depth, bottom_meta_data, grad)
    B, H, W, Ch = bottom_data.shape
    meta = bottom_meta_data.reshape(B, -1).contiguous().float()
    out = torch.empty((B, H, W, Ch), dtype=torch.float32, device=bottom_data.device)
    rc = _lib.load().pcnn_backproject_bwd(_lib.ptr(grad.contiguous().float()),
                                          _lib.ptr(bottom_depth.contiguous().float()), _lib.ptr(meta), meta.shape[1],
                                          B, H, W, Ch, int(grid_size), _lib.ptr(out), _lib.stream_ptr())
    _lib.check(rc, "backproject_grad")
    return out
