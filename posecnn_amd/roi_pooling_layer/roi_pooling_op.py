"""Drop-in for lib/roi_pooling_layer/roi_pooling_op.py (:4-7): `roi_pool` /
`roi_pool_grad` over NHWC features (REGISTER_OP("RoiPool") / "RoiPoolGrad",
roi_pooling_op.cc:29-50), backed by libposecnn_hip.so.

roi_pool(data (B,H,W,C), rois (R, >=6), pooled_height, pooled_width,
         spatial_scale, pool_channel) -> (top (R,PH,PW,C or 1), argmax int32)
roi_pool_grad(data, rois, argmax, grad, ...) -> d data  (roi_pooling_op_grad.py:33-50)
`num_rois` (optional device int32 scalar tensor) bounds the rows used, for the
capacity-sized RoI buffers of the fused pose step.  `batch_base` is subtracted
from the rows' batch column: an image-sharded rank holds images
[batch_base, batch_base + B) while the Hough rows carry the global index.
"""
import torch

from .. import _lib


def roi_pool(bottom_data, bottom_rois, pooled_height, pooled_width, spatial_scale, pool_channel=0, name=None,
             num_rois=None, layout=0, out=None, accumulate=False, batch_base=0):
    """accumulate=True: out[0] += pooled (out required), argmax written to out[1]."""
    _lib.require_gpu(bottom_data, bottom_rois)
    if bottom_data.dim() != 4:
        raise ValueError("data must be 4-dimensional")  # roi_pooling_op.cc:92-93
    if bottom_rois.dim() != 2:
        raise ValueError("rois must be 2-dimensional")  # :96-97
    data = bottom_data.contiguous().float()
    rois = bottom_rois.contiguous().float()
    if layout == 0:
        B, H, W, C = data.shape
    else:
        B, C, H, W = data.shape
    R, stride = rois.shape
    Co = 1 if pool_channel else C
    shape = (R, pooled_height, pooled_width, Co) if layout == 0 else (R, Co, pooled_height, pooled_width)
    if out is None:
        if accumulate:
            raise ValueError("accumulate=True needs out=(top, argmax)")
        top = torch.empty(shape, dtype=torch.float32, device=data.device)
        arg = torch.empty(shape, dtype=torch.int32, device=data.device)
    else:
        top, arg = out
    lib = _lib.load()
    fn = lib.pcnn_roi_pool_fwd_accumulate if accumulate else lib.pcnn_roi_pool_fwd
    rc = fn(_lib.ptr(data), B, H, W, C, layout, _lib.ptr(rois), R, stride, int(batch_base), _lib.ptr(num_rois),
            float(spatial_scale), int(pooled_height), int(pooled_width), int(pool_channel), _lib.ptr(top),
            _lib.ptr(arg), _lib.stream_ptr())
    _lib.check(rc, "roi_pool")
    return top, arg


def roi_pool_pair(data_a, scale_a, data_b, scale_b, rois, pooled_height, pooled_width, num_rois=None, out=None,
                  batch_base=0, pixel_argmax=False):
    """pool_a + pool_b and both argmax tensors in one pass (vgg16_convs.py:177-184:
    roi_pool(conv5_3, 1/16) + roi_pool(conv4_3, 1/8)); NHWC, all channels.
    Equal to roi_pool(data_a) then roi_pool(data_b, accumulate=True).
    Argmax tensors of dtype int16 (or pixel_argmax=True) hold the compact form:
    the uint16 pixel index h*W + w (flat argmax = pixel*C + c; 0xFFFF = empty
    bin), which roi_pool_grad accepts as well."""
    _lib.require_gpu(data_a, data_b, rois)
    if data_a.dim() != 4 or data_b.dim() != 4 or rois.dim() != 2:
        raise ValueError("data must be 4-dimensional and rois 2-dimensional")
    da, db = data_a.contiguous().float(), data_b.contiguous().float()
    B, Ha, Wa, C = da.shape
    Bb, Hb, Wb, Cb = db.shape
    if (Bb, Cb) != (B, C):
        raise ValueError("both maps need the same batch and channel count")
    rois = rois.contiguous().float()
    R, stride = rois.shape
    shape = (R, pooled_height, pooled_width, C)
    if out is None:
        adt = torch.int16 if pixel_argmax else torch.int32
        out = (torch.empty(shape, dtype=torch.float32, device=da.device),
               torch.empty(shape, dtype=adt, device=da.device),
               torch.empty(shape, dtype=adt, device=da.device))
    top, arg_a, arg_b = out
    if arg_a.dtype != arg_b.dtype or arg_a.dtype not in (torch.int16, torch.int32):
        raise ValueError("argmax tensors must both be int32 (flat index) or int16 (pixel index)")
    fn = _lib.load().pcnn_roi_pool_fwd_pair_px if arg_a.dtype == torch.int16 else _lib.load().pcnn_roi_pool_fwd_pair
    rc = fn(_lib.ptr(da), Ha, Wa, float(scale_a), _lib.ptr(db), Hb, Wb, float(scale_b), B, C, _lib.ptr(rois), R, stride,
            int(batch_base), _lib.ptr(num_rois), int(pooled_height), int(pooled_width), _lib.ptr(top), _lib.ptr(arg_a),
            _lib.ptr(arg_b), _lib.stream_ptr())
    _lib.check(rc, "roi_pool_pair")
    return top, arg_a, arg_b


def roi_pool_grad(bottom_data, bottom_rois, argmax, grad, pooled_height, pooled_width, spatial_scale,
                  pool_channel=0, name=None, num_rois=None, layout=0, out=None, batch_base=0):
    _lib.require_gpu(bottom_data, bottom_rois, argmax, grad)
    rois = bottom_rois.contiguous().float()
    if layout == 0:
        B, H, W, C = bottom_data.shape
    else:
        B, C, H, W = bottom_data.shape
    R, stride = rois.shape
    lib = _lib.load()
    ws = _lib.workspace(lib.pcnn_roi_pool_bwd_workspace_size(B, R), bottom_data.device, "roi_bwd")
    dd = out if out is not None else torch.empty(bottom_data.shape, dtype=torch.float32, device=bottom_data.device)
    if argmax.dtype == torch.int16:  # pixel-index argmax of roi_pool_pair(pixel_argmax=True)
        if layout != 0 or pool_channel:
            raise ValueError("a pixel-index argmax needs NHWC data and pool_channel 0")
        rc = lib.pcnn_roi_pool_bwd_px(_lib.ptr(grad.contiguous()), _lib.ptr(argmax.contiguous()), B, H, W, C,
                                      _lib.ptr(rois), R, stride, int(batch_base), _lib.ptr(num_rois),
                                      float(spatial_scale), int(pooled_height), int(pooled_width), _lib.ptr(dd),
                                      _lib.ptr(ws), ws.numel(), _lib.stream_ptr())
    else:
        rc = lib.pcnn_roi_pool_bwd(_lib.ptr(grad.contiguous()), _lib.ptr(argmax.contiguous()), B, H, W, C, layout,
                                   _lib.ptr(rois), R, stride, int(batch_base), _lib.ptr(num_rois),
                                   float(spatial_scale), int(pooled_height), int(pooled_width), int(pool_channel),
                                   _lib.ptr(dd), _lib.ptr(ws), ws.numel(), _lib.stream_ptr())
    _lib.check(rc, "roi_pool_grad")
    return dd


class RoiPoolFunction(torch.autograd.Function):
    """autograd binding (the TF gradient registration, roi_pooling_op_grad.py:29-50)."""

    @staticmethod
    def forward(ctx, data, rois, pooled_height, pooled_width, spatial_scale, pool_channel=0, layout=0):
        top, arg = roi_pool(data, rois, pooled_height, pooled_width, spatial_scale, pool_channel, layout=layout)
        ctx.save_for_backward(data, rois, arg)
        ctx.params = (pooled_height, pooled_width, spatial_scale, pool_channel, layout)
        return top, arg

    @staticmethod
    def backward(ctx, grad, _garg):
        data, rois, arg = ctx.saved_tensors
        ph, pw, sc, pc, layout = ctx.params
        return roi_pool_grad(data, rois, arg, grad, ph, pw, sc, pc, layout=layout), None, None, None, None, None, None
