"""Class-compact vertex wire format.

The reference's `vertex_pred` layer (lib/networks/vgg16_convs.py:152-163: a
1x1 conv 128 -> 3C plus bias_add, network.py:168-185) writes a (B,H,W,3C)
map — 264 B per pixel at C = 22 — of which the Hough vote reads only the three
channels of each voter's own class (hough_voting_gpu_op.cu.cc:276-280).
`vertex_pred_compact` evaluates the layer only at those channels, given the
label map, and writes (B,H,W,3); `hough_voting_gpu_capacity(...,
vertex_compact=True)` votes from it with outputs identical to the full map's.
"""
import torch

from . import _lib


def vertex_pred_compact(feat, weights, biases, label, out=None, stream=None):
    """feat (B,H,W,K) NHWC, weights (K,3C) or the reference's (1,1,K,3C) kernel,
    biases (3C), label (B,H,W) int -> (B,H,W,3) float32."""
    _lib.require_gpu(feat, weights, biases, label)
    if feat.dim() != 4 or label.dim() != 3:
        raise ValueError("feat must be (B,H,W,K) and label (B,H,W)")
    B, H, W, K = feat.shape
    w = weights.reshape(K, -1).contiguous().float()
    if w.shape[1] % 3 or biases.numel() != w.shape[1]:
        raise ValueError("weights must be (K, 3C) with a 3C bias")
    C = w.shape[1] // 3
    feat = feat.contiguous().float()
    lab = label.contiguous().to(torch.int32)
    if out is None:
        out = torch.empty((B, H, W, 3), dtype=torch.float32, device=feat.device)
    rc = _lib.load().pcnn_vertex_pred_compact(_lib.ptr(feat), _lib.ptr(w), _lib.ptr(biases.contiguous().float()),
                                              _lib.ptr(lab), B, H, W, K, C, _lib.ptr(out), _lib.stream_ptr(stream))
    _lib.check(rc, "vertex_pred_compact")
    return out
