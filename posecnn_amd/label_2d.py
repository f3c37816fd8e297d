"""`argmax_2d` of lib/networks/network.py:433-434 (`tf.to_int32(tf.argmax(input,
3))`), the producer of label_2d from prob_normalized in vgg16_convs.py:144-146,
as a HIP kernel (pcnn_argmax_2d): the first maximum over the class axis wins,
and a NaN wins at its first occurrence (numpy / tf.argmax).

The Hough op can also consume prob directly with this argmax fused into its
compaction pass: hough_voting_gpu_layer.hough_voting_gpu_op.
hough_voting_gpu_from_prob / hough_voting_gpu_capacity(prob=...).
"""
import torch

from . import _lib


def argmax_2d(prob, out=None, stream=None):
    _lib.require_gpu(prob)
    if prob.dim() != 4:
        raise ValueError("argmax_2d takes a 4-D (B,H,W,C) tensor")
    B, H, W, C = prob.shape
    prob = prob.contiguous().float()
    if out is None:
        out = torch.empty((B, H, W), dtype=torch.int32, device=prob.device)
    rc = _lib.load().pcnn_argmax_2d(_lib.ptr(prob), B, H, W, C, _lib.ptr(out), _lib.stream_ptr(stream))
    _lib.check(rc, "argmax_2d")
    return out
