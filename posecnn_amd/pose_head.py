"""Pose head of vgg16_convs (lib/networks/vgg16_convs.py:186-200) on the HIP
MFMA GEMM: pool5 + pool4 -> fc6 (relu) -> fc7 (relu) -> fc8 -> tanh ->
* poses_weight -> l2_normalize, forward and backward, with every row count
read on the device (capacity-sized RoI buffers, no host sync).

Weights follow Network.fc (network.py:393-423): `weights` [in, out] with
truncated-normal(0, 0.001) init (network.py:415), `biases` [out] zero; the
reshape of the (R,7,7,512) pooled features is NHWC-flat ((h*7+w)*512+c).
drop6 / drop7 (vgg16_convs.py:189,191, tf.nn.dropout) are fused into the fc6 /
fc7 forward epilogues and the relu-mask epilogues of the backward (keep_prob
0.5 in training, train.py:421; 1, the identity, at test time).
"""
import torch

from . import _lib


def gemm(A, B, C, a_trans=0, b_trans=0, A2=None, bias=None, act=0, mask=None, M_dev=None, K_dev=None, M=None,
         N=None, K=None, precision=2, drop=None, keep_prob=1.0, drop_gen=None, stream=None):
    """C[M,N] = epilogue(op(A) (+ op(A2)) @ op(B)); see pcnn_gemm / pcnn_gemm_drop in
    include/posecnn_hip.h.  drop (uint8 (M, >=N) 0/1) applies tf.nn.dropout after
    the activation, (v / keep_prob) * drop; with mask, keep_prob scales the kept
    gradient (v / keep_prob: the backward of relu + dropout).  drop_gen =
    (seed, step_dev, stream_id): the reduce draws the keep bits itself (as
    dropout_mask would) and writes them into drop (pcnn_gemm_drop_gen)."""
    _lib.require_gpu(A, B, C)
    for t in (A, B, C, A2, bias, mask):
        if t is not None and (t.dtype != torch.float32 or t.stride(-1) != 1):
            raise ValueError("gemm operands must be fp32 with unit inner stride")
    if drop is not None and (drop.dtype != torch.uint8 or drop.stride(-1) != 1 or not drop.is_cuda):
        raise ValueError("gemm: drop must be a uint8 device tensor with unit inner stride")
    if M is None:
        M = A.shape[1] if a_trans else A.shape[0]
    if K is None:
        K = A.shape[0] if a_trans else A.shape[1]
    if N is None:
        N = B.shape[0] if b_trans else B.shape[1]
    lib = _lib.load()
    ws = _lib.workspace(lib.pcnn_gemm_workspace_size(M, N, K, int(M_dev is not None), precision), C.device, "gemm",
                        stream)
    if drop_gen is not None:
        if drop is None or mask is not None:
            raise ValueError("gemm: drop_gen needs the drop output buffer and no mask (forward only)")
        seed, step_dev, sid = drop_gen
        if step_dev is not None and (step_dev.dtype != torch.int64 or not step_dev.is_cuda):
            raise ValueError("gemm: drop_gen's step counter must be an int64 device tensor")
        rc = lib.pcnn_gemm_drop_gen(M, N, K, _lib.ptr(A), _lib.ptr(A2), A.stride(0), int(a_trans), _lib.ptr(B),
                                    B.stride(0), int(b_trans), _lib.ptr(C), C.stride(0), _lib.ptr(bias), int(act),
                                    _lib.ptr(drop), drop.stride(0), float(keep_prob), int(seed) & ((1 << 64) - 1),
                                    _lib.ptr(step_dev), int(sid), _lib.ptr(M_dev), _lib.ptr(K_dev), int(precision),
                                    _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    elif drop is None and keep_prob == 1.0:
        rc = lib.pcnn_gemm(M, N, K, _lib.ptr(A), _lib.ptr(A2), A.stride(0), int(a_trans), _lib.ptr(B), B.stride(0),
                           int(b_trans), _lib.ptr(C), C.stride(0), _lib.ptr(bias), int(act), _lib.ptr(mask),
                           mask.stride(0) if mask is not None else 0, _lib.ptr(M_dev), _lib.ptr(K_dev),
                           int(precision), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    else:
        rc = lib.pcnn_gemm_drop(M, N, K, _lib.ptr(A), _lib.ptr(A2), A.stride(0), int(a_trans), _lib.ptr(B),
                                B.stride(0), int(b_trans), _lib.ptr(C), C.stride(0), _lib.ptr(bias), int(act),
                                _lib.ptr(mask), mask.stride(0) if mask is not None else 0, _lib.ptr(drop),
                                drop.stride(0) if drop is not None else 0, float(keep_prob), _lib.ptr(M_dev),
                                _lib.ptr(K_dev), int(precision), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "gemm")
    return C


def tp_bytes(rows, K):
    """Bytes of the tiled three-plane (hi / mid / lo bf16) form of a rows x K operand."""
    return int(_lib.load().pcnn_tp_bytes(int(rows), int(K)))


def split_tp(src, rows, K, out, row_stride, k_stride, rows_dev=None, K_dev=None, stream=None):
    """out (uint8, >= tp_bytes(rows, K)) <- the tiled planes of the fp32 view
    src[row * row_stride + k * k_stride] (zeros past rows_dev / K_dev); see
    pcnn_split_tp in include/posecnn_hip.h."""
    _lib.require_gpu(src, out)
    if src.dtype != torch.float32 or out.dtype != torch.uint8 or not out.is_contiguous():
        raise ValueError("split_tp: fp32 source, contiguous uint8 destination")
    rc = _lib.load().pcnn_split_tp(_lib.ptr(src), int(row_stride), int(k_stride), int(rows), _lib.ptr(rows_dev),
                                   int(K), _lib.ptr(K_dev), _lib.ptr(out), out.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "split_tp")
    return out


def gemm_tp(A_tp, B_tp, C, M, N, K, bias=None, act=0, mask=None, drop=None, keep_prob=1.0, M_dev=None, K_dev=None,
            stream=None):
    """C[M,N] = epilogue(A @ B) from the tiled planes of op(A) (M x K) and of
    op(B)^T (N x K) (split_tp); bit-identical to gemm(..., precision=2)."""
    _lib.require_gpu(A_tp, B_tp, C)
    for t in (C, bias, mask):
        if t is not None and (t.dtype != torch.float32 or t.stride(-1) != 1):
            raise ValueError("gemm_tp: fp32 outputs / epilogue operands with unit inner stride")
    if drop is not None and (drop.dtype != torch.uint8 or drop.stride(-1) != 1):
        raise ValueError("gemm_tp: drop must be uint8 with unit inner stride")
    lib = _lib.load()
    ws = _lib.workspace(lib.pcnn_gemm_workspace_size(M, N, K, int(M_dev is not None), 2), C.device, "gemm", stream)
    rc = lib.pcnn_gemm_tp(int(M), int(N), int(K), _lib.ptr(A_tp), _lib.ptr(B_tp), _lib.ptr(C), C.stride(0),
                          _lib.ptr(bias), int(act), _lib.ptr(mask), mask.stride(0) if mask is not None else 0,
                          _lib.ptr(drop), drop.stride(0) if drop is not None else 0, float(keep_prob),
                          _lib.ptr(M_dev), _lib.ptr(K_dev), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(stream))
    _lib.check(rc, "gemm_tp")
    return C


def dropout_mask(mask, keep_prob, seed, step_dev=None, stream_id=0, rows_dev=None, stream=None):
    """The binary tensor of tf.nn.dropout, floor(keep_prob + U[0,1)), into the
    uint8 (rows, cols) `mask` (Philox4x32-10 keyed on seed, the device step
    counter step_dev (int64 (1,)) and stream_id; rows past *rows_dev untouched)."""
    _lib.require_gpu(mask)
    if mask.dtype != torch.uint8 or mask.dim() != 2 or mask.stride(1) != 1:
        raise ValueError("dropout_mask: uint8 (rows, cols) mask with unit inner stride")
    if step_dev is not None and (step_dev.dtype != torch.int64 or not step_dev.is_cuda):
        raise ValueError("dropout_mask: step_dev must be an int64 device tensor")
    rc = _lib.load().pcnn_dropout_mask(_lib.ptr(mask), mask.shape[0], mask.shape[1], mask.stride(0),
                                       _lib.ptr(rows_dev), int(seed) & ((1 << 64) - 1), _lib.ptr(step_dev),
                                       int(stream_id), float(keep_prob), _lib.stream_ptr(stream))
    _lib.check(rc, "dropout_mask")
    return mask


def colsum(X, out, M_dev=None, stream=None):
    rc = _lib.load().pcnn_colsum(_lib.ptr(X), X.shape[0], X.shape[1], X.stride(0), _lib.ptr(M_dev), _lib.ptr(out),
                                 _lib.stream_ptr(stream))
    _lib.check(rc, "colsum")
    return out


def head_fwd(y8, poses_weight, tanh_out, pred, num_rois=None, stream=None):
    R, D = y8.shape
    rc = _lib.load().pcnn_pose_head_fwd(_lib.ptr(y8), _lib.ptr(poses_weight), R, _lib.ptr(num_rois), D,
                                        _lib.ptr(tanh_out), _lib.ptr(pred), _lib.stream_ptr(stream))
    _lib.check(rc, "pose_head_fwd")


def head_bwd(d_pred, tanh_out, poses_weight, pred, d_y8, num_rois=None, d_pred_scale=None, stream=None):
    """d_y8 from d_pred; with d_pred_scale (device scalar) d_pred is taken as
    d_pred_scale[0] * d_pred -- the ADD-loss gradient op folded into this pass."""
    R, D = d_pred.shape
    rc = _lib.load().pcnn_pose_head_bwd(_lib.ptr(d_pred), _lib.ptr(d_pred_scale), _lib.ptr(tanh_out),
                                        _lib.ptr(poses_weight), _lib.ptr(pred), R, _lib.ptr(num_rois), D,
                                        _lib.ptr(d_y8), _lib.stream_ptr(stream))
    _lib.check(rc, "pose_head_bwd")


def truncated_normal(shape, std, generator, device):
    t = torch.empty(shape, dtype=torch.float32, device=device)
    torch.nn.init.trunc_normal_(t, 0.0, std, -2 * std, 2 * std, generator=generator)
    return t


class PoseHeadWeights:
    """fc6 / fc7 / fc8 variables of the pose head (vgg16_convs.py:186-192)."""

    def __init__(self, num_classes, device, in_dim=7 * 7 * 512, units=4096, seed=0):
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        D = 4 * num_classes
        self.w6 = truncated_normal((in_dim, units), 0.001, g, device)
        self.b6 = torch.zeros(units, device=device)
        self.w7 = truncated_normal((units, units), 0.001, g, device)
        self.b7 = torch.zeros(units, device=device)
        self.w8 = truncated_normal((units, D), 0.001, g, device)
        self.b8 = torch.zeros(D, device=device)
        self.in_dim, self.units, self.D = in_dim, units, D

    def grads_like(self):
        return {k: torch.empty_like(getattr(self, k)) for k in ("w6", "b6", "w7", "b7", "w8", "b8")}
