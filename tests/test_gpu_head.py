"""GPU parity of the pose-head tail (vgg16_convs.py:193-197: tanh -> * poses_weight
-> tf.nn.l2_normalize(dim=1)) forward and backward against torch autograd in
fp64, including the folded ADD-loss gradient scale (AveragedistanceBackward,
average_distance_loss_op_gpu.cu.cc:346-354) and the device-side row count."""
import numpy as np
import pytest
import torch

from posecnn_amd import pose_head as ph
from posecnn_amd.average_distance_loss import average_distance_loss_op as adl

pytestmark = pytest.mark.gpu
D = torch.device("cuda")


def _ref(y8, pw):
    m = torch.tanh(y8) * pw
    ss = (m * m).sum(1, keepdim=True)
    return m / torch.sqrt(torch.clamp(ss, min=1e-12))  # x * rsqrt(max(sum x^2, eps))


def test_pose_head_tail_vs_autograd(hip):
    g = torch.Generator().manual_seed(4)
    R, C, live = 41, 22, 33
    y8 = torch.randn(R, 4 * C, generator=g)
    pw = torch.zeros(R, 4 * C)
    cls = torch.randint(1, C, (R,), generator=g)
    for r in range(R):
        pw[r, 4 * cls[r]:4 * cls[r] + 4] = 1.0  # poses_weight: the row's class channels
    pw[5] = 0.0  # a row without weight: the l2 norm clamps at eps
    nr = torch.tensor([live], dtype=torch.int32, device=D)
    t8 = torch.full((R, 4 * C), 7.0, device=D)
    pred = torch.full((R, 4 * C), 7.0, device=D)
    ph.head_fwd(y8.to(D), pw.to(D), t8, pred, num_rois=nr)
    y = y8[:live].double().requires_grad_()
    p = _ref(y, pw[:live].double())
    np.testing.assert_allclose(pred[:live].cpu().numpy(), p.detach().numpy(), rtol=2e-6, atol=1e-7)
    assert (pred[live:] == 7.0).all()

    dpred = torch.randn(R, 4 * C, generator=g)
    scale = torch.tensor([0.7])
    p.backward(scale.double() * dpred[:live].double())
    dy8 = torch.full((R, 4 * C), 7.0, device=D)
    ph.head_bwd(dpred.to(D), t8, pw.to(D), pred, dy8, num_rois=nr, d_pred_scale=scale.to(D))
    np.testing.assert_allclose(dy8[:live].cpu().numpy(), y.grad.numpy(), rtol=1e-5, atol=1e-7)
    assert (dy8[live:] == 7.0).all()

    # folded scale == the separate gradient op followed by the unscaled pass, bit for bit
    dp = adl.average_distance_loss_grad(dpred.to(D), scale.to(D), num_rois=nr, out=torch.zeros(R, 4 * C, device=D))
    dy8b = torch.full((R, 4 * C), 7.0, device=D)
    ph.head_bwd(dp, t8, pw.to(D), pred, dy8b, num_rois=nr)
    np.testing.assert_array_equal(dy8[:live].cpu().numpy(), dy8b[:live].cpu().numpy())
