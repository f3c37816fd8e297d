"""my_tools pth module surface (posecnn_amd/pth.py) on the GPU: NCHW/5-column
RoI pooling equals the NHWC op, autograd backward matches the explicit
gradient ops, HoughVoting equals hough_voting_gpu."""
import numpy as np
import pytest
import torch

from posecnn_amd import pth, synth
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv
from posecnn_amd.roi_pooling_layer import roi_pooling_op as rp
from posecnn_amd.average_distance_loss import average_distance_loss_op as adl

pytestmark = pytest.mark.gpu
D = torch.device("cuda")


def test_roi_pooling_module_nchw(hip):
    rng = np.random.default_rng(11)
    B, H, W, C = 2, 30, 40, 32
    nhwc = torch.from_numpy(rng.normal(size=(B, H, W, C)).astype(np.float32)).to(D)
    x1 = rng.uniform(0, 500, 9); y1 = rng.uniform(0, 400, 9)
    r7 = np.stack([np.sort(rng.integers(0, B, 9)), np.zeros(9), x1, y1, x1 + 120, y1 + 90, np.zeros(9)], 1)
    rois7 = torch.from_numpy(r7.astype(np.float32)).to(D)
    rois5 = rois7[:, [0, 2, 3, 4, 5]].contiguous()
    ref, arg = rp.roi_pool(nhwc, rois7, 7, 7, 1 / 16, 0)
    nchw = nhwc.permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    out = pth._RoIPooling(7, 7, 1 / 16)(nchw, rois5)
    np.testing.assert_array_equal(out.detach().permute(0, 2, 3, 1).cpu().numpy(), ref.cpu().numpy())
    g = torch.randn_like(out)
    out.backward(g)
    gref = rp.roi_pool_grad(nhwc, rois7, arg, g.permute(0, 2, 3, 1).contiguous(), 7, 7, 1 / 16, 0)
    np.testing.assert_array_equal(nchw.grad.permute(0, 2, 3, 1).cpu().numpy(), gref.cpu().numpy())


def test_hough_and_add_modules(hip):
    fr = synth.make_frames(1, H=120, W=160, num_classes=6, objects_per_image=3, seed=12)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(D)
    hvm = pth.HoughVoting(6, -1.0, 0.02, skip_pixels=3, is_train=True)
    outs = hvm(t(fr["label"]), t(fr["vertex"]), t(fr["extents"]), t(fr["gt"]), t(fr["meta"]))
    ref = hv.hough_voting_gpu(t(fr["label"]), t(fr["vertex"]), t(fr["extents"]), t(fr["meta"]), t(fr["gt"]),
                              1, -1.0, 0.02, 3)
    for a, b in zip(outs, ref):
        np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    pts, sym = synth.rescaled_points(6)
    R = outs[0].shape[0]
    pred = torch.nn.functional.normalize(torch.randn(R, 24, device=D), dim=1).requires_grad_(True)
    loss = pth.AverageDistanceLoss(6, 0.01)(pred, outs[2], outs[3], t(pts), t(sym))
    loss.backward()
    l2, diff = adl.average_distance_loss(pred.detach(), outs[2], outs[3], t(pts), t(sym), 0.01)
    np.testing.assert_array_equal(loss.detach().cpu().numpy(), l2.cpu().numpy())
    np.testing.assert_array_equal(pred.grad.cpu().numpy(), diff.cpu().numpy())
