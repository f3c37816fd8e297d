"""End-to-end parity of the fused pose step (posecnn_amd/pipeline.py) against
an fp64 torch autograd restatement of the graph it runs
(vgg16_convs.py:184-200 + TF's gradients):

    x = pool5 + pool4 -> fc6 (relu) -> fc7 (relu) -> fc8 -> tanh * poses_weight
      -> l2_normalize -> average_distance_loss  (network.py:393-445)

The RoI pools, the Hough op and the ADD loss have their own bit-exact /
1e-4 parity tests against the oracle; here the step's pooled rows and its ADD
gradient (`step.diff`, d loss / d pred) are taken as given, and everything the
step chains around them -- the split-bf16 x3 GEMMs, bias / ReLU epilogues, the
ReLU masks of the backward, the bias column sums, the tail's tanh / l2-norm
backward and the RoI-pool backward routing of dX -- is checked against fp64,
on a small configuration (64 channels, 256 units)."""
import numpy as np
import pytest
import torch

from posecnn_amd import synth
from posecnn_amd.pipeline import PoseStep

pytestmark = pytest.mark.gpu
D = torch.device("cuda")
B, H, W, C, CH, UNITS = 2, 120, 160, 22, 64, 256


def _close(a, ref, rt=1e-4):
    """relative to the tensor's scale: |a - ref| <= rt * (|ref| + max |ref|)"""
    np.testing.assert_allclose(a, ref, rtol=rt, atol=rt * float(np.abs(ref).max()))


@pytest.mark.parametrize("drop", ["none", "philox", "external"])
def test_pose_step_vs_fp64_autograd(hip, orc, drop):
    """drop: "none" = keep_prob 1 (the test-time graph); "philox" = keep_prob
    0.5 with the step's own drawn masks; "external" = keep_prob 0.5 with masks
    supplied through set_drop_masks.  The fp64 graph applies drop6 / drop7 as
    tf.nn.dropout does, (x / keep_prob) * binary (vgg16_convs.py:189,191), and
    autograd gives TF's backward of it."""
    fr = synth.make_frames(B, H=H, W=W, num_classes=C, objects_per_image=4, seed=91)
    g = torch.Generator().manual_seed(3)
    conv4 = torch.randn((B, H // 8, W // 8, CH), generator=g)
    conv5 = torch.randn((B, H // 16, W // 16, CH), generator=g)
    pts, sym = synth.rescaled_points(C)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(D)
    inputs = dict(label=t(fr["label"]), vertex=t(fr["vertex"]), extents=t(fr["extents"]), meta=t(fr["meta"]),
                  gt=t(fr["gt"]), conv4=conv4.to(D), conv5=conv5.to(D), points=t(pts), symmetry=t(sym))
    keep = 1.0 if drop == "none" else 0.5
    step = PoseStep(B, H, W, C, D, channels=CH, units=UNITS, is_train=1, skip_pixels=3, keep_prob=keep)
    if drop == "external":
        gm = torch.Generator().manual_seed(11)
        cap = step.drop6.shape[0]
        step.set_drop_masks((torch.rand((cap, UNITS), generator=gm) < 0.5).to(D),
                            (torch.rand((cap, UNITS), generator=gm) < 0.5).to(D))
    # non-zero biases so the bias epilogues and column sums are exercised
    w = step.weights
    for b in (w.b6, w.b7, w.b8):
        b.copy_(torch.randn(b.shape, generator=g) * 1e-3)
    step.step(inputs)
    torch.cuda.synchronize()
    n = int(step.hough["num_rois"][1].item())
    assert n > 8, "the synthetic frames should produce RoI rows"
    f64 = lambda x: x.detach().double().cpu()

    x = f64(step.pool[:n].reshape(n, -1))
    W6, W7, W8 = (f64(v).requires_grad_() for v in (w.w6, w.w7, w.w8))
    b6, b7, b8 = (f64(v).requires_grad_() for v in (w.b6, w.b7, w.b8))
    x.requires_grad_()
    if keep < 1.0:
        m6, m7 = f64(step.drop6[:n]), f64(step.drop7[:n])
        for m_ in (m6, m7):  # Bernoulli(keep_prob) masks
            assert set(np.unique(m_.numpy())) <= {0.0, 1.0}
            assert abs(float(m_.mean()) - keep) < 0.03
        if drop == "philox":
            assert not torch.equal(m6, m7)
    else:
        m6 = m7 = None
    dropout = lambda y, m_: y if m_ is None else (y / keep) * m_  # tf.nn.dropout
    y6 = dropout(torch.relu(x @ W6 + b6), m6)
    y7 = dropout(torch.relu(y6 @ W7 + b7), m7)
    y8 = y7 @ W8 + b8
    pw = f64(step.hough["weight"][:n])
    m = torch.tanh(y8) * pw
    pred = m / torch.sqrt(torch.clamp((m * m).sum(1, keepdim=True), min=1e-12))

    _close(step.y6[:n].cpu().numpy(), y6.detach().numpy())
    _close(step.y7[:n].cpu().numpy(), y7.detach().numpy())
    _close(step.pred[:n].cpu().numpy(), pred.detach().numpy())

    # the ADD loss against the oracle on the step's own prediction (1e-4, its contract)
    ol, od, _ = orc.average_distance_loss(step.pred[:n].cpu().numpy(), step.hough["target"][:n].cpu().numpy(),
                                              step.hough["weight"][:n].cpu().numpy(), pts, sym, 0.01)
    np.testing.assert_allclose(step.loss.cpu().numpy(), ol, rtol=1e-4)
    np.testing.assert_allclose(step.diff[:n].cpu().numpy(), od, rtol=1e-4, atol=1e-7)

    pred.backward(f64(step.diff[:n]))
    gr = step.grads
    for k, ref in (("w8", W8), ("b8", b8), ("w7", W7), ("b7", b7), ("w6", W6), ("b6", b6)):
        _close(gr[k].cpu().numpy(), ref.grad.numpy())
    dx = step.dx[:n].cpu().numpy()
    _close(dx, x.grad.numpy())

    # dX routed into both feature maps by the RoI-pool backward: the oracle's
    # backward of the step's own dX and argmax (flat index = pixel * C + c)
    box = step.hough["box"][:n].cpu().numpy()
    for arg, data, dconv, s in ((step.arg5, conv5, step.dconv5, 1.0 / 16), (step.arg4, conv4, step.dconv4, 1.0 / 8)):
        a = arg[:n].cpu().numpy().astype(np.int64)
        if arg.dtype == torch.int16:
            a &= 0xFFFF
            a = np.where(a == 0xFFFF, -1, a * CH + np.arange(CH))
        od = orc.roi_pool_bwd(dx.reshape(n, 7, 7, CH), a.astype(np.int32), tuple(data.shape), box, 7, 7, s, 0)
        np.testing.assert_array_equal(dconv.cpu().numpy(), od)


def test_step_side_prep_placement_is_bitwise_neutral(hip):
    """PoseStep(side_prep=False) runs the dropout masks and the ADD row
    classification on the step's own stream (no fork / join) instead of the
    side stream: the same kernels on the same data, so every output of two
    steps (masks drawn from the device step counter each step) is bit-identical."""
    fr = synth.make_frames(B, H=H, W=W, num_classes=C, objects_per_image=4, seed=92)
    g = torch.Generator().manual_seed(5)
    conv4 = torch.randn((B, H // 8, W // 8, CH), generator=g)
    conv5 = torch.randn((B, H // 16, W // 16, CH), generator=g)
    pts, sym = synth.rescaled_points(C)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(D)
    inputs = dict(label=t(fr["label"]), vertex=t(fr["vertex"]), extents=t(fr["extents"]), meta=t(fr["meta"]),
                  gt=t(fr["gt"]), conv4=conv4.to(D), conv5=conv5.to(D), points=t(pts), symmetry=t(sym))
    outs = []
    weights = None
    for side_prep in (True, False):
        step = PoseStep(B, H, W, C, D, channels=CH, units=UNITS, is_train=1, skip_pixels=3, weights=weights,
                        side_prep=side_prep)
        weights = step.weights
        res = []
        for _ in range(2):
            loss = step.step(inputs)
            torch.cuda.synchronize()
            res.append([loss.clone(), step.drop6.clone(), step.drop7.clone(), step.y7.clone(), step.dx.clone(),
                        step.dconv4.clone(), step.grads["w6"].clone(), step.grads["b7"].clone()])
        outs.append(res)
    for a_step, b_step in zip(*outs):
        for a, b in zip(a_step, b_step):
            assert torch.equal(a, b)
    assert not torch.equal(outs[0][0][1], outs[0][1][1])  # the second step drew new masks


def test_forward_alone_draws_masks_in_mask_kernel_mode(hip):
    """with drop_in_reduce=False the keep masks come from
    draw_drop_masks(); forward() called on its own (after a vote, without
    step()) must draw this pass's masks itself rather than use the zeroed
    buffers (every unit dropped) or the previous pass's masks."""
    fr = synth.make_frames(B, H=H, W=W, num_classes=C, objects_per_image=4, seed=93)
    g = torch.Generator().manual_seed(6)
    conv4 = torch.randn((B, H // 8, W // 8, CH), generator=g).to(D)
    conv5 = torch.randn((B, H // 16, W // 16, CH), generator=g).to(D)
    pts, sym = synth.rescaled_points(C)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(D)
    step = PoseStep(B, H, W, C, D, channels=CH, units=UNITS, is_train=1, skip_pixels=3, drop_in_reduce=False,
                    backward=False)
    assert step.keep == 0.5
    step.vote(t(fr["label"]), t(fr["vertex"]), t(fr["extents"]), t(fr["meta"]), t(fr["gt"]))
    drawn = []
    for _ in range(2):
        step.forward(conv4, conv5, t(pts), t(sym))
        torch.cuda.synchronize()
        n = int(step.hough["num_rois"][1].item())
        m6 = step.drop6[:n].double()
        assert abs(float(m6.mean()) - 0.5) < 0.03  # drawn (zeroed buffers would read 0)
        x = step.pool[:n].reshape(n, -1).double()
        w = step.weights
        y6 = torch.relu(x @ w.w6.double() + w.b6.double()) / 0.5 * m6
        _close(step.y6[:n].cpu().numpy(), y6.cpu().numpy())
        drawn.append(step.drop6[:n].clone())
    assert not torch.equal(drawn[0], drawn[1])  # each forward pass draws its own masks
