"""BASELINE.json configs[2] at its real size, and the per-rank share of
configs[4] -- the step the bench times, checked end to end.

configs[2]: B = 8 frames of 640x480, C = 22 YCB classes, train mode, conv4_3 /
conv5_3 with 512 channels, 4096-unit fc6 / fc7 (vgg16_convs.py:167-200), the
default fp32-faithful GEMMs.  Checked, on the step's own intermediate values:
  * the Hough rows against the oracle (bit-exact);
  * pool5 + pool4 against the oracle's two RoI pools (bit-exact sum);
  * each layer of the head with drop6 / drop7 at keep_prob 0.5 on
    externally supplied masks (y6, y7, y8, pred; dy8, dy7, dy6, dX and every
    weight / bias gradient) against float64 (torch on the GPU) of that
    layer on the step's own fp32 inputs, at fp32-GEMM tolerance (2e-5 of the
    tensor's scale); the ADD loss / gradient against the oracle (1e-4, its
    contract);
  * both RoI-pool backwards against the oracle on the step's dX (bit-exact).
configs[4] per rank: LINEMOD, C = 16 (15 objects, linemod.py:35-37), 8 frames
of the 32-frame global batch (index_size = 128 / 32 = 4, rows rebased by the
rank's batch offset), symmetric classes per linemod.py:44; the Hough rows and
the ADD loss against the oracle on that rank's frames."""
import numpy as np
import pytest
import torch

from posecnn_amd import synth
from posecnn_amd.pipeline import PoseStep

pytestmark = pytest.mark.gpu
D = torch.device("cuda")


def _close(a, ref, rt):
    """|a - ref| <= rt * (|ref| + max |ref|), on the GPU"""
    a, ref = a.double(), ref.double()
    scale = float(ref.abs().max())
    bad = (a - ref).abs() > rt * (ref.abs() + scale)
    assert not bool(bad.any()), f"{int(bad.sum())} of {bad.numel()} beyond {rt}; max err " \
                                f"{float((a - ref).abs().max()):.3e}, scale {scale:.3e}"


def _inputs(fr, conv_hw4, conv_hw5, pts, sym, seed):
    g = torch.Generator(device=D)
    g.manual_seed(seed)
    B = fr["label"].shape[0]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(D)
    return dict(label=t(fr["label"]), vertex=t(fr["vertex"]), extents=t(fr["extents"]), meta=t(fr["meta"]),
                gt=t(fr["gt"]), conv4=torch.randn((B,) + conv_hw4 + (512,), generator=g, device=D),
                conv5=torch.randn((B,) + conv_hw5 + (512,), generator=g, device=D), points=t(pts), symmetry=t(sym))


def test_configs2_full_step(hip, orc):
    B, H, W, C = 8, 480, 640, 22
    fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=3)
    pts, sym = synth.rescaled_points(C)
    inp = _inputs(fr, (60, 80), (30, 40), pts, sym, 1234)
    step = PoseStep(B, H, W, C, D, is_train=1, skip_pixels=10)  # train: drop6 / drop7 at keep_prob 0.5
    keep = step.keep
    assert keep == 0.5
    # externally supplied dropout keep masks (the step's Philox draw is checked in test_gpu_step.py)
    gm = torch.Generator(device=D)
    gm.manual_seed(17)
    m6 = torch.rand((step.drop6.shape[0], 4096), generator=gm, device=D) < keep
    m7 = torch.rand((step.drop7.shape[0], 4096), generator=gm, device=D) < keep
    step.set_drop_masks(m6, m7)
    w = step.weights
    gb = torch.Generator(device=D)
    gb.manual_seed(5)
    for b in (w.b6, w.b7, w.b8):  # non-zero biases so the bias epilogues and column sums are exercised
        b.copy_(torch.randn(b.shape, generator=gb, device=D) * 1e-3)
    step.step(inp)
    torch.cuda.synchronize()
    n = int(step.hough["num_rois"][1].item())
    assert n > 300, n

    # Hough rows (bit-exact)
    ob, op, ot, ow, od, on = orc.hough_voting(fr["label"], fr["vertex"], fr["extents"], fr["meta"], fr["gt"], 1,
                                              -1.0, 0.02, 10)
    assert on == n
    np.testing.assert_array_equal(step.hough["box"][:n].cpu().numpy(), ob)
    np.testing.assert_array_equal(step.hough["pose"][:n].cpu().numpy(), op)
    np.testing.assert_array_equal(step.hough["target"][:n].cpu().numpy(), ot)
    np.testing.assert_array_equal(step.hough["weight"][:n].cpu().numpy(), ow)

    # pool5 + pool4 (bit-exact)
    c4, c5 = inp["conv4"].cpu().numpy(), inp["conv5"].cpu().numpy()
    p5, a5 = orc.roi_pool_fwd(c5, ob, 7, 7, 1.0 / 16)
    p4, a4 = orc.roi_pool_fwd(c4, ob, 7, 7, 1.0 / 8)
    np.testing.assert_array_equal(step.pool[:n].cpu().numpy(), p5 + p4)

    # every layer against fp64 on the step's own fp32 inputs to that layer (a
    # ReLU mask decided on an fp32 activation within rounding of 0 would
    # otherwise flip whole terms between the two graphs), on the GPU
    f = lambda t_: t_[:n].double()
    x = step.pool[:n].reshape(n, -1).double()
    W6, W7, W8 = (v.double() for v in (w.w6, w.w7, w.w8))
    d6, d7 = m6[:n].double(), m7[:n].double()
    dropout = lambda y, m_: (y / keep) * m_  # tf.nn.dropout (network.py:574-577)
    _close(step.y6[:n], dropout(torch.relu(x @ W6 + w.b6.double()), d6), 2e-5)
    _close(step.y7[:n], dropout(torch.relu(f(step.y6) @ W7 + w.b7.double()), d7), 2e-5)
    _close(step.y8[:n], f(step.y7) @ W8 + w.b8.double(), 2e-5)
    y8 = f(step.y8).requires_grad_()
    pw = step.hough["weight"][:n].double()
    m = torch.tanh(y8) * pw
    pred = m / torch.sqrt(torch.clamp((m * m).sum(1, keepdim=True), min=1e-12))  # network.py:440-445
    _close(step.pred[:n], pred.detach(), 2e-5)

    ol, odf, _ = orc.average_distance_loss(step.pred[:n].cpu().numpy(), ot, ow, pts, sym, 0.01)
    np.testing.assert_allclose(step.loss.cpu().numpy(), ol, rtol=1e-4)
    np.testing.assert_allclose(step.diff[:n].cpu().numpy(), odf, rtol=1e-4, atol=1e-7)

    pred.backward(f(step.diff))
    _close(step.dy8[:n], y8.grad, 2e-5)
    gr = step.grads
    dy8, dy7, dy6 = f(step.dy8), f(step.dy7), f(step.dy6)
    _close(gr["w8"], f(step.y7).T @ dy8, 2e-5)
    _close(gr["b8"], dy8.sum(0), 2e-5)
    # TF's backward of relu -> dropout: ReluGrad((g * binary) / keep_prob); y7 is the dropped activation
    _close(step.dy7[:n], (dy8 @ W8.T) * d7 / keep * (step.y7[:n] > 0), 2e-5)
    _close(gr["w7"], f(step.y6).T @ dy7, 2e-5)
    _close(gr["b7"], dy7.sum(0), 2e-5)
    _close(step.dy6[:n], (dy7 @ W7.T) * d6 / keep * (step.y6[:n] > 0), 2e-5)
    _close(gr["w6"], x.T @ dy6, 2e-5)
    _close(gr["b6"], dy6.sum(0), 2e-5)
    _close(step.dx[:n], dy6 @ W6.T, 2e-5)
    del W6, x

    # both RoI-pool backwards on the step's dX and argmax (pixel index -> flat index)
    dx = step.dx[:n].cpu().numpy().reshape(n, 7, 7, 512)
    for arg, data, dconv, s in ((step.arg5, c5, step.dconv5, 1.0 / 16), (step.arg4, c4, step.dconv4, 1.0 / 8)):
        a = arg[:n].cpu().numpy().astype(np.int64) & 0xFFFF
        a = np.where(a == 0xFFFF, -1, a * 512 + np.arange(512)).astype(np.int32)
        od_ = orc.roi_pool_bwd(dx, a, data.shape, ob, 7, 7, s, 0)
        np.testing.assert_array_equal(dconv.cpu().numpy(), od_)


def test_configs4_linemod_rank(hip, orc):
    """One rank of configs[4] (rank 1 of 4: frames 8-15 of a global batch of 32)."""
    B, H, W, C, rank, gB = 8, 480, 640, 16, 1, 32
    fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=4, seed=5, image_offset=rank * B,
                           extents=synth.models()["linemod_extents"])
    pts, sym = synth.linemod_points()
    assert sym.any(), "LINEMOD has symmetric classes (linemod.py:44)"
    inp = _inputs(fr, (60, 80), (30, 40), pts, sym, 77)
    step = PoseStep(B, H, W, C, D, is_train=1, skip_pixels=10, global_batch=gB, batch_base=rank * B)
    step.step(inp)
    torch.cuda.synchronize()
    n = int(step.hough["num_rois"][1].item())
    ob, op, ot, ow, od, on = orc.hough_voting(fr["label"], fr["vertex"], fr["extents"], fr["meta"], fr["gt"], 1,
                                              -1.0, 0.02, 10, global_batch=gB, batch_base=rank * B)
    assert on == n and n > 0
    # index_size = 4 maxima per image: at most 4 * 9 rows per image
    assert n <= B * 4 * 9
    np.testing.assert_array_equal(step.hough["box"][:n].cpu().numpy(), ob)
    np.testing.assert_array_equal(step.hough["pose"][:n].cpu().numpy(), op)
    np.testing.assert_array_equal(step.hough["target"][:n].cpu().numpy(), ot)
    np.testing.assert_array_equal(step.hough["weight"][:n].cpu().numpy(), ow)
    assert (ob[:, 0] >= rank * B).all() and (ob[:, 0] < (rank + 1) * B).all()
    # ADD loss with the LINEMOD symmetry on the step's prediction; the single-rank
    # normaliser is this rank's row count (the sharded run all-reduces it)
    cls = np.argmax(ow[:, ::4] > 0, axis=1)
    assert sym[cls].any(), "the frames should carry a symmetric-class row"
    ol, odf, _ = orc.average_distance_loss(step.pred[:n].cpu().numpy(), ot, ow, pts, sym, 0.01)
    np.testing.assert_allclose(step.loss.cpu().numpy(), ol, rtol=1e-4)
    np.testing.assert_allclose(step.diff[:n].cpu().numpy(), odf, rtol=1e-4, atol=1e-7)
