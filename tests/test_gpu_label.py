"""GPU parity of the label producers against the oracle:
argmax_2d (network.py:433-434), Hardlabel fwd/bwd (hard_label_op_gpu.cu.cc:
17-29, 56-64) and the Hough op with the argmax fused into its compaction pass
(pcnn_hough_voting_prob), all bit-exact."""
import numpy as np
import pytest
import torch

from posecnn_amd import synth
from posecnn_amd.label_2d import argmax_2d
from posecnn_amd.hard_label_layer import hard_label_op as hl
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv

pytestmark = pytest.mark.gpu
D = torch.device("cuda")


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(D)


def _prob_from_label(rng, label, C, ties=True):
    """Softmax-like scores whose argmax is `label`, with exact ties, NaNs and
    near-ties sprinkled in (the argmax must follow numpy's rules, not the label)."""
    B, H, W = label.shape
    p = rng.uniform(0.0, 0.5, size=(B, H, W, C)).astype(np.float32)
    b, y, x = np.indices(label.shape)
    p[b, y, x, label] = rng.uniform(0.6, 1.0, size=label.shape).astype(np.float32)
    if ties:
        m = rng.random(label.shape) < 0.01
        p[m, 0] = p[m].max(axis=1)                 # tie with class 0 -> class 0 wins
        n = rng.random(label.shape) < 0.001
        p[n, C - 1] = np.nan                       # NaN wins
        q = rng.random(label.shape) < 0.01
        p[q, 3] = np.nextafter(p[q].max(axis=1), np.float32(2))  # one ulp above
    return p


@pytest.mark.parametrize("B,H,W,C", [(2, 48, 64, 22), (1, 7, 9, 3), (3, 33, 65, 16), (1, 17, 19, 130),
                                      (2, 5, 13, 1)])
def test_argmax_2d(hip, orc, B, H, W, C):
    rng = np.random.default_rng(B * 100 + C)
    label = rng.integers(0, C, size=(B, H, W)).astype(np.int32)
    p = _prob_from_label(rng, label, C, ties=C > 3)
    got = argmax_2d(T(p)).cpu().numpy()
    np.testing.assert_array_equal(got, orc.argmax_2d(p))


@pytest.mark.parametrize("thr", [0.9, 0.5])
def test_hard_label(hip, orc, thr):
    rng = np.random.default_rng(5)
    B, H, W, C = 2, 9, 11, 5
    p = rng.uniform(0, 1, size=(B, H, W, C)).astype(np.float32)
    gt = rng.integers(-1, C, size=(B, H, W)).astype(np.int32)
    gt[0, 0, :3] = [C, C + 7, -5]  # out of range -> zero rows
    top = hl.hard_label(T(p), T(gt), thr)
    np.testing.assert_array_equal(top.cpu().numpy(), orc.hard_label(p, gt, thr))
    gp, gg = hl.hard_label_grad(T(p), T(gt), top, thr)
    assert not gp.any() and not gg.any() and gg.shape == (B, H, W)
    with pytest.raises(ValueError):
        hl.hard_label(T(p), T(gt), 0.0)


@pytest.mark.parametrize("is_train,thr_vote", [(0, -1.0), (1, -1.0), (0, 0.5)])
def test_hough_from_prob_matches_label_path(hip, orc, is_train, thr_vote):
    """prob -> fused argmax + vote == oracle vote on numpy's argmax, bit for bit."""
    rng = np.random.default_rng(11 + is_train)
    fr = synth.make_frames(2, H=96, W=128, num_classes=22, objects_per_image=4, seed=21)
    p = _prob_from_label(rng, fr["label"], 22)
    lab = orc.argmax_2d(p)
    label_2d, box, pose, tgt, wgt, dom = hv.hough_voting_gpu_from_prob(
        T(p), T(fr["vertex"]), T(fr["extents"]), T(fr["meta"]), T(fr["gt"]), is_train, thr_vote, 0.02, 2)
    np.testing.assert_array_equal(label_2d.cpu().numpy(), lab)
    ob, op, ot, ow, od, on = orc.hough_voting(lab, fr["vertex"], fr["extents"], fr["meta"], fr["gt"], is_train,
                                              thr_vote, 0.02, 2)
    assert on > 0
    np.testing.assert_array_equal(box.cpu().numpy(), ob)
    np.testing.assert_array_equal(pose.cpu().numpy(), op)
    np.testing.assert_array_equal(tgt.cpu().numpy(), ot)
    np.testing.assert_array_equal(wgt.cpu().numpy(), ow)
    np.testing.assert_array_equal(dom.cpu().numpy(), od)


def test_hough_from_prob_full_frame_matches_label_path(hip):
    """At the bench size (640x480, 22 classes) the fused path equals the
    two-op path (argmax_2d kernel, then the label-input Hough op) on device."""
    fr = synth.make_frames(2, 480, 640, num_classes=22, objects_per_image=6, seed=3)
    rng = np.random.default_rng(3)
    p = T(_prob_from_label(rng, fr["label"], 22))
    args = (T(fr["vertex"]), T(fr["extents"]), T(fr["meta"]), T(fr["gt"]), 1, -1.0, 0.02, 10)
    a = hv.hough_voting_gpu_capacity(None, *args, prob=p)
    lab = argmax_2d(p)
    assert torch.equal(a["label"], lab)
    b = hv.hough_voting_gpu_capacity(lab, *args)
    n = int(a["num_rois"][1].item())
    assert n == int(b["num_rois"][1].item()) and n > 1
    for k in ("box", "pose", "target", "weight", "domain"):
        assert torch.equal(a[k][:n], b[k][:n]), k


@pytest.mark.parametrize("B,H,W,K,C", [(2, 24, 32, 128, 22), (1, 9, 13, 16, 4)])
def test_vertex_pred_compact(hip, orc, B, H, W, K, C):
    """Class-compact vertex_pred bit-exact vs the oracle's
    k-ordered fp32 restatement; labels outside [0, C) -> zeros."""
    from posecnn_amd.vertex_pred import vertex_pred_compact
    rng = np.random.default_rng(K + C)
    feat = rng.normal(size=(B, H, W, K)).astype(np.float32)
    w = (rng.normal(size=(1, 1, K, 3 * C)) * 0.05).astype(np.float32)
    b = rng.normal(size=3 * C).astype(np.float32)
    lab = rng.integers(0, C, size=(B, H, W)).astype(np.int32)
    lab[0, 0, :2] = [-1, C]
    out = vertex_pred_compact(T(feat), T(w), T(b), T(lab))
    np.testing.assert_array_equal(out.cpu().numpy(), orc.vertex_pred_compact(feat, w, b, lab))


@pytest.mark.parametrize("is_train,thr_vote", [(1, -1.0), (0, 0.5)])
def test_hough_from_compact_vertex_matches_full(hip, is_train, thr_vote):
    """The vote on the class-compact (B,H,W,3) map equals the vote on the full
    (B,H,W,3C) map, bit for bit, at the bench size (640x480, 22 classes)."""
    fr = synth.make_frames(2, 480, 640, num_classes=22, objects_per_image=6, seed=3)
    lab = fr["label"]
    b, y, x = np.indices(lab.shape)
    v3 = np.stack([fr["vertex"][b, y, x, 3 * lab + j] for j in range(3)], axis=-1).astype(np.float32)
    args = (T(fr["extents"]), T(fr["meta"]), T(fr["gt"]), is_train, thr_vote, 0.02, 10)
    a = hv.hough_voting_gpu_capacity(T(lab), T(fr["vertex"]), *args)
    c = hv.hough_voting_gpu_capacity(T(lab), T(v3), *args, vertex_compact=True)
    n = int(a["num_rois"][1].item())
    assert n == int(c["num_rois"][1].item()) and n > 1
    for k in ("box", "pose", "target", "weight", "domain"):
        assert torch.equal(a[k][:n], c[k][:n]), k
