"""GPU parity of the device box NMS + pose combination (pcnn_box_nms) against
the reference's own NMS outputs (golden) and the oracle (ties, device row
count, capacity, the Hough op's test-mode rows)."""
import os

import numpy as np
import pytest
import torch

from posecnn_amd import synth
from posecnn_amd.utils import nms as dn
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv

pytestmark = pytest.mark.gpu
D = torch.device("cuda")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nms_golden.npz")


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(D)


def test_nms_matches_reference_golden(hip):
    z = np.load(GOLD)
    for k in z.files:
        if not k.endswith("_dets"):
            continue
        case = k[: -len("_dets")]
        thr = float(case.rsplit("_", 1)[1])
        assert dn.nms(T(z[k]), thr) == z[case + "_keep"].tolist(), case


@pytest.mark.parametrize("R,seed", [(1, 0), (37, 1), (405, 2), (1152, 3)])
def test_nms_ties_and_combine_vs_oracle(hip, orc, R, seed):
    rng = np.random.default_rng(seed)
    d = np.zeros((R, 7), np.float32)
    d[:, 1] = rng.integers(-1, 4, R)
    xy = rng.uniform(0, 300, (R, 2))
    d[:, 2:4] = xy
    d[:, 4:6] = xy + rng.uniform(-5, 120, (R, 2))  # some negative extents
    d[:, 6] = rng.integers(0, 8, R)  # many equal scores
    keep = orc.box_nms(d, 0.5)
    assert dn.nms(T(d), 0.5) == keep.tolist()
    init = rng.normal(size=(R, 7)).astype(np.float32)
    pred = rng.normal(size=(R, 16)).astype(np.float32)
    ro, po = orc.nms_combine(d, init, pred, keep)
    r, p, n = dn.nms_combine(T(d), T(init), T(pred), 0.5)
    k = int(n.item())
    assert k == len(keep)
    np.testing.assert_array_equal(r[:k].cpu().numpy(), ro)
    np.testing.assert_array_equal(p[:k].cpu().numpy(), po)


def test_nms_device_row_count(hip, orc):
    rng = np.random.default_rng(9)
    d = np.zeros((64, 7), np.float32)
    d[:, 1] = 1
    d[:, 2:4] = rng.uniform(0, 50, (64, 2))
    d[:, 4:6] = d[:, 2:4] + 40
    d[:, 6] = rng.permutation(64)
    keep, n = dn.nms_device(T(d), 0.5, num_rois=torch.tensor([23], dtype=torch.int32, device=D))
    ref = orc.box_nms(d[:23], 0.5)
    assert int(n.item()) == len(ref)
    assert keep[: len(ref)].cpu().tolist() == ref.tolist()


def test_nms_on_hough_rows(hip, orc):
    """The inference chain of test.py:190-211: test-mode Hough rows -> NMS ->
    combined poses, against the oracle on the same rows."""
    fr = synth.make_frames(2, 120, 160, num_classes=8, objects_per_image=4, seed=5)
    box, pose, tgt, wgt, dom = hv.hough_voting_gpu(T(fr["label"]), T(fr["vertex"]), T(fr["extents"]),
                                                   T(fr["meta"]), T(fr["gt"]), 0, -1.0, 0.02, 2)
    b = box.cpu().numpy()
    pred = np.random.default_rng(1).normal(size=(b.shape[0], 32)).astype(np.float32)
    keep = orc.box_nms(b, 0.5)
    ro, po = orc.nms_combine(b, pose.cpu().numpy(), pred, keep)
    r, p, n = dn.nms_combine(box, pose, T(pred), 0.5)
    k = int(n.item())
    np.testing.assert_array_equal(r[:k].cpu().numpy(), ro)
    np.testing.assert_array_equal(p[:k].cpu().numpy(), po)
