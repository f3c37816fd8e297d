"""GPU parity against the stored golden vectors (tests/golden/golden.npz):
bit-exact for the Hough op, RoI pool, backprojection; the ADD loss within the
north-star 1e-4 relative tolerance (its per-row sums are reduced in a
different, fixed order on the GPU)."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402

from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv
from posecnn_amd.roi_pooling_layer import roi_pooling_op as rp
from posecnn_amd.average_distance_loss import average_distance_loss_op as adl
from posecnn_amd.backprojecting_layer import backprojecting_op as bp

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(HERE, "golden", "golden.npz"), allow_pickle=False)
D = torch.device("cuda")


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(D)


@pytest.mark.parametrize("case", mg.HOUGH_CASES, ids=[c[0] for c in mg.HOUGH_CASES])
def test_hough_golden(hip, case):
    name, B, H, W, C, obj, seed, train, vthr, skip = case
    fr = mg.hough_frames(B, H, W, C, obj, seed)
    outs = hv.hough_voting_gpu(T(fr["label"]), T(fr["vertex"]), T(fr["extents"]), T(fr["meta"]), T(fr["gt"]),
                               train, vthr, 0.02, skip)
    for k, v in zip(("box", "pose", "target", "weight", "domain"), outs):
        np.testing.assert_array_equal(v.cpu().numpy(), GOLD[f"{name}/{k}"], err_msg=f"{name}/{k}")


@pytest.mark.parametrize("pc", [0, 1])
def test_roi_pool_golden(hip, pc):
    data, rois, top_diff = GOLD["roi/data"], GOLD["roi/rois"], GOLD["roi/top_diff"]
    top, arg = rp.roi_pool(T(data), T(rois), 7, 7, 1.0 / 16, pc)
    np.testing.assert_array_equal(top.cpu().numpy(), GOLD[f"roi{pc}/top"])
    np.testing.assert_array_equal(arg.cpu().numpy(), GOLD[f"roi{pc}/argmax"])
    td = top_diff if not pc else top_diff[..., :1].copy()
    g = rp.roi_pool_grad(T(data), T(rois), arg, T(td), 7, 7, 1.0 / 16, pc)
    np.testing.assert_array_equal(g.cpu().numpy(), GOLD[f"roi{pc}/bottom_diff"])


def test_add_loss_golden(hip):
    args = [T(GOLD[f"add/{k}"]) for k in ("pred", "target", "weight", "points", "symmetry")]
    loss, diff = adl.average_distance_loss(*args, 0.01)
    np.testing.assert_allclose(loss.cpu().numpy(), GOLD["add/loss"], rtol=1e-4)
    np.testing.assert_allclose(diff.cpu().numpy(), GOLD["add/diff"], rtol=1e-4, atol=1e-7)


def test_backproject_golden(hip):
    data, label, depth, meta, label3d, top_diff, G = mg.bp_inputs()
    td, tl, tf = bp.backproject(T(data), T(label), T(depth), T(meta), T(label3d), G, 1, 0.05)
    np.testing.assert_array_equal(td.cpu().numpy(), GOLD["bp/top_data"])
    np.testing.assert_array_equal(tl.cpu().numpy(), GOLD["bp/top_label"])
    np.testing.assert_array_equal(tf.cpu().numpy(), GOLD["bp/top_flag"])
    gb = bp.backproject_grad(T(data), T(depth), T(meta), T(top_diff), G, 1, 0.05)
    np.testing.assert_array_equal(gb.cpu().numpy(), GOLD["bp/bottom_diff"])
