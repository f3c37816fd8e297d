"""Class-aware box NMS (lib/utils/nms.py:3-32) and pose combination
(lib/fcn/test.py:197-211): the oracle against the reference's own outputs
(tests/golden/nms_golden.npz, made by importing the reference module in
tests/golden/make_nms_golden.py) and hand-derived cases."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nms_golden.npz")


def _cases():
    z = np.load(GOLD)
    return [k[: -len("_dets")] for k in z.files if k.endswith("_dets")]


@pytest.mark.parametrize("case", _cases())
def test_oracle_matches_reference_nms(orc, case):
    z = np.load(GOLD)
    d, keep = z[case + "_dets"], z[case + "_keep"]
    thr = float(case.rsplit("_", 1)[1])
    np.testing.assert_array_equal(orc.box_nms(d, thr), keep)


def test_nms_known_answers(orc):
    # two same-class boxes overlapping 81/(100+100-81) = 0.68 > 0.5: the lower
    # score goes; a third of another class survives the same overlap
    d = np.array([[0, 1, 0, 0, 9, 9, 5.0],
                  [0, 1, 1, 1, 10, 10, 7.0],
                  [0, 2, 1, 1, 10, 10, 1.0],
                  [0, 1, 50, 50, 60, 60, 3.0]], np.float32)
    np.testing.assert_array_equal(orc.box_nms(d, 0.5), [1, 3, 2])
    np.testing.assert_array_equal(orc.box_nms(d, 0.7), [1, 0, 3, 2])  # 0.68 <= 0.7 keeps both
    # ties: lower row first (numpy leaves the order unspecified)
    t = d.copy()
    t[:, 6] = 4.0
    np.testing.assert_array_equal(orc.box_nms(t, 0.5), [0, 2, 3])


def test_combine_poses(orc):
    rois = np.array([[0, 2, 0, 0, 9, 9, 5.0], [0, -1, 0, 0, 9, 9, 4.0]], np.float32)
    init = np.arange(14, dtype=np.float32).reshape(2, 7)
    pred = np.arange(24, dtype=np.float32).reshape(2, 12) + 100
    ro, po = orc.nms_combine(rois, init, pred, np.array([1, 0], np.int32))
    np.testing.assert_array_equal(ro, rois[[1, 0]])
    np.testing.assert_array_equal(po[0], init[1])  # class -1: pose unchanged
    np.testing.assert_array_equal(po[1, :4], pred[0, 8:12])  # class 2 -> columns 8..11
    np.testing.assert_array_equal(po[1, 4:], init[0, 4:])
