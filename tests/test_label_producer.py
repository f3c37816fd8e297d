"""CPU checks of the label-producer oracle: argmax_2d
(network.py:433-434) and Hardlabel (hard_label_op.cc:94-106,
hard_label_op_gpu.cu.cc:17-29) on hand-derived known answers, (the C-ABI
exports are checked in test_abi.py)."""
import numpy as np

from oracle import oracle


def test_argmax_2d_known_answers():
    p = np.zeros((1, 1, 5, 4), np.float32)
    p[0, 0, 0] = [0.1, 0.7, 0.1, 0.1]          # plain max -> 1
    p[0, 0, 1] = [0.4, 0.1, 0.4, 0.1]          # tie -> first (0)
    p[0, 0, 2] = [0.1, 0.2, 0.3, 0.3]          # tie at the end -> 2
    p[0, 0, 3] = [0.1, np.nan, 0.9, np.nan]    # NaN wins at its first occurrence -> 1
    p[0, 0, 4] = [-np.inf, -np.inf, -5, -np.inf]
    np.testing.assert_array_equal(oracle.argmax_2d(p)[0, 0], [1, 0, 2, 1, 2])


def test_hard_label_known_answers():
    thr = 0.9
    prob = np.full((1, 1, 6, 3), 1 / 3, np.float32)
    prob[0, 0, 1, 0] = 0.95   # background confident -> no label
    gt = np.array([[[0, 0, 2, -1, 1, 3]]], np.int32)
    top = oracle.hard_label(prob, gt, thr)
    want = np.zeros((1, 1, 6, 3), np.float32)
    want[0, 0, 0, 0] = 1      # bg with prob 1/3 < 0.9 -> hard example
    want[0, 0, 2, 2] = 1      # foreground always labelled
    want[0, 0, 4, 1] = 1
    np.testing.assert_array_equal(top, want)  # gt -1 and out-of-range 3 -> zero rows


def test_vertex_pred_compact_known_answer():
    # 1 pixel per class, K = 4: out = (((0 + x0 w0) + x1 w1) + x2 w2) + x3 w3 + b at the class columns
    K, C = 4, 3
    x = np.arange(1, 1 + 3 * K, dtype=np.float32).reshape(1, 1, 3, K)
    w = np.arange(K * 3 * C, dtype=np.float32).reshape(K, 3 * C) / 8
    b = np.arange(3 * C, dtype=np.float32) / 2
    lab = np.array([[[0, 2, 5]]], np.int32)  # 5: out of range -> zeros
    out = oracle.vertex_pred_compact(x, w, b, lab)
    for px, l in enumerate([0, 2]):
        want = (x[0, 0, px] @ w[:, 3 * l:3 * l + 3]) + b[3 * l:3 * l + 3]  # small integers / 8: exact
        np.testing.assert_array_equal(out[0, 0, px], want)
    assert not out[0, 0, 2].any()
