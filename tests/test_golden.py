"""Golden fixtures (tests/golden/golden.npz, written by make_golden.py):
the oracle and the synthetic generator must reproduce them bit for bit."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402

GOLD = np.load(os.path.join(HERE, "golden", "golden.npz"), allow_pickle=False)


@pytest.mark.parametrize("case", mg.HOUGH_CASES, ids=[c[0] for c in mg.HOUGH_CASES])
def test_synth_inputs_unchanged(case):
    name, B, H, W, C, obj, seed = case[:7]
    fr = mg.hough_frames(B, H, W, C, obj, seed)
    assert mg.sha(fr["label"], fr["vertex"], fr["meta"], fr["gt"]) == str(GOLD[f"{name}/sha"])


def test_oracle_reproduces_golden(orc):
    got = mg.compute(orc)
    assert set(got) == set(GOLD.files)
    for k in GOLD.files:
        if GOLD[k].dtype.kind in "US":
            assert str(got[k]) == str(GOLD[k]), k
        else:
            np.testing.assert_array_equal(got[k], GOLD[k], err_msg=k)
