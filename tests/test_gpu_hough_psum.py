"""The distance sum at the Hough maxima (hough_voting_gpu_op.cu.cc:269-298),
round 5: the reference's in-order fp32 sum is rebuilt in parallel
(hough_peak.hip, exact_cell_par: parity transducers per binade run, the
binade crossings added by one lane with the real fp32 add, every prediction
verified) instead of one lane's dependent chain.  The bar is the same bits as
the serial chain: every output column against the oracle's sequential loop,
and against the kernel's own serial path (PCNN_HOUGH_SUM=serial).  diag[3]
counts maxima that fell back to the serial chain."""
import os

import numpy as np
import pytest
import torch

from posecnn_amd import synth
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv

pytestmark = pytest.mark.gpu


def _run(fr, is_train, skip, serial=False, vote_thr=-1.0):
    d = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(d)  # noqa: E731
    old = os.environ.pop("PCNN_HOUGH_SUM", None)
    if serial:
        os.environ["PCNN_HOUGH_SUM"] = "serial"
    try:
        o = hv.hough_voting_gpu_capacity(t(fr["label"]), t(fr["vertex"]), t(fr["extents"]), t(fr["meta"]),
                                         t(fr["gt"]), is_train, vote_thr, 0.02, skip)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("PCNN_HOUGH_SUM", None)
        if old is not None:
            os.environ["PCNN_HOUGH_SUM"] = old
    n = int(o["num_rois"][1].item())
    res = [o[k][:n].cpu().numpy() for k in ("box", "pose", "target", "weight", "domain")]
    return res, hv.hough_voting_diag(o)


def _exact(orc, fr, is_train, skip, vote_thr=-1.0):
    res, diag = _run(fr, is_train, skip, vote_thr=vote_thr)
    ser, dser = _run(fr, is_train, skip, serial=True, vote_thr=vote_thr)
    assert diag[0] == 0 and dser[0] == 0 and dser[3] == 0
    ref = orc.hough_voting(fr["label"], fr["vertex"], fr["extents"], fr["meta"], fr["gt"], is_train, vote_thr, 0.02,
                           skip)
    for a, s_, r in zip(res, ser, ref[:5]):
        np.testing.assert_array_equal(a, r)
        np.testing.assert_array_equal(s_, r)
    return res, diag


def test_psum_bench_frames(hip, orc):
    """configs[2]'s own frames (B = 8, 640x480, skip 10; bench.py seed 3): the
    parallel sum gives the serial bits, and no maximum needs the fallback."""
    fr = synth.make_frames(8, 480, 640, num_classes=22, objects_per_image=6, seed=3)
    res, diag = _exact(orc, fr, 1, 10)
    assert res[0].shape[0] > 300
    assert diag[3] == 0, f"{diag[3]} maxima fell back to the serial chain"


def _tie_depths(n, rng):
    """n depths d = 1 + (2j + 1) 2^-13 together with a float32 log-depth z
    whose (float)exp((double)z) is exactly d (the op's depth, cu.cc:280):
    every add of such a d to a running sum in [2048, 4096) is an exact
    half-ulp tie (round half to even), in [1024, 2048) exact."""
    d = (1.0 + (2 * rng.integers(0, 2 ** 11, n) + 1) * 2.0 ** -13).astype(np.float32)
    z = np.log(d.astype(np.float64)).astype(np.float32)
    for k in range(n):
        zi = z[k]
        for step in range(12):
            if np.float32(np.exp(np.float64(zi))) == d[k]:
                break
            zi = np.nextafter(zi, np.float32(np.inf) if np.exp(np.float64(zi)) < d[k] else np.float32(-np.inf))
        z[k] = zi
    ok = np.exp(z.astype(np.float64)).astype(np.float32) == d
    return d, z, ok


@pytest.mark.parametrize("skip,r", [(1, 62), (2, 62), (1, 95)])
def test_psum_half_ulp_ties(hip, orc, skip, r):
    """A disc of thousands of voters whose vectors point exactly at its centre
    and whose depths make every add in the [2048, 4096) binade a half-ulp tie
    (and cross binades on the way): the parity transducers carry the
    round-half-even choices; the sum, the pose and the box are the serial
    chain's bits.  The cases take each of the peak kernel's paths: 6 k
    voters (8 per thread), 12 k (24 per thread) and 28 k (past 24 per
    thread: the serial chain, counted in diag[3])."""
    H, W, C = 240, 320, 4
    fr = synth.make_frames(1, H, W, num_classes=C, objects_per_image=1, seed=21)
    fr["extents"] = np.full((C, 3), 0.3, np.float32)  # T ~ 190 px at 1 m: every disc voter passes the box test
    rng = np.random.default_rng(5)
    cy, cx = 120, 160
    yy, xx = np.mgrid[0:H, 0:W]
    disc = (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
    label = np.zeros((1, H, W), np.int32)
    label[0][disc] = 2
    vert = rng.uniform(-1, 1, (1, H, W, 3 * C)).astype(np.float32)
    dx, dy = (cx - xx).astype(np.float64), (cy - yy).astype(np.float64)
    nrm = np.sqrt(dx * dx + dy * dy)
    nrm[nrm == 0] = 1
    vert[0, :, :, 6] = (dx / nrm).astype(np.float32)
    vert[0, :, :, 7] = (dy / nrm).astype(np.float32)
    npx = int(disc.sum())
    d, z, ok = _tie_depths(npx, rng)
    assert ok.mean() > 0.9
    zz = vert[0, :, :, 8].copy()
    zz[disc] = z
    vert[0, :, :, 8] = zz
    fr["label"], fr["vertex"] = label, vert
    fr["gt"] = fr["gt"][:0]
    res, diag = _exact(orc, fr, 0, skip)
    assert res[0].shape[0] == 1 and res[1][0, 6] > 0.9  # one maximum, its distance ~1 m
    nv = (npx + skip - 1) // skip
    assert (diag[3] >= 1) == (nv > 24 * 1024), (nv, diag[3])
