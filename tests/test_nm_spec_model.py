"""CPU model of the device Nelder-Mead's speculative rounds (csrc/icp.hip
k_nm_spec): every iteration evaluates the reflection, the expansion and both
contractions in one round, the initial simplex and a shrink four points per
round, and the search takes the values in the sequential order, counting only
those it uses.  Because the objective is a pure function of the point, the
simplex, the evaluation count and the result must be those of the sequential
search (posecnn_amd/synthesize/icp.py nelder_mead, the driver the device
search is tested against bit for bit on the GPU).  This model restates the
kernel's control flow in Python and checks that claim on objectives with
plateaus, ties and clamped optima, where reflection, expansion, both
contractions and shrinks all occur."""
import numpy as np
import pytest

from posecnn_amd.synthesize.icp import nelder_mead

W = 4  # points per round (kNmSpecW)


def nelder_mead_spec(f, x0, lb, ub, max_eval, log):
    """k_nm_spec's control flow; log collects the size of every round."""
    x0 = np.asarray(x0, np.float64)
    lb, ub = np.asarray(lb, np.float64), np.asarray(ub, np.float64)
    n = x0.size
    clamp = lambda p: np.minimum(np.maximum(p, lb), ub)  # noqa: E731

    def rnd(points):
        log.append(len(points))
        return [f(p) for p in points]

    pts = [x0.copy()]
    for i in range(n):
        step = min(0.25 * (ub[i] - lb[i]), 0.75 * (ub[i] - x0[i]), 0.75 * (x0[i] - lb[i]))
        p = x0.copy()
        p[i] = x0[i] + step
        pts.append(p)
    vals = []
    for i0 in range(0, n + 1, W):
        vals += rnd(pts[i0:i0 + W])
    pts, vals = np.array(pts), np.array(vals)
    nev = n + 1
    while nev < max_eval:
        order = np.argsort(vals, kind="stable")
        pts, vals = pts[order], vals[order]
        cen = pts[0].copy()
        for i in range(1, n):
            cen = cen + pts[i]
        cen = cen / n
        xr = clamp(cen + (cen - pts[n]))
        cand = [xr, clamp(cen + 2.0 * (cen - pts[n])), clamp(cen + 0.5 * (xr - cen)), clamp(cen + 0.5 * (pts[n] - cen))]
        fs = rnd(cand)
        fr = fs[0]
        nev += 1
        v0, vn1, vn = vals[0], vals[n - 1], vals[n]
        if fr < v0 and nev < max_eval:
            nev += 1
            take_e = fs[1] < fr
            pts[n], vals[n] = (cand[1], fs[1]) if take_e else (cand[0], fr)
        elif fr < vn1:
            pts[n], vals[n] = cand[0], fr
        elif nev < max_eval:
            nev += 1
            kc = 3 if fr >= vn else 2
            if fs[kc] < min(fr, vn):
                pts[n], vals[n] = cand[kc], fs[kc]
            else:
                m = min(n, max_eval - nev)
                new = [clamp(pts[0] + 0.5 * (pts[i] - pts[0])) for i in range(1, m + 1)]
                fv = []
                for i0 in range(0, m, W):
                    fv += rnd(new[i0:i0 + W])
                for i in range(m):
                    pts[1 + i], vals[1 + i] = new[i], fv[i]
                nev += max(m, 0)
    b = int(np.argmin(vals))
    return pts[b], vals[b], nev


def _objectives():
    rng = np.random.default_rng(11)
    A = rng.normal(size=(7, 7))
    H = A @ A.T + 0.1 * np.eye(7)
    c = rng.uniform(-0.05, 0.05, 7)
    yield lambda p: float((p - c) @ H @ (p - c))                                    # smooth bowl
    yield lambda p: float(np.round(np.sum(np.abs(p - c)) * 20) / 20)                  # plateaus and ties
    yield lambda p: float(np.sum((p - 0.5) ** 2))                                     # optimum outside the bounds
    yield lambda p: float(np.float32(np.sum(np.sin(7 * p) * np.cos(3 * p[::-1]))))  # float32 values, many minima


@pytest.mark.parametrize("max_eval", [5, 8, 12, 30, 50, 200])
def test_speculative_rounds_match_sequential_search(max_eval):
    x0 = np.array([0.99, 0.02, -0.01, 0.0, 0.002, -0.001, 0.01])
    r = np.array([0.1, 0.1, 0.1, 0.1, 0.01, 0.01, 0.1])
    for f in _objectives():
        hx, hf = nelder_mead(f, x0, x0 - r, x0 + r, max_eval)
        log = []
        sx, sf, nev = nelder_mead_spec(f, x0, x0 - r, x0 + r, max_eval, log)
        np.testing.assert_array_equal(sx, hx)
        assert sf == hf
        assert nev == max(8, max_eval)
        assert sum(1 for k in log if k == W) >= 1
        if max_eval >= 50:  # fewer rounds than evaluations: the point of the speculation
            assert len(log) < nev
