"""CPU model of the Hough peak's parallel in-order fp32 sum (csrc/hough_peak.hip,
exact_cell_par): thread-contiguous runs, binades
predicted from exact prefix sums, parity transducers composed within a
binade, the crossings added by one "lane" with the real fp32 add, every
prediction verified.  It must reproduce the serial loop fl(s + d) bit for
bit (the reference's sum, hough_voting_gpu_op.cu.cc:269-291) or report a
fallback -- on random, tie-heavy and wide-range sequences."""
import numpy as np
import pytest

f32 = np.float32
NT = 64  # "threads"

def serial(d):
    s = f32(0)
    for x in d:
        s = f32(s + x)
    return s

def binade(x):  # E with 2^E <= x < 2^(E+1), x > 0
    return int(np.floor(np.log2(x))) if x > 0 else -999

def trans(q):
    """parity transducer of adding q (= d/u, exact) to an integer S: returns (inc0, inc1)"""
    fl = np.floor(q); fr = q - fl; fl = int(fl)
    if fr > 0.5: return (fl + 1, fl + 1)
    if fr < 0.5: return (fl, fl)
    return tuple(fl + (((p + fl) & 1)) for p in (0, 1))

def compose(A, B):  # A then B; transducer = (inc0, inc1)
    out = []
    for p in (0, 1):
        i = A[p]
        q = (p + i) & 1
        out.append(i + B[q])
    return tuple(out)

ID = (0, 0)

def par(d):
    """The parallel form; None = fallback to the serial chain."""
    n = len(d)
    P = np.cumsum(d.astype(np.float64))  # exact-ish prefixes
    E = [binade(p) for p in P]
    event = [k == 0 or E[k] != E[k - 1] for k in range(n)]
    # per-term transducer in units of u = 2^(E-23) of its segment
    T = []
    for k in range(n):
        if event[k]:
            T.append(None)
        else:
            u = 2.0 ** (E[k] - 23)
            q = float(d[k]) / u
            if q >= 2.0 ** 23: return None  # a "non-event" that cannot be in-binade
            T.append(trans(q))
    # chunking into NT threads (contiguous), local summaries + exclusive scan
    m = (n + NT - 1) // NT
    chunks = [(t * m, min(n, (t + 1) * m)) for t in range(NT)]
    summ = []
    for a, b in chunks:
        has, tr = False, ID
        for k in range(a, b):
            if event[k]: has, tr = True, ID
            else: tr = compose(tr, T[k])
        summ.append((has, tr))
    X = []  # exclusive prefix (tail since last event)
    acc = (False, ID)
    for s in summ:
        X.append(acc)
        acc = (True, s[1]) if s[0] else (acc[0], compose(acc[1], s[1]))
    # event records: (k, transducer of the segment ending just before it)
    ev = []
    for t, (a, b) in enumerate(chunks):
        tr = X[t][1]
        for k in range(a, b):
            if event[k]:
                ev.append((k, tr)); tr = ID
            else:
                tr = compose(tr, T[k])
    final_tr = acc[1]
    # serial walk over events
    s = f32(0); seg_start = {}
    for (k, tr) in ev:
        if s != 0:
            u = 2.0 ** (binade(float(s)) - 23)
            S = int(float(s) / u)
            S2 = S + tr[S & 1]
            if S2 >= 2 ** 24: return None
            s = f32(S2 * u)
        s = f32(s + d[k])
        if binade(float(s)) != E[k]: return None  # event landed elsewhere
        seg_start[k] = s
    u = 2.0 ** (binade(float(s)) - 23); S = int(float(s) / u)
    S2 = S + final_tr[S & 1]
    if S2 >= 2 ** 24: return None
    # verification of in-segment terms (each stays inside its binade)
    cur = None
    for k in range(n):
        if event[k]:
            cur = int(float(seg_start[k]) / 2.0 ** (E[k] - 23)); continue
        c2 = cur + T[k][cur & 1]
        if not (2 ** 23 <= cur and c2 < 2 ** 24): return None
        cur = c2
    return f32(S2 * u)



@pytest.mark.parametrize("kind", [0, 1, 2, 3])
def test_parallel_sum_model_matches_serial(kind):
    rng = np.random.default_rng(1 + kind)
    exact = 0
    for trial in range(25):
        n = int(rng.integers(1, 2500))
        if kind == 0:
            d = np.exp(rng.normal(0.2, 0.3, n)).astype(f32)          # depths ~1 m
        elif kind == 1:
            d = rng.integers(1, 64, n).astype(f32) * f32(0.25)       # many exact ties
        elif kind == 2:
            d = (rng.integers(1, 2 ** 12, n) * 2.0 ** -12 + 1).astype(f32)
        else:
            d = np.exp(rng.normal(0, 2, n)).astype(f32)               # wide spread
        got = par(d)
        if got is None:
            continue
        assert got == serial(d)
        exact += 1
    assert exact >= 20
