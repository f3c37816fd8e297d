# Analysis (not collected by pytest): how often a reordered (tree)
# Sigma-d would need the serial fallback.  For each (image, class) maximum of the
# configs[2] frames: voting voters at the argmax, the serial fp32 sum, a rigorous
# running-error bound on it, the T(distance) interval, and whether a cone voter can flip.
import sys, time, numpy as np
sys.path.insert(0, '.')
from posecnn_amd import synth
from oracle import oracle as orc
orc.build()
B, H, W, C = 8, 480, 640, 22
SEED = int(sys.argv[1]) if len(sys.argv) > 1 else 3
fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=SEED)
t0 = time.time()
box, pose, *_ , n = orc.hough_voting(fr["label"], fr["vertex"], fr["extents"], fr["meta"], fr["gt"], 0, -1.0, 0.02, 10)
print("oracle", time.time() - t0, "s, rows", n)
f32 = np.float32
ext = fr["extents"].astype(np.float32)
def project_box(cls, meta, d):
    xh = f32(np.float64(ext[cls, 0]) * 0.5); yh = f32(np.float64(ext[cls, 1]) * 0.5); zh = f32(np.float64(ext[cls, 2]) * 0.5)
    fx, fy, px, py = f32(meta[0]), f32(meta[4]), f32(meta[2]), f32(meta[5])
    zf = f32(zh + d); zb = f32(-zh + d)
    xs, ys = [], []
    for i in range(8):
        X = -xh if i & 1 else xh; Y = -yh if i & 2 else yh; Z = zb if i & 4 else zf
        xs.append(f32(f32(fx * f32(X / Z)) + px)); ys.append(f32(f32(fy * f32(Y / Z)) + py))
    w = f32(f32(max(xs) - min(xs)) + f32(1)); h = f32(f32(max(ys) - min(ys)) + f32(1))
    return f32(max(w, h) * f32(0.6))
u = 2.0 ** -24
stats = []
for r in range(n):
    b, cls = int(box[r, 0]), int(box[r, 1])
    cx = int(round((float(box[r, 2]) + float(box[r, 4])) / 2)); cy = int(round((float(box[r, 3]) + float(box[r, 5])) / 2))
    lab = fr["label"][b].reshape(-1); meta = fr["meta"][b].reshape(-1)
    idx = np.nonzero(lab == cls)[0][::10]
    x = (idx % W).astype(np.int64); y = (idx // W).astype(np.int64)
    vm = fr["vertex"][b].reshape(-1, 3 * C)[idx]
    uu, vv = vm[:, 3 * cls].astype(f32), vm[:, 3 * cls + 1].astype(f32)
    d = np.exp(vm[:, 3 * cls + 2].astype(np.float64)).astype(f32)
    T = np.array([project_box(cls, meta, di) for di in d], f32)
    dx = (cx - x).astype(f32); dy = (cy - y).astype(f32)
    n1 = np.sqrt(uu * uu + vv * vv); n2 = np.sqrt(dx * dx + dy * dy); dot = uu * dx + vv * dy
    with np.errstate(invalid='ignore', divide='ignore'):
        cone = (dot / (n1 * n2)) > f32(0.9)
    adx, ady = np.abs(dx), np.abs(dy)
    vote = cone & (adx < T) & (ady < T)
    dv = d[vote]
    ser = np.add.accumulate(dv, dtype=f32)
    S = float(ser[-1]); cnt = int(vote.sum())
    bound = u * float(np.sum(ser[1:].astype(np.float64))) * 1.0000001
    tree = float(np.sum(dv.astype(np.float64)))  # ~exact
    dist_ser = f32(f32(S) / f32(cnt))
    assert abs(dist_ser - float(pose[r, 6])) <= 0, (dist_ser, pose[r, 6])
    lo = f32((tree - bound - 2 * u * tree) / cnt); hi = f32((tree + bound + 2 * u * tree) / cnt)
    Ts = [project_box(cls, meta, f32(v)) for v in (lo, hi)]
    Tlo, Thi = min(Ts) * (1 - 8 * 2 ** -24), max(Ts) * (1 + 8 * 2 ** -24)
    amb_int = int(np.ceil(Tlo)) != int(np.ceil(Thi))
    flip = False
    if amb_int:
        ks = np.arange(np.ceil(Tlo) - 1, np.ceil(Thi) + 1)
        sel = cone & ((np.isin(adx, ks) & (ady < Thi)) | (np.isin(ady, ks) & (adx < Thi)))
        flip = bool(sel.any())
    stats.append((b, cls, cnt, S, bound / S, Tlo, Thi, amb_int, flip, abs(S - tree) / S))
st = np.array([(s[2], s[4], s[6] - s[5], s[7], s[8], s[9]) for s in stats])
print("slots", len(st), "mean count", st[:, 0].mean(), "max", st[:, 0].max())
print("rel bound mean %.2e max %.2e; actual serial err mean %.2e max %.2e" % (st[:, 1].mean(), st[:, 1].max(), st[:, 5].mean(), st[:, 5].max()))
print("T band width mean %.4f max %.4f" % (st[:, 2].mean(), st[:, 2].max()))
print("integer in band:", int(st[:, 3].sum()), " voter could flip (fallback):", int(st[:, 4].sum()))
