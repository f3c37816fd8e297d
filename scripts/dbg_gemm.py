import sys, numpy as np, torch
sys.path.insert(0, ".")
from posecnn_amd import pose_head as ph
D = torch.device("cuda")
def run(M, N, K, at=0, bt=0, a2=False, fill=None):
    rng = np.random.default_rng(0)
    A = rng.normal(size=(M, K)).astype(np.float32) if fill is None else np.full((M, K), fill[0], np.float32)
    B = rng.normal(size=(K, N)).astype(np.float32) if fill is None else np.full((K, N), fill[1], np.float32)
    As = A.T.copy() if at else A
    Bs = B.T.copy() if bt else B
    C = torch.full((M, N), -7.0, device=D)
    ph.gemm(torch.from_numpy(As).to(D), torch.from_numpy(Bs).to(D), C, a_trans=at, b_trans=bt, precision=1)
    torch.cuda.synchronize()
    ref = A.astype(np.float64) @ B
    c = C.cpu().numpy()
    err = np.abs(c - ref)
    bad = np.argwhere(err > 1e-3 * (1 + np.abs(ref)))
    print(M, N, K, at, bt, "maxerr", err.max(), "nbad", len(bad), "first", bad[:4].tolist(), c.flat[:3], ref.flat[:3], flush=True)
run(256, 256, 32, fill=(1.0, 1.0))
run(256, 256, 64, fill=(1.0, 1.0))
run(256, 256, 32)
run(256, 256, 64)
run(256, 256, 1024)
run(512, 512, 4096)
run(200, 300, 1000)
run(200, 300, 1000, 0, 1)
run(200, 300, 1000, 1, 0)
run(200, 300, 1000, 1, 1)
