"""Per-K-step cost of the x3 GEMM tile against its live 32-row blocks: one
M tile of m rows (1..256) x 256 tiles along N (tile mode, one tile per
workgroup), K = 4096.  Also the stream-K form of fc6 dX / fc7 fwd at R rows
with and without the schedule's partial-tile weighting.
    python scripts/gemm_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posecnn_amd import pose_head as ph  # noqa: E402

D = torch.device("cuda")
g = torch.Generator(device=D).manual_seed(0)


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


K, N = 4096, 256 * 256
A = torch.randn(256, K, generator=g, device=D)
B = torch.randn(K, N, generator=g, device=D) * 1e-3
C = torch.empty(256, N, device=D)
full = None
for m in (256, 224, 192, 160, 128, 96, 64, 32):
    us = timeit(lambda: ph.gemm(A[:m], B, C[:m], precision=1))
    full = full or us
    print(f"tile-mode m={m:3d} live blocks={(m + 31) // 32}: {us:8.1f} us  ({us / full:.3f} of full, "
          f"{us / 128:.3f} us per K step)", flush=True)
