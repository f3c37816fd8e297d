"""Time the pose step's nine FC GEMMs (R RoI rows, fp32 in HBM) one by one
with HIP events; prints us and achieved TFLOP/s per shape.
    python scripts/gemm_bench.py [--rows 405] [--precision 2[,1,0,-1]] [--iters 20]
(precision -1: the weight gradients on pre-split tiled planes, csrc/gemm_tp.hip)"""
import argparse
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from posecnn_amd import pose_head as ph  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rows", type=int, default=405)
p.add_argument("--precision", default="2")
p.add_argument("--iters", type=int, default=20)
p.add_argument("--only", default="")
p.add_argument("--kc", action="store_true", help="also fc6 dW from k-contiguous (transposed) copies of X / dY")
a = p.parse_args()
D = torch.device("cuda")
CAP, K6, U, O = 1152, 25088, 4096, 88
g = torch.Generator(device=D).manual_seed(0)
r = lambda *s: torch.randn(*s, generator=g, device=D)
x5, x4, w6, w7, w8 = r(CAP, K6), r(CAP, K6), r(K6, U) * 1e-3, r(U, U) * 1e-3, r(U, O) * 1e-3
y6, y7, y8 = r(CAP, U), r(CAP, U), torch.empty(CAP, O, device=D)
dy8, dy7, dy6, dx = r(CAP, O), r(CAP, U), r(CAP, U), torch.empty(CAP, K6, device=D)
gw6, gw7, gw8 = torch.empty(K6, U, device=D), torch.empty(U, U, device=D), torch.empty(U, O, device=D)
nr = torch.tensor([a.rows], dtype=torch.int32, device=D)
R = a.rows


def cases_for(P):
    return [
        ("fc6_fwd", 2 * R * K6 * U, lambda: ph.gemm(x5, w6, y6, act=1, M_dev=nr, precision=P)),
        ("fc7_fwd", 2 * R * U * U, lambda: ph.gemm(y6, w7, y7, act=1, M_dev=nr, precision=P)),
        ("fc8_fwd", 2 * R * U * O, lambda: ph.gemm(y7, w8, y8, M_dev=nr, precision=P)),
        ("fc8_dw", 2 * R * U * O, lambda: ph.gemm(y7, dy8, gw8, a_trans=1, K_dev=nr, M=U, N=O, K=CAP, precision=P)),
        ("fc8_dx", 2 * R * U * O, lambda: ph.gemm(dy8, w8, dy7, b_trans=1, mask=y7, M_dev=nr, precision=P)),
        ("fc7_dw", 2 * R * U * U, lambda: ph.gemm(y6, dy7, gw7, a_trans=1, K_dev=nr, M=U, N=U, K=CAP, precision=P)),
        ("fc7_dx", 2 * R * U * U, lambda: ph.gemm(dy7, w7, dy6, b_trans=1, mask=y6, M_dev=nr, precision=P)),
        ("fc6_dw", 2 * R * K6 * U, lambda: ph.gemm(x5, dy6, gw6, a_trans=1, K_dev=nr, M=K6, N=U, K=CAP,
                                                   precision=P)),
        ("fc6_dx", 2 * R * K6 * U, lambda: ph.gemm(dy6, w6, dx, b_trans=1, M_dev=nr, precision=P)),
    ]


def kc_cases(P):
    """fc6 dW with one or both operands stored k-contiguous (the transposes timed on their own)."""
    x5t, dy6t = x5.t().contiguous(), dy6.t().contiguous()  # (K6, CAP), (U, CAP)
    return [
        ("tr_x5", 0, lambda: x5t.copy_(x5.t())),
        ("tr_dy6", 0, lambda: dy6t.copy_(dy6.t())),
        ("fc6_dw_akc", 2 * R * K6 * U, lambda: ph.gemm(x5t, dy6, gw6, K_dev=nr, M=K6, N=U, K=CAP, precision=P)),
        ("fc6_dw_bkc", 2 * R * K6 * U, lambda: ph.gemm(x5, dy6t, gw6, a_trans=1, b_trans=1, K_dev=nr, M=K6, N=U,
                                                       K=CAP, precision=P)),
        ("fc6_dw_kc", 2 * R * K6 * U, lambda: ph.gemm(x5t, dy6t, gw6, b_trans=1, K_dev=nr, M=K6, N=U, K=CAP,
                                                      precision=P)),
    ]


def tp_cases():
    """The fc6 / fc7 GEMMs on pre-split tiled planes (gemm_tp), the split
    producers timed on their own."""
    K6cap = CAP
    a6, b6 = [torch.empty(ph.tp_bytes(n, K6cap), dtype=torch.uint8, device=D) for n in (K6, U)]
    a7, b7 = [torch.empty(ph.tp_bytes(n, K6cap), dtype=torch.uint8, device=D) for n in (U, U)]
    for src, rows, out in ((x5, K6, a6), (dy6, U, b6), (y6, U, a7), (dy7, U, b7)):
        ph.split_tp(src, rows, CAP, out, 1, rows, K_dev=nr)
    # forward / dX shapes: op(B)^T of fc6 fwd is W6^T (4096 rows x K6), of fc6 dX W6 itself (K6 rows x 4096)
    ax, w6f, dyx, w6d = (torch.empty(ph.tp_bytes(n, k), dtype=torch.uint8, device=D)
                         for n, k in ((CAP, K6), (U, K6), (CAP, U), (K6, U)))
    ph.split_tp(x5, CAP, K6, ax, K6, 1, rows_dev=nr)
    ph.split_tp(w6, U, K6, w6f, 1, U)
    ph.split_tp(dy6, CAP, U, dyx, U, 1, rows_dev=nr)
    ph.split_tp(w6, K6, U, w6d, U, 1)
    return [
        ("split_w6", 0, lambda: ph.split_tp(w6, U, K6, w6f, 1, U)),
        ("fc6_fwd_tp", 2 * R * K6 * U, lambda: ph.gemm_tp(ax, w6f, y6, CAP, U, K6, act=1, M_dev=nr)),
        ("fc6_dx_tp", 2 * R * K6 * U, lambda: ph.gemm_tp(dyx, w6d, dx, CAP, K6, U, M_dev=nr)),
        ("split_x6T", 0, lambda: ph.split_tp(x5, K6, CAP, a6, 1, K6, K_dev=nr)),
        ("split_dy6T", 0, lambda: ph.split_tp(dy6, U, CAP, b6, 1, U, K_dev=nr)),
        ("fc6_dw_tp", 2 * R * K6 * U, lambda: ph.gemm_tp(a6, b6, gw6, K6, U, CAP, K_dev=nr)),
        ("fc7_dw_tp", 2 * R * U * U, lambda: ph.gemm_tp(a7, b7, gw7, U, U, CAP, K_dev=nr)),
    ]


for P in [int(v) for v in a.precision.split(",")]:
    print(f"precision {P}", flush=True)
    tot = 0.0
    for name, flops, fn in (cases_for(P) + (kc_cases(P) if a.kc else []) if P >= 0 else tp_cases()):
        if a.only and name not in a.only.split(","):
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        tot += us
        print(f"{name:10s} {us:9.1f} us  {flops / us / 1e6:8.1f} TFLOP/s", flush=True)
    print(f"total    {tot:9.1f} us", flush=True)
