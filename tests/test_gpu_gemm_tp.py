"""The x6 GEMM on pre-split tiled planes (csrc/gemm_tp.hip): the planes are
the exact three-way split, and the product is bit-identical to the staged x6
kernel (pcnn_gemm precision 2) on the same fp32 operands -- same plan, same
MFMA order -- on the fc6 / fc7 weight-gradient shapes of the step (device-side
K = R rows of a 1152 capacity) and on forward-style shapes (device-side M,
split-K slabs, bias / relu / dropout epilogues)."""
import numpy as np
import pytest
import torch

from posecnn_amd import pose_head as ph

pytestmark = pytest.mark.gpu
D = torch.device("cuda")
CAP = 1152


def _tp(src, rows, K, rs, ks, rows_dev=None, K_dev=None):
    out = torch.full((ph.tp_bytes(rows, K),), 0xAB, dtype=torch.uint8, device=D)
    return ph.split_tp(src, rows, K, out, rs, ks, rows_dev=rows_dev, K_dev=K_dev)


def test_planes_are_the_exact_split(hip):
    g = torch.Generator(device=D).manual_seed(1)
    X = torch.randn((70, 40), generator=g, device=D)  # rows 70 (3 row blocks), K 40 (3 k steps)
    tp = _tp(X, 70, 40, 40, 1).cpu().numpy().view(np.uint16).reshape(3, 3, 3, 64, 8)  # rb, ks, plane, lane, 8
    x = X.cpu().numpy()
    f = lambda h: (h.astype(np.uint32) << 16).view(np.float32)  # noqa: E731
    for rb in range(3):
        for ks in range(3):
            for lane in range(64):
                row, k0 = rb * 32 + (lane & 31), ks * 16 + 8 * (lane >> 5)
                hi, mid, lo = (f(tp[rb, ks, p, lane]) for p in range(3))
                want = np.array([x[row, k] if row < 70 and k < 40 else 0.0 for k in range(k0, k0 + 8)], np.float32)
                np.testing.assert_array_equal((hi.astype(np.float64) + mid + lo).astype(np.float32), want)
                assert np.all(np.abs(mid) <= np.abs(hi) * 2.0 ** -8) and np.all(np.abs(lo) <= np.abs(hi) * 2.0 ** -16)


@pytest.mark.parametrize("R,K6", [(405, 25088), (1152, 4096), (37, 4096)])
def test_weight_grad_bit_identical(hip, R, K6):
    """dW = X^T dY with X (CAP, K6), dY (CAP, 4096), K = R rows on the device."""
    g = torch.Generator(device=D).manual_seed(R)
    U = 4096
    X = torch.randn((CAP, K6), generator=g, device=D)
    dY = torch.randn((CAP, U), generator=g, device=D) * 1e-3
    nr = torch.tensor([R], dtype=torch.int32, device=D)
    ref = torch.empty((K6, U), device=D)
    ph.gemm(X, dY, ref, a_trans=1, K_dev=nr, M=K6, N=U, K=CAP, precision=2)
    At = _tp(X, K6, CAP, 1, K6, K_dev=nr)     # rows = features, k = RoI rows
    Bt = _tp(dY, U, CAP, 1, U, K_dev=nr)
    C = torch.full((K6, U), 7.0, device=D)
    ph.gemm_tp(At, Bt, C, K6, U, CAP, K_dev=nr)
    assert torch.equal(C, ref)


@pytest.mark.parametrize("M,N,K,mdev", [(405, 4096, 4096, 405), (1152, 512, 96, 0), (77, 300, 1000, 77)])
def test_forward_shapes_bit_identical(hip, M, N, K, mdev):
    g = torch.Generator(device=D).manual_seed(M + N)
    A = torch.randn((CAP if mdev else M, K), generator=g, device=D)
    W = torch.randn((K, N), generator=g, device=D) * 0.03
    b = torch.randn((N,), generator=g, device=D) * 0.1
    Md = torch.tensor([mdev], dtype=torch.int32, device=D) if mdev else None
    rows = A.shape[0]
    drop = (torch.rand((rows, N), generator=g, device=D) < 0.5).to(torch.uint8)
    ref = torch.zeros((rows, N), device=D)
    ph.gemm(A, W, ref, bias=b, act=1, M_dev=Md, precision=2, drop=drop, keep_prob=0.5)
    At = _tp(A, rows, K, K, 1, rows_dev=Md)   # op(A) rows x K
    Bt = _tp(W, N, K, 1, N)                   # op(B)^T: rows = N, k stride N
    C = torch.zeros((rows, N), device=D)
    ph.gemm_tp(At, Bt, C, rows, N, K, bias=b, act=1, M_dev=Md, drop=drop, keep_prob=0.5)
    m = mdev or M
    assert torch.equal(C[:m], ref[:m])
