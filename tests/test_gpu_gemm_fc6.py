"""fp32-faithfulness of the default pose-head GEMM (precision 2: exact
three-way split-bf16 x6 MFMA) on the real fc6 / fc7 shapes of the configs[2]
step (vgg16_convs.py:186-192, network.py:393-423): R = 405 RoI rows of a
1152-row capacity (device-side row count), fc6 25088 -> 4096, fc7 4096 ->
4096, forward, data gradient and weight gradient.

The reference computes these layers as fp32 matmuls.  Each result is checked
against an fp64 GEMM of the same operands (torch on the GPU) two ways:
  * the precision-0 tolerance, rtol 2e-5 (atol 2e-5 of the result's scale);
  * as accurate as an fp32 GEMM: its max / mean absolute error against fp64
    at most 2x that of torch's own fp32 matmul of the same operands (the
    split-bf16 x3 path, ~2^-16 per product, fails this by an order of
    magnitude; printed for contrast).
Operand scales are the step's: pooled features ~N(0, 1), weights
N(0, 0.001^2) (network.py:415), data gradients from the ADD loss."""
import pytest
import torch

from posecnn_amd import pose_head as ph

pytestmark = pytest.mark.gpu
D = torch.device("cuda")
R, CAP, K6, U = 405, 1152, 25088, 4096


def _errs(C, ref):
    e = (C.double() - ref).abs()
    return float(e.max()), float(e.mean())


def _check(name, C, ref, c32):
    scale = float(ref.abs().max())
    emax, emean = _errs(C, ref)
    fmax, fmean = _errs(c32, ref)
    print(f"{name}: x6 max/mean err {emax:.3e}/{emean:.3e}  fp32 torch {fmax:.3e}/{fmean:.3e}  scale {scale:.3e}")
    assert emax <= 2 * fmax and emean <= 2 * fmean, name
    ok = (C.double() - ref).abs() <= 2e-5 * ref.abs() + 2e-5 * scale
    assert bool(ok.all()), f"{name}: {int((~ok).sum())} elements outside rtol 2e-5"


def _x3_err(fn, ref):
    C = fn(1)
    return _errs(C, ref)


@pytest.fixture(scope="module")
def ops():
    g = torch.Generator(device=D)
    g.manual_seed(17)
    x = torch.randn((CAP, K6), generator=g, device=D)
    w6 = torch.randn((K6, U), generator=g, device=D) * 1e-3
    w7 = torch.randn((U, U), generator=g, device=D) * 1e-3
    b6 = torch.randn((U,), generator=g, device=D) * 1e-3
    dy = torch.randn((CAP, U), generator=g, device=D) * 1e-4
    nr = torch.tensor([R], dtype=torch.int32, device=D)
    torch.backends.cuda.matmul.allow_tf32 = False
    return dict(x=x, w6=w6, w7=w7, b6=b6, dy=dy, nr=nr)


def test_fc6_forward(hip, ops):
    x, w6, b6, nr = ops["x"], ops["w6"], ops["b6"], ops["nr"]

    def run(prec):
        C = torch.zeros((CAP, U), device=D)
        ph.gemm(x, w6, C, bias=b6, M_dev=nr, precision=prec)
        return C[:R]
    C = run(2)
    ref = x[:R].double() @ w6.double() + b6.double()
    c32 = x[:R] @ w6 + b6
    _check("fc6 fwd", C, ref, c32)
    print("fc6 fwd x3 max/mean err %.3e/%.3e" % _x3_err(run, ref))


def test_fc6_data_grad(hip, ops):
    dy, w6, nr = ops["dy"], ops["w6"], ops["nr"]

    def run(prec):
        C = torch.zeros((CAP, K6), device=D)
        ph.gemm(dy, w6, C, b_trans=1, M_dev=nr, precision=prec)
        return C[:R]
    C = run(2)
    ref = dy[:R].double() @ w6.double().T
    c32 = dy[:R] @ w6.T
    _check("fc6 dX", C, ref, c32)
    print("fc6 dX x3 max/mean err %.3e/%.3e" % _x3_err(run, ref))


def test_fc6_weight_grad(hip, ops):
    x, dy, nr = ops["x"], ops["dy"], ops["nr"]

    def run(prec):
        C = torch.empty((K6, U), device=D)
        ph.gemm(x, dy, C, a_trans=1, K_dev=nr, M=K6, N=U, K=CAP, precision=prec)
        return C
    C = run(2)
    ref = x[:R].double().T @ dy[:R].double()
    c32 = x[:R].T @ dy[:R]
    _check("fc6 dW", C, ref, c32)
    del C
    print("fc6 dW x3 max/mean err %.3e/%.3e" % _x3_err(run, ref))


def test_fc7_forward_relu(hip, ops):
    x, w7, nr = ops["x"], ops["w7"], ops["nr"]
    y6 = torch.relu(x[:, :U] * 0.05)
    C = torch.zeros((CAP, U), device=D)
    ph.gemm(y6, w7, C, act=1, M_dev=nr, precision=2)
    ref = torch.relu(y6[:R].double() @ w7.double())
    c32 = torch.relu(y6[:R] @ w7)
    _check("fc7 fwd", C[:R], ref, c32)
    assert not C[R:].any()


def test_x6_edge_semantics(hip):
    """x6's stated operand range: finite |x| <= 3.3895314e38 (the largest
    bf16, 0x7F7F) -- there it tracks fp32 (values up to 1e38 here).  A larger
    finite fp32 rounds its hi plane to inf, and an inf / NaN operand makes its
    mid plane NaN: the output elements that operand reaches are NaN (fp32 gives
    +-inf for inf * finite, a finite value for the near-FLT_MAX case), and every
    other element is unaffected (a row of A reaches only its own output row)."""
    g = torch.Generator(device=D)
    g.manual_seed(3)
    M, K, N = 64, 256, 128
    A = torch.randn((M, K), generator=g, device=D)
    B = torch.randn((K, N), generator=g, device=D) * 1e-3
    A[1, 5] = 1e38                      # in range: finite, fp32-faithful
    A[2, 7] = float("inf")
    A[3, 9] = float("nan")
    A[4, 11] = 3.4e38                   # finite fp32, above the largest bf16
    C = torch.zeros((M, N), device=D)
    ph.gemm(A, B, C, precision=2)
    ref = A.double() @ B.double()
    fin = torch.ones(M, dtype=torch.bool, device=D)
    fin[2:5] = False
    ok = (C[fin].double() - ref[fin]).abs() <= 2e-5 * ref[fin].abs() + 2e-5 * ref[fin].abs().max()
    assert bool(ok.all())
    assert torch.isfinite(C[1]).all() and abs(float(C[1, 0]) / float(ref[1, 0]) - 1) < 1e-6
    for r in (2, 3, 4):
        assert bool(torch.isnan(C[r]).all()), r
    assert bool(torch.isfinite((A[4:5] @ B)).all())  # the fp32 matmul stays finite there
