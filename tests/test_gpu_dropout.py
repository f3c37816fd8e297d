"""drop6 / drop7 of the pose head on the GPU (csrc/dropout.hip and the
dropout epilogue of k_gemm_reduce):
  * Philox4x32-10 against the Random123 known answers, the keep-mask kernel
    bit-exact against oracle/philox.py (device row count, step counter,
    stream ids, a graph replay drawing a fresh mask);
  * pcnn_gemm_drop at every precision on split-K and whole-tile shapes,
    forward ((relu(v + b) / keep) * mask, tf.nn.dropout) and backward
    (mask > 0 ? v / keep : 0) against float64."""
import numpy as np
import pytest
import torch

from oracle import philox
from posecnn_amd import _lib
from posecnn_amd import pose_head as ph
from test_dropout_oracle import KAT

pytestmark = pytest.mark.gpu
D = torch.device("cuda")


def test_philox_kernel_known_answers(hip):
    # uint32 words carried in int32 tensors (bit views)
    bits = lambda a: torch.from_numpy(np.array(a, np.uint32).view(np.int32)).to(D)
    ctr, key = bits([c for c, _, _ in KAT]), bits([k for _, k, _ in KAT])
    out = torch.zeros((len(KAT), 4), dtype=torch.int32, device=D)
    _lib.check(hip.pcnn_philox_check(_lib.ptr(ctr), _lib.ptr(key), len(KAT), _lib.ptr(out), _lib.stream_ptr()),
               "philox")
    want = np.array([w for _, _, w in KAT], np.uint32)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)


def test_dropout_mask_matches_oracle(hip):
    rows, cols, seed = 1152, 4096, 0x5EED + (3 << 40)
    m = torch.full((rows, cols), 7, dtype=torch.uint8, device=D)
    step = torch.tensor([5], dtype=torch.int64, device=D)
    nr = torch.tensor([405], dtype=torch.int32, device=D)
    ph.dropout_mask(m, 0.5, seed, step, 6, rows_dev=nr)
    torch.cuda.synchronize()
    want = philox.dropout_mask(405, cols, seed, 5, 6, 0.5)
    np.testing.assert_array_equal(m[:405].cpu().numpy(), want)
    assert bool((m[405:] == 7).all())  # rows past the device count untouched
    # keep 0.75, a pitch wider than the columns, no device count
    m2 = torch.zeros((64, 520), dtype=torch.uint8, device=D)
    ph.dropout_mask(m2[:, :512], 0.75, 99, step, 2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m2[:, :512].cpu().numpy(), philox.dropout_mask(64, 512, 99, 5, 2, 0.75))
    assert not bool(m2[:, 512:].any())


def test_dropout_mask_graph_replay_draws_new_masks(hip):
    """The step counter lives on the device: replays of one captured graph
    draw the masks of consecutive steps."""
    m = torch.zeros((32, 256), dtype=torch.uint8, device=D)
    step = torch.zeros((1,), dtype=torch.int64, device=D)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside the capture
        ph.dropout_mask(m, 0.5, 1, step, 0)
        step.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ph.dropout_mask(m, 0.5, 1, step, 0)
        step.add_(1)
    torch.cuda.synchronize()
    step.zero_()
    seen = []
    for i in range(3):
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(m.cpu().numpy(), philox.dropout_mask(32, 256, 1, i, 0, 0.5))
        seen.append(m.cpu().numpy().copy())
    assert not np.array_equal(seen[0], seen[1])


@pytest.mark.parametrize("precision", [2, 1, 0])
@pytest.mark.parametrize("shape", [(405, 4096, 4096, True), (1152, 512, 96, False), (77, 300, 1000, True)])
def test_gemm_dropout_vs_fp64(hip, precision, shape):
    """shape = (M, N, K, device-side M): (405, 4096, 4096) is fc7's forward
    (split-K, dropout in the slab reduce); (1152, 512, 96) a static-M
    whole-tile shape (dropout as the in-place pass)."""
    M, N, K, mdev = shape
    g = torch.Generator(device=D)
    g.manual_seed(M + N + K + precision)
    A = torch.randn((M, K), generator=g, device=D)
    Bm = torch.randn((K, N), generator=g, device=D) * 0.05
    bias = torch.randn((N,), generator=g, device=D) * 0.1
    keep = 0.5 if M != 77 else 0.7
    drop = (torch.rand((M, N), generator=g, device=D) < keep).to(torch.uint8)
    C = torch.full((M, N), 3.0, device=D)
    Md = torch.tensor([M], dtype=torch.int32, device=D) if mdev else None
    ph.gemm(A, Bm, C, bias=bias, act=1, M_dev=Md, precision=precision, drop=drop, keep_prob=keep)
    ref = ((torch.relu(A.double() @ Bm.double() + bias.double()) / keep) * drop.double())
    tol = 1e-4 if precision == 1 else 2e-5
    err = (C.double() - ref).abs().max().item()
    assert err <= tol * ref.abs().max().item(), err
    assert bool((C[drop == 0] == 0).all())  # dropped elements are exact zeros
    # backward: dY_prev = mask > 0 ? (dY @ W^T) / keep : 0 with mask = the dropped activation
    dY = torch.randn((M, K), generator=g, device=D)
    dX = torch.full((M, N), 3.0, device=D)
    W_ = torch.randn((N, K), generator=g, device=D) * 0.05  # B stored (N, K): b_trans
    ph.gemm(dY, W_, dX, b_trans=1, mask=C, M_dev=Md, precision=precision, keep_prob=keep)
    refb = (dY.double() @ W_.double().T) / keep * (C > 0).double()
    err = (dX.double() - refb).abs().max().item()
    assert err <= tol * refb.abs().max().item(), err


def test_gemm_drop_rejects_bad_keep(hip):
    A = torch.zeros((4, 4), device=D)
    with pytest.raises(ValueError):
        ph.gemm(A, A, A.clone(), keep_prob=0.0)
    with pytest.raises(ValueError):
        ph.gemm(A, A, A.clone(), keep_prob=1.5)
    with pytest.raises(ValueError):
        ph.gemm(A, A, A.clone(), drop=torch.ones((4, 4), device=D), keep_prob=0.5)  # not uint8


@pytest.mark.parametrize("precision", [2, 0])
@pytest.mark.parametrize("shape", [(405, 4096, 4096, True), (1152, 512, 96, False), (77, 300, 1000, True)])
def test_gemm_drop_gen_matches_mask_kernel(hip, precision, shape):
    """pcnn_gemm_drop_gen (keep bits drawn in the reduce epilogue) against the
    mask kernel + pcnn_gemm_drop: the same output bit for bit and the same
    bits stored (oracle/philox.py), rows past the device-side M untouched --
    on the split-K float4 reduce (fc7's forward), the in-place whole-tile pass
    and the element-wise reduce (an output pitch that is not a multiple of 4)."""
    M, N, K, mdev = shape
    g = torch.Generator(device=D)
    g.manual_seed(M * 7 + N + K)
    A = torch.randn((M, K), generator=g, device=D)
    Bm = torch.randn((K, N), generator=g, device=D) * 0.05
    bias = torch.randn((N,), generator=g, device=D) * 0.1
    keep, seed, sid = 0.5, 0x5EED + (1 << 40), 6
    step = torch.tensor([9], dtype=torch.int64, device=D)
    m_eff = M - 3 if mdev else M
    Md = torch.tensor([m_eff], dtype=torch.int32, device=D) if mdev else None
    mask = torch.full((M, N), 7, dtype=torch.uint8, device=D)
    ph.dropout_mask(mask, keep, seed, step, sid, rows_dev=Md)
    pad = 1 if M == 77 else 0  # an output pitch that is not a multiple of 4: the element-wise reduce
    C_ref = torch.zeros((M, N + pad), device=D)[:, :N]
    ph.gemm(A, Bm, C_ref, bias=bias, act=1, M_dev=Md, precision=precision, drop=mask, keep_prob=keep)
    drop = torch.full((M, N), 7, dtype=torch.uint8, device=D)
    C = torch.zeros((M, N + pad), device=D)[:, :N]
    ph.gemm(A, Bm, C, bias=bias, act=1, M_dev=Md, precision=precision, drop=drop, keep_prob=keep,
            drop_gen=(seed, step, sid))
    torch.cuda.synchronize()
    assert torch.equal(C, C_ref)
    np.testing.assert_array_equal(drop[:m_eff].cpu().numpy(), philox.dropout_mask(m_eff, N, seed, 9, sid, keep))
    assert bool((drop[m_eff:] == 7).all())
    with pytest.raises(ValueError):
        ph.gemm(A, Bm, C, drop=drop, mask=C_ref, keep_prob=keep, drop_gen=(seed, step, sid))
