"""The completion-event hook of the C-ABI (pcnn_set_completion_event): the op's
last kernel records the armed event through its own completion signal, so a
second stream forked on that event sees the op's output; an op without the
hook leaves the event pending, and pcnn_completion_event_pending reports and
clears it (the pose step then falls back to an event-record marker)."""
import pytest
import torch

from posecnn_amd import _lib
from posecnn_amd import pose_head as ph

pytestmark = pytest.mark.gpu
D = torch.device("cuda")


def _event():
    ev = torch.cuda.Event()
    ev.record()  # created (torch waits only on created events)
    torch.cuda.synchronize()
    return ev


@pytest.mark.parametrize("M,N,K", [(405, 4096, 4096), (405, 88, 4096), (300, 512, 1024)])
def test_gemm_last_kernel_records_the_event(hip, M, N, K):
    """The forked stream reads C only behind the event; the copy it makes is
    the finished product (split-K shapes: the reduce records it)."""
    lib = _lib.load()
    g = torch.Generator(device=D).manual_seed(3)
    A = torch.randn((M, K), generator=g, device=D)
    B = torch.randn((K, N), generator=g, device=D) * 1e-2
    C = torch.zeros((M, N), device=D)
    md = torch.tensor([M], dtype=torch.int32, device=D)
    ref = ph.gemm(A, B, torch.empty_like(C), M_dev=md)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    for _ in range(3):
        C.zero_()
        ev = _event()
        lib.pcnn_set_completion_event(ev.cuda_event)
        ph.gemm(A, B, C, M_dev=md)
        assert lib.pcnn_completion_event_pending() == 0  # taken by the op's last launch
        side.wait_event(ev)
        with torch.cuda.stream(side):
            got = C.clone()
        torch.cuda.synchronize()
        assert torch.equal(got, ref)


def test_op_without_hook_leaves_the_event_pending(hip):
    lib = _lib.load()
    y8 = torch.randn((16, 88), device=D)
    w = torch.ones((16, 88), device=D)
    t8, pred = torch.empty_like(y8), torch.empty_like(y8)
    ev = _event()
    lib.pcnn_set_completion_event(ev.cuda_event)
    ph.head_fwd(y8, w, t8, pred)
    assert lib.pcnn_completion_event_pending() == 1
    assert lib.pcnn_completion_event_pending() == 0  # cleared by the first query
    torch.cuda.synchronize()
