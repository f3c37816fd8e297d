"""Image-sharded pose step on 2 ranks vs the single-device step over the whole
batch: rank r's pooled RoI rows, its dconv4_3 / dconv5_3
images, the all-reduced loss and its row block of the fc6/fc7/fc8 weight
gradients (exchange.GradShard) must reproduce the single-device run.

The box has one GPU and RCCL wants one GPU per rank, so the two ranks share
cuda:0 and talk over gloo through host copies (_HostStaged, test-only); the
step code is the one that runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B_RANK, H, W, C, CH, UNITS = 2, 120, 160, 22, 64, 256
pytestmark = pytest.mark.gpu


class _Done:
    def wait(self):
        pass


class _HostStaged:
    """gloo collectives on host copies of device tensors (test-only)."""

    def __init__(self, d):
        self.d = d

    def get_world_size(self):
        return self.d.get_world_size()

    def get_rank(self):
        return self.d.get_rank()

    def _ret(self, async_op):
        torch.cuda.synchronize()
        return _Done() if async_op else None

    def all_reduce(self, t, async_op=False):
        h = t.cpu()
        self.d.all_reduce(h)
        t.copy_(h)
        return self._ret(async_op)

    def all_gather_into_tensor(self, out, inp, async_op=False):
        h = torch.empty(out.shape, dtype=out.dtype)
        self.d.all_gather_into_tensor(h, inp.cpu())
        out.copy_(h)
        return self._ret(async_op)

    def all_to_all_single(self, out, inp, async_op=False):
        h = torch.empty(out.shape, dtype=out.dtype)
        self.d.all_to_all_single(h, inp.contiguous().cpu())
        out.copy_(h)
        return self._ret(async_op)


class _Work:
    """Async handle of _HostStagedAsync: the gloo op runs on host copies; the
    device tensor receives the result only in wait(), as an H2D copy enqueued
    on the waiter's current stream -- a step that reads a collective's output
    before waiting on its handle reads stale data and fails the comparison."""

    def __init__(self, work, finish):
        self.work, self.finish = work, finish

    def wait(self):
        self.work.wait()
        self.finish()


class _HostStagedAsync(_HostStaged):
    """gloo collectives with real async work handles and no device-wide sync:
    the D2H copy of the input orders only against the current stream, the
    collective itself runs asynchronously, and the result lands at wait()."""

    def _go(self, fn, dst, h, async_op):
        work = fn()
        finish = lambda: dst.copy_(h, non_blocking=False)
        if not async_op:
            work.wait()
            finish()
            return None
        return _Work(work, finish)

    def all_reduce(self, t, async_op=False):
        h = t.cpu()
        return self._go(lambda: self.d.all_reduce(h, async_op=True), t, h, async_op)

    def all_gather_into_tensor(self, out, inp, async_op=False):
        h = torch.empty(out.shape, dtype=out.dtype)
        src = inp.cpu()
        return self._go(lambda: self.d.all_gather_into_tensor(h, src, async_op=True), out, h, async_op)

    def all_to_all_single(self, out, inp, async_op=False):
        h = torch.empty(out.shape, dtype=out.dtype)
        src = inp.contiguous().cpu()
        return self._go(lambda: self.d.all_to_all_single(h, src, async_op=True), out, h, async_op)


def _inputs(world, seed=77):
    from posecnn_amd import synth
    fr = synth.make_frames(B_RANK * world, H=H, W=W, num_classes=C, objects_per_image=4, seed=seed)
    g = torch.Generator().manual_seed(5 + seed - 77)
    fr["conv4"] = torch.randn((B_RANK * world, H // 8, W // 8, CH), generator=g).numpy()
    fr["conv5"] = torch.randn((B_RANK * world, H // 16, W // 16, CH), generator=g).numpy()
    fr["points"], fr["symmetry"] = synth.rescaled_points(C)
    return fr


def _run(fr, sl, global_batch, batch_base, d):
    from posecnn_amd.pipeline import PoseStep
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    inputs = {k: t(fr[k][sl]) for k in ("label", "vertex", "meta", "conv4", "conv5")}
    inputs.update(extents=t(fr["extents"]), gt=t(fr["gt"]), points=t(fr["points"]), symmetry=t(fr["symmetry"]))
    nb = inputs["label"].shape[0]
    step = PoseStep(nb, H, W, C, dev, channels=CH, units=UNITS, is_train=1, skip_pixels=3,
                    global_batch=global_batch, batch_base=batch_base, dist=d, keep_prob=1.0)
    for _ in range(2):  # second step: stale rows of the first must not leak into the gradients
        step.step(inputs)
    torch.cuda.synchronize()
    n = int(step.hough["num_rois"][0].item())
    out = dict(n=np.array(n), pool=step.pool[:n].cpu().numpy(), loss=step.loss.cpu().numpy(),
               dconv4=step.dconv4.cpu().numpy(), dconv5=step.dconv5.cpu().numpy(),
               box=step.hough["box"][:n].cpu().numpy())
    for k, v in step.grads.items():
        out["g_" + k] = v.cpu().numpy()
    return out


def _device_inputs(fr, sl):
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    inputs = {k: t(fr[k][sl]) for k in ("label", "vertex", "meta", "conv4", "conv5")}
    inputs.update(extents=t(fr["extents"]), gt=t(fr["gt"]), points=t(fr["points"]), symmetry=t(fr["symmetry"]))
    return inputs


def _run_pipelined(frs, sl, global_batch, batch_base, d, pipeline):
    """Three consecutive sharded steps over distinct minibatches; pipelined:
    each step is handed the next minibatch, whose vote and RoI-pool forward run
    on the prefetch stream beside the current step's collectives."""
    from posecnn_amd.pipeline import PoseStep
    batches = [_device_inputs(fr, sl) for fr in frs]
    step = PoseStep(B_RANK, H, W, C, torch.device("cuda", 0), channels=CH, units=UNITS, is_train=1, skip_pixels=3,
                    global_batch=global_batch, batch_base=batch_base, dist=d, keep_prob=1.0, pipeline=pipeline)
    out = {}
    for k, inp in enumerate(batches):
        if pipeline:
            step.step(inp, batches[k + 1] if k + 1 < len(batches) else None)
        else:
            step.step(inp)
        torch.cuda.synchronize()
        n = int(step.hough["num_rois"][0].item())
        out[f"n{k}"] = np.array(n)
        for name, v in (("pool", step.pool[:n]), ("loss", step.loss), ("dconv4", step.dconv4),
                        ("dconv5", step.dconv5), ("box", step.hough["box"][:n])):
            out[f"{name}{k}"] = v.cpu().numpy()
        for gk, v in step.grads.items():
            out[f"g_{gk}{k}"] = v.cpu().numpy()
    return out


def _worker(rank, world, port, out_dir, mode="sync"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wrap = _HostStagedAsync(dist) if mode in ("async", "pipelined") else _HostStaged(dist)
        sl = slice(rank * B_RANK, (rank + 1) * B_RANK)
        if mode == "pipelined":
            frs = [_inputs(world, 77 + k) for k in range(3)]
            ref = _run_pipelined(frs, sl, B_RANK * world, rank * B_RANK, wrap, False)
            o = _run_pipelined(frs, sl, B_RANK * world, rank * B_RANK, wrap, True)
            o.update({"ref_" + k: v for k, v in ref.items()})
        else:
            o = _run(_inputs(world), sl, B_RANK * world, rank * B_RANK, wrap)
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **o)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_sharded_step_matches_single_device(hip, tmp_path, mode):
    """mode "async": the collectives return real async handles whose results
    land only at wait(), so the step's wait placement (loss, rows, weight
    gradient shards, reused exchange buffers across two steps) is exercised;
    RCCL's own stream ordering stays unpinned until a multi-GPU run."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world, join=True)
    fr = _inputs(world)
    ref = _run(fr, slice(0, B_RANK * world), B_RANK * world, 0, None)
    ranks = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    n = [int(o["n"]) for o in ranks]
    assert sum(n) == int(ref["n"]) and min(n) > 0
    off = 0
    for r, o in enumerate(ranks):
        sl = slice(off, off + n[r])
        np.testing.assert_array_equal(o["box"], ref["box"][sl])       # global batch column
        np.testing.assert_array_equal(o["pool"], ref["pool"][sl])     # pooled from the rank's own maps
        assert np.abs(o["pool"]).sum() > 0
        img = slice(r * B_RANK, (r + 1) * B_RANK)
        for k in ("dconv4", "dconv5"):
            np.testing.assert_allclose(o[k], ref[k][img], rtol=1e-6, atol=1e-12)
            assert np.abs(o[k]).sum() > 0
        np.testing.assert_allclose(o["loss"], ref["loss"], rtol=1e-5)  # all-reduced, global normaliser
        for k in ("w6", "w7", "w8"):
            blk = ref["g_" + k].shape[0] // world
            want = ref["g_" + k][r * blk:(r + 1) * blk]
            assert o["g_" + k].shape == want.shape
            np.testing.assert_allclose(o["g_" + k], want, rtol=1e-4, atol=1e-4 * np.abs(want).max())
        for k in ("b6", "b7", "b8"):
            want = ref["g_" + k]
            np.testing.assert_allclose(o["g_" + k], want, rtol=1e-4, atol=1e-4 * np.abs(want).max())
        off += n[r]


def test_sharded_pipelined_steps_bit_identical(hip, tmp_path):
    """The bench's default N > 1 path: each rank's pipelined step (the next
    minibatch's vote and pool on the prefetch stream while this step's loss
    all-reduce, RoI row exchange and weight-gradient shards are in flight,
    async collective handles) over three distinct minibatches, bit for bit the
    unpipelined sharded step's outputs on the same rank."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), "pipelined"), nprocs=world, join=True)
    for r in range(world):
        o = dict(np.load(tmp_path / f"rank{r}.npz"))
        keys = [k for k in o if not k.startswith("ref_")]
        assert len({int(o[f"n{k}"]) for k in range(3)}) > 1 or not np.array_equal(o["box0"], o["box1"])
        for k in keys:
            np.testing.assert_array_equal(o[k], o["ref_" + k], err_msg=f"rank {r} {k}")
        assert all(int(o[f"n{k}"]) > 0 for k in range(3))
