"""BASELINE.json configs[3] at its real per-rank geometry: global batch 64
sharded 8 ways (8 frames of 640x480 per rank, index_size = 128 / 64 = 2,
hough_voting_gpu_op.cu.cc:734), 512-channel conv4_3 / conv5_3, 4096-unit
fc6 / fc7, train mode -- against the single-device step over all 64 frames.

Checked per rank: the all-gathered RoI / pose rows the sharded step ends with
(PoseStep.detections, exchange.RoiExchange; bit-exact and rank-major, i.e.
the single-device row order of hough_voting_gpu_op.cc:369-377), the rank's
own box rows and pooled rows (bit-exact), the all-reduced ADD loss (global
normaliser), its dconv4_3 / dconv5_3 images, its row block of dW6 / dW7 /
dW8 and the full bias gradients.

The box has one GPU and RCCL wants one GPU per rank, so the eight ranks share
cuda:0 and exchange over gloo through host copies with real async handles
(test_gpu_dist._HostStagedAsync); only RCCL's transport itself is not
exercised here.  Every rank synthesises only its own frames (seeded per
global image index, synth.make_frames), the parent the whole batch while the
ranks run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_gpu_dist import _HostStagedAsync

WORLD, B_RANK, H, W, C, CH, UNITS = 8, 8, 480, 640, 22, 512, 4096
SEED = 3  # configs[2]/[3] frames (bench.py)
pytestmark = pytest.mark.gpu


def _features(b0, nb):
    """conv4_3 / conv5_3 for global images [b0, b0 + nb), seeded per image."""
    c4 = np.empty((nb, H // 8, W // 8, CH), np.float32)
    c5 = np.empty((nb, H // 16, W // 16, CH), np.float32)
    for i in range(nb):
        rng = np.random.default_rng(9000 + b0 + i)
        c4[i] = rng.standard_normal(c4.shape[1:], dtype=np.float32)
        c5[i] = rng.standard_normal(c5.shape[1:], dtype=np.float32)
    return c4, c5


def _frames(b0, nb):
    from posecnn_amd import synth
    fr = synth.make_frames(nb, H, W, num_classes=C, objects_per_image=6, seed=SEED, image_offset=b0)
    fr["conv4"], fr["conv5"] = _features(b0, nb)
    fr["points"], fr["symmetry"] = synth.rescaled_points(C)
    return fr


def _run(fr, batch_base, d):
    from posecnn_amd.pipeline import PoseStep
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    inputs = {k: t(fr[k]) for k in ("label", "vertex", "meta", "conv4", "conv5", "extents", "gt", "points",
                                     "symmetry")}
    nb = inputs["label"].shape[0]
    step = PoseStep(nb, H, W, C, dev, channels=CH, units=UNITS, is_train=1, skip_pixels=10,
                    global_batch=WORLD * B_RANK, batch_base=batch_base, dist=d, keep_prob=1.0)
    for _ in range(2):  # the second step must not see stale rows of the first
        step.step(inputs)
    torch.cuda.synchronize()
    n = int(step.hough["num_rois"][0].item())
    out = dict(n=np.array(n), box=step.hough["box"][:n].cpu().numpy(), pose=step.hough["pose"][:n].cpu().numpy(),
               pool=step.pool[:n].cpu().numpy(), loss=step.loss.cpu().numpy(),
               dconv4=step.dconv4.cpu().numpy(), dconv5=step.dconv5.cpu().numpy(),
               y6=step.y6[:n].cpu().numpy(), y7=step.y7[:n].cpu().numpy(), dy6=step.dy6[:n].cpu().numpy(),
               dy7=step.dy7[:n].cpu().numpy(), dy8=step.dy8[:n].cpu().numpy())
    if step.detections is not None:
        rows, total = step.detections
        tot = int(total.item())
        out["g_total"] = np.array(tot)
        out["g_rows"] = rows[:tot].cpu().numpy()
        out["g_tail"] = np.array(float(rows[tot:].abs().sum().item()))
    for k, v in step.grads.items():
        out["g_" + k] = v.cpu().numpy()
    del step
    torch.cuda.empty_cache()
    return out


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fr = _frames(rank * B_RANK, B_RANK)
        o = _run(fr, rank * B_RANK, _HostStagedAsync(dist))
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


@pytest.mark.timeout(600)
def test_configs3_sharded_step_matches_single_device(hip, tmp_path):
    ctx = mp.spawn(_worker, args=(WORLD, _free_port(), str(tmp_path)), nprocs=WORLD, join=False)
    fr = _frames(0, WORLD * B_RANK)  # the single-device batch, synthesised while the ranks run
    while not ctx.join():
        pass
    ref = _run(fr, 0, None)
    del fr
    n_ref = int(ref["n"])
    ref_rows = np.concatenate([ref["box"], ref["pose"]], 1)
    ranks = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(WORLD)]
    # the layer inputs / output gradients of all ranks, rank-major (= the
    # global row order): the sharded weight gradient must be their product
    dev = torch.device("cuda")
    cat = lambda k: torch.from_numpy(np.concatenate([o[k] for o in ranks])).to(dev).double()  # noqa: E731
    XdY = {"w6": (cat("pool").reshape(n_ref, -1), cat("dy6")), "w7": (cat("y6"), cat("dy7")),
           "w8": (cat("y7"), cat("dy8"))}
    off = 0
    for r in range(WORLD):
        o = ranks[r]
        n = int(o["n"])
        assert n > 0
        sl = slice(off, off + n)
        # the RoI / pose all-gather inside the sharded step: every rank ends
        # with the single-device rows, in the single-device order
        assert int(o["g_total"]) == n_ref
        np.testing.assert_array_equal(o["g_rows"], ref_rows)
        assert float(o["g_tail"]) == 0.0
        np.testing.assert_array_equal(o["box"], ref["box"][sl])   # global batch column, index_size 2
        np.testing.assert_array_equal(o["pose"], ref["pose"][sl])
        np.testing.assert_array_equal(o["pool"], ref["pool"][sl])  # pooled from the rank's own maps
        assert np.abs(o["pool"]).sum() > 0
        img = slice(r * B_RANK, (r + 1) * B_RANK)
        for k in ("dconv4", "dconv5"):
            # the rank's feature-map gradients are its own images' (a wrong image
            # offset or RoI rebase would be off by O(1)); they match the
            # single-device step up to the ReLU-mask flips of its activations
            # (the exact chain dY -> dX -> RoI-pool backward is test_gpu_step_full's)
            np.testing.assert_allclose(o[k], ref[k][img], rtol=1e-3, atol=1e-3 * np.abs(ref[k]).max())
            assert np.abs(o[k]).sum() > 0
        np.testing.assert_allclose(o["loss"], ref["loss"], rtol=1e-5)  # all-reduced, global normaliser
        # this rank's row block of each weight gradient (GradShard: all-to-all of
        # the inputs' column blocks + all-gather of dY) against float64
        # X_all[:, rows_r]^T dY_all of every rank's own rows.  (Against the
        # single-device step the products differ where a ReLU mask decided on an
        # activation within rounding of 0 flips between the two runs' GEMMs.)
        for k in ("w6", "w7", "w8"):
            X, dY = XdY[k]
            blk = X.shape[1] // WORLD
            want = (X[:, r * blk:(r + 1) * blk].T @ dY).cpu().numpy()
            assert o["g_" + k].shape == want.shape
            np.testing.assert_allclose(o["g_" + k], want, rtol=2e-5, atol=2e-5 * np.abs(want).max())
            # and the single-device step's block, up to those mask flips
            ref_blk = ref["g_" + k][r * blk:(r + 1) * blk]
            assert np.abs(o["g_" + k] - ref_blk).max() <= 0.02 * np.abs(ref_blk).max()
        for k, dk in (("b6", "dy6"), ("b7", "dy7"), ("b8", "dy8")):
            want = cat(dk).sum(0).cpu().numpy()
            np.testing.assert_allclose(o["g_" + k], want, rtol=2e-5, atol=2e-5 * np.abs(want).max())
        off += n
    assert off == n_ref
