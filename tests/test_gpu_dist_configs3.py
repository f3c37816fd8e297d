"""BASELINE.json configs[3] at its real per-rank geometry: global batch 64
sharded 8 ways (8 frames of 640x480 per rank, index_size = 128 / 64 = 2,
hough_voting_gpu_op.cu.cc:734), 512-channel conv4_3 / conv5_3, 4096-unit
fc6 / fc7, train mode -- against the single-device step over all 64 frames.

Train mode WITH drop6 / drop7 at keep_prob 0.5 (vgg16_convs.py:189,191;
train.py:421): every rank gets its own externally drawn keep masks
(PoseStep.set_drop_masks), and the single-device step gets their rank-major
concatenation, so both graphs drop the same units of the same RoI rows.

Checked per rank: the all-gathered RoI / pose rows the sharded step ends with
(PoseStep.detections, exchange.RoiExchange; bit-exact and rank-major, i.e.
the single-device row order of hough_voting_gpu_op.cc:369-377), the rank's
own box rows and pooled rows (bit-exact), the all-reduced ADD loss (global
normaliser), and against float64 on the rank's own fp32 layer inputs (2e-5
of the tensor's scale, the bar of test_gpu_step_full): its fc6 / fc7
activations with the dropout, its dX = dY6 W6^T, its row block of dW6 / dW7 /
dW8 and the full bias gradients; its dconv4_3 / dconv5_3 images are
bit-exact against the oracle's RoI-pool backward of its own dX and argmax.
Against the single-device step the activations and gradients can differ where
a ReLU mask decided on an activation within rounding of 0 flips between the
two runs' GEMMs (their split-K plans differ with M), so that comparison is a
coarse sanity bound only; the float64 checks are the parity bars.

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
KEEP = 0.5  # drop6 / drop7 keep_prob in training (train.py:421)
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


def _rank_masks(rank, rows):
    """drop6 / drop7 keep masks (rows, UNITS) of one rank, seeded per rank."""
    g = torch.Generator(device="cuda")
    g.manual_seed(700 + rank)
    return tuple((torch.rand((rows, UNITS), generator=g, device="cuda") < KEEP).to(torch.uint8) for _ in range(2))


def _run(fr, batch_base, d, masks):
    from posecnn_amd.pipeline import PoseStep
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    inputs = {k: t(fr[k]) for k in ("label", "vertex", "meta", "conv4", "conv5", "extents", "gt", "points",
                                     "symmetry")}
    nb = inputs["label"].shape[0]
    step = PoseStep(nb, H, W, C, dev, channels=CH, units=UNITS, is_train=1, skip_pixels=10,
                    global_batch=WORLD * B_RANK, batch_base=batch_base, dist=d, keep_prob=KEEP)
    m6, m7 = masks(step.drop6.shape[0]) if callable(masks) else masks
    step.set_drop_masks(m6, m7)
    for _ in range(2):  # the second step must not see stale rows of the first
        step.step(inputs)
    torch.cuda.synchronize()
    n = int(step.hough["num_rois"][0].item())
    u16 = lambda a: a[:n].cpu().numpy().view(np.uint16)  # noqa: E731  (pixel-index argmax, 0xFFFF empty)
    out = dict(n=np.array(n), box=step.hough["box"][:n].cpu().numpy(), pose=step.hough["pose"][:n].cpu().numpy(),
               pool=step.pool[:n].cpu().numpy(), loss=step.loss.cpu().numpy(),
               dconv4=step.dconv4.cpu().numpy(), dconv5=step.dconv5.cpu().numpy(),
               y6=step.y6[:n].cpu().numpy(), y7=step.y7[:n].cpu().numpy(), dy6=step.dy6[:n].cpu().numpy(),
               dy7=step.dy7[:n].cpu().numpy(), dy8=step.dy8[:n].cpu().numpy(), dx=step.dx[:n].cpu().numpy(),
               arg5=u16(step.arg5), arg4=u16(step.arg4), m6=m6[:n].cpu().numpy(), m7=m7[:n].cpu().numpy())
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
        o = _run(fr, rank * B_RANK, _HostStagedAsync(dist), lambda rows: _rank_masks(rank, rows))
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
def test_configs3_sharded_step_matches_single_device(hip, orc, tmp_path):
    from posecnn_amd.pipeline import CAP
    ctx = mp.spawn(_worker, args=(WORLD, _free_port(), str(tmp_path)), nprocs=WORLD, join=False)
    fr = _frames(0, WORLD * B_RANK)  # the single-device batch, synthesised while the ranks run
    while not ctx.join():
        pass
    ranks = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(WORLD)]
    # the single-device step drops the same units of the same rows: the ranks'
    # masks in rank-major (= global row) order
    dev = torch.device("cuda")
    gm = []
    for k in ("m6", "m7"):
        m = np.zeros((CAP, UNITS), np.uint8)
        cat_m = np.concatenate([o[k] for o in ranks])
        m[:cat_m.shape[0]] = cat_m
        gm.append(torch.from_numpy(m).to(dev))
    conv = [_features(r * B_RANK, B_RANK) for r in range(WORLD)]  # each rank's conv4_3 / conv5_3
    ref = _run(fr, 0, None, tuple(gm))
    del fr
    n_ref = int(ref["n"])
    ref_rows = np.concatenate([ref["box"], ref["pose"]], 1)
    # the layer inputs / output gradients of all ranks, rank-major (= the
    # global row order): the sharded weight gradient must be their product
    cat = lambda k: torch.from_numpy(np.concatenate([o[k] for o in ranks])).to(dev).double()  # noqa: E731
    XdY = {"w6": (cat("pool").reshape(n_ref, -1), cat("dy6")), "w7": (cat("y6"), cat("dy7")),
           "w8": (cat("y7"), cat("dy8"))}
    from posecnn_amd import pose_head as ph
    wts = ph.PoseHeadWeights(C, dev, in_dim=49 * CH, units=UNITS)  # the step's weights (fixed seed)
    W6, W7 = wts.w6.double(), wts.w7.double()
    scale_close = lambda got, want: np.testing.assert_allclose(  # noqa: E731
        got, want, rtol=2e-5, atol=2e-5 * max(np.abs(want).max(), 1e-30))
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
        np.testing.assert_allclose(o["loss"], ref["loss"], rtol=1e-5)  # all-reduced, global normaliser
        # the forward layers with the dropout, against float64 on the rank's own inputs
        x = torch.from_numpy(o["pool"].reshape(n, -1)).to(dev).double()
        d6 = torch.from_numpy(o["m6"]).to(dev).double()
        d7 = torch.from_numpy(o["m7"]).to(dev).double()
        assert 0.4 < float(d6.mean()) < 0.6 and 0.4 < float(d7.mean()) < 0.6  # dropout is really on
        y6_64 = torch.relu(x @ W6) / KEEP * d6  # tf.nn.dropout (network.py:574-577), zero biases
        scale_close(o["y6"], y6_64.cpu().numpy())
        y6 = torch.from_numpy(o["y6"]).to(dev).double()
        scale_close(o["y7"], (torch.relu(y6 @ W7) / KEEP * d7).cpu().numpy())
        # the data-gradient chain: dX = dY6 W6^T against float64, then both RoI-pool
        # backwards bit-exact against the oracle on the rank's own dX and argmax
        dx64 = torch.from_numpy(o["dy6"]).to(dev).double() @ W6.T
        scale_close(o["dx"], dx64.cpu().numpy())
        del x, y6_64, dx64
        c4, c5 = conv[r]
        box_local = o["box"].copy()
        box_local[:, 0] -= r * B_RANK  # the rank's own feature maps (batch column rebased)
        dx = o["dx"].reshape(n, 7, 7, CH)
        for arg, data, k, s_ in ((o["arg5"], c5, "dconv5", 1.0 / 16), (o["arg4"], c4, "dconv4", 1.0 / 8)):
            a = arg.astype(np.int64)
            a = np.where(a == 0xFFFF, -1, a * CH + np.arange(CH)).astype(np.int32)
            want = orc.roi_pool_bwd(dx, a, data.shape, box_local, 7, 7, s_, 0)
            np.testing.assert_array_equal(o[k], want)
            assert np.abs(o[k]).sum() > 0
            # and the single-device step's images of this rank, up to those mask flips
            img = slice(r * B_RANK, (r + 1) * B_RANK)
            assert np.abs(o[k] - ref[k][img]).max() <= 0.02 * np.abs(ref[k][img]).max()
        # this rank's row block of each weight gradient (GradShard: all-to-all of
        # the inputs' column blocks + all-gather of dY) against float64
        # X_all[:, rows_r]^T dY_all of every rank's own rows
        for k in ("w6", "w7", "w8"):
            X, dY = XdY[k]
            blk = X.shape[1] // WORLD
            want = (X[:, r * blk:(r + 1) * blk].T @ dY).cpu().numpy()
            assert o["g_" + k].shape == want.shape
            scale_close(o["g_" + k], want)
            # and the single-device step's block, up to those mask flips (a coarse bound)
            ref_blk = ref["g_" + k][r * blk:(r + 1) * blk]
            assert np.abs(o["g_" + k] - ref_blk).max() <= 0.02 * np.abs(ref_blk).max()
        for k, dk in (("b6", "dy6"), ("b7", "dy7"), ("b8", "dy8")):
            want = cat(dk).sum(0).cpu().numpy()
            scale_close(o["g_" + k], want)
        off += n
    assert off == n_ref
