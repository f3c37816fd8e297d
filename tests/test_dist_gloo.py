"""Image sharding + RoI exchange on 2 CPU ranks (gloo): per-rank votes with
index_size = MAX_ROI / global batch and the batch column rebased to the global
image index, gathered and compacted by posecnn_amd.exchange.RoiExchange (the
same code that runs over RCCL on GPUs), reproduce a single-process run on the
whole batch row for row.  The per-rank votes come from the
oracle (test infrastructure) so the test needs no GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from posecnn_amd import synth

B_RANK, H, W, C = 2, 96, 128, 6
CAP = 128 * 9


def _frames(world):
    return synth.make_frames(B_RANK * world, H=H, W=W, num_classes=C, objects_per_image=3, seed=31)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, is_train):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as orc
    from posecnn_amd.exchange import RoiExchange
    fr = _frames(world)
    sl = slice(rank * B_RANK, (rank + 1) * B_RANK)
    box, pose, _, _, _, n = orc.hough_voting(fr["label"][sl], fr["vertex"][sl], fr["extents"], fr["meta"][sl],
                                             fr["gt"], is_train, -1.0, 0.02, 3, batch_base=rank * B_RANK,
                                             global_batch=B_RANK * world, exact_rows=False)
    x = RoiExchange(dist, CAP, torch.device("cpu"))
    rows, total = x(torch.from_numpy(box), torch.from_numpy(pose),
                    torch.tensor([n, max(n, 1)], dtype=torch.int32))
    if rank == 0:
        np.save(os.path.join(out_dir, "rows.npy"), rows.numpy())
        np.save(os.path.join(out_dir, "total.npy"), total.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("is_train", [0, 1])
def test_sharded_exchange_matches_single_device(orc, tmp_path, is_train):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), is_train), nprocs=world, join=True)
    rows = np.load(tmp_path / "rows.npy")
    total = int(np.load(tmp_path / "total.npy")[0])
    fr = _frames(world)
    box, pose, _, _, _, n = orc.hough_voting(fr["label"], fr["vertex"], fr["extents"], fr["meta"], fr["gt"],
                                             is_train, -1.0, 0.02, 3)
    assert total == n and n > 0
    np.testing.assert_array_equal(rows[:n, :7], box[:n])
    np.testing.assert_array_equal(rows[:n, 7:], pose[:n])
    assert not rows[n:].any()
    # rows are image-major with global batch indices
    assert (np.diff(rows[:n, 0]) >= 0).all() and rows[:n, 0].max() < world * B_RANK
