"""Cross-rank RoI exchange for image-sharded runs.

Each rank votes on its own images (index_size = MAX_ROI / global batch, batch
column rebased to the global image index) into capacity-sized slots with a
device-side row count.  One all-gather of the padded slots and the counts,
then a device-side scatter compacts the live rows rank-major — the canonical
row order of a single-device run over the whole batch, because the reference
emits RoIs image by image (hough_voting_gpu_op.cc:369-377) and rank r holds
images [r*B, (r+1)*B).  No host sync: the compaction positions come from an
exclusive scan of the gathered counts, dead slots land on a trash row.

Backend-agnostic: "nccl" (RCCL over xGMI) for GPU tensors in production,
"gloo" for CPU tensors in the multi-process tests.
"""
import torch

ROW = 14  # box (7) + pose (7)


class RoiExchange:
    def __init__(self, dist, cap, device):
        self.dist = dist
        self.ws = dist.get_world_size()
        self.cap = cap
        f32 = dict(dtype=torch.float32, device=device)
        i32 = dict(dtype=torch.int32, device=device)
        self.l_rows = torch.zeros((cap, ROW), **f32)
        self.g_rows = torch.zeros((self.ws * cap, ROW), **f32)
        self.g_counts = torch.zeros((self.ws * 2,), **i32)
        # compacted global rows (+1 trash row for dead slots) and the live total
        self.rows = torch.zeros((self.ws * cap + 1, ROW), **f32)
        self.total = torch.zeros((1,), **i32)
        idx = torch.arange(self.ws * cap, device=device)
        self._rank = idx // cap
        self._local = (idx % cap).to(torch.int32)

    def __call__(self, box, pose, num_rois):
        """box (cap,7), pose (cap,7), num_rois (2,) int32 [rows, max(rows,1)].
        Returns (rows (ws*cap, 14) with the global rows first, total (1,) int32)."""
        d = self.dist
        self.l_rows[:, :7].copy_(box)
        self.l_rows[:, 7:].copy_(pose)
        d.all_gather_into_tensor(self.g_counts, num_rois)
        d.all_gather_into_tensor(self.g_rows, self.l_rows)
        counts = self.g_counts.view(self.ws, 2)[:, 0]
        offs = torch.cumsum(counts, 0, dtype=torch.int32) - counts  # exclusive scan
        live = self._local < counts[self._rank]
        pos = torch.where(live, offs[self._rank] + self._local,
                          torch.full_like(self._local, self.ws * self.cap)).long()
        self.rows.zero_()
        self.rows.index_copy_(0, pos, self.g_rows)  # duplicates only on the trash row
        self.total.copy_(counts.sum(dtype=torch.int32).view(1))
        return self.rows[:-1], self.total
