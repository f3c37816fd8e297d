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
        self._pending = []

    def __call__(self, box, pose, num_rois):
        """box (cap,7), pose (cap,7), num_rois (2,) int32 [rows, max(rows,1)].
        Returns (rows (ws*cap, 14) with the global rows first, total (1,) int32)."""
        self.start(box, pose, num_rois)
        return self.finish()

    def start(self, box, pose, num_rois):
        """Issue the two all-gathers asynchronously (the pose step starts them
        right after the vote; they overlap the rest of the step)."""
        d = self.dist
        self.l_rows[:, :7].copy_(box)
        self.l_rows[:, 7:].copy_(pose)
        self._pending = [d.all_gather_into_tensor(self.g_counts, num_rois, async_op=True),
                         d.all_gather_into_tensor(self.g_rows, self.l_rows, async_op=True)]

    def finish(self):
        """Join the all-gathers and compact the live rows rank-major on the device.

        The returned tensors are views of this exchange's own buffers, valid
        until its next start() / gather(): a caller that keeps a step's rows
        clones them (PoseStep.step stores clones in `detections`)."""
        for w in self._pending:
            if w is not None:
                w.wait()
        self._pending = []
        counts = self.g_counts.view(self.ws, 2)[:, 0]
        offs = torch.cumsum(counts, 0, dtype=torch.int32) - counts  # exclusive scan
        live = self._local < counts[self._rank]
        pos = torch.where(live, offs[self._rank] + self._local,
                          torch.full_like(self._local, self.ws * self.cap)).long()
        self.rows.zero_()
        self.rows.index_copy_(0, pos, self.g_rows)  # duplicates only on the trash row
        self.total.copy_(counts.sum(dtype=torch.int32).view(1))
        return self.rows[:-1], self.total


class GradShard:
    """Data-parallel weight gradients of the pose head, owned by row block.

    Every fc layer's weight gradient is a sum over RoI rows, dW = X^T dY
    (network.py:393-423 backward), and an image-sharded step holds only its
    own rows.  The rows of all ranks together never exceed the op's capacity
    (MAX_ROI * 9 = 1152, hough_voting_gpu_op.cc:94), far below the layers'
    fan-in, so the factors are much smaller than the product: fc6's 411 MB dW
    against X (<= 1152 x 25088) and dY (<= 1152 x 4096).  Rank r owns rows
    [r*in/ws, (r+1)*in/ws) of each weight gradient (the ZeRO-2 split) and gets
    them as one local GEMM over every rank's rows:

        dW[rows_r] = X_all[:, rows_r]^T @ dY_all

    X_all[:, rows_r] arrives by one all-to-all of column blocks (each rank
    sends ws-1 blocks of slot x in/ws), dY_all by one all-gather.  At 8 ranks
    of 144 rows that is 50 MB received per rank for fc6 + fc7 + fc8, against
    the 837 MB per rank (2 (ws-1)/ws x 478 MB) of a ring all-reduce.  The X exchange of a layer starts
    as soon as its input exists in the forward and overlaps the rest of the
    step; only the dY gathers sit behind the backward chain.  Bias gradients
    (colsum of dY_all) are computed in full on every rank.

    Rows past a rank's live count are zeroed in dY before the gather, so the
    padded slot rows add exact zeros.  `gemm`/`colsum` are passed in: the step
    uses the HIP kernels (pose_head.gemm / colsum), the CPU gloo test a
    reference matmul.
    """

    def __init__(self, dist, slot, layers, device):
        self.dist = dist
        self.ws = dist.get_world_size()
        self.rank = dist.get_rank()
        self.slot = slot
        self.layers = dict(layers)  # name -> (in_dim, out_dim)
        f32 = dict(dtype=torch.float32, device=device)
        self.x_send, self.x_recv, self.dy_send, self.dy_all, self.pending = {}, {}, {}, {}, {}
        for name, (din, dout) in self.layers.items():
            if din % self.ws:
                raise ValueError(f"{name}: fan-in {din} does not split over {self.ws} ranks")
            blk = din // self.ws
            self.x_send[name] = torch.zeros((self.ws, slot, blk), **f32)
            self.x_recv[name] = torch.zeros((self.ws * slot, blk), **f32)
            self.dy_send[name] = torch.zeros((slot, dout), **f32)
            self.dy_all[name] = torch.zeros((self.ws * slot, dout), **f32)
        self.row_ids = torch.arange(slot, device=device, dtype=torch.int32).view(slot, 1)

    def rows(self, name):
        """This rank's row block of layer `name`'s weight gradient."""
        blk = self.layers[name][0] // self.ws
        return slice(self.rank * blk, (self.rank + 1) * blk)

    def send_input(self, name, X):
        """X (>= slot rows, in_dim): this rank's layer input; column block j goes to rank j."""
        blk = self.layers[name][0] // self.ws
        self.x_send[name].copy_(X[:self.slot].view(self.slot, self.ws, blk).transpose(0, 1))
        self.pending[name + ".x"] = self.dist.all_to_all_single(self.x_recv[name], self.x_send[name], async_op=True)

    def send_grad(self, name, dY, num_rows):
        """dY (>= slot rows, out_dim); rows >= num_rows (device int, shape (1,)) are sent as zeros."""
        live = self.row_ids < num_rows.view(1, 1)
        torch.where(live, dY[:self.slot], torch.zeros((), dtype=dY.dtype, device=dY.device), out=self.dy_send[name])
        self.pending[name + ".dy"] = self.dist.all_gather_into_tensor(self.dy_all[name], self.dy_send[name],
                                                                      async_op=True)

    def reduce(self, name, gw_rows, gb, gemm, colsum):
        """gw_rows (in_dim/ws, out_dim) <- dW[rows_r]; gb (out_dim,) <- full bias gradient."""
        for k in (name + ".x", name + ".dy"):
            w = self.pending.pop(k, None)
            if w is not None:
                w.wait()
        din, dout = self.layers[name]
        colsum(self.dy_all[name], gb)  # short launch ahead of the long dW GEMM
        gemm(self.x_recv[name], self.dy_all[name], gw_rows, a_trans=1, M=din // self.ws, N=dout,
             K=self.ws * self.slot)
