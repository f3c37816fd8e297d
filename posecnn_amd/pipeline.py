"""The hot path as one sync-free step (vgg16_convs.py:167-200 + the backward
TF derives for it): hough_voting_gpu -> roi_pool(conv5_3, 1/16) +
roi_pool(conv4_3, 1/8) -> fc6/fc7/fc8 -> tanh * poses_weight -> l2_normalize
-> average_distance_loss(margin 0.01), then backward through the loss, the
pose head and both RoI pools (the Hough op's gradient is identically zero,
hough_voting_gpu_op.cc:440-484, and is not materialised).

Every buffer is capacity-sized (MAX_ROI * 9 = 1152 RoI rows) and every kernel
reads the RoI row count from the device, so a step issues no host sync and can
be captured in a HIP graph.

Image sharding (one process per GPU): rank r votes on images
[r*B, (r+1)*B) with index_size = MAX_ROI / global_batch and the batch column
rebased to the global image index (the RoI pools subtract batch_base again to
index the rank's own feature maps).  Collectives (RCCL, torch.distributed
"nccl"): an all-reduce of the row count gives the ADD-loss normaliser (the
global row count, so per-rank losses sum to the single-device loss); the
pose-head weight gradients are reduced by row block through their factors
(posecnn_amd/exchange.py GradShard: rank r ends with rows_r of the global
dW6/dW7/dW8 and the full bias gradients); the loss scalar is all-reduced.
The detected RoIs + initial poses are all-gathered in single-device row
order (exchange.RoiExchange; BASELINE.json configs[3] "RCCL all-gather of
RoIs/poses"): step() starts the gather right after the vote, it overlaps the
rest of the step and is joined at the step's end (`self.detections`);
`gather_detections()` runs the same exchange on its own.
"""
import contextlib

import torch

from . import _lib
from . import pose_head as ph
from .hough_voting_gpu_layer import hough_voting_gpu_op as hv
from .roi_pooling_layer import roi_pooling_op as rp
from .average_distance_loss import average_distance_loss_op as adl
from .exchange import GradShard, RoiExchange

CAP = hv.CAPACITY
_nullctx = contextlib.nullcontext


class PoseStep:
    def __init__(self, B, H, W, num_classes, device, conv4_hw=None, conv5_hw=None, channels=512, units=4096,
                 is_train=1, skip_pixels=10, vote_threshold=-1.0, vote_percentage=0.02, margin=0.01,
                 global_batch=None, batch_base=0, weights=None, dist=None, backward=True, precision=2,
                 overlap_weight_grads=True, pixel_argmax=True, keep_prob=None, drop_seed=0x5EED, side_prep=True,
                 drop_in_reduce=True, pipeline=False, prefetch_at="loss", fuse_loss_tail=True,
                 defer_side_join=False, signal_forks=True, pool_at_tail=False):
        self.B, self.H, self.W, self.C = B, H, W, num_classes
        self.dev = device
        self.is_train, self.skip, self.vthr, self.vper, self.margin = is_train, skip_pixels, vote_threshold, \
            vote_percentage, margin
        self.global_batch = global_batch or B
        self.batch_base = batch_base
        self.dist = dist  # torch.distributed module (initialised) or None
        self.backward = backward
        # FC GEMMs: 2 = exact three-way split-bf16 x6 MFMA (fp32-faithful, the default), 1 = split-bf16 x3
        # MFMA (fp32-class, ~2^-16 per product), 0 = fp32 MFMA
        self.prec = precision
        self.h4, self.w4 = conv4_hw or (H // 8, W // 8)
        self.h5, self.w5 = conv5_hw or (H // 16, W // 16)
        self.Ch = channels
        D = 4 * num_classes
        self.D = D
        self.weights = weights or ph.PoseHeadWeights(num_classes, device, in_dim=49 * channels, units=units)
        f32 = dict(dtype=torch.float32, device=device)
        i32 = dict(dtype=torch.int32, device=device)
        K6 = 49 * channels
        # argmax as uint16 pixel indices (half the bytes of the flat int32 form,
        # written by the pool pair and re-read by both pool backwards) when
        # both maps have fewer than 0xFFFF pixels
        px = pixel_argmax and max(self.h4 * self.w4, self.h5 * self.w5) < 0xFFFF
        adt = dict(dtype=torch.int16 if px else torch.int32, device=device)

        def minibatch_set():
            """The per-minibatch buffers: the Hough outputs, pool5 + pool4
            (vgg16_convs.py:184), both argmax maps, the ADD row classes."""
            return dict(hough=dict(box=torch.zeros((CAP, 7), **f32), pose=torch.zeros((CAP, 7), **f32),
                                   target=torch.zeros((CAP, D), **f32), weight=torch.zeros((CAP, D), **f32),
                                   domain=torch.zeros((CAP,), **i32), num_rois=torch.zeros((2,), **i32)),
                        pool=torch.zeros((CAP, 7, 7, channels), **f32),
                        arg5=torch.zeros((CAP, 7, 7, channels), **adt),
                        arg4=torch.zeros((CAP, 7, 7, channels), **adt),
                        add_ws=None, prepped=False)
        # pipeline=True: two sets; step(inputs, next_inputs) runs the forward /
        # backward of `inputs` on one while the vote, RoI-pool forward and ADD
        # row classification of `next_inputs` fill the other on a third stream
        # the loss's row tail + the pose head's backward in one pass, the scalar
        # loss on the side stream (step() only; False: separate launches, A/B)
        self.fuse_loss_tail = fuse_loss_tail
        self.pipeline = bool(pipeline)
        self._sets = [minibatch_set() for _ in range(2 if self.pipeline else 1)]
        self._cur = 0           # the set the step's forward / backward uses (and the attributes show)
        self._primed = None     # pipelined: (set index, inputs) voted + pooled ahead by the previous step
        # where the next minibatch's front chain forks off: "start" (beside the
        # fc6 forward), "fwd" (the same point on the device -- ordered after the
        # step's start by an event -- but issued by the host after the fc6
        # forward's launch, so the chain's first kernel is queued first),
        # "loss" (after fc8's forward), "bwd" (after the head backward) or
        # "tail" (after fc6 dX is launched: beside fc6 dW and the RoI-pool
        # backward)
        self.prefetch_at = prefetch_at
        if prefetch_at not in ("loss", "bwd", "start", "fwd", "tail"):
            raise ValueError("prefetch_at must be 'start', 'fwd', 'loss', 'bwd' or 'tail'")
        self._fork_ev = torch.cuda.Event() if self.pipeline else None
        self._fork_recorded = False
        self.pre_stream = torch.cuda.Stream(device=device) if self.pipeline else None
        self._next = None       # (inputs, set index) of the minibatch to prefetch during this step
        self.y6 = torch.zeros((CAP, units), **f32)
        self.y7 = torch.zeros((CAP, units), **f32)
        self.y8 = torch.zeros((CAP, D), **f32)
        self.t8 = torch.zeros((CAP, D), **f32)
        self.pred = torch.zeros((CAP, D), **f32)
        self.loss = torch.zeros((1,), **f32)
        self.diff = torch.zeros((CAP, D), **f32)
        self.one = torch.ones((1,), **f32)
        self.dy8 = torch.zeros((CAP, D), **f32)
        self.dy7 = torch.zeros((CAP, units), **f32)
        self.dy6 = torch.zeros((CAP, units), **f32)
        self.dx = torch.zeros((CAP, K6), **f32)
        self.gshard = None
        if dist is not None:
            # rows a rank can emit: B images x index_size maxima x (9 jitters | 1), or the dummy row
            per_max = 9 if is_train else 1
            slot = max(1, min(CAP, B * (hv.MAX_ROI // self.global_batch) * per_max))
            self.gshard = GradShard(dist, slot, [("w6", (K6, units)), ("w7", (units, units)), ("w8", (units, D))],
                                    device)
        self.grads = self.weights.grads_like()
        if self.gshard is not None:  # this rank's row block of each weight gradient
            for k in ("w6", "w7", "w8"):
                self.grads[k] = self.grads[k][self.gshard.rows(k)].contiguous()
        # drop6 / drop7 (vgg16_convs.py:189,191): keep_prob 0.5 in training
        # (train.py:421), 1 at test time (test.py:173); fused into the fc6 / fc7
        # epilogues (forward) and the relu-mask epilogues of fc8 / fc7 dX
        self.keep = float(keep_prob if keep_prob is not None else (0.5 if is_train else 1.0))
        if not 0.0 < self.keep <= 1.0:
            raise ValueError("keep_prob must be in (0, 1]")
        self.drop6 = self.drop7 = None
        self._drop_external = False
        self.drop_in_reduce = drop_in_reduce  # keep bits drawn in the fc6 / fc7 reduce epilogues
        self._bump_drop_step = False
        self._drawn = False  # this step's keep masks drawn by draw_drop_masks() (mask-kernel mode)
        if self.keep < 1.0:
            u8 = dict(dtype=torch.uint8, device=device)
            self.drop6 = torch.zeros((CAP, units), **u8)
            self.drop7 = torch.zeros((CAP, units), **u8)
            self.drop_step = torch.zeros((1,), dtype=torch.int64, device=device)  # Philox counter word, bumped per step
            rank = dist.get_rank() if dist is not None else 0  # independent masks per rank
            self.drop_seed = (int(drop_seed) + rank * 0x9E3779B97F4A7C15) & ((1 << 64) - 1)
            self._drop_ready = None
            self._drop_ev = torch.cuda.Event()
        self.dconv4 = torch.zeros((B, self.h4, self.w4, channels), **f32)
        self.dconv5 = torch.zeros((B, self.h5, self.w5, channels), **f32)
        self.norm_rows = torch.zeros((1,), **i32)
        self.timer = None  # optional {name: [(start_event, end_event), ...]} (bench.py)
        # optional {gemm name: [(start_event, end_event), ...]}: HIP events around each FC GEMM on the
        # stream it runs on, with the step's stream overlap left on (the in-step kernel times, bench.py)
        self.gemm_timer = None
        self.xchg = None  # RoiExchange, built on the first sharded step / gather_detections()
        self.detections = None  # sharded step: (global rows (ws*CAP, 14) = [box | pose], total (1,)) of the last step
        self._pending = {}  # async collectives of the current step
        self._in_step = False  # forward() inside step(): the loss all-reduce is joined at the step's end
        # weight-gradient branch of the backward (None: everything on the caller's stream)
        self.side_stream = torch.cuda.Stream(device=device) if overlap_weight_grads else None
        # the post-vote side work (the ADD loss's row classification, and the
        # dropout keep masks when drop_in_reduce is off): on the side stream
        # beside the RoI pool (True), or on the step's stream with no fork /
        # join (False: the row classification right before the loss)
        self.side_prep = side_prep and self.side_stream is not None
        # pipelined, single device: the weight-gradient stream is not joined at
        # the end of the step; the next step waits for it only where it first
        # rewrites what that stream reads (y6 before the fc6 forward: an event
        # after fc7's weight gradient; dy6 before fc7 dX, and the other set's
        # buffers before the prefetch or an un-prefetched front chain: the end
        # of the stream), so the next step's fc6 forward starts beside this
        # step's fc6 dW.  step() then returns before the weight gradients and
        # the loss are ordered on the caller's stream: join() (or a device
        # synchronize) before reading them there.
        self.defer_side_join = bool(defer_side_join) and self.pipeline and dist is None and \
            self.side_stream is not None
        self._side_mid_ev = torch.cuda.Event() if self.defer_side_join else None
        self._side_done_ev = torch.cuda.Event() if self.defer_side_join else None
        self._side_pending = False
        # the chain's forks to the weight-gradient stream (after the fused loss
        # tail, fc8 dX and fc7 dX) wait on an event the op's last kernel records
        # through its own completion signal (pcnn_set_completion_event) instead
        # of an event-record marker, which leaves the chain's stream idle ~7 us
        # per fork; eager, single device (under graph capture: markers)
        self.signal_forks = bool(signal_forks) and self.side_stream is not None and dist is None
        self._fork_evs = {}
        # pipelined: the prefetched minibatch's RoI-pool forward issued on the
        # prefetch stream only once fc6 dX is launched (beside the tail),
        # its vote and ADD row classes at the fork point
        self.pool_at_tail = bool(pool_at_tail) and self.pipeline
        self._pool_pending = None
        if self.signal_forks:
            for k in ("loss", "fc8_dx", "fc7_dx"):
                ev = torch.cuda.Event()
                ev.record()  # creates the event (torch waits only on created events)
                self._fork_evs[k] = ev
        self._mid_covers_pre = False  # the mid event was recorded after the prefetch it follows was joined
        self._mid_waited = False      # this step's stream already waited for the previous step's mid event

    # ------------------------------------------------------------------
    def _t(self, name):
        """HIP-event bracket on the current stream (no-op unless self.timer is set)."""
        step = self

        class _Ctx:
            def __enter__(self_):
                if step.timer is not None:
                    self_.e0 = torch.cuda.Event(enable_timing=True)
                    self_.e0.record()

            def __exit__(self_, *a):
                if step.timer is not None:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    step.timer.setdefault(name, []).append((self_.e0, e1))
        return _Ctx()

    def join(self):
        """Order everything the step's other streams issued (the deferred
        weight-gradient stream, the prefetch stream) before the caller's
        current stream's later work."""
        cur = torch.cuda.current_stream()
        for st in (self.side_stream, self.pre_stream):
            if st is not None:
                cur.wait_stream(st)
        self._side_pending = False

    def _side_wait(self, ev_name, stream=None):
        """Deferred join: `stream` (default the current one) waits for the
        previous step's weight-gradient stream up to the named event."""
        if self._side_pending:
            (stream or torch.cuda.current_stream()).wait_event(getattr(self, ev_name))

    def _arm_fork(self, name):
        """Arm the completion event `name` for the next library op on this
        thread (eager, signal_forks); returns it, or None."""
        if not self.signal_forks or self.timer is not None or torch.cuda.is_current_stream_capturing():
            return None
        ev = self._fork_evs[name]
        _lib.load().pcnn_set_completion_event(ev.cuda_event)
        return ev

    @staticmethod
    def _fork_taken(ev):
        """The armed event if the op's last kernel recorded it, else None (and
        the hook cleared): the caller then forks with a marker."""
        if ev is None:
            return None
        return None if _lib.load().pcnn_completion_event_pending() else ev

    def _fork_side(self, side, ev):
        """`side` continues after the chain's last op: on its completion event
        when it was taken, else behind an event-record marker."""
        if ev is not None:
            side.wait_event(ev)
        else:
            side.wait_stream(torch.cuda.current_stream())

    # the current minibatch set's buffers (after a pipelined step: the set that
    # step trained on, not the one its prefetch filled)
    hough = property(lambda self: self._sets[self._cur]["hough"])
    pool = property(lambda self: self._sets[self._cur]["pool"])
    arg5 = property(lambda self: self._sets[self._cur]["arg5"])
    arg4 = property(lambda self: self._sets[self._cur]["arg4"])
    add_ws = property(lambda self: self._sets[self._cur]["add_ws"])

    def vote(self, label, vertex, extents, meta, gt, s=None):
        s = self._cur if s is None else s
        self._sets[s]["pooled"] = False
        with self._t("hough_voting_gpu"):
            return hv.hough_voting_gpu_capacity(label, vertex, extents, meta, gt, self.is_train, self.vthr,
                                                self.vper, self.skip, global_batch=self.global_batch,
                                                batch_base=self.batch_base, out=self._sets[s]["hough"])

    def add_prep(self, points, symmetry, s=None, stream=None):
        """The ADD loss's row classification (it reads only the Hough weights):
        on the side stream right after the vote, joined before the loss
        (`stream` given: on that stream, already ordered after the vote)."""
        s = self._cur if s is None else s
        st = self._sets[s]
        if st["add_ws"] is None:
            st["add_ws"] = torch.empty(adl.workspace_bytes(CAP, self.C, points.shape[1]), dtype=torch.uint8,
                                       device=self.dev)
        h = st["hough"]
        side = None
        if stream is None:
            side = self.side_stream if self.timer is None and self.side_prep else None
            if side is not None:
                side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream or side or torch.cuda.current_stream()):
            adl.average_distance_loss_prep(h["weight"], symmetry, points.shape[1], st["add_ws"],
                                           num_rois=h["num_rois"][1:2], points=points)
        st["prepped"] = "side" if side is not None else "stream"

    def pool_fwd(self, conv4, conv5, s=None):
        """pool5 + pool4 (vgg16_convs.py:177-184) and both argmax maps, one pass."""
        s = self._cur if s is None else s
        st = self._sets[s]
        with self._t("roi_pool_fwd"):
            rp.roi_pool_pair(conv5, 1.0 / 16.0, conv4, 1.0 / 8.0, st["hough"]["box"], 7, 7,
                             num_rois=st["hough"]["num_rois"][1:2], out=(st["pool"], st["arg5"], st["arg4"]),
                             batch_base=self.batch_base)
        st["pooled"] = True

    def _front(self, inputs, s, stream=None):
        """A minibatch's weight-independent front chain into set s: the vote,
        the ADD row classification and the RoI-pool forward (`stream`: all of
        it there, in that order)."""
        ctx = torch.cuda.stream(stream) if stream is not None else _nullctx()
        with ctx:
            self.vote(inputs["label"], inputs["vertex"], inputs["extents"], inputs["meta"], inputs["gt"], s=s)
            if stream is not None:
                self.add_prep(inputs["points"], inputs["symmetry"], s=s, stream=stream)
                if self.pool_at_tail and stream is self.pre_stream:
                    self._pool_pending = (inputs, s)
                else:
                    self.pool_fwd(inputs["conv4"], inputs["conv5"], s=s)

    def _issue_pending_pool(self):
        """The prefetched minibatch's RoI-pool forward (pool_at_tail), on the
        prefetch stream behind its vote."""
        if self._pool_pending is None:
            return
        inputs, s = self._pool_pending
        self._pool_pending = None
        with torch.cuda.stream(self.pre_stream):
            self.pool_fwd(inputs["conv4"], inputs["conv5"], s=s)

    def _prefetch(self):
        """The next minibatch's front chain on the prefetch stream (pipelined
        step): ordered after everything the step had issued on its stream at
        the fork point ("fwd": at the step's start, through the event recorded
        there) -- so after the previous step, which last used that set -- and
        joined by the next step before it reads the set."""
        if self._next is None:
            return
        nxt, s = self._next
        self._next = None
        if self.timer is not None:  # per-op timing runs the ops one by one on the step's stream
            self._side_wait("_side_done_ev")  # the set's hough rows / pool / ADD workspace
            self._side_pending = False
            self._front(nxt, s, stream=torch.cuda.current_stream())
        else:
            if self._fork_recorded:
                self.pre_stream.wait_event(self._fork_ev)
            else:
                self.pre_stream.wait_stream(torch.cuda.current_stream())
            self._side_wait("_side_done_ev", self.pre_stream)  # the set's hough rows / pool / ADD workspace
            self._front(nxt, s, stream=self.pre_stream)
        self._fork_recorded = False
        self._primed = (s, nxt)

    def set_drop_masks(self, m6, m7):
        """Use fixed dropout keep masks ((rows, units) 0/1, copied into the
        capacity buffers) instead of drawing new ones every step (tests)."""
        if self.keep >= 1.0:
            raise ValueError("set_drop_masks: the step has keep_prob 1 (no dropout)")
        for dst, m in ((self.drop6, m6), (self.drop7, m7)):
            dst.zero_()
            dst[:m.shape[0]].copy_(m.to(torch.uint8))
        self._drop_external = True

    def draw_drop_masks(self):
        """This step's drop6 / drop7 keep masks (Philox, keyed on the device
        step counter so graph replays draw new ones) as separate launches, on
        the side stream (the fc6 forward waits for them) or, without side_prep,
        on the step's stream.  Only with drop_in_reduce=False: by default the
        fc6 / fc7 forward reduces draw the same bits in their epilogue
        (pcnn_gemm_drop_gen) and store them for the backward."""
        if self.keep >= 1.0 or self._drop_external or self.drop_in_reduce:
            return
        self._drawn = True
        nr = self.hough["num_rois"][1:2]
        side = self.side_stream if self.timer is None and self.side_prep else None
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side or torch.cuda.current_stream()):
            ph.dropout_mask(self.drop6, self.keep, self.drop_seed, self.drop_step, 6, rows_dev=nr)
            ph.dropout_mask(self.drop7, self.keep, self.drop_seed, self.drop_step, 7, rows_dev=nr)
            self.drop_step.add_(1)
            if side is not None:
                self._drop_ev.record(side)
                self._drop_ready = self._drop_ev

    def exchange(self):
        """Global ADD-loss normaliser = max(sum of per-rank rows, 1): an
        all-reduce of one int (async; the loss kernel waits for it)."""
        h = self.hough
        if self.dist is None:  # single device: the loss normaliser is the op's own row count
            self.norm_rows = h["num_rois"][1:2]
            return
        with self._t("allreduce_rows"):
            self.norm_rows.copy_(h["num_rois"][0:1])
            self._pending["rows"] = self.dist.all_reduce(self.norm_rows, async_op=True)

    def _wait(self, key):
        w = self._pending.pop(key, None)
        if w is not None:
            w.wait()

    def gather_detections(self):
        """All-gather of the detected RoI boxes + initial poses (RCCL): returns
        (rows (ws*CAP, 14) = [box(7) | pose(7)], total (1,) int32), the global
        rows first in single-device order (image-major).  Single device: the
        op's own rows."""
        h = self.hough
        if self.dist is None:
            return torch.cat([h["box"], h["pose"]], 1), h["num_rois"][0:1]
        return self._exchange_rows()(h["box"], h["pose"], h["num_rois"])

    def _exchange_rows(self):
        if self.xchg is None:
            self.xchg = RoiExchange(self.dist, CAP, self.dev)
        return self.xchg

    def forward(self, conv4, conv5, points, symmetry):
        h = self.hough
        nr = h["num_rois"][1:2]  # output row count (incl. dummy row)
        w = self.weights
        K6 = 49 * self.Ch
        st = self._sets[self._cur]
        if not (self.pipeline and st.get("pooled")):  # pipelined: pooled ahead by the previous step's prefetch
            self.pool_fwd(conv4, conv5)
        x = self.pool.view(CAP, K6)
        gs = self.gshard if self.backward else None
        if gs is not None:  # fc6 input column blocks to their owners (overlaps the forward)
            gs.send_input("w6", x)
        dk = dict(keep_prob=self.keep) if self.keep < 1.0 else {}
        if not self._drawn:  # forward() on its own in mask-kernel mode: this pass's masks (a no-op otherwise)
            self.draw_drop_masks()
        self._drawn = False
        if self.keep < 1.0 and getattr(self, "_drop_ready", None) is not None:
            torch.cuda.current_stream().wait_event(self._drop_ready)  # this step's keep masks (side stream)
            self._drop_ready = None
        gen = self.keep < 1.0 and self.drop_in_reduce and not self._drop_external
        g6 = dict(drop_gen=(self.drop_seed, self.drop_step, 6)) if gen else {}
        g7 = dict(drop_gen=(self.drop_seed, self.drop_step, 7)) if gen else {}
        if not self._mid_waited:
            self._side_wait("_side_mid_ev")  # the previous step's fc7 weight gradient read y6
        self._mid_waited = False
        with self._t("gemm_fc6_fwd"):
            self._g("fc6_fwd", x, w.w6, self.y6, bias=w.b6, act=1, M_dev=nr, drop=self.drop6, **dk, **g6)
        if self.prefetch_at == "fwd":  # forked at the step's start (event), issued after the fc6 forward
            self._prefetch()
        if gs is not None:
            gs.send_input("w7", self.y6)
        with self._t("gemm_fc7_fc8_fwd"):
            self._g("fc7_fwd", self.y6, w.w7, self.y7, bias=w.b7, act=1, M_dev=nr, drop=self.drop7, **dk, **g7)
            if gs is not None:
                gs.send_input("w8", self.y7)
            self._g("fc8_fwd", self.y7, w.w8, self.y8, bias=w.b8, act=0, M_dev=nr)
        if self.prefetch_at == "loss":  # the next minibatch's vote + pool beside the loss and the backward
            self._prefetch()
        if gen:  # the step counter moves on once both masks are drawn
            if self._in_step and self.backward:
                self._bump_drop_step = True  # at the end of the data-gradient chain, beside the dW tail
            else:
                self.drop_step.add_(1)
        if self.dist is not None:
            self._wait("rows")
            self.norm_rows.clamp_(min=1)
        with self._t("head_add_loss_fwd"):
            ph.head_fwd(self.y8, h["weight"], self.t8, self.pred, num_rois=nr)
            if not st["prepped"]:  # forward() called without step()
                self.add_prep(points, symmetry)
            if st["prepped"] == "side":
                torch.cuda.current_stream().wait_stream(self.side_stream)  # the row classes (add_prep)
            st["prepped"] = False
            # the previous step's in-place loss all-reduce must be done before
            # the loss kernel rewrites self.loss (its handle orders it on this stream)
            self._wait("loss")
            side = self.side_stream
            self._head_bwd_done = fuse = (self.fuse_loss_tail and self._in_step and self.backward and
                                          self.timer is None and side is not None and self.D <= 256)
            if fuse:
                # the loss's row tail and the pose head's backward in one pass
                # (dY8 straight from the row sums), the scalar loss beside the
                # backward on the side stream: nothing on the chain reads it
                ev = self._arm_fork("loss")
                adl.average_distance_loss_head_bwd(self.pred, h["target"], h["weight"], points, symmetry,
                                                   self.margin, self.t8, self.one, self.diff, self.dy8, st["add_ws"],
                                                   num_rois=nr, loss_norm_rows_dev=self.norm_rows)
                self._fork_side(side, self._fork_taken(ev))
                with torch.cuda.stream(side):
                    adl.average_distance_loss_total(CAP, self.C, points.shape[1], st["add_ws"], self.loss,
                                                    num_rois=nr)
                    if self.dist is not None:  # joined at the end of the step
                        self._pending["loss"] = self.dist.all_reduce(self.loss, async_op=True)
                return self.loss
            adl.average_distance_loss(self.pred, h["target"], h["weight"], points, symmetry, self.margin,
                                      num_rois=nr, loss_norm_rows_dev=self.norm_rows, out=(self.loss, self.diff),
                                      workspace=st["add_ws"], prepared=True)
        if self.dist is not None:  # nothing downstream reads the global loss: joined at the end of the step
            self._pending["loss"] = self.dist.all_reduce(self.loss, async_op=True)
            if not self._in_step:  # called on its own: the returned loss is the reduced one
                self._wait("loss")
        return self.loss

    def backward_pass(self, conv4, conv5):
        """Backward through the ADD loss, the pose head and both RoI pools.

        The data-gradient chain (fc8 dX -> fc7 dX -> fc6 dX -> RoI-pool
        backward) stays on the step's stream; the weight / bias gradients are
        leaves of the graph and run on a side stream that joins at the end, so
        their launches fill the gaps and tails of the chain (HIP-graph branches
        when captured).  Image-sharded: each layer's dY goes to the all-gather
        as soon as it exists and the side stream computes this rank's row
        block of the global weight gradient (GradShard)."""
        h = self.hough
        nr = h["num_rois"][1:2]
        w, g = self.weights, self.grads
        K6 = 49 * self.Ch
        main = torch.cuda.current_stream()
        side = self.side_stream if self.timer is None else None  # per-op timing runs the ops one by one
        gs = self.gshard
        x = self.pool.view(CAP, K6)

        def weight_grads(name, X, dY, K_loc, M, N, fork=True, fork_ev=None):
            if side is not None and fork:
                self._fork_side(side, fork_ev)
            if gs is not None:
                gs.send_grad(name, dY, nr)
            with torch.cuda.stream(side or main):
                if gs is not None:
                    gs.reduce(name, g[name], g["b" + name[1:]],
                              lambda A, B_, C_, **kw: self._g(f"fc{name[1:]}_dw", A, B_, C_, **kw), ph.colsum)
                else:
                    # the bias sum first: a short launch ahead of the long dW GEMM, not
                    # a tail after it (fc6: it ran 44 us behind the dW, beside the pool bwd)
                    ph.colsum(dY, g["b" + name[1:]], M_dev=nr)
                    self._g(f"fc{name[1:]}_dw", X, dY, g[name], a_trans=1, K_dev=nr, M=M, N=N, K=K_loc)

        # the fused loss tail already forked the side stream right after dY8
        # (forward()) and nothing has been queued on this stream since: the
        # fc8 weight gradient reuses that fork (each fork is a marker packet
        # that leaves the chain's stream idle ~7 us)
        fused_fork = getattr(self, "_head_bwd_done", False) and side is not None
        if not getattr(self, "_head_bwd_done", False):  # (fused into the loss's row tail inside step())
            with self._t("add_loss_head_bwd"):
                # average_distance_loss_grad (top_diff[0] * bottom_diff) folded into
                # the head backward: one pass over the (R, 4C) rows instead of two
                ph.head_bwd(self.diff, self.t8, h["weight"], self.pred, self.dy8, num_rois=nr,
                            d_pred_scale=self.one)
        self._head_bwd_done = False
        if self.prefetch_at == "bwd":
            self._prefetch()
        with self._t("gemm_fc8_fc7_dw_bias"):  # fc8 weight / bias gradients
            weight_grads("w8", self.y7, self.dy8, CAP, w.units, self.D, fork=not fused_fork)
        dk = dict(keep_prob=self.keep) if self.keep < 1.0 else {}  # relu + dropout backward: kept grads / keep_prob
        ev = self._arm_fork("fc8_dx") if side is not None else None
        with self._t("gemm_fc8_fc7_dx"):
            self._g("fc8_dx", self.dy8, w.w8, self.dy7, b_trans=1, mask=self.y7, M_dev=nr, **dk)
        ev = self._fork_taken(ev)
        with self._t("gemm_fc8_fc7_dw_bias"):  # fc7 weight / bias gradients
            weight_grads("w7", self.y6, self.dy7, CAP, w.units, w.units, fork_ev=ev)
        defer = self.defer_side_join and side is not None
        self._side_wait("_side_done_ev")  # (deferred join) the previous step's fc6 dW / bias read dy6
        self._side_pending = False
        if defer:
            # the mid event also covers the next minibatch's prefetch (when it
            # was issued by now) and the dropout counter bump, so the next step
            # starts behind one cross-stream wait instead of two or three
            # (not while a HIP graph is captured: that step keeps both waits)
            self._mid_covers_pre = (self._primed is not None and self._pool_pending is None and
                                    not torch.cuda.is_current_stream_capturing())
            if self._mid_covers_pre:
                side.wait_stream(self.pre_stream)
            if self._bump_drop_step and self._mid_covers_pre:
                with torch.cuda.stream(side):  # after this step's fc6 / fc7 forward reduces read it (joined above)
                    self.drop_step.add_(1)
                self._bump_drop_step = False
            self._side_mid_ev.record(side)  # after this step's last reader of y6 / y7 / dy7 / dy8
        ev = self._arm_fork("fc7_dx") if side is not None else None
        with self._t("gemm_fc8_fc7_dx"):
            self._g("fc7_dx", self.dy7, w.w7, self.dy6, b_trans=1, mask=self.y6, M_dev=nr, **dk)
        ev = self._fork_taken(ev)
        with self._t("gemm_fc6_dw"):  # fc6 weight / bias gradients (A = pool5 + pool4)
            weight_grads("w6", x, self.dy6, CAP, K6, w.units, fork_ev=ev)
        with self._t("gemm_fc6_dx"):
            self._g("fc6_dx", self.dy6, w.w6, self.dx, b_trans=1, M_dev=nr)
        if self.prefetch_at == "tail":
            self._prefetch()
        self._issue_pending_pool()
        dxp = self.dx.view(CAP, 7, 7, self.Ch)
        with self._t("roi_pool_bwd"):  # both pools receive d(pool5 + pool4) = dx
            rp.roi_pool_grad(conv5, h["box"], self.arg5, dxp, 7, 7, 1.0 / 16.0, 0, num_rois=nr, out=self.dconv5,
                             batch_base=self.batch_base)
            rp.roi_pool_grad(conv4, h["box"], self.arg4, dxp, 7, 7, 1.0 / 8.0, 0, num_rois=nr, out=self.dconv4,
                             batch_base=self.batch_base)
        if self._bump_drop_step:  # next step's dropout draws (off the critical path: the side stream's tail runs)
            self.drop_step.add_(1)
            self._bump_drop_step = False
        if defer:
            self._side_done_ev.record(side)
            self._side_pending = True
        elif side is not None:
            main.wait_stream(side)

    def _gemm(self, A, B, C, **kw):
        return ph.gemm(A, B, C, precision=self.prec, **kw)

    def _g(self, name, A, B, C, **kw):
        """One FC GEMM at the step's precision, bracketed by HIP events on the
        stream it is launched on when gemm_timer is set."""
        if self.gemm_timer is None:
            return ph.gemm(A, B, C, precision=self.prec, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ph.gemm(A, B, C, precision=self.prec, **kw)
        e1.record()
        self.gemm_timer.setdefault(name, []).append((e0, e1))
        return C

    def step(self, inputs, next_inputs=None):
        """One training step over the minibatch `inputs`.

        Pipelined (PoseStep(pipeline=True)): the vote, ADD row classification
        and RoI-pool forward of `next_inputs` (the minibatch of the following
        call) run on the prefetch stream beside this step's loss and backward
        (`prefetch_at`), into the other buffer set; the following step(
        next_inputs, ...) starts from them.  They depend only on a minibatch's
        inputs, not on the weights (vgg16_convs.py:167-184: the Hough op and
        the RoI pools read the network's label / vertex / conv maps), so every
        output is the unpipelined step's, bit for bit.  A call whose inputs
        were not prefetched runs its own front chain first."""
        if self.pipeline:
            return self._step_pipelined(inputs, next_inputs)
        if next_inputs is not None:
            raise ValueError("next_inputs needs PoseStep(pipeline=True)")
        self.vote(inputs["label"], inputs["vertex"], inputs["extents"], inputs["meta"], inputs["gt"])
        self.draw_drop_masks()
        if self.side_prep:  # else forward() classifies the rows right before the loss
            self.add_prep(inputs["points"], inputs["symmetry"])
        return self._train(inputs)

    def _step_pipelined(self, inputs, next_inputs):
        main = torch.cuda.current_stream()
        if self._primed is not None and self._primed[1] is inputs:
            self._cur = self._primed[0]
            if self._side_pending and self._mid_covers_pre:  # deferred join: one wait covers the prefetch too
                main.wait_event(self._side_mid_ev)
                self._mid_waited = True
            else:
                main.wait_stream(self.pre_stream)  # this minibatch's vote / prep / pool (previous step's prefetch)
        else:  # not prefetched (first step, or other inputs): its front chain here, on the step's stream
            self._side_wait("_side_done_ev")  # it rewrites the set the previous step's weight gradients read
            self._side_pending = False
            self._front(inputs, self._cur, stream=main)
        self._primed = None
        self._next = (next_inputs, 1 - self._cur) if next_inputs is not None else None
        self.draw_drop_masks()
        if self.prefetch_at == "start":
            self._prefetch()
        elif self.prefetch_at == "fwd" and self._next is not None and self.timer is None:
            self._fork_ev.record(main)
            self._fork_recorded = True
        loss = self._train(inputs)
        self._prefetch()  # (no-op unless the fork point was never reached)
        self._issue_pending_pool()
        return loss

    def _train(self, inputs):
        """Forward + backward of the minibatch whose vote is in the current set."""
        self.exchange()
        if self.dist is not None:  # the RoI / pose all-gather: started here, joined at the end of the step
            with self._t("allgather_rois"):
                h = self.hough
                self._exchange_rows().start(h["box"], h["pose"], h["num_rois"])
        self._in_step = True
        try:
            loss = self.forward(inputs["conv4"], inputs["conv5"], inputs["points"], inputs["symmetry"])
            if self.backward:
                self.backward_pass(inputs["conv4"], inputs["conv5"])
        finally:
            self._in_step = False
        self._wait("loss")
        if self.dist is not None:
            # clones: the exchange reuses its buffers on the next step and on
            # gather_detections(), so a kept step's rows must not alias them
            rows, total = self.xchg.finish()
            self.detections = (rows.clone(), total.clone())
        return loss
