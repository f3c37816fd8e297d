"""The pipelined pose step (PoseStep(pipeline=True)): the next minibatch's
vote, ADD row classification and RoI-pool forward run on the prefetch stream
beside the current step's loss and backward, into a second buffer set.  These
depend only on a minibatch's inputs (vgg16_convs.py:167-184), so every output
of every step must be bit-identical to the unpipelined step on the same
minibatch -- checked over three consecutive steps with different frames, at
each fork point, plus the fallback for inputs that were not prefetched."""
import numpy as np
import pytest
import torch

from posecnn_amd import synth
from posecnn_amd.pipeline import PoseStep

pytestmark = pytest.mark.gpu
D = torch.device("cuda")
B, H, W, C, CH, UNITS = 2, 120, 160, 22, 64, 256


def _batches(n):
    pts, sym = synth.rescaled_points(C)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(D)
    out = []
    for k in range(n):
        fr = synth.make_frames(B, H=H, W=W, num_classes=C, objects_per_image=4, seed=120 + k)
        g = torch.Generator().manual_seed(40 + k)
        out.append(dict(label=t(fr["label"]), vertex=t(fr["vertex"]), extents=t(fr["extents"]), meta=t(fr["meta"]),
                        gt=t(fr["gt"]), conv4=torch.randn((B, H // 8, W // 8, CH), generator=g).to(D),
                        conv5=torch.randn((B, H // 16, W // 16, CH), generator=g).to(D), points=t(pts),
                        symmetry=t(sym)))
    return out


def _snap(step):
    n = int(step.hough["num_rois"][1].item())
    h = step.hough
    return dict(n=n, box=h["box"][:n].clone(), pose=h["pose"][:n].clone(), target=h["target"][:n].clone(),
                weight=h["weight"][:n].clone(), pool=step.pool[:n].clone(), arg5=step.arg5[:n].clone(),
                arg4=step.arg4[:n].clone(), loss=step.loss.clone(), diff=step.diff[:n].clone(),
                drop6=step.drop6[:n].clone() if step.drop6 is not None else None, y7=step.y7[:n].clone(), dx=step.dx[:n].clone(),
                dconv4=step.dconv4.clone(), dconv5=step.dconv5.clone(), dy8=step.dy8[:n].clone(),
                **{"g_" + k: v.clone() for k, v in step.grads.items()})


def _run(batches, weights, **kw):
    step = PoseStep(B, H, W, C, D, channels=CH, units=UNITS, is_train=1, skip_pixels=3, weights=weights, **kw)
    res = []
    for k, inp in enumerate(batches):
        nxt = batches[k + 1] if kw.get("pipeline") and k + 1 < len(batches) else None
        step.step(inp, nxt) if kw.get("pipeline") else step.step(inp)
        torch.cuda.synchronize()
        res.append(_snap(step))
    return step, res


@pytest.mark.parametrize("fork", ["start", "fwd", "loss", "bwd", "tail"])
def test_pipelined_steps_bit_identical(hip, fork):
    batches = _batches(3)
    ref_step, ref = _run(batches, None)
    assert len({r["n"] for r in ref}) > 1 or not torch.equal(ref[0]["box"], ref[1]["box"])  # distinct minibatches
    _, got = _run(batches, ref_step.weights, pipeline=True, prefetch_at=fork)
    for k, (a, b) in enumerate(zip(ref, got)):
        assert a["n"] == b["n"] > 8, (k, a["n"], b["n"])
        for key in a:
            if key == "n" or a[key] is None:
                continue
            assert torch.equal(a[key], b[key]), f"step {k}: {key} differs (fork {fork})"


def _run_overlapped(batches, weights, **kw):
    """Consecutive steps with no host synchronisation in between: each step's
    outputs are copied on the stream that produced them right after step()
    returns (the chain's on the step's stream, the loss and weight gradients on
    the weight-gradient stream), so a deferred join's next step really runs
    beside the previous step's weight gradients."""
    step = PoseStep(B, H, W, C, D, channels=CH, units=UNITS, is_train=1, skip_pixels=3, weights=weights, **kw)
    main_keys = ("box", "pose", "target", "weight")
    res = []
    for k, inp in enumerate(batches):
        step.step(inp, batches[k + 1] if k + 1 < len(batches) else None)
        h = step.hough
        r = {key: h[key].clone() for key in main_keys}
        r["num_rois"] = h["num_rois"].clone()
        for key in ("pool", "arg5", "arg4", "diff", "y7", "dx", "dconv4", "dconv5", "dy8"):
            r[key] = getattr(step, key).clone()
        r["drop6"] = step.drop6.clone() if step.drop6 is not None else None
        with torch.cuda.stream(step.side_stream):
            r["loss"] = step.loss.clone()
            for gk, v in step.grads.items():
                r["g_" + gk] = v.clone()
        res.append(r)
    step.join()
    torch.cuda.synchronize()
    out = []
    for r in res:
        n = int(r.pop("num_rois")[1].item())
        out.append({key: (v[:n] if v is not None and key not in ("loss", "dconv4", "dconv5") and
                          not key.startswith("g_") else v) for key, v in r.items()} | {"n": n})
    return step, out


@pytest.mark.parametrize("fork,pool_at_tail", [("start", False), ("fwd", False), ("loss", False), ("loss", True)])
def test_pipelined_deferred_join_bit_identical(hip, fork, pool_at_tail):
    """PoseStep(defer_side_join=True): the weight-gradient stream is not joined
    at the end of a step; over three consecutive steps with no host sync, every
    output is still the unpipelined step's, bit for bit (pool_at_tail: the
    prefetched RoI-pool forward issued beside the tail)."""
    batches = _batches(3)
    ref_step, ref = _run(batches, None)
    step, got = _run_overlapped(batches, ref_step.weights, pipeline=True, prefetch_at=fork, defer_side_join=True,
                                pool_at_tail=pool_at_tail)
    assert step.defer_side_join
    for k, (a, b) in enumerate(zip(ref, got)):
        assert a["n"] == b["n"] > 8, (k, a["n"], b["n"])
        for key in b:
            if key == "n" or b[key] is None:
                continue
            assert torch.equal(a[key], b[key]), f"step {k}: {key} differs (fork {fork}, deferred join)"


def test_pipelined_step_without_prefetch_and_mismatched_inputs(hip):
    """A call whose inputs are not the previous call's next_inputs runs its
    own front chain (no stale prefetched set is used)."""
    batches = _batches(3)
    ref_step, ref = _run(batches, None, keep_prob=1.0)  # no dropout: step 2 here is the reference's step 3
    step = PoseStep(B, H, W, C, D, channels=CH, units=UNITS, is_train=1, skip_pixels=3, weights=ref_step.weights,
                    pipeline=True, keep_prob=1.0)
    step.step(batches[0], batches[1])  # prefetches batch 1 ...
    torch.cuda.synchronize()
    step.step(batches[2])  # ... but batch 2 comes: voted here
    torch.cuda.synchronize()
    got = _snap(step)
    for key in ("box", "pool", "loss", "dconv4", "g_w6"):
        assert torch.equal(ref[2][key], got[key]), key
    with pytest.raises(ValueError):
        PoseStep(B, H, W, C, D, channels=CH, units=UNITS, weights=ref_step.weights).step(batches[0], batches[1])


def test_fused_loss_tail_bit_identical(hip):
    """The loss's row tail fused with the pose head's backward (dY8 straight
    from the row sums; the scalar loss on the side stream) against the
    separate launches (pcnn_add_loss_fwd_prepared + pcnn_pose_head_bwd):
    every output of two steps bit-identical."""
    batches = _batches(2)
    ref_step, ref = _run(batches, None, fuse_loss_tail=False)
    _, got = _run(batches, ref_step.weights, fuse_loss_tail=True)
    for k, (a, b) in enumerate(zip(ref, got)):
        for key in a:
            if key == "n" or a[key] is None:
                assert a[key] == b[key]
                continue
            assert torch.equal(a[key], b[key]), f"step {k}: {key} differs"
