"""Synthetic frame generator (posecnn_amd/synth.py): per-image seeding makes a
sharded run see exactly the frames of the single-device run."""
import numpy as np

from posecnn_amd import synth


def test_shards_equal_whole_batch():
    whole = synth.make_frames(4, H=60, W=80, num_classes=6, objects_per_image=2, seed=9)
    parts = [synth.make_frames(2, H=60, W=80, num_classes=6, objects_per_image=2, seed=9, image_offset=o)
             for o in (0, 2)]
    for k in ("label", "vertex", "meta"):
        np.testing.assert_array_equal(whole[k], np.concatenate([p[k] for p in parts]))
    np.testing.assert_array_equal(whole["gt"], np.concatenate([p["gt"] for p in parts]))
    assert set(whole["gt"][:, 0].astype(int)) == {0, 1, 2, 3}  # global image index


def test_vertex_targets_point_at_centres():
    fr = synth.make_frames(1, H=120, W=160, num_classes=6, objects_per_image=1, seed=3, dir_noise=0.0,
                           depth_noise=0.0)
    cls = int(fr["gt"][0, 1])
    K = fr["K"]
    t = fr["gt"][0, 10:13]
    cx, cy = K[0, 0] * t[0] / t[2] + K[0, 2], K[1, 1] * t[1] / t[2] + K[1, 2]
    ys, xs = np.nonzero(fr["label"][0] == cls)
    u = fr["vertex"][0, ys, xs, 3 * cls]
    v = fr["vertex"][0, ys, xs, 3 * cls + 1]
    far = np.hypot(cx - xs, cy - ys) > 2
    dots = (u * (cx - xs) + v * (cy - ys)) / np.hypot(cx - xs, cy - ys)
    assert np.all(dots[far] > 0.999)
    np.testing.assert_allclose(np.exp(fr["vertex"][0, ys, xs, 3 * cls + 2]), t[2], rtol=1e-5)
    assert fr["meta"].shape == (1, 1, 1, 48)
    np.testing.assert_allclose(fr["meta"][0, 0, 0, :9].reshape(3, 3) @ fr["meta"][0, 0, 0, 9:18].reshape(3, 3),
                               np.eye(3), atol=1e-5)
