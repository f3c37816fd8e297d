"""The dropout keep-mask restatement (oracle/philox.py) pinned by the Random123
known-answer vectors of Philox4x32-10, plus the properties of tf.nn.dropout's
binary tensor floor(keep_prob + U[0,1)) (CPU only)."""
import numpy as np

from oracle import philox

# Random123 kat_vectors: philox4x32 R=10 (counter, key) -> output
KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        np.testing.assert_array_equal(philox.philox4x32_10(ctr, key)[0], np.array(want, np.uint32))


def test_uniform_construction():
    u = philox.uniform01(np.array([0, 0x7FFFFF, 0xFFFFFFFF, 0x800000], np.uint32))
    assert u.dtype == np.float32
    np.testing.assert_array_equal(u, np.array([0.0, 1.0 - 2.0 ** -23, 1.0 - 2.0 ** -23, 0.0], np.float32))


def test_mask_properties():
    m = philox.dropout_mask(405, 4096, seed=0x5EED, step=0, stream_id=6, keep_prob=0.5)
    assert m.shape == (405, 4096) and m.dtype == np.uint8 and set(np.unique(m)) == {0, 1}
    assert abs(m.mean() - 0.5) < 0.005
    # keep_prob 1 keeps everything (floor(1 + U) = 1); 0.9 keeps ~90 %
    assert philox.dropout_mask(16, 64, 1, 0, 0, 1.0).all()
    assert abs(philox.dropout_mask(64, 1024, 1, 0, 0, 0.9).mean() - 0.9) < 0.01
    # distinct streams / steps / seeds draw independent masks; rows are a prefix of a taller draw
    other = [philox.dropout_mask(405, 4096, 0x5EED, 0, 7, 0.5), philox.dropout_mask(405, 4096, 0x5EED, 1, 6, 0.5),
             philox.dropout_mask(405, 4096, 0x5EEE, 0, 6, 0.5)]
    for o in other:
        assert 0.45 < (o == m).mean() < 0.55
    np.testing.assert_array_equal(philox.dropout_mask(1152, 4096, 0x5EED, 0, 6, 0.5)[:405], m)
