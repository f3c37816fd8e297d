"""TEST INFRASTRUCTURE ONLY (never imported by posecnn_amd/): numpy
restatement of the pose head's dropout keep masks (csrc/dropout.hip).

tf.nn.dropout (TF 1.x nn_ops.py, called by Network.dropout,
lib/networks/network.py:574-577, on drop6 / drop7, vgg16_convs.py:189,191)
computes binary = floor(keep_prob + U[0,1)) and returns (x / keep_prob) *
binary.  U is drawn here by Philox4x32-10 (Salmon, Moraes, Dror, Shaw:
"Parallel random numbers: as easy as 1, 2, 3", SC'11; the Random123
constants), with TF's uint32 -> float construction (random_distributions.h
Uint32ToFloat).  Pinned by the Random123 known-answer vectors
(tests/test_dropout_oracle.py).  TF's assignment of Philox streams to
elements is not reproducible here, so the mask VALUES are parity-unpinned
against TF: any i.i.d. Bernoulli(keep_prob) draw is a legal execution."""
import numpy as np

M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_M32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr (n, 4) uint32 counters, key (n, 2) uint32 keys -> (n, 4) uint32."""
    c = np.asarray(ctr, np.uint64).reshape(-1, 4).copy()
    k = np.asarray(key, np.uint64).reshape(-1, 2).copy()
    if k.shape[0] == 1 and c.shape[0] > 1:
        k = np.repeat(k, c.shape[0], 0)
    for _ in range(10):
        p0 = np.uint64(M0) * c[:, 0]
        p1 = np.uint64(M1) * c[:, 2]
        h0, l0 = p0 >> np.uint64(32), p0 & _M32
        h1, l1 = p1 >> np.uint64(32), p1 & _M32
        c = np.stack([h1 ^ c[:, 1] ^ k[:, 0], l1, h0 ^ c[:, 3] ^ k[:, 1], l0], 1)
        k = (k + np.array([W0, W1], np.uint64)) & _M32
    return c.astype(np.uint32)


def uniform01(x):
    """TF's Uint32ToFloat: 23 random mantissa bits -> [1, 2) - 1 (float32)."""
    bits = (np.asarray(x, np.uint32) & np.uint32(0x7FFFFF)) | np.uint32(0x3F800000)
    return bits.view(np.float32) - np.float32(1.0)


def dropout_mask(rows, cols, seed, step, stream_id, keep_prob):
    """The (rows, cols) uint8 keep mask pcnn_dropout_mask writes: element quad
    e = r * cols / 4 + c / 4 takes Philox block (e lo, e hi, stream_id, step)
    under key (seed lo, seed hi); byte j of the quad is floor(keep + U(word j))."""
    q4 = cols // 4
    e = np.arange(rows * q4, dtype=np.uint64)
    ctr = np.stack([e & _M32, e >> np.uint64(32), np.full_like(e, stream_id), np.full_like(e, step & 0xFFFFFFFF)], 1)
    key = np.array([[seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF]], np.uint64)
    u = uniform01(philox4x32_10(ctr, key))
    keep = np.floor(np.float32(keep_prob) + u) >= np.float32(1.0)
    return keep.astype(np.uint8).reshape(rows, cols)
