"""Index decode of the flattened pair enumeration in k_pair_queue16 (csrc/hip/count.hip),
checked exhaustively in float32 for every row length the u8 block counts allow (<= 255):

* off-diagonal tiles: pair t = j * ci + i  ->  j = mulhi(t << 8, ceil(2^24 / ci)), i = t - j * ci
  (and the earlier float form j = int((t + 0.5) * rcp(ci)), also with the reciprocal one ulp off);
* diagonal tiles: t = j (j - 1) / 2 + i, i < j  ->  j = int((1 + sqrt(8 t + 1)) / 2) with a +-1
  fix-up (also with the square root one ulp off).
"""
import numpy as np


def test_offdiag_decode_exhaustive():
    for c in range(1, 256):
        t = np.arange(c * 255, dtype=np.int64)
        r = np.float32(1.0) / np.float32(c)
        for rr in (r, np.nextafter(r, np.float32(0)), np.nextafter(r, np.float32(1))):
            j = ((t.astype(np.float32) + np.float32(0.5)) * np.float32(rr)).astype(np.int64)
            i = t - j * c
            assert ((i >= 0) & (i < c)).all(), c


def test_diag_decode_exhaustive():
    t = np.arange(255 * 254 // 2, dtype=np.int64)
    s = np.sqrt(np.float32(8.0) * t.astype(np.float32) + np.float32(1.0)).astype(np.float32)
    for s2 in (s, np.nextafter(s, np.float32(np.inf)), np.nextafter(s, np.float32(-np.inf))):
        j = ((np.float32(1.0) + s2.astype(np.float32)) * np.float32(0.5)).astype(np.int64)
        j = np.where(j * (j - 1) // 2 > t, j - 1, np.where(j * (j + 1) // 2 <= t, j + 1, j))
        i = t - j * (j - 1) // 2
        assert ((i >= 0) & (i < j) & (j * (j - 1) // 2 + i == t)).all()


def test_offdiag_magic_decode_exhaustive():
    for c in range(2, 256):
        m = (0x1000000 + c - 1) // c
        assert m < (1 << 24)
        t = np.arange(c * 255, dtype=np.uint64)
        j = ((t << np.uint64(8)) * np.uint64(m)) >> np.uint64(32)
        assert np.array_equal(j, t // np.uint64(c)), c
