"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

CPU restatement of the reference's hash dedupe (src/videotofaces/dupes.py:11-59):
ahash = cv2.cvtColor(BGR2GRAY) -> cv2.resize(gray, (8, 8)) -> tiny > mean (cv2 is absent
here: OpenCV's published uint8 fixed point is restated -- cvtColor coefficients 1868/9617/4899
>> 14, INTER_LINEAR 11-bit coefficients as oracle.facenet._coefs, INTER_AREA for an exact 2x
downscale; parity-UNPINNED), and remove_dupes_overall('hash')'s Hamming distance matrix with
the strict-lower-triangle mask (pinned by tests/golden/dupes.npz from the reference's own
function).
"""
import numpy as np

from .facenet import _coefs


def gray(img):
    """cv2.cvtColor(img, COLOR_BGR2GRAY) for uint8."""
    i = img.astype(np.int64)
    return ((i[..., 0] * 1868 + i[..., 1] * 9617 + i[..., 2] * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def resize8(g):
    """cv2.resize(gray, (8, 8)) INTER_LINEAR (uint8 fixed point; INTER_AREA fast path at 2x)."""
    h, w = g.shape
    if (h, w) == (8, 8):
        return g.copy()
    src = g.astype(np.int64)
    if (h, w) == (16, 16):
        return ((src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    sx0, sx1, a0, a1, ex = _coefs(w, 8)
    sy0, sy1, b0, b1, _ = _coefs(h, 8)

    def hrow(rows):
        r = src[rows]
        v = r[:, sx0] * a0[None, :] + r[:, sx1] * a1[None, :]
        v[:, ex] = r[:, sx0[ex]] * 2048
        return v
    h0, h1 = hrow(sy0), hrow(sy1)
    t = (((h0 >> 4) * b0[:, None]) >> 16) + (((h1 >> 4) * b1[:, None]) >> 16)
    return np.clip((t + 2) >> 2, 0, 255).astype(np.uint8)


def ahash(img):
    """dupes.ahash (dupes.py:11-15) -> 64-element 0/1 int array."""
    tiny = resize8(gray(img))
    return 1 * (tiny > np.mean(tiny)).flatten()


def hamming_lower(H):
    """dupes.py:55-64 hash branch: D (uint16) + (1 - tri(N, -1)) * 10000, row min / argmin."""
    H = np.asarray(H)
    n = H.shape[0]
    D = (H[:, None, :] != H[None, :, :]).sum(2).astype(np.uint16)
    D += (1 - np.tri(n, k=-1).astype(D.dtype)) * 10000
    return D.min(axis=1), D.argmin(axis=1)
