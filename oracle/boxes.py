"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, bench.py cpu_baseline leg).

Vectorised numpy restatement of the reference's box post-processing between detector and
encoder (src/videotofaces/detection.py:126-162): check_box 165-171, filter_boxes 174-180,
adjust_boxes 220-262 and the (frame, face) flatten of process_frames_batch 139-145.  Each step
below names the reference lines it restates; the reference's per-box Python loop becomes array
operations applied to all boxes at once, with the same integer / double arithmetic.  Pinned by
tests/golden/boxes.npz (the reference's own filter_boxes / adjust_boxes on random and edge-case
boxes, tests/golden/make_golden.py gen_boxes).
"""
import numpy as np


def _round_out(rows):
    """filter_boxes 176: (floor x1, floor y1, ceil x2, ceil y2) of the float32 box, as ints."""
    r = np.asarray(rows, np.float32).reshape(-1, 5)
    x1, y1 = np.floor(r[:, 0]).astype(np.int64), np.floor(r[:, 1]).astype(np.int64)
    x2, y2 = np.ceil(r[:, 2]).astype(np.int64), np.ceil(r[:, 3]).astype(np.int64)
    return x1, y1, x2, y2, r[:, 4]


def passes(rows, img_size, mscore, msize, mborder):
    """check_box 165-171 negated: keep mask of the rounded boxes.  The score test is float32
    against float32(mscore) (numpy float32 scalar vs Python float under NEP 50)."""
    H, W = img_size
    x1, y1, x2, y2, s = _round_out(rows)
    low = s < np.float32(mscore)
    small = ((x2 - x1) < msize) | ((y2 - y1) < msize)
    if mborder:
        edge = (x1 < mborder) | (y1 < mborder) | (x2 > W - mborder) | (y2 > H - mborder)
    else:
        edge = np.zeros_like(low)
    return ~(low | small | edge)


def _scale(a1, a2, s_lo, s_hi, lim):
    """adjust_boxes 228-233 for one axis: centre in double, floor/ceil after the frame clamp."""
    n = (a2 - a1).astype(np.float64)
    c = a1.astype(np.float64) + n / 2
    lo = c - s_lo * n / 2
    hi = c + s_hi * n / 2
    return np.floor(np.maximum(lo, 0.0)).astype(np.int64), np.ceil(np.minimum(hi, float(lim))).astype(np.int64)


def _widen(a1, a2, d, lim, sel):
    """adjust_boxes 237-243 / 245-250 on the rows in `sel`: grow by d, then push back inside."""
    a1, a2 = a1.copy(), a2.copy()
    a1 = np.where(sel, a1 - d // 2, a1)
    a2 = np.where(sel, a2 + d - d // 2, a2)
    neg = sel & (a1 < 0)
    a2 = np.where(neg, np.minimum(a2 - a1, lim), a2)
    a1 = np.where(neg, 0, a1)
    over = sel & (a2 > lim)
    a1 = np.where(over, np.maximum(a1 - (a2 - lim), 0), a1)
    a2 = np.where(over, lim, a2)
    return a1, a2


def adjust(x1, y1, x2, y2, img_size, scale, square):
    """adjust_boxes 220-262 on integer corner arrays."""
    if isinstance(scale, int):
        scale = (scale,) * 4
    sx1, sx2, sy1, sy2 = scale
    H, W = img_size
    x1, x2 = _scale(x1, x2, sx1, sx2, W)
    y1, y2 = _scale(y1, y2, sy1, sy2, H)
    if square:
        w, h = x2 - x1, y2 - y1
        x1, x2 = _widen(x1, x2, h - w, W, h > w)
        y1, y2 = _widen(y1, y2, w - h, H, w > h)
        w, h = x2 - x1, y2 - y1
        dx = w - H
        shrink_x = w > H
        x1 = np.where(shrink_x, x1 + dx // 2, x1)
        x2 = np.where(shrink_x, x2 - (dx - dx // 2), x2)
        dy = h - W
        shrink_y = ~shrink_x & (h > W)
        y1 = np.where(shrink_y, y1 + dy // 2, y1)
        y2 = np.where(shrink_y, y2 - (dy - dy // 2), y2)
    return x1, y1, x2, y2


def rows_to_crops(rows_per_frame, img_size, mscore=0.4, msize=50, mborder=5, scale=(1.5, 1.5, 2.2, 1.2),
                  square=True, frame_offset=0, do_adjust=True):
    """process_frames_batch 139-145: per frame filter + adjust, flattened in (frame, face) order
    -> (int32 [N,5] frame_offset + frame, x1, y1, x2, y2; int64 [N] source row within its frame)."""
    out, src = [], []
    for f, rows in enumerate(rows_per_frame):
        rows = np.asarray(rows, np.float32).reshape(-1, 5)
        keep = passes(rows, img_size, mscore, msize, mborder)
        x1, y1, x2, y2, _ = _round_out(rows[keep])
        if do_adjust:
            x1, y1, x2, y2 = adjust(x1, y1, x2, y2, img_size, scale, square)
        out.append(np.stack([np.full_like(x1, frame_offset + f), x1, y1, x2, y2], 1))
        src.append(np.nonzero(keep)[0])
    if not out:
        return np.zeros((0, 5), np.int32), np.zeros(0, np.int64)
    return np.concatenate(out).astype(np.int32), np.concatenate(src)
