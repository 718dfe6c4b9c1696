"""Detection stage host logic (drop-in for src/videotofaces/detection.py).

get_detector_model keeps the reference's style coupling (detection.py:22-29).  The box
post-processing (filter_boxes 174-217, adjust_boxes 220-262, get_crops 161-162) is the
reference's integer logic, kept on the host (a few boxes per frame); frames may stay in HBM:
``detect_and_crop`` returns crop rectangles that the encoder consumes on device
(vtf_facenet_encode_crops), replacing the reference's JPEG write/read hand-off.
"""
import numpy as np


def get_detector_model(style, det_model, device):
    if style == 'anime':
        from .detectors.rcnn import AnimeFRCNN
        return AnimeFRCNN(device)
    if style == 'live':
        if det_model == 'mtcnn':
            from .detectors.mtcnn import RealMTCNN
            return RealMTCNN(device)
        from .detectors.yolo import RealYOLO
        return RealYOLO(device)
    return 0


def check_box(box, img_size, mscore, msize, mborder):
    """detection.py:165-171"""
    x1, y1, x2, y2, score = box
    H, W = img_size
    c1 = score < mscore
    c2 = x2 - x1 < msize or y2 - y1 < msize
    c3 = mborder and (x1 < mborder or y1 < mborder or x2 > W - mborder or y2 > H - mborder)
    return (c1, c2, c3)


def filter_boxes(boxes, img_size, mscore, msize, mborder):
    """detection.py:174-180 (the rejects / frames saving side effects are IO, not here)."""
    boxes = [(int(np.floor(x1)), int(np.floor(y1)), int(np.ceil(x2)), int(np.ceil(y2)), score)
             for (x1, y1, x2, y2, score) in boxes]
    return [b for b in boxes if not any(check_box(b, img_size, mscore, msize, mborder))]


def adjust_boxes(boxes, img_size, scale, square):
    """detection.py:220-262"""
    if isinstance(scale, int):
        scale = (scale, scale, scale, scale)
    (sx1, sx2, sy1, sy2) = scale
    H, W = img_size
    adjusted = []
    for (x1, y1, x2, y2, score) in boxes:
        w, h = x2 - x1, y2 - y1
        xc, yc = x1 + w / 2, y1 + h / 2
        x1 = int(np.floor(max(0, xc - sx1 * w / 2)))
        x2 = int(np.ceil(min(W, xc + sx2 * w / 2)))
        y1 = int(np.floor(max(0, yc - sy1 * h / 2)))
        y2 = int(np.ceil(min(H, yc + sy2 * h / 2)))
        w, h = x2 - x1, y2 - y1
        if square:
            if h > w:
                d = h - w
                x1 -= d // 2
                x2 += d - d // 2
                if x1 < 0: x2 += abs(x1); x1 = 0; x2 = min(W, x2)  # noqa: E701,E702
                if x2 > W: x1 -= x2 - W; x2 = W; x1 = max(0, x1)  # noqa: E701,E702
            elif w > h:
                d = w - h
                y1 -= d // 2
                y2 += d - d // 2
                if y1 < 0: y2 += abs(y1); y1 = 0; y2 = min(H, y2)  # noqa: E701,E702
                if y2 > H: y1 -= y2 - H; y2 = H; y1 = max(0, y1)  # noqa: E701,E702
            w, h = x2 - x1, y2 - y1
            if w > H:
                d = w - H
                x1 += d // 2
                x2 -= d - d // 2
            elif h > W:
                d = h - W
                y1 += d // 2
                y2 -= d - d // 2
        adjusted.append((x1, y1, x2, y2, score))
    return adjusted


def get_crops(img, boxes):
    """detection.py:161-162"""
    return [img[y1: y2, x1: x2] for (x1, y1, x2, y2, _) in boxes]


DEFAULT_DET_PARAMS = dict(mscore=0.4, msize=50, mborder=5, scale=(1.5, 1.5, 2.2, 1.2), square=True)


def normalize_detout(detout):
    """detection.py:131-136: YOLO/RCNN tuples -> [n,5] arrays like MTCNN's."""
    if isinstance(detout, tuple):
        b, s, _ = detout
        return [np.concatenate((bi, si[:, None]), axis=1) for bi, si in zip(b, s)]
    return detout


def boxes_to_crops(detout, img_size, frame_offset=0, mscore=0.4, msize=50, mborder=5,
                   scale=(1.5, 1.5, 2.2, 1.2), square=True):
    """process_frames_batch steps 2-5 (detection.py:133-152): filter, adjust, flatten in
    (frame, face) order -> int32 [N,5] (frame index, x1, y1, x2, y2)."""
    out = []
    for i, b in enumerate(normalize_detout(detout)):
        bx = adjust_boxes(filter_boxes(b, img_size, mscore, msize, mborder), img_size, scale, square)
        out.extend((frame_offset + i, x1, y1, x2, y2) for (x1, y1, x2, y2, _) in bx)
    return np.array(out, np.int32).reshape(-1, 5)
