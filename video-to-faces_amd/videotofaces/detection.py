"""Detection stage host logic (drop-in for src/videotofaces/detection.py).

get_detector_model keeps the reference's style coupling (detection.py:22-29); detect_faces /
process_frames_batch mirror the detection stage (detection.py:32-158) with the frames of a
det-batch uploaded to HBM once (detector, average hashes of the crops).  The box
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


# ------------------------------------------------------------------ detection stage (detection.py:32-158)
def frame_source(path, video_reader='opencv'):
    """(n_frames, fps, read(indices) -> uint8 [B,H,W,3] BGR) for a video file (OpenCV, as
    detection.py:82-111), a .npy file of frames, or an in-memory uint8 array (fps 1)."""
    import numpy as np
    if isinstance(path, np.ndarray):
        arr = path
        return arr.shape[0], 1, lambda idx: arr[idx]
    if str(path).lower().endswith('.npy'):
        arr = np.load(path, mmap_mode='r')
        return arr.shape[0], 1, lambda idx: np.ascontiguousarray(arr[idx])
    try:
        import cv2
    except ImportError:
        raise RuntimeError('decoding %s needs OpenCV (cv2), which is not installed; pass frames as a .npy file or '
                           'a uint8 array [F,H,W,3] instead' % path)
    cap = cv2.VideoCapture(path)
    n, fps = round(cap.get(cv2.CAP_PROP_FRAME_COUNT)), round(cap.get(cv2.CAP_PROP_FPS))
    state = {'c': 0}

    def read(idx):
        out = []
        step = idx[1] - idx[0] if len(idx) > 1 else 1
        for i in idx:
            if step > 50:
                cap.set(cv2.CAP_PROP_POS_FRAMES, i - 1)
                _, f = cap.read()
            else:
                for _ in range(state['c'], i + 1):
                    cap.grab()
                state['c'] = i + 1
                _, f = cap.retrieve()
            out.append(f)
        return np.stack(out)
    return n, fps, read


def process_frames_batch(frames, indices, model, det_params, save_params, hash_thr, hashes):
    """detection.py:126-158 with the frames uploaded to HBM once: detect, filter/adjust on the
    host (integer box logic), average hashes of the crops on device, nearest-5 hash dedupe,
    JPEG save.  Returns (file names, updated `hashes` list)."""
    import os.path as osp
    import numpy as np
    import torch
    from .dupes import ahash_crops, ahash, nearest_dupes
    from .utils import resize_keep_ratio, imwrite
    _, mscore, msize, mborder, scale, square = det_params
    out_dir, out_prefix, resize_to, _, _, _ = save_params
    imsize = frames.shape[1:3]
    fr_dev = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    boxes = normalize_detout(model(fr_dev))
    faces, rects = [], []
    for b, fi, fidx in zip(boxes, range(len(frames)), indices):
        bx = adjust_boxes(filter_boxes(b, imsize, mscore, msize, mborder), imsize, scale, square)
        for j, (x1, y1, x2, y2, _) in enumerate(bx):
            faces.append((frames[fi][y1:y2, x1:x2], out_prefix + '%06d_%u.jpg' % (fidx, j)))
            rects.append((fi, x1, y1, x2, y2))
    if resize_to:
        faces = [(resize_keep_ratio(img, resize_to), fn) for (img, fn) in faces]
    if hash_thr and hash_thr != -1 and faces:
        if resize_to:  # the reference hashes the resized face (detection.py:149-153)
            hs = [int(sum(int(v) << k for k, v in enumerate(ahash(img)))) for img, _ in faces]
        else:
            hs = ahash_crops(fr_dev, np.array(rects))
        flags, _ = nearest_dupes(list(zip(hs, [fn for _, fn in faces])), hashes, hash_thr)
        faces = [f for f, d in zip(faces, flags) if not d]
    for img, fn in faces:
        imwrite(osp.join(out_dir, 'faces', fn), np.ascontiguousarray(img))
    return [fn for _, fn in faces], hashes


def detect_faces(files, model, vid_params, det_params, save_params, hash_thr):
    """detection.py:32-65: every video in det-batches of sampled frames, then the overall hash
    dedupe.  Saving annotated frames / rejects (debug IO) is not mirrored."""
    import os
    import os.path as osp
    import numpy as np
    from .dupes import remove_dupes_overall, unpack_hash
    video_step, video_fragment, video_area, video_reader = vid_params
    bs = det_params[0]
    out_dir, out_prefix = save_params[0], save_params[1]
    os.makedirs(osp.join(out_dir, 'faces'), exist_ok=True)
    if len(files) > 1:
        print('File count: ' + str(len(files)))
    fnames, hashes_all = [], []
    for k, f in enumerate(files):
        print('Processing ' + (f if isinstance(f, str) else 'in-memory frames'))
        sp = (out_dir, out_prefix + ('' if len(files) == 1 else '%02d_' % (k + 1)), *save_params[2:])
        n, fps, read = frame_source(f, video_reader)
        step = max(1, round(fps * video_step))
        bgn = step if not video_fragment or video_fragment[0] < 0 else max(step, round(60 * video_fragment[0] * fps))
        end = n if not video_fragment or video_fragment[1] < 0 else min(n, round(60 * video_fragment[1] * fps + 1))
        fi = list(range(bgn, end, step))
        hashes = []
        for j in range(-(len(fi) // -bs)):
            bi = fi[bs * j:bs * (j + 1)]
            frames = read(bi)
            if video_area:
                cx1, cy1, cx2, cy2 = video_area
                frames = frames[:, cy1:cy2, cx1:cx2, :]
            fn_b, hashes = process_frames_batch(frames, bi, model, det_params, sp, hash_thr, hashes)
            fnames.extend(fn_b)
        hashes_all.extend(h for (h, _) in hashes)  # the kept faces' hashes (detection.py:123)
    if hash_thr and hash_thr != -1 and fnames:
        _, fnames = remove_dupes_overall(np.stack([unpack_hash(h) for h in hashes_all]), fnames,
                                         ('hash', hash_thr, save_params[5], out_dir))
    paths = [osp.join(out_dir, 'faces', fn) for fn in fnames]
    print()
    print('Saved a total of %u faces to: %s' % (len(paths), osp.join(out_dir, 'faces')))
    print()
    return paths
