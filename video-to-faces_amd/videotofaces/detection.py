"""Detection stage host logic (drop-in for src/videotofaces/detection.py).

get_detector_model keeps the reference's style coupling (detection.py:22-29); detect_faces /
process_frames_batch mirror the detection stage (detection.py:32-158) with the frames of a
det-batch uploaded to HBM once (detector, average hashes of the crops).  The box
post-processing (filter_boxes 174-217, adjust_boxes 220-262, get_crops 161-162) runs on the
device (vtf_boxes_to_crops, csrc/boxes.hip) straight on the detector's rows in HBM:
``detect_crops`` returns device crop rectangles that the encoders consume on device
(vtf_*_encode_crops), replacing the reference's JPEG write/read hand-off.
"""
import ctypes

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


def _rows_to_crops(rows, img_size, params, frame_offset=0, device=None):
    """Host detector rows (list of [n_i,5] fp32 arrays, one per frame) through the device box
    kernel (vtf_boxes_to_crops) -> (crops int32 [N,5], source row per crop, per-frame counts)."""
    import torch
    from . import _native as nat
    dev = nat.require_gpu(device)
    B = len(rows)
    counts = np.array([len(r) for r in rows], np.int32)
    flat = np.concatenate([np.asarray(r, np.float32).reshape(-1, 5) for r in rows]) if B else np.zeros((0, 5), np.float32)
    n = flat.shape[0]
    if B == 0:
        return np.zeros((0, 5), np.int32), np.zeros(0, np.int32), counts
    d_rows = torch.from_numpy(np.ascontiguousarray(flat)).to(dev)
    d_crops = torch.empty((max(n, 1), 5), dtype=torch.int32, device=dev)
    d_src = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    fc = np.zeros(B, np.int32)
    m = ctypes.c_int64(0)
    H, W = int(img_size[0]), int(img_size[1])
    with torch.cuda.device(dev):
        nat.check(nat.lib().vtf_boxes_to_crops(nat.ptr(d_rows), counts.ctypes.data, B, H, W, ctypes.byref(params),
                                               int(frame_offset), nat.ptr(d_crops), nat.ptr(d_src), fc.ctypes.data,
                                               max(n, 1), ctypes.byref(m), nat.stream_ptr(dev)))
    k = m.value
    return d_crops[:k].cpu().numpy(), d_src[:k].cpu().numpy(), fc


def filter_boxes(boxes, img_size, mscore, msize, mborder, *debug_io, device=None):
    """filter_boxes (detection.py:174-217) on the device box kernel: integer-rounded boxes that
    pass check_box (score, size, border), as (x1, y1, x2, y2, score) tuples.  The reference's
    save_frames / save_rejects debug IO (its trailing arguments) is not mirrored.
    This per-call wrapper (one H2D, a launch and a D2H) keeps the reference's signature; the
    pipeline never calls it -- detect_crops runs the same kernel once per det-batch on the
    detector's device rows.  There is deliberately no host implementation in the product (the
    library is the only compute path; the test suite's numpy restatement is pinned by
    tests/golden/boxes.npz)."""
    from . import _native as nat
    b = np.asarray(boxes, np.float32).reshape(-1, 5)
    cr, src, _ = _rows_to_crops([b], img_size, nat.BoxParams.make(mscore, msize, mborder, adjust=False),
                                device=device)
    return [(int(c[1]), int(c[2]), int(c[3]), int(c[4]), b[i, 4]) for c, i in zip(cr, src)]


def adjust_boxes(boxes, img_size, scale, square, device=None):
    """adjust_boxes (detection.py:220-262) on the device box kernel; boxes are filter_boxes
    output (integer corners, score)."""
    from . import _native as nat
    b = np.asarray([tuple(x) for x in boxes], np.float32).reshape(-1, 5)
    keep_all = nat.BoxParams.make(float('-inf'), float('-inf'), 0, scale, square)
    cr, src, _ = _rows_to_crops([b], img_size, keep_all, device=device)
    return [(int(c[1]), int(c[2]), int(c[3]), int(c[4]), boxes[i][4]) for c, i in zip(cr, src)]


def get_crops(img, boxes):
    """detection.py:161-162: the frame slice of every (x1, y1, x2, y2, score) box."""
    out = []
    for b in boxes:
        x1, y1, x2, y2 = b[:4]
        out.append(img[y1:y2, x1:x2])
    return out


DEFAULT_DET_PARAMS = dict(mscore=0.4, msize=50, mborder=5, scale=(1.5, 1.5, 2.2, 1.2), square=True)


def normalize_detout(detout):
    """detection.py:131-136: YOLO/RCNN tuples -> [n,5] arrays like MTCNN's."""
    if isinstance(detout, tuple):
        b, s, _ = detout
        return [np.concatenate((bi, si[:, None]), axis=1) for bi, si in zip(b, s)]
    return detout


def boxes_to_crops(detout, img_size, frame_offset=0, mscore=0.4, msize=50, mborder=5,
                   scale=(1.5, 1.5, 2.2, 1.2), square=True, device=None):
    """process_frames_batch steps 2-5 (detection.py:133-152) for host detector output, on the
    device box kernel -> int32 [N,5] (frame_offset + frame, x1, y1, x2, y2) in (frame, face)
    order."""
    from . import _native as nat
    rows = normalize_detout(detout)
    cr, _, _ = _rows_to_crops(rows, img_size, nat.BoxParams.make(mscore, msize, mborder, scale, square),
                              frame_offset, device)
    return cr


def detect_crops(model, frames_dev, frame_offset=0, mscore=0.4, msize=50, mborder=5,
                 scale=(1.5, 1.5, 2.2, 1.2), square=True):
    """model(frames) + process_frames_batch steps 2-5 with nothing on the host but counts:
    -> (device int32 crops [N,5], host per-frame counts).  model: RealMTCNN / RealYOLO /
    AnimeFRCNN or their handles (their detect_crops)."""
    from . import _native as nat
    return model.detect_crops(frames_dev, nat.BoxParams.make(mscore, msize, mborder, scale, square), frame_offset)


# ------------------------------------------------------------------ detection stage (detection.py:32-158)
def frame_source(path, video_reader='opencv', device=None):
    """(n_frames, fps, read(indices) -> uint8 [B,H,W,3] BGR) for a video file (OpenCV, as
    detection.py:82-111), a YUV4MPEG2 stream (.y4m: decoded frames converted on the GPU, read()
    returns them in HBM of `device`, videotofaces/video.py), a .npy file of frames, or an
    in-memory uint8 array (fps 1)."""
    import numpy as np
    if isinstance(path, np.ndarray):
        arr = path
        return arr.shape[0], 1, lambda idx: arr[idx]
    if str(path).lower().endswith('.npy'):
        arr = np.load(path, mmap_mode='r')
        return arr.shape[0], 1, lambda idx: np.ascontiguousarray(arr[idx])
    if str(path).lower().endswith('.y4m'):
        from .video import Y4MReader
        r = Y4MReader(path)
        return r.n_frames, r.fps, lambda idx: r.read(idx, device)
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


class _HostFrames:
    """frames[fi][y1:y2, x1:x2] of device frames: only the face crops come back to the host."""

    def __init__(self, dev):
        self.dev = dev

    def __getitem__(self, fi):
        return _HostFrame(self.dev[fi])


class _HostFrame:
    def __init__(self, t):
        self.t = t

    def __getitem__(self, key):
        return self.t[key].cpu().numpy()


def process_frames_batch(frames, indices, model, det_params, save_params, hash_thr, hashes):
    """detection.py:126-158 with the frames uploaded to HBM once: detect and filter/adjust the
    boxes on device (detect_crops), average hashes of the crops on device, nearest-5 hash
    dedupe, JPEG save.  Returns (file names, updated `hashes` list)."""
    import os.path as osp
    import numpy as np
    import torch
    from .dupes import ahash_crops, ahash, nearest_dupes
    from .utils import resize_keep_ratio, imwrite
    from . import _native as nat
    _, mscore, msize, mborder, scale, square = det_params
    out_dir, out_prefix, resize_to, _, _, _ = save_params
    if isinstance(frames, torch.Tensor):  # frames already in HBM (a .y4m source; strided views are fine)
        fr_dev = frames.to(nat.device_of(model))
        frames = _HostFrames(fr_dev)
    else:
        fr_dev = torch.from_numpy(np.ascontiguousarray(frames)).to(nat.device_of(model))
    # detector + box post-processing on device; only the crop rectangles come back for the
    # JPEG slices and file names
    with torch.inference_mode():
        d_crops, _ = detect_crops(model, fr_dev, 0, mscore, msize, mborder, scale, square)
    rects = d_crops.cpu().numpy()
    faces, seen = [], {}
    for fi, x1, y1, x2, y2 in rects.tolist():
        j = seen.get(fi, 0)
        seen[fi] = j + 1
        faces.append((frames[fi][y1:y2, x1:x2], out_prefix + '%06d_%u.jpg' % (indices[fi], j)))
    if resize_to:
        faces = [(resize_keep_ratio(img, resize_to), fn) for (img, fn) in faces]
    if hash_thr and hash_thr != -1 and faces:
        if resize_to:  # the reference hashes the resized face (detection.py:149-153)
            hs = [int(sum(int(v) << k for k, v in enumerate(ahash(img, fr_dev.device)))) for img, _ in faces]
        else:
            hs = ahash_crops(fr_dev, rects)
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
    from . import _native as nat
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
        n, fps, read = frame_source(f, video_reader, nat.device_of(model))
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
