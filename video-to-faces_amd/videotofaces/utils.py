"""Small host helpers (src/videotofaces/utils/image.py)."""


def crop_to_area(img, area):
    """utils/image.py:17-22"""
    h, w = img.shape[:2]
    px1, py1, px2, py2 = area
    x1, x2 = int(px1 * w), int(px2 * w + 1)
    y1, y2 = int(py1 * h), int(py2 * h + 1)
    return img[y1:y2, x1:x2, :]


def resize_keep_ratio(img, to_area, upscale=True):
    """utils/image.py:4-14 (cv2.resize INTER_LINEAR restated on the host, uint8 fixed point)."""
    h, w = img.shape[:2]
    aw, ah = to_area if isinstance(to_area, tuple) else (to_area, to_area)
    scale = min(aw / w, ah / h)
    if scale != 1 and (upscale or scale < 1):
        img = resize_linear(img, int(h * scale), int(w * scale))
    return img


def _lin_coefs(src, dst):
    import numpy as np
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * (1.0 / (dst / src)) - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0, 0
    edge = s >= src - 1
    f[edge], s[edge] = 0, src - 1
    c0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    c1 = np.rint(f * np.float32(2048)).astype(np.int64)
    return s, np.minimum(s + 1, src - 1), c0, c1, edge


def resize_linear(img, H, W):
    """OpenCV uint8 INTER_LINEAR resize of an HxWx3 image (the kernels' lin_coef arithmetic)."""
    import numpy as np
    h, w = img.shape[:2]
    if (h, w) == (H, W):
        return img.copy()
    sx0, sx1, a0, a1, ex = _lin_coefs(w, W)
    sy0, sy1, b0, b1, _ = _lin_coefs(h, H)
    src = img.astype(np.int64)

    def hrow(rows):
        r = src[rows]
        v = r[:, sx0] * a0[None, :, None] + r[:, sx1] * a1[None, :, None]
        v[:, ex] = r[:, sx0[ex]] * 2048
        return v
    h0, h1 = hrow(sy0), hrow(sy1)
    t = (((h0 >> 4) * b0[:, None, None]) >> 16) + (((h1 >> 4) * b1[:, None, None]) >> 16)
    return np.clip((t + 2) >> 2, 0, 255).astype(np.uint8)


def imwrite(path, img):
    """cv2.imwrite of a BGR uint8 image (Pillow when OpenCV is absent)."""
    try:
        import cv2
        return cv2.imwrite(path, img)
    except ImportError:
        from PIL import Image
        Image.fromarray(img[:, :, ::-1]).save(path, quality=95)
        return True
