"""Small host helpers (src/videotofaces/utils/image.py)."""


def crop_to_area(img, area):
    """utils/image.py:17-22"""
    h, w = img.shape[:2]
    px1, py1, px2, py2 = area
    x1, x2 = int(px1 * w), int(px2 * w + 1)
    y1, y2 = int(py1 * h), int(py2 * h + 1)
    return img[y1:y2, x1:x2, :]
