"""Known-answer tests of the reference (tests/test_*.py of sephirot-github/video-to-faces) with
REAL weights: they run when the reference's checkpoints are supplied locally and skip cleanly
otherwise (the weights are remote downloads, unreachable here).

* checkpoints: $VTF_WEIGHTS_DIR or ./weights, under the reference's own file names
  (utils/weights.py:51-72: mtcnn_joined.pt, yolov3_wider.pt, frcnn_anime.pt, facenet_vgg.pt,
  vit_anime_b16.pt), read with torch.load(weights_only=True) and converted by synth.load_real;
* images: tests/kat_images/ -- the reference's test JPEGs (tests/images/, data fixtures);
  decoded with cv2.imread when OpenCV is importable, else Pillow (libjpeg either way; a decoder
  whose IDCT differs from OpenCV's can move the 4th decimal, which these KATs would report);
* expected values: the numbers of the reference's assertions, cited file:line.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
IMG = os.path.join(HERE, 'kat_images')
WDIR = os.environ.get('VTF_WEIGHTS_DIR', os.path.join(os.getcwd(), 'weights'))


def _weights(name):
    p = os.path.join(WDIR, name + '.pt')
    if not os.path.isfile(p):
        pytest.skip('real weights %s not supplied (set VTF_WEIGHTS_DIR); the reference downloads them' % p)
    return p


def _imread(name):
    p = os.path.join(IMG, name)
    try:
        import cv2
        return cv2.imread(p)
    except ImportError:
        from PIL import Image
        return np.asarray(Image.open(p).convert('RGB'))[:, :, ::-1].copy()


def test_kat_mtcnn():
    """tests/test_mtcnn.py:12-26"""
    from videotofaces.detectors.mtcnn import RealMTCNN
    m = RealMTCNN('cuda:0', min_face_size=20, weights=_weights('mtcnn_joined'))
    res = m([_imread('irl_det_%u.jpg' % i) for i in (1, 2, 3, 4)])
    assert [r.shape for r in res] == [(15, 5), (5, 5), (51, 5), (28, 5)]
    np.testing.assert_almost_equal(res[0][7], [682.8788, 122.9998, 739.7405, 192.9459, 0.9997], decimal=4)
    np.testing.assert_almost_equal(res[1][-1], [927.6433, 221.3357, 974.1216, 276.0959, 0.9989], decimal=4)
    np.testing.assert_almost_equal(res[2][44], [162.0115, 53.9863, 173.8801, 67.2544, 0.8978], decimal=4)
    np.testing.assert_almost_equal(res[3][22], [150.9578, 234.9925, 199.8160, 301.9932, 0.9934], decimal=4)


def test_kat_yolo():
    """tests/test_yolo.py:12-26"""
    from videotofaces.detectors.yolo import RealYOLO
    m = RealYOLO('cuda:0', weights=_weights('yolov3_wider'))
    b, s, _ = m([_imread('irl_det_%u.jpg' % i) for i in (1, 2, 3, 4)])
    res = [np.hstack([b[i], s[i][:, None]]) for i in range(len(b))]
    assert [r.shape for r in res] == [(20, 5), (10, 5), (100, 5), (93, 5)]
    np.testing.assert_almost_equal(res[0][10], [286.4944, 335.9040, 354.3441, 426.0989, 0.9969], decimal=4)
    np.testing.assert_almost_equal(res[3][25], [460.0020, 143.5856, 493.6367, 193.8361, 0.8309], decimal=4)


def test_kat_rcnn():
    """tests/test_rcnn.py:12-30"""
    from videotofaces.detectors.rcnn import AnimeFRCNN
    m = AnimeFRCNN('cuda:0', weights=_weights('frcnn_anime'))
    b, s, _ = m([_imread('anime_det_%u.jpg' % i) for i in (1, 2, 3, 4)])
    assert [x.shape for x in b] == [(14, 4), (64, 4), (6, 4), (4, 4)]
    np.testing.assert_almost_equal(b[0][10], [751.9342, 276.2107, 783.7333, 311.8178], decimal=4)
    np.testing.assert_almost_equal(b[1][50], [329.8422, 381.0872, 367.5275, 419.2162], decimal=4)
    np.testing.assert_almost_equal(b[2][3], [404.4612, 164.2291, 520.1513, 310.8856], decimal=4)
    np.testing.assert_almost_equal(b[3][1], [752.1040, 98.5442, 1095.4589, 422.9254], decimal=4)
    np.testing.assert_almost_equal(s[0][5:10], [0.9873, 0.9793, 0.9594, 0.9509, 0.8711], decimal=4)
    np.testing.assert_almost_equal(s[1][-5:], [0.6398, 0.5793, 0.5513, 0.4126, 0.2921], decimal=4)
    np.testing.assert_almost_equal(s[2], [0.9989, 0.9956, 0.7671, 0.7199, 0.6205, 0.0755], decimal=4)
    np.testing.assert_almost_equal(s[3], [0.9991, 0.9988, 0.9988, 0.9686], decimal=4)


def test_kat_facenet():
    """tests/test_facenet.py:12-22"""
    from videotofaces.encoders.facenet import FaceNet
    m = FaceNet('cuda:0', weights=_weights('facenet_vgg'))
    emb = m([_imread('irl_enc_%u.jpg' % i) for i in (1, 2, 3, 4)])
    assert emb.shape == (4, 512)
    np.testing.assert_almost_equal(emb[0][100:108], [0.0068, -0.0066, -0.0551, -0.0322, -0.0331, -0.0548, 0.0612,
                                                     -0.0518], decimal=4)
    np.testing.assert_almost_equal(emb[1][:8], [-0.0300, 0.0069, -0.0658, -0.0612, 0.0508, -0.0651, 0.0128, 0.0467],
                                   decimal=4)
    np.testing.assert_almost_equal(emb[2][-8:], [-0.0204, 0.0470, 0.0248, 0.0154, -0.0144, -0.0156, 0.0506, -0.0088],
                                   decimal=4)
    np.testing.assert_almost_equal(emb[3][400:408], [0.0297, -0.0122, -0.0281, 0.0492, -0.0473, 0.0425, -0.0185,
                                                     -0.0171], decimal=4)


def test_kat_vit():
    """tests/test_vit.py:12-20"""
    from videotofaces.encoders.vit import AnimeVIT
    m = AnimeVIT('cuda:0', weights=_weights('vit_anime_b16'))
    emb = m([_imread('anime_enc_%u.jpg' % i) for i in (1, 2)])
    assert emb.shape == (2, 768)
    np.testing.assert_almost_equal(emb[0][100:105], [-0.4530, -2.1694, 0.0624, -0.7991, -0.3798], decimal=4)
    np.testing.assert_almost_equal(emb[1][640:645], [0.3255, -0.6816, -0.1108, 0.2946, 1.7022], decimal=4)
