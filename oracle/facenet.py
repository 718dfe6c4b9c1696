"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

CPU restatement of InceptionResnetV1 (src/videotofaces/encoders/facenet.py:10-154) with
torch-CPU functional ops, and of FaceNet.__call__'s blob step (facenet.py:178-183) for the
post-resize tensor.  Pinned against tests/golden/facenet.npz (reference module outputs).
"""
import numpy as np
import torch
import torch.nn.functional as F


class _P:
    def __init__(self, params):
        self.p = {k: torch.from_numpy(np.asarray(v)) for k, v in params.items()}

    def __getitem__(self, k):
        return self.p[k]


def _cu(P, x, pre, s=1, p=0):
    """conv_unit: Conv2d(no bias) -> BatchNorm2d(eps 1e-3) -> ReLU (facenet.py:10-11, basic.py:38-45)"""
    x = F.conv2d(x, P[pre + '.conv.weight'], None, s, p)
    x = F.batch_norm(x, P[pre + '.bn.running_mean'], P[pre + '.bn.running_var'], P[pre + '.bn.weight'],
                     P[pre + '.bn.bias'], False, 0.0, 1e-3)
    return F.relu(x, inplace=True)  # nn.ReLU(inplace=True) (basic.py:26): same values


def _block35(P, x, pre, scale):
    x0 = _cu(P, x, pre + '.branch0')
    x1 = _cu(P, _cu(P, x, pre + '.branch1.0'), pre + '.branch1.1', p=1)
    x2 = _cu(P, _cu(P, _cu(P, x, pre + '.branch2.0'), pre + '.branch2.1', p=1), pre + '.branch2.2', p=1)
    out = F.conv2d(torch.cat((x0, x1, x2), 1), P[pre + '.conv2d.weight'], P[pre + '.conv2d.bias'])
    return F.relu(out * scale + x)


def _block17(P, x, pre, scale):
    x0 = _cu(P, x, pre + '.branch0')
    x1 = _cu(P, x, pre + '.branch1.0')
    x1 = _cu(P, x1, pre + '.branch1.1', p=(0, 3))
    x1 = _cu(P, x1, pre + '.branch1.2', p=(3, 0))
    out = F.conv2d(torch.cat((x0, x1), 1), P[pre + '.conv2d.weight'], P[pre + '.conv2d.bias'])
    return F.relu(out * scale + x)


def _block8(P, x, pre, scale, relu=True):
    x0 = _cu(P, x, pre + '.branch0')
    x1 = _cu(P, x, pre + '.branch1.0')
    x1 = _cu(P, x1, pre + '.branch1.1', p=(0, 1))
    x1 = _cu(P, x1, pre + '.branch1.2', p=(1, 0))
    out = F.conv2d(torch.cat((x0, x1), 1), P[pre + '.conv2d.weight'], P[pre + '.conv2d.bias'])
    out = out * scale + x
    return F.relu(out) if relu else out


def inception_resnet_v1(params, x):
    """InceptionResnetV1.forward (facenet.py:150-154): [N,3,160,160] -> [N,512] L2-normalised."""
    P = _P(params)
    with torch.inference_mode():
        x = _cu(P, x, 'stem.0', s=2)
        x = _cu(P, x, 'stem.1')
        x = _cu(P, x, 'stem.2', p=1)
        x = F.max_pool2d(x, 3, 2)
        x = _cu(P, x, 'stem.4')
        x = _cu(P, x, 'stem.5')
        x = _cu(P, x, 'stem.6', s=2)
        for b in range(5):
            x = _block35(P, x, 'main.0.%d' % b, 0.17)
        x0 = _cu(P, x, 'main.1.branch0', s=2)
        x1 = _cu(P, _cu(P, _cu(P, x, 'main.1.branch1.0'), 'main.1.branch1.1', p=1), 'main.1.branch1.2', s=2)
        x = torch.cat((x0, x1, F.max_pool2d(x, 3, 2)), 1)
        for b in range(10):
            x = _block17(P, x, 'main.2.%d' % b, 0.1)
        x0 = _cu(P, _cu(P, x, 'main.3.branch0.0'), 'main.3.branch0.1', s=2)
        x1 = _cu(P, _cu(P, x, 'main.3.branch1.0'), 'main.3.branch1.1', s=2)
        x2 = _cu(P, _cu(P, _cu(P, x, 'main.3.branch2.0'), 'main.3.branch2.1', p=1), 'main.3.branch2.2', s=2)
        x = torch.cat((x0, x1, x2, F.max_pool2d(x, 3, 2)), 1)
        for b in range(5):
            x = _block8(P, x, 'main.4.%d' % b, 0.2)
        x = _block8(P, x, 'main.5', 1.0, relu=False)
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        x = F.linear(x, P['main.8.weight'])
        x = F.batch_norm(x, P['main.9.running_mean'], P['main.9.running_var'], P['main.9.weight'], P['main.9.bias'],
                         False, 0.0, 1e-3)
        return F.normalize(x, p=2, dim=1)


def blob_from_u8_nchw(u8, mean=127.5, scale=1 / 128):
    """blobFromImages tail for an already-sized RGB uint8 NCHW tensor: (x - mean) * scale."""
    return (u8.float() - mean) * scale


def _coefs(src, dst):
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


def resize_linear_u8(img, S):
    """OpenCV uint8 INTER_LINEAR (resizeGeneric_ fixed point + SIMD vertical rounding), numpy.
    cv2 is absent here: this restatement is parity-UNPINNED (used to check the GPU kernel)."""
    h, w = img.shape[:2]
    if (h, w) == (S, S):
        return img.copy()
    sx0, sx1, a0, a1, ex = _coefs(w, S)
    sy0, sy1, b0, b1, _ = _coefs(h, S)
    src = img.astype(np.int64)

    def hrow(rows):
        r = src[rows]                                   # [S, w, C]
        v = r[:, sx0] * a0[None, :, None] + r[:, sx1] * a1[None, :, None]
        v[:, ex] = r[:, sx0[ex]] * 2048
        return v
    h0, h1 = hrow(sy0), hrow(sy1)
    t = (((h0 >> 4) * b0[:, None, None]) >> 16) + (((h1 >> 4) * b1[:, None, None]) >> 16)
    return np.clip((t + 2) >> 2, 0, 255).astype(np.uint8)
