"""GPU parity: ViT-B/16 and ViT-L/16 encoders vs reference goldens (encoders/vit.py)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def g():
    return np.load(os.path.join(GOLDEN, 'vit.npz'))


@pytest.mark.parametrize('precision', ['fp32', 'f16x'])
@pytest.mark.parametrize('isL', [False, True])
def test_vit_fp32_vs_golden(g, isL, precision):
    """Both GEMM operand modes (fp32 MFMA; split-fp16 fp32-grade products) at the fp32 tolerance."""
    from videotofaces.encoders.vit import ViT
    m = ViT('cuda:0', isL=isL, precision=precision)
    x = (torch.from_numpy(g['u8']).float() - 127.5) * np.float32(1 / 127.5)
    if isL:
        x = x[:1]
    emb = m(x).cpu().numpy()
    ref = g['vit_l' if isL else 'vit_b']
    err = np.abs(emb - ref).max()
    print('vit', 'L' if isL else 'B', precision, 'max abs err', err)
    # north-star fp32 tolerance; outputs are LayerNorm'ed (|x| ~ 0.8)
    np.testing.assert_allclose(emb, ref, atol=1e-4, rtol=0)


def test_vit_encode_crops_matches_blob_path():
    from videotofaces import synth
    from videotofaces.encoders.vit import ViT
    from videotofaces.encoders.facenet import blob_from_images
    m = ViT('cuda:0')
    fr = synth.make_frames(1, 240, 320, seed=8)
    crops = np.array([[0, 20, 10, 200, 230], [0, 100, 50, 228, 178]], np.int32)
    a = m.encode_crops(torch.from_numpy(fr).cuda(), crops).cpu().numpy()
    imgs = [fr[0, y1:y2, x1:x2] for _, x1, y1, x2, y2 in crops]
    b = m(blob_from_images(imgs, 128, 127.5, 1 / 127.5, torch.device('cuda:0'))).cpu().numpy()
    np.testing.assert_array_equal(a, b)


def test_vit_split_guard_falls_back_to_fp32(g):
    """An operand past the fp16 range (>= 2^14) trips the guard: the f16x handle re-runs the
    forward on fp32 MFMA, so its output equals the fp32 handle's bit for bit."""
    from videotofaces.encoders.vit import ViT
    x = (torch.from_numpy(g['u8']).float() - 127.5) * np.float32(1 / 127.5)
    x = x * 40000.0
    a = ViT('cuda:0', precision='f16x')(x).cpu().numpy()
    b = ViT('cuda:0', precision='fp32')(x).cpu().numpy()
    np.testing.assert_array_equal(a, b)
