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


def test_vit_blob_128_matches_restated_inter_linear():
    """A-E3: AnimeVIT's blobFromImages(1/127.5, 128x128, 127.5, swapRB) (vit.py:141) on device vs
    the oracle's INTER_LINEAR restatement, bit-exact, for down- and up-sampled crops (incl. the
    224x224 crops of config 4)."""
    from videotofaces.encoders.facenet import blob_from_images
    from oracle.facenet import resize_linear_u8
    rng = np.random.default_rng(4)
    sizes = [(224, 224), (128, 128), (73, 91), (300, 211), (1, 5), (129, 127), (850, 870)]
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for (h, w) in sizes]
    out = blob_from_images(imgs, 128, 127.5, 1 / 127.5, torch.device('cuda:0')).cpu().numpy()
    for i, im in enumerate(imgs):
        r = resize_linear_u8(im, 128)[:, :, ::-1].transpose(2, 0, 1).astype(np.float32)
        np.testing.assert_array_equal(out[i], (r - 127.5) * np.float32(1 / 127.5), err_msg=str(sizes[i]))


def test_encode_crops_validates_host_crops():
    """Host crop lists are checked against the frames before anything is read (VTF_E_ARG); a
    device crop list with a bad frame index encodes a zero image instead of reading outside."""
    from videotofaces import synth
    from videotofaces.encoders.vit import ViT
    from videotofaces._native import NativeError
    m = ViT('cuda:0')
    fr = torch.from_numpy(synth.make_frames(2, 64, 96, seed=1)).cuda()
    for bad in ([2, 0, 0, 10, 10], [-1, 0, 0, 10, 10], [0, 5, 0, 5, 10], [0, 0, 0, 97, 10], [0, 0, 60, 10, 65]):
        with pytest.raises(NativeError, match='crop 0'):
            m.encode_crops(fr, np.array([bad], np.int32))
    good = np.array([[1, 0, 0, 96, 64]], np.int32)
    zero = torch.tensor([[7, 0, 0, 96, 64]], dtype=torch.int32, device='cuda:0')
    a = m.encode_crops(fr, torch.from_numpy(good).cuda()).cpu().numpy()
    np.testing.assert_array_equal(a, m.encode_crops(fr, good).cpu().numpy())
    z = m.encode_crops(fr, zero).cpu().numpy()
    ref = m(torch.full((1, 3, 128, 128), -1.0)).cpu().numpy()  # a zero image: (0 - 127.5) / 127.5
    np.testing.assert_array_equal(z, ref)
