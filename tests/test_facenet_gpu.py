"""GPU parity: FaceNet (InceptionResnetV1) on libvtf_hip.so vs reference goldens / oracle."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def g():
    return np.load(os.path.join(GOLDEN, 'facenet.npz'))


@pytest.fixture(scope='module')
def fp32():
    from videotofaces.encoders.facenet import InceptionResnetV1
    return InceptionResnetV1('cuda:0', precision='fp32')


def test_fp32_vs_golden(g, fp32):
    x = (torch.from_numpy(g['u8']).float() - 127.5) * (1 / 128)
    emb = fp32(x).cpu().numpy()
    # north-star tolerance for fp32 embeddings
    np.testing.assert_allclose(emb, g['emb'], atol=1e-4, rtol=0)
    np.testing.assert_allclose(np.linalg.norm(emb, axis=1), 1.0, atol=1e-5)


def test_bf16_drift_reported(g):
    from videotofaces.encoders.facenet import InceptionResnetV1
    m = InceptionResnetV1('cuda:0', precision='bf16')
    x = (torch.from_numpy(g['u8']).float() - 127.5) * (1 / 128)
    emb = m(x).cpu().numpy()
    cos = (emb * g['emb']).sum(1)
    print('bf16 vs fp32-reference cosine:', cos, 'max abs', np.abs(emb - g['emb']).max())
    assert cos.min() > 0.99


@pytest.mark.parametrize('n,split', [(128, '1'), (5, '1'), (1, '1'), (128, '0'), (5, '0')])
def test_bf16_fused_blocks_bit_identical(n, split, g, monkeypatch):
    """The fused bf16 blocks (csrc/facenet_fused.hip: Block17 and the Block35 branches one launch
    per block with the activations in LDS, the stem's 32-channel 3x3 convs as patch convs) run the
    unfused kernels' MFMA k order and epilogue arithmetic: with the unfused launches' small-grid
    split-K turned off in both runs (VTF_NO_SPLITK=1, every output one k-ordered chain) the two
    paths give the same embeddings bit for bit.  Block17's stage 4 runs as its own GEMM launch over
    the batch (VTF_B17_SPLIT=1) or inside the per-image launch (0, default).  The fused Block17 and
    Block8-middle kernels stream their weights from padded-stride copies (facenet_runtime.hip
    pad_rows, VTF_FN_WPAD), the unfused launches from the dense rows: equal bits check those too.
    The Block35 launch also runs its block tail (1x1 96 -> 256 + residual) on the rows it just
    wrote (VTF_B35_TAIL, default on) with the unfused conv's chain and epilogue.
    Both paths stay within the drift bar of the fp32 golden."""
    from videotofaces.encoders.facenet import InceptionResnetV1
    m = InceptionResnetV1('cuda:0', precision='bf16')
    u8 = torch.from_numpy(np.random.default_rng(n).integers(0, 256, (n, 3, 160, 160), dtype=np.uint8))
    x = (u8.float() - 127.5) * (1 / 128)
    monkeypatch.setenv('VTF_NO_SPLITK', '1')  # both runs: the layers outside the fused blocks too
    monkeypatch.setenv('VTF_B17_SPLIT', split)
    fused = m(x).cpu().numpy()
    monkeypatch.setenv('VTF_FN_FUSED', '0')
    plain = m(x).cpu().numpy()
    print('fused vs unfused (no split-K): max |diff| %.3g' % np.abs(fused - plain).max())
    np.testing.assert_array_equal(fused, plain)
    monkeypatch.delenv('VTF_NO_SPLITK')
    xg = (torch.from_numpy(g['u8']).float() - 127.5) * (1 / 128)
    for mode in ('1', '0'):
        monkeypatch.setenv('VTF_FN_FUSED', mode)
        e = m(xg).cpu().numpy()
        assert (e * g['emb']).sum(1).min() > 0.99, mode


@pytest.mark.parametrize('n', [128, 7])
def test_bf16_stem_head_bit_identical(n, monkeypatch):
    """k_stem_head (csrc/facenet_fused.hip: the blob of the device crops and conv2d_1a in one launch,
    the 160x160 blob kept in LDS) computes k_blob's pixels and k_conv's MFMA chain / epilogue for
    that layer: with split-K off in both runs the embeddings equal the unfused path's (k_blob to
    HBM, then k_conv) bit for bit.  Crops: 160x160 (the direct-copy case), smaller / larger than the
    blob, 1-pixel wide, at the frame edges and partly outside, and (device crops) a frame index
    outside the frames (a zero image)."""
    from videotofaces import synth
    from videotofaces.encoders.facenet import InceptionResnetV1
    m = InceptionResnetV1('cuda:0', precision='bf16')
    fr = torch.from_numpy(synth.make_frames(3, 240, 320, seed=5)).cuda()
    rng = np.random.default_rng(n)
    fixed = [[0, 0, 0, 160, 160], [1, 10, 20, 110, 130], [2, 100, 50, 320, 240], [0, 5, 5, 6, 200],
             [1, 300, 200, 340, 260], [2, 0, 0, 320, 240], [7, 0, 0, 50, 50]]
    rows = []
    for i in range(n):
        if i < len(fixed):
            rows.append(fixed[i])
            continue
        x1, y1 = int(rng.integers(0, 300)), int(rng.integers(0, 220))
        rows.append([int(rng.integers(0, 3)), x1, y1, x1 + int(rng.integers(1, 260)), y1 + int(rng.integers(1, 200))])
    crops = torch.tensor(rows, dtype=torch.int32, device='cuda')
    monkeypatch.setenv('VTF_NO_SPLITK', '1')
    fused = m.encode_crops(fr, crops).cpu().numpy()
    monkeypatch.setenv('VTF_FN_FUSED', '0')
    plain = m.encode_crops(fr, crops).cpu().numpy()
    print('stem head vs blob + k_conv: max |diff| %.3g' % np.abs(fused - plain).max())
    np.testing.assert_array_equal(fused, plain)


def test_blob_kernel_matches_restated_inter_linear():
    from videotofaces.encoders.facenet import blob_from_images
    from oracle.facenet import resize_linear_u8
    rng = np.random.default_rng(3)
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for (h, w) in [(160, 160), (73, 91), (300, 211), (1, 5), (161, 159)]]
    out = blob_from_images(imgs, 160, 127.5, 1 / 128, torch.device('cuda:0')).cpu().numpy()
    for i, im in enumerate(imgs):
        r = resize_linear_u8(im, 160)[:, :, ::-1].transpose(2, 0, 1).astype(np.float32)
        np.testing.assert_array_equal(out[i], (r - 127.5) * np.float32(1 / 128))


def test_encode_crops_vs_oracle(fp32):
    from videotofaces import synth
    from oracle.facenet import resize_linear_u8, inception_resnet_v1
    fr = synth.make_frames(2, 200, 320, seed=2)
    crops = np.array([[0, 10, 20, 110, 130], [1, 100, 50, 260, 190], [0, 0, 0, 160, 160], [1, 300, 150, 320, 200]], np.int32)
    emb = fp32.encode_crops(torch.from_numpy(fr).cuda(), crops).cpu().numpy()
    blobs = []
    for f, x1, y1, x2, y2 in crops:
        r = resize_linear_u8(fr[f, y1:y2, x1:x2], 160)[:, :, ::-1].transpose(2, 0, 1)
        blobs.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * (1 / 128))
    ref = inception_resnet_v1(synth.make_params('facenet'), torch.stack(blobs)).numpy()
    np.testing.assert_allclose(emb, ref, atol=1e-4)


@pytest.mark.parametrize('area', [None, (0.1, 0.05, 0.9, 0.8)])
def test_encode_faces_order_vs_oracle(tmp_path, area):
    """A-E5: grouping.encode_faces (grouping.py:29-40) over face files in batches of 3: the
    concatenated [N,512] rows are in path order and equal the oracle on the same images (PNG, so
    the file round trip is lossless), with and without enc_area (utils/image.py:17-22)."""
    from PIL import Image
    from videotofaces import synth
    from videotofaces.encoders.facenet import FaceNet
    from videotofaces.grouping import encode_faces
    from oracle.facenet import resize_linear_u8, inception_resnet_v1
    fr = synth.make_frames(1, 300, 400, seed=12)[0]
    rects = [(0, 0, 120, 150), (50, 40, 90, 70), (200, 100, 399, 299), (10, 200, 70, 300), (300, 0, 400, 64),
             (120, 120, 280, 280), (5, 5, 37, 29)]
    paths = []
    for i, (x1, y1, x2, y2) in enumerate(rects):
        p = str(tmp_path / ('face_%02d.png' % i))
        Image.fromarray(np.ascontiguousarray(fr[y1:y2, x1:x2, ::-1])).save(p)  # BGR frame -> RGB file
        paths.append(p)
    X = encode_faces(paths, FaceNet('cuda:0'), 3, area)
    blobs = []
    for x1, y1, x2, y2 in rects:
        im = fr[y1:y2, x1:x2]
        if area:
            h, w = im.shape[:2]
            im = im[int(area[1] * h):int(area[3] * h + 1), int(area[0] * w):int(area[2] * w + 1)]
        r = resize_linear_u8(im, 160)[:, :, ::-1].transpose(2, 0, 1)
        blobs.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * (1 / 128))
    ref = inception_resnet_v1(synth.make_params('facenet'), torch.stack(blobs)).numpy()
    assert X.shape == (len(rects), 512)
    np.testing.assert_allclose(X, ref, rtol=0, atol=1e-4)
