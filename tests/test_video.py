"""The frame source of process_video (src/videotofaces/detection.py:68-111) on YUV4MPEG2 streams:
container parsing and frame sampling on the CPU; on the GPU, vtf_yuv_to_bgr (csrc/video.hip)
bit for bit against the numpy restatement (oracle/yuv.py) and the whole video_to_faces run on a
.y4m file against the same run on the restatement's frames.  Against the reference's own decoder
(cv2 / FFmpeg / decord, all absent here) the conversion is parity-unpinned."""
import os

import numpy as np
import pytest

from oracle import yuv as oy


def write_y4m(*a, **k):
    from videotofaces.video import write_y4m as w
    return w(*a, **k)


def _planes(rng, B, H, W, chroma):
    return rng.integers(0, 256, (B, oy.frame_bytes(H, W, chroma)), dtype=np.uint8)


def test_y4m_parse_and_offsets(tmp_path):
    from videotofaces.video import Y4MReader
    rng = np.random.default_rng(0)
    H, W = 9, 17  # odd: chroma 5 x 9
    p = _planes(rng, 4, H, W, 420)
    f = str(tmp_path / 'a.y4m')
    write_y4m(f, p, H, W, fps='30000:1001', frame_params=[None, 'Ip', None, 'XFOO=1'])
    r = Y4MReader(f)
    assert (r.width, r.height, r.chroma, r.fps, r.n_frames, r.full_range) == (W, H, 420, 30, 4, False)
    assert r.frame_bytes == H * W + 2 * 5 * 9
    np.testing.assert_array_equal(r.planes([3, 0, 2]), p[[3, 0, 2]])
    r.close()
    # truncated last frame dropped; full-range tag; other chroma layouts
    with open(f, 'ab') as fh:
        fh.write(b'FRAME\n' + bytes(10))
    assert Y4MReader(f).n_frames == 4
    for chroma in (422, 444, 400):
        g = str(tmp_path / ('c%d.y4m' % chroma))
        q = _planes(rng, 2, 6, 10, chroma)
        write_y4m(g, q, 6, 10, chroma=chroma, extra=' XCOLORRANGE=FULL')
        r = Y4MReader(g)
        assert (r.chroma, r.full_range, r.n_frames, r.frame_bytes) == (chroma, True, 2, oy.frame_bytes(6, 10, chroma))
        np.testing.assert_array_equal(r.planes([1]), q[1:2])
    bad = tmp_path / 'b.y4m'
    bad.write_bytes(b'NOTY4M W2 H2\n')
    with pytest.raises(ValueError):
        Y4MReader(str(bad))
    with pytest.raises(IndexError):
        Y4MReader(f).planes([4])


def test_oracle_conversion_anchors():
    """BT.601 limited range: black (16, 128, 128) -> 0, white (235, 128, 128) -> 255, and the
    integer transform within 1 level of the float equations; a round trip through the test-data
    encoder stays within a few levels on smooth content."""
    H, W = 2, 2
    pl = np.array([[16] * 4 + [128, 128], [235] * 4 + [128, 128]], np.uint8)
    out = oy.yuv_to_bgr(pl, H, W)
    assert (out[0] == 0).all() and (out[1] == 255).all()
    rng = np.random.default_rng(1)
    p = _planes(rng, 3, 8, 8, 444)
    got = oy.yuv_to_bgr(p, 8, 8, 444).astype(np.float64)
    Y, U, V = (p[:, i * 64:(i + 1) * 64].reshape(3, 8, 8).astype(np.float64) for i in range(3))
    yy = 1.164 * np.maximum(Y - 16, 0)
    ref = np.stack([yy + 2.018 * (U - 128), yy - 0.813 * (V - 128) - 0.391 * (U - 128), yy + 1.596 * (V - 128)], -1)
    assert np.abs(got - np.clip(np.floor(ref + 0.5), 0, 255)).max() <= 1
    x = np.tile(np.linspace(40, 200, 16).astype(np.uint8)[None, None, :, None], (1, 16, 1, 3))
    from videotofaces import synth
    back = oy.yuv_to_bgr(synth.bgr_to_yuv420(x), 16, 16).astype(int)
    assert np.abs(back - x).max() <= 3


def test_sampling_matches_reference_rule():
    """detection.py:85-91: step = round(fps * video_step), begin at one step (or the fragment's
    start), end at the frame count (or the fragment's end + 1)."""
    assert oy.sample_indices(100, 30, 1) == list(range(30, 100, 30))
    assert oy.sample_indices(10000, 25, 2, (1, 2)) == list(range(1500, 3001, 50))
    assert oy.sample_indices(10000, 25, 2, (-1, 0.5)) == list(range(50, 751, 50))


@pytest.mark.gpu
@pytest.mark.parametrize('H,W,chroma,full', [(720, 1280, 420, False), (9, 17, 420, False), (9, 16, 420, False),
                                             (8, 12, 422, False), (8, 12, 420, True),
                                             (6, 8, 444, True), (5, 7, 400, False), (1080, 1920, 420, True)])
def test_yuv_to_bgr_bit_exact(H, W, chroma, full):
    import torch
    from videotofaces.video import yuv_to_bgr
    rng = np.random.default_rng(H * W + chroma)
    p = _planes(rng, 3, H, W, chroma)
    got = yuv_to_bgr(p, H, W, chroma, full).cpu().numpy()
    np.testing.assert_array_equal(got, oy.yuv_to_bgr(p, H, W, chroma, full))
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_yuv_to_bgr_strided_output():
    """output rows and frames at strides wider than the frame (a video_area-style view), and an
    input frame stride with padding; the bytes outside the frames stay untouched."""
    import torch
    from videotofaces import _native as nat
    H, W = 10, 12
    rng = np.random.default_rng(7)
    fb = oy.frame_bytes(H, W, 420)
    p = _planes(rng, 2, H, W, 420)
    pad = np.zeros((2, fb + 20), np.uint8)
    pad[:, :fb] = p
    d_in = torch.from_numpy(pad).cuda()
    big = torch.full((2, H + 3, W + 5, 3), 77, dtype=torch.uint8, device='cuda')
    view = big[:, 1:1 + H, 2:2 + W]
    nat.check(nat.lib().vtf_yuv_to_bgr(nat.ptr(d_in), 2, H, W, 420, 0, fb + 20, nat.ptr(view), view.stride(0),
                                       view.stride(1), nat.stream_ptr(torch.device('cuda:0'))))
    got = big.cpu().numpy()
    np.testing.assert_array_equal(got[:, 1:1 + H, 2:2 + W], oy.yuv_to_bgr(p, H, W))
    mask = np.ones(got.shape, bool)
    mask[:, 1:1 + H, 2:2 + W] = False
    assert (got[mask] == 77).all()


@pytest.mark.gpu
def test_y4m_read_sampled_frames(tmp_path):
    from videotofaces.video import Y4MReader
    rng = np.random.default_rng(3)
    H, W = 72, 128
    p = _planes(rng, 7, H, W, 420)
    f = str(tmp_path / 'v.y4m')
    write_y4m(f, p, H, W, fps='25:1')
    r = Y4MReader(f)
    idx = [6, 1, 3]
    got = r.read(idx).cpu().numpy()
    np.testing.assert_array_equal(got, oy.yuv_to_bgr(p[idx], H, W))
    assert r.read([]).shape == (0, H, W, 3)


@pytest.mark.gpu
def test_video_to_faces_on_y4m_matches_decoded_frames(tmp_path):
    """The whole detection stage on a .y4m file (decode + sampling + detection + crops + hash
    dedupe + JPEG save) writes the same faces, byte for byte, as the same call on the
    restatement's decoded frames passed as an array with the same frame sampling."""
    from videotofaces import synth, video_to_faces
    src = synth.make_frames(12, seed=5)
    H, W = src.shape[1:3]
    planes = synth.bgr_to_yuv420(src)
    f = str(tmp_path / 'clip.y4m')
    write_y4m(f, planes, H, W, fps='2:1')
    dec = oy.yuv_to_bgr(planes, H, W)
    # in-memory frames run at fps 1 with frame indices 0..: give them the y4m's sampled frames
    idx = oy.sample_indices(12, 2, 1.0)
    assert idx == list(range(2, 12, 2))
    kw = dict(mode='detection', style='live', det_batch_size=4, det_min_size=10, video_step=1.0)
    out_a = tmp_path / 'a'
    out_b = tmp_path / 'b'
    out_a.mkdir()
    out_b.mkdir()
    video_to_faces(f, out_dir=str(out_a), **kw)
    video_to_faces(np.ascontiguousarray(dec[[0] + idx]), out_dir=str(out_b), **kw)
    fa = sorted(os.listdir(out_a / 'faces'))
    fb = sorted(os.listdir(out_b / 'faces'))
    assert fa, 'no faces written from the y4m stream'
    assert sorted(_map_name(x, idx) for x in fa) == fb
    for x in fa:
        assert (out_a / 'faces' / x).read_bytes() == (out_b / 'faces' / _map_name(x, idx)).read_bytes()


def _map_name(name, idx):
    """y4m frame idx[j] is frame j + 1 of the in-memory array (which samples 1, 2, ...): the
    file name '<frame %06d>_<face>.jpg' of one run in the other's numbering."""
    stem, rest = name.split('_', 1)
    return '%06d' % (idx.index(int(stem)) + 1) + '_' + rest


@pytest.mark.gpu
def test_video_to_faces_on_y4m_with_video_area(tmp_path):
    """video_area on a .y4m source crops the device frames as a strided view (no copy): the faces
    equal the same call on the restatement's decoded frames with the same area."""
    from videotofaces import synth, video_to_faces
    src = synth.make_frames(8, seed=9)
    H, W = src.shape[1:3]
    planes = synth.bgr_to_yuv420(src)
    f = str(tmp_path / 'clip.y4m')
    write_y4m(f, planes, H, W, fps='1:1')
    dec = oy.yuv_to_bgr(planes, H, W)
    area = (101, 37, 1181, 683)
    kw = dict(mode='detection', style='live', det_batch_size=4, det_min_size=10, video_step=1.0, video_area=area)
    out_a, out_b = tmp_path / 'a', tmp_path / 'b'
    out_a.mkdir()
    out_b.mkdir()
    video_to_faces(f, out_dir=str(out_a), **kw)
    video_to_faces(np.ascontiguousarray(dec), out_dir=str(out_b), **kw)
    fa, fb = sorted(os.listdir(out_a / 'faces')), sorted(os.listdir(out_b / 'faces'))
    assert fa and fa == fb
    for x in fa:
        assert (out_a / 'faces' / x).read_bytes() == (out_b / 'faces' / x).read_bytes()
