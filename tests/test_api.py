"""CPU: the public API's host logic (prep.py mirror) and the end-to-end video_to_faces run on a
GPU (in-memory frames, YOLO + FaceNet, clustering) -- the reference's plugin surface."""
import os

import numpy as np
import pytest


def test_clusters_and_validation():
    from videotofaces import prep
    assert prep.get_clusters(None) == list(range(2, 9))
    assert prep.get_clusters('2-9') == list(range(2, 10))
    assert prep.get_clusters('5,3,3') == [3, 5]
    assert prep.get_clusters(4) == [4]
    assert prep.get_clusters('9-2') is None
    fr = np.zeros((1, 8, 8, 3), np.uint8)
    assert prep.validate_args('full', fr, None, 'live', 'clustering', 'opencv', 'yolo', 'facenet_vgg')
    assert not prep.validate_args('full', fr, None, 'live', 'clustering', 'opencv', 'yolo', 'vit_l')
    assert prep.validate_args('full', fr, None, 'live', 'clustering', 'opencv', 'yolo', 'vit_l', decoupled=True)
    assert not prep.validate_args('full', None, None, 'live', 'clustering', 'opencv', 'yolo', 'facenet_vgg')
    assert not prep.validate_args('both', fr, None, 'live', 'clustering', 'opencv', 'yolo', 'facenet_vgg')


def test_video_list_and_grouping_paths(tmp_path):
    from videotofaces import prep
    for n in ('b.mp4', 'a.mkv', 'c.txt'):
        (tmp_path / n).write_text('x')
    assert prep.get_video_list(str(tmp_path), 'mp4;mkv') == [str(tmp_path / 'a.mkv'), str(tmp_path / 'b.mp4')]
    (tmp_path / 'faces').mkdir()
    (tmp_path / 'faces' / 'f.jpg').write_text('x')
    assert prep.get_paths_for_grouping(str(tmp_path)) == [str(tmp_path / 'faces' / 'f.jpg')]


@pytest.mark.gpu
def test_video_to_faces_in_memory(tmp_path):
    from videotofaces import synth, video_to_faces
    frames = synth.make_frames(8, seed=3)
    video_to_faces(frames, style='live', out_dir=str(tmp_path), det_batch_size=4, det_min_size=10,
                   clusters='2-3', enc_batch_size=16, enc_dup_thr=-1)  # synthetic encoders: near-identical embeddings
    faces = os.path.join(str(tmp_path), 'faces')
    got = [os.path.join(dp, f) for dp, _, fs in os.walk(faces) for f in fs if f.endswith('.jpg')]
    assert got, 'no faces written'
    assert os.path.exists(os.path.join(faces, 'log_clustering.csv'))
