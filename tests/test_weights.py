"""Real-weight import: synth.load_real is the positional state_dict copy of
utils/weights.py:36-48 (plus the R-CNN RoI-head reorder of rcnn.py:159-166).  The real
checkpoints are not available offline, so these tests write checkpoints of the right shapes
under foreign names and check where every tensor lands."""
import numpy as np
import pytest
import torch

from videotofaces import synth
from videotofaces.specs import spec


def _ckpt(model, tmp_path, wrap=None):
    src = {}
    for i, (_, shape) in enumerate(spec(model)):
        src['src_%04d' % i] = torch.full(tuple(shape), float(i), dtype=torch.float32) if len(shape) else \
            torch.tensor(float(i))
    path = tmp_path / (model + '.pt')
    torch.save({wrap: src} if wrap else src, path)
    return path


@pytest.mark.parametrize('model', ['mtcnn', 'facenet', 'yolo'])
def test_load_real_positional(model, tmp_path):
    """Tensor i of the checkpoint becomes parameter i of the reference module, whatever its name."""
    p = synth.load_real(model, _ckpt(model, tmp_path))
    names = [n for n, _ in spec(model)]
    assert list(p) == names
    for i, (name, shape) in enumerate(spec(model)):
        assert tuple(p[name].shape) == tuple(shape)
        assert np.all(p[name] == i)


def test_load_real_rcnn_roi_head_reorder(tmp_path):
    """AnimeFRCNN.wconv (rcnn.py:158-165): the last 8 checkpoint tensors swap halves (MMDet
    stores the RoI head's representation FCs and its cls/reg FCs the other way round)."""
    sp = spec('rcnn')
    n = len(sp)
    # the checkpoint in MMDet order: module tensors n-8..n-5 stored last, n-4..n-1 before them
    ref_shapes = [tuple(s) for _, s in sp]
    mm_order = list(range(n - 8)) + list(range(n - 4, n)) + list(range(n - 8, n - 4))
    src = {'src_%04d' % j: torch.full(ref_shapes[i], float(i)) for j, i in enumerate(mm_order)}
    path = tmp_path / 'rcnn.pt'
    torch.save({'state_dict': src}, path)
    p = synth.load_real('rcnn', path)
    for i, (name, shape) in enumerate(sp):
        assert tuple(p[name].shape) == tuple(shape)
        assert np.all(p[name] == i), name


def test_load_real_refuses_pickled_objects(tmp_path):
    """weights_only=True: a checkpoint holding an arbitrary object is refused, not executed."""
    path = tmp_path / 'bad.pt'
    torch.save({'x': object()}, path)
    with pytest.raises(Exception):
        synth.load_real('mtcnn', path)
