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


@pytest.mark.parametrize('model', ['vit_b', 'vit_l'])
def test_load_real_vit_wconv(model, tmp_path):
    """AnimeVIT.wconv (vit.py:112-127): the checkpoint lists the positional embedding after the
    patch conv, each block's norm1 after its attention tensors and norm2 after its MLP, and
    carries text / decoder / MLM / classifier tensors the encoder drops.  Every tensor must
    land on its ViT parameter (value = spec index), the skipped ones nowhere."""
    sp = spec(model)
    idx = {n: i for i, (n, _) in enumerate(sp)}
    shp = {n: tuple(s) for n, s in sp}
    src = []

    def put(ref_name, key):
        src.append((key, torch.full(shp[ref_name], float(idx[ref_name]))))

    def junk(key):
        src.append((key, torch.full((3,), -1.0)))

    junk('text_embeddings.word.weight')
    put('class_token', 'model.cls_token')
    put('patch_embedding.weight', 'model.patch.w')
    put('patch_embedding.bias', 'model.patch.b')
    put('pos_embedding', 'model.positional_embedding.pe')
    depth = 24 if model == 'vit_l' else 12
    for b in range(depth):
        p = 'transformer.blocks.%d.' % b
        for t in ('attn.proj_q', 'attn.proj_k', 'attn.proj_v', 'proj'):
            put(p + t + '.weight', 'model.blk%d.%s.w' % (b, t))
            put(p + t + '.bias', 'model.blk%d.%s.b' % (b, t))
        put(p + 'norm1.weight', 'model.blk%d.norm1.w' % b)
        put(p + 'norm1.bias', 'model.blk%d.norm1.b' % b)
        for t in ('pwff.fc1', 'pwff.fc2'):
            put(p + t + '.weight', 'model.blk%d.%s.w' % (b, t))
            put(p + t + '.bias', 'model.blk%d.%s.b' % (b, t))
        put(p + 'norm2.weight', 'model.blk%d.norm2.w' % b)
        put(p + 'norm2.bias', 'model.blk%d.norm2.b' % b)
        if b == 3:
            junk('decoder.layer%d.w' % b)
    put('norm.weight', 'model.norm.w')
    put('norm.bias', 'model.norm.b')
    for k in ('mlm_head.dense.w', 'model.fc.weight', 'model.fc.bias', 'class_head.1.weight'):
        junk(k)
    path = tmp_path / (model + '.pt')
    torch.save(dict(src), path)
    p = synth.load_real(model, path)
    assert list(p) == [n for n, _ in sp]
    for i, (name, shape) in enumerate(sp):
        assert tuple(p[name].shape) == tuple(shape)
        assert np.all(p[name] == i), name


def test_load_real_facenet_drops_logits(tmp_path):
    """FaceNet.no_classify (facenet.py:165-168): the classifier tensors are popped wherever they
    sit in the checkpoint; everything else copies positionally."""
    sp = spec('facenet')
    src = {}
    for i, (_, shape) in enumerate(sp):
        if i == 5:
            src['logits.weight'] = torch.full((7, 512), -1.0)
        src['t%04d' % i] = torch.full(tuple(shape), float(i)) if len(shape) else torch.tensor(float(i))
    src['logits.bias'] = torch.full((7,), -1.0)
    path = tmp_path / 'facenet.pt'
    torch.save(src, path)
    p = synth.load_real('facenet', path)
    for i, (name, _) in enumerate(sp):
        assert np.all(p[name] == i), name


def test_load_real_shape_mismatch_names_the_tensor(tmp_path):
    sp = spec('mtcnn')
    src = {'t%03d' % i: torch.zeros(tuple(s)) for i, (_, s) in enumerate(sp)}
    src['t002'] = torch.zeros(5)
    path = tmp_path / 'mtcnn.pt'
    torch.save(src, path)
    with pytest.raises(ValueError, match='t002'):
        synth.load_real('mtcnn', path)


def test_load_real_refuses_pickled_objects(tmp_path):
    """weights_only=True: a checkpoint holding an arbitrary object is refused, not executed."""
    path = tmp_path / 'bad.pt'
    torch.save({'x': object()}, path)
    with pytest.raises(Exception):
        synth.load_real('mtcnn', path)
