"""Parameter specs (name, shape) for every model on the hot path.

The names and their ORDER are exactly the reference modules' ``state_dict()`` keys, so
that (a) synthetic weights generated here can be loaded into the reference modules with
``load_state_dict`` when golden vectors are made, and (b) the native runtime can consume a
flat fp32 buffer in this order (``num_batches_tracked`` entries are skipped when packing).

Reference structures mirrored:
  MTCNN             src/videotofaces/detectors/mtcnn.py:12-121
  InceptionResnetV1 src/videotofaces/encoders/facenet.py:10-154 (+ backbones/basic.py:5-45)
  YOLOv3            src/videotofaces/detectors/yolo.py:17-129
  ViT               src/videotofaces/encoders/vit.py:9-102
"""


def _conv(prefix, cin, cout, kh, kw, bias=True):
    out = [(prefix + '.weight', (cout, cin, kh, kw))]
    if bias:
        out.append((prefix + '.bias', (cout,)))
    return out


def _bn(prefix, c):
    return [(prefix + '.weight', (c,)), (prefix + '.bias', (c,)),
            (prefix + '.running_mean', (c,)), (prefix + '.running_var', (c,)),
            (prefix + '.num_batches_tracked', ())]


def _lin(prefix, cin, cout, bias=True):
    out = [(prefix + '.weight', (cout, cin))]
    if bias:
        out.append((prefix + '.bias', (cout,)))
    return out


def _prelu(prefix, c):
    return [(prefix + '.weight', (c,))]


def _conv_unit(prefix, cin, cout, kh, kw):
    # backbones/basic.py:5-45 ConvUnit with bn -> conv has no bias
    return _conv(prefix + '.conv', cin, cout, kh, kw, bias=False) + _bn(prefix + '.bn', cout)


def mtcnn_spec():
    s = []
    # PNet mtcnn.py:12-25
    s += _conv('pnet.conv1', 3, 10, 3, 3) + _prelu('pnet.prelu1', 10)
    s += _conv('pnet.conv2', 10, 16, 3, 3) + _prelu('pnet.prelu2', 16)
    s += _conv('pnet.conv3', 16, 32, 3, 3) + _prelu('pnet.prelu3', 32)
    s += _conv('pnet.conv4_1', 32, 2, 1, 1) + _conv('pnet.conv4_2', 32, 4, 1, 1)
    # RNet mtcnn.py:41-56
    s += _conv('rnet.conv1', 3, 28, 3, 3) + _prelu('rnet.prelu1', 28)
    s += _conv('rnet.conv2', 28, 48, 3, 3) + _prelu('rnet.prelu2', 48)
    s += _conv('rnet.conv3', 48, 64, 2, 2) + _prelu('rnet.prelu3', 64)
    s += _lin('rnet.dense4', 576, 128) + _prelu('rnet.prelu4', 128)
    s += _lin('rnet.dense5_1', 128, 2) + _lin('rnet.dense5_2', 128, 4)
    # ONet mtcnn.py:79-99
    s += _conv('onet.conv1', 3, 32, 3, 3) + _prelu('onet.prelu1', 32)
    s += _conv('onet.conv2', 32, 64, 3, 3) + _prelu('onet.prelu2', 64)
    s += _conv('onet.conv3', 64, 64, 3, 3) + _prelu('onet.prelu3', 64)
    s += _conv('onet.conv4', 64, 128, 2, 2) + _prelu('onet.prelu4', 128)
    s += _lin('onet.dense5', 1152, 256) + _prelu('onet.prelu5', 256)
    s += _lin('onet.dense6_1', 256, 2) + _lin('onet.dense6_2', 256, 4) + _lin('onet.dense6_3', 256, 10)
    return s


def facenet_spec():
    s = []
    # stem facenet.py:126-134 (indices 0..6; 3 is MaxPool)
    stem = [(0, 3, 32, 3, 3), (1, 32, 32, 3, 3), (2, 32, 64, 3, 3),
            (4, 64, 80, 1, 1), (5, 80, 192, 3, 3), (6, 192, 256, 3, 3)]
    for i, cin, cout, kh, kw in stem:
        s += _conv_unit('stem.%d' % i, cin, cout, kh, kw)
    # 5 x Block35 facenet.py:14-33
    for b in range(5):
        p = 'main.0.%d' % b
        s += _conv_unit(p + '.branch0', 256, 32, 1, 1)
        s += _conv_unit(p + '.branch1.0', 256, 32, 1, 1) + _conv_unit(p + '.branch1.1', 32, 32, 3, 3)
        s += _conv_unit(p + '.branch2.0', 256, 32, 1, 1) + _conv_unit(p + '.branch2.1', 32, 32, 3, 3)
        s += _conv_unit(p + '.branch2.2', 32, 32, 3, 3)
        s += _conv(p + '.conv2d', 96, 256, 1, 1)
    # Mixed_6a facenet.py:84-101
    s += _conv_unit('main.1.branch0', 256, 384, 3, 3)
    s += _conv_unit('main.1.branch1.0', 256, 192, 1, 1) + _conv_unit('main.1.branch1.1', 192, 192, 3, 3)
    s += _conv_unit('main.1.branch1.2', 192, 256, 3, 3)
    # 10 x Block17 facenet.py:36-56
    for b in range(10):
        p = 'main.2.%d' % b
        s += _conv_unit(p + '.branch0', 896, 128, 1, 1)
        s += _conv_unit(p + '.branch1.0', 896, 128, 1, 1) + _conv_unit(p + '.branch1.1', 128, 128, 1, 7)
        s += _conv_unit(p + '.branch1.2', 128, 128, 7, 1)
        s += _conv(p + '.conv2d', 256, 896, 1, 1)
    # Mixed_7a facenet.py:104-120
    s += _conv_unit('main.3.branch0.0', 896, 256, 1, 1) + _conv_unit('main.3.branch0.1', 256, 384, 3, 3)
    s += _conv_unit('main.3.branch1.0', 896, 256, 1, 1) + _conv_unit('main.3.branch1.1', 256, 256, 3, 3)
    s += _conv_unit('main.3.branch2.0', 896, 256, 1, 1) + _conv_unit('main.3.branch2.1', 256, 256, 3, 3)
    s += _conv_unit('main.3.branch2.2', 256, 256, 3, 3)

    def block8(p):
        out = _conv_unit(p + '.branch0', 1792, 192, 1, 1)
        out += _conv_unit(p + '.branch1.0', 1792, 192, 1, 1) + _conv_unit(p + '.branch1.1', 192, 192, 1, 3)
        out += _conv_unit(p + '.branch1.2', 192, 192, 3, 1)
        out += _conv(p + '.conv2d', 384, 1792, 1, 1)
        return out
    # 5 x Block8 + Block8(relu=False) facenet.py:59-81, 142-143
    for b in range(5):
        s += block8('main.4.%d' % b)
    s += block8('main.5')
    # Linear 1792->512 (no bias) + BatchNorm1d facenet.py:146-147
    s += _lin('main.8', 1792, 512, bias=False) + _bn('main.9', 512)
    return s


def yolo_spec():
    s = []

    def cu(p, cin, cout, k):
        return _conv_unit(p, cin, cout, k, k)
    # Darknet53 yolo.py:34-47
    s += cu('backbone.conv1', 3, 32, 3)
    L, C = [1, 2, 8, 8, 4], [(32, 64), (64, 128), (128, 256), (256, 512), (512, 1024)]
    for i in range(5):
        p = 'backbone.conv_res_block%d' % (i + 1)
        s += cu(p + '.conv', C[i][0], C[i][1], 3)
        for j in range(L[i]):
            c = C[i][1]
            s += cu(p + '.res%d.conv1' % j, c, c // 2, 1) + cu(p + '.res%d.conv2' % j, c // 2, c, 3)

    # neck yolo.py:57-94
    def det_block(p, cin, cout):
        return (cu(p + '.layers.0', cin, cout, 1) + cu(p + '.layers.1', cout, cout * 2, 3)
                + cu(p + '.layers.2', cout * 2, cout, 1) + cu(p + '.layers.3', cout, cout * 2, 3)
                + cu(p + '.layers.4', cout * 2, cout, 1))
    cbone, cneck, chead = [256, 512, 1024], [128, 256, 512], [256, 512, 1024]
    s += det_block('neck.detect1', cbone[2], cneck[2])
    s += cu('neck.conv1', cneck[2], cneck[1], 1)
    s += det_block('neck.detect2', cbone[1] + cneck[1], cneck[1])
    s += cu('neck.conv2', cneck[1], cneck[0], 1)
    s += det_block('neck.detect3', cbone[0] + cneck[0], cneck[0])
    # head yolo.py:97-112
    for i, (ci, cm) in enumerate([(cneck[2], chead[2]), (cneck[1], chead[1]), (cneck[0], chead[0])]):
        s += cu('head.convs_bridge.%d' % i, ci, cm, 3)
    for i, cm in enumerate([chead[2], chead[1], chead[0]]):
        s += _conv('head.convs_pred.%d' % i, cm, 18, 1, 1)
    return s


def vit_spec(dim=768, depth=12, img=128, patch=16):
    s = [('class_token', (1, 1, dim)), ('pos_embedding', (1, (img // patch) ** 2 + 1, dim))]
    s += _conv('patch_embedding', 3, dim, patch, patch)
    for i in range(depth):
        p = 'transformer.blocks.%d' % i
        s += [(p + '.norm1.weight', (dim,)), (p + '.norm1.bias', (dim,))]
        s += _lin(p + '.attn.proj_q', dim, dim) + _lin(p + '.attn.proj_k', dim, dim) + _lin(p + '.attn.proj_v', dim, dim)
        s += _lin(p + '.proj', dim, dim)
        s += [(p + '.norm2.weight', (dim,)), (p + '.norm2.bias', (dim,))]
        s += _lin(p + '.pwff.fc1', dim, dim * 4) + _lin(p + '.pwff.fc2', dim * 4, dim)
    s += [('norm.weight', (dim,)), ('norm.bias', (dim,))]
    return s


def rcnn_spec():
    """FasterRCNN (detectors/rcnn.py:127-139): ResNet50 body (backbones/resnet.py:11-54,
    BN eps 1e-5), FPN (rcnn.py:16-31, ConvUnits with bias and no BN), RPN (34-47), RoI head
    (85-92)."""
    s = _conv_unit('body.layers.0.0', 3, 64, 7, 7)
    cin = 64
    for li, (w, n) in enumerate(zip((64, 128, 256, 512), (3, 4, 6, 3))):
        for b in range(n):
            p = 'body.layers.%d.%d' % (li + 1, b)
            stride = 2 if (b == 0 and li > 0) else 1
            s += _conv_unit(p + '.u1', cin, w, 1, 1) + _conv_unit(p + '.u2', w, w, 3, 3)
            s += _conv_unit(p + '.u3', w, w * 4, 1, 1)
            if stride > 1 or cin != w * 4:
                s += _conv_unit(p + '.downsample', cin, w * 4, 1, 1)
            cin = w * 4
    for i, c in enumerate((256, 512, 1024, 2048)):
        s += _conv('fpn.conv_laterals.%d.conv' % i, c, 256, 1, 1)
    for i in range(4):
        s += _conv('fpn.conv_smooths.%d.conv' % i, 256, 256, 3, 3)
    s += _conv('rpn.conv.conv', 256, 256, 3, 3) + _conv('rpn.log', 256, 3, 1, 1) + _conv('rpn.reg', 256, 12, 1, 1)
    s += _lin('roi.fc.0', 256 * 7 * 7, 1024) + _lin('roi.fc.1', 1024, 1024)
    s += _lin('roi.cls', 1024, 2) + _lin('roi.reg', 1024, 4)
    return s


SPECS = {
    'mtcnn': mtcnn_spec,
    'rcnn': rcnn_spec,
    'facenet': facenet_spec,
    'yolo': yolo_spec,
    'vit_b': lambda: vit_spec(768, 12),
    'vit_l': lambda: vit_spec(1024, 24),
}


def spec(model):
    return SPECS[model]()
