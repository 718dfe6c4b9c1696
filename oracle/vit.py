"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

CPU restatement of ViT (src/videotofaces/encoders/vit.py:9-102) with torch-CPU functional
ops; pinned against tests/golden/vit.npz (reference module outputs).
"""
import numpy as np
import torch
import torch.nn.functional as F


def vit(params, x, dim, depth):
    P = {k: torch.from_numpy(np.asarray(v)) for k, v in params.items()}
    heads = dim // 64
    with torch.inference_mode():
        x = F.conv2d(x, P['patch_embedding.weight'], P['patch_embedding.bias'], stride=16)
        x = x.flatten(2).transpose(1, 2)
        x = torch.cat((P['class_token'].expand(x.shape[0], -1, -1), x), dim=1)
        x = x + P['pos_embedding']
        for i in range(depth):
            p = 'transformer.blocks.%d.' % i
            h = F.layer_norm(x, (dim,), P[p + 'norm1.weight'], P[p + 'norm1.bias'], 1e-12)
            q, k, v = [F.linear(h, P[p + 'attn.proj_%s.weight' % n], P[p + 'attn.proj_%s.bias' % n]) for n in 'qkv']
            q, k, v = [t.view(*t.shape[:2], heads, -1).transpose(1, 2) for t in (q, k, v)]
            s = F.softmax(q @ k.transpose(2, 3) / (64 ** .5), dim=-1)
            h = (s @ v).transpose(1, 2).reshape(*x.shape[:2], -1)
            x = x + F.linear(h, P[p + 'proj.weight'], P[p + 'proj.bias'])
            h = F.layer_norm(x, (dim,), P[p + 'norm2.weight'], P[p + 'norm2.bias'], 1e-12)
            h = F.linear(F.gelu(F.linear(h, P[p + 'pwff.fc1.weight'], P[p + 'pwff.fc1.bias'])),
                         P[p + 'pwff.fc2.weight'], P[p + 'pwff.fc2.bias'])
            x = x + h
        return F.layer_norm(x[:, 0], (dim,), P['norm.weight'], P['norm.bias'], 1e-12)
