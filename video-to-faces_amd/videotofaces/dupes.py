"""Near-duplicate removal (drop-in for src/videotofaces/dupes.py).

The embedding branch of remove_dupes_overall (dupes.py:51-68) runs on the GPU as one fused
cosine-distance + strict-lower-triangle row-min kernel (vtf_cosine_dedupe): no N x N
matrix (the reference materialises an fp32 N x N plus an fp64 N x N mask).
"""
import ctypes
import os
import os.path as osp

import numpy as np
import torch

from . import _native as nat


def cosine_dedupe_device(X):
    """X: CUDA fp32 [N,D] -> (mins f32 [N], inds i64 [N]) exactly as dupes.py:60-64 computes
    them: min / first argmin over j < i of clip(1 - cos(X_i, X_j), 0, 2); row 0 -> (10000, 0)."""
    X = X.to(torch.float32).contiguous()
    n, d = X.shape
    mins = torch.empty(n, dtype=torch.float32, device=X.device)
    inds = torch.empty(n, dtype=torch.int64, device=X.device)
    nat.check(nat.lib().vtf_cosine_dedupe(nat.ptr(X), n, d, nat.ptr(mins), nat.ptr(inds), nat.stream_ptr(X.device)))
    return mins.cpu().numpy(), inds.cpu().numpy()


def hamming_lower(H):
    """hash branch (dupes.py:55-57): Hamming distances of 64-bit average hashes, strict lower
    triangle min/argmin (host numpy; the GPU popcount kernel is the next §8f item)."""
    H = np.asarray(H).astype(np.uint8)
    n = H.shape[0]
    D = (H[:, None, :] != H[None, :, :]).sum(2).astype(np.uint16) if n else np.zeros((0, 0), np.uint16)
    D = D + (1 - np.tri(n, k=-1).astype(D.dtype)) * 10000
    return D.min(axis=1), D.argmin(axis=1)


def remove_dupes_overall(X, filenames, dup_params):
    measure_type, threshold, save_dupes, out_dir = dup_params
    if measure_type == 'hash':
        mins, inds = hamming_lower(X)
    else:
        dev = torch.device('cuda:0')
        mins, inds = cosine_dedupe_device(torch.from_numpy(np.ascontiguousarray(X, np.float32)).to(dev))
    idx = (mins <= threshold).nonzero()[0]
    sidx = set(idx.tolist())
    dupes = [fn for i, fn in enumerate(filenames) if i in sidx]
    goods = [fn for i, fn in enumerate(filenames) if i not in sidx]
    X = np.delete(X, idx, axis=0)
    if out_dir is not None:
        if not save_dupes:
            for fn in dupes:
                p = osp.join(out_dir, 'faces', osp.basename(fn))
                if osp.exists(p):
                    os.remove(p)
        else:
            mdigit, mname = ('2', 'hash_diff') if measure_type == 'hash' else ('3', 'distance')
            dup_dir = osp.join(out_dir, 'intermediate', 'dupes' + mdigit)
            os.makedirs(dup_dir, exist_ok=True)
            for fn in dupes:
                fn = osp.basename(fn)
                os.replace(osp.join(out_dir, 'faces', fn), osp.join(dup_dir, fn))
            with open(osp.join(out_dir, 'intermediate', 'log_dupes' + mdigit + '.csv'), 'w') as f:
                f.write('file_name,nearest_in_prev,' + mname + ',marked_as_duplicate\n')
                for i in range(1, len(filenames)):
                    f.write('%s,%s,%s,%s\n' % (filenames[i], filenames[inds[i]], str(mins[i]), '1' if i in sidx else '0'))
    if measure_type != 'hash' and len(idx):
        print('Removed %u near-duplicates' % idx.shape[0])
    return X, goods
