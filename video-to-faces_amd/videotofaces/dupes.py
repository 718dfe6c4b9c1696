"""Near-duplicate removal (drop-in for src/videotofaces/dupes.py).

The embedding branch of remove_dupes_overall (dupes.py:51-68) runs on the GPU as one fused
cosine-distance + strict-lower-triangle row-min kernel (vtf_cosine_dedupe): no N x N
matrix (the reference materialises an fp32 N x N plus an fp64 N x N mask).  The hash branch
(dupes.py:11-59): average hashes of the face crops straight from the frames in HBM
(vtf_ahash_crops) and the all-pairs Hamming row-min as a popcount kernel
(vtf_hamming_dedupe) instead of a Python-lambda pairwise_distances.
"""
import ctypes
import math
import os
import os.path as osp

import numpy as np
import torch

from . import _native as nat


def cosine_dedupe_device(X, sharded=False, replicated=False):
    """X: CUDA fp32 [N,D] -> (mins f32 [N], inds i64 [N]) exactly as dupes.py:60-64 computes
    them, in sklearn's bits: min / first argmin over j < i of clip(1 - cos(X_i, X_j), 0, 2);
    row 0 -> (10000, 0).  sharded=True (a collective: every rank of the default process group
    must call it with the same X, which is checked) splits the rows across the ranks
    (cosine_dedupe_sharded); replicated=True: the caller has already checked that."""
    X = X.to(torch.float32).contiguous()
    if sharded and _world() > 1:
        if not replicated:
            from .parallel import check_replicated
            check_replicated(X.cpu().numpy(), 'cosine_dedupe_device')
        return cosine_dedupe_sharded(X)
    return cosine_dedupe_rows(X, 0, X.shape[0])


def cosine_dedupe_rows(X, lo, hi):
    """rows [lo, hi) of cosine_dedupe_device (lo a multiple of 128, hi one or N)."""
    n, d = X.shape
    mins = torch.empty(hi - lo, dtype=torch.float32, device=X.device)
    inds = torch.empty(hi - lo, dtype=torch.int64, device=X.device)
    if hi > lo:
        nat.check(nat.lib().vtf_cosine_dedupe_rows(nat.ptr(X), n, d, lo, hi, nat.ptr(mins), nat.ptr(inds),
                                                   nat.stream_ptr(X.device)))
    return mins.cpu().numpy(), inds.cpu().numpy()


def _world():
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def dedupe_shards(n, world, tile=128):
    """Row boundaries of the lower-triangle dedupe across `world` ranks: tile-aligned and
    balanced by triangle area (rank r ends near n * sqrt((r+1) / world))."""
    nt = -(-n // tile)
    b = [min(n, int(round(nt * math.sqrt(r / world))) * tile) for r in range(world + 1)]
    b[0], b[-1] = 0, n
    for r in range(1, world + 1):
        b[r] = max(b[r], b[r - 1])
    return b


def cosine_dedupe_sharded(X, rows_fn=None):
    """the N x N dedupe row-block sharded across the ranks of the default process
    group (each holds the gathered X), then one tensor all-gather-v (RCCL on GPUs) of the per-row
    (min, argmin), packed as two float64 words a row (both exact: fp32 minima, indices < 2^31).
    rows_fn(lo, hi) -> (mins, inds) computes a shard (default: the device kernel)."""
    import torch.distributed as dist
    from .parallel import all_gather_cpu
    world, rank = dist.get_world_size(), dist.get_rank()
    n = X.shape[0]
    b = dedupe_shards(n, world)
    mins, inds = (rows_fn or (lambda lo, hi: cosine_dedupe_rows(X, lo, hi)))(b[rank], b[rank + 1])
    pk = torch.from_numpy(np.stack([np.asarray(mins, np.float32).astype(np.float64),
                                    np.asarray(inds, np.int64).astype(np.float64)], 1).reshape(-1, 2))
    allv = all_gather_cpu(pk).numpy()
    return allv[:, 0].astype(np.float32), allv[:, 1].astype(np.int64)


def pack_hashes(H):
    """ahash bit arrays [N,64] (0/1, dupes.py:15 `1 * diff.flatten()`) -> uint64 [N], bit k =
    element k; packed uint64 input passes through."""
    H = np.asarray(H)
    if H.dtype == np.uint64 and H.ndim == 1:
        return H
    H = H.reshape(-1, 64).astype(np.uint64)
    return (H << np.arange(64, dtype=np.uint64)).sum(axis=1, dtype=np.uint64) if len(H) else np.zeros(0, np.uint64)


def unpack_hash(h):
    """uint64 -> the reference's 64-element 0/1 int array."""
    return ((np.uint64(h) >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(np.int64)


def ahash_crops(frames_dev, crops):
    """dupes.ahash (dupes.py:11-15) of every crop (int [N,5] frame, x1, y1, x2, y2) of the
    CUDA uint8 frames [B,H,W,3] -> uint64 [N] (vtf_ahash_crops)."""
    c = np.ascontiguousarray(crops, dtype=np.int32).reshape(-1, 5)
    out = np.zeros(c.shape[0], np.uint64)
    if c.shape[0] == 0:
        return out
    B, H, W = frames_dev.shape[:3]
    nat.check(nat.lib().vtf_ahash_crops(nat.ptr(frames_dev), B, H, W, frames_dev.stride(0), frames_dev.stride(1),
                                        c.ctypes.data, c.shape[0], out.ctypes.data, nat.stream_ptr(frames_dev.device)))
    return out


def ahash(img, device=None):
    """dupes.ahash (dupes.py:11-15) of one uint8 BGR image -> 64-element 0/1 array."""
    t = torch.from_numpy(np.ascontiguousarray(img)[None]).to(nat.require_gpu(device))
    h, w = img.shape[:2]
    return unpack_hash(ahash_crops(t, [[0, 0, 0, w, h]])[0])


def hamming_lower(H, device=None):
    """hash branch distances (dupes.py:55-64) on the GPU: min / first argmin over j < i of the
    Hamming distance of the 64-bit average hashes; row 0 -> (10000, 0)."""
    h = pack_hashes(H)
    n = h.shape[0]
    if n == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int64)
    dev = nat.require_gpu(device)
    d = torch.from_numpy(h.view(np.int64)).to(dev)
    mins = torch.empty(n, dtype=torch.int32, device=dev)
    inds = torch.empty(n, dtype=torch.int64, device=dev)
    nat.check(nat.lib().vtf_hamming_dedupe(nat.ptr(d), n, nat.ptr(mins), nat.ptr(inds), nat.stream_ptr(dev)))
    return mins.cpu().numpy(), inds.cpu().numpy()


def nearest_dupes(hashes, prev, hash_thr):
    """remove_dupes_nearest's decision loop (dupes.py:18-36) on packed hashes: `prev` is the
    running list of (hash, name) of kept faces (the reference's `hashes`), updated in place.
    Returns (dupe flags, log rows (fn, nearest fn, diff, is_dupe))."""
    flags, log = [], []
    for h, fn in hashes:
        h = int(h)
        if not prev:
            prev.append((h, fn))
            flags.append(False)
            continue
        diffs = [(bin(h ^ p).count('1'), pfn) for (p, pfn) in prev[-5:]]
        md, md_fn = min(diffs, key=lambda a: a[0])
        log.append((fn, md_fn, md, md <= hash_thr))
        if md <= hash_thr:
            flags.append(True)
        else:
            prev.append((h, fn))
            flags.append(False)
    return flags, log


def remove_dupes_overall(X, filenames, dup_params, device=None, sharded=False):
    """dupes.py:51-93; `device` (an addition) picks the GPU, default cuda:0.  sharded=True (an
    addition, a collective over the default process group: every rank passes the same X) splits
    the embedding dedupe's rows across the ranks; only rank 0 then touches out_dir."""
    measure_type, threshold, save_dupes, out_dir = dup_params
    if measure_type == 'hash':
        mins, inds = hamming_lower(X, device)
    else:
        dev = nat.require_gpu(device)
        mins, inds = cosine_dedupe_device(torch.from_numpy(np.ascontiguousarray(X, np.float32)).to(dev), sharded)
    if sharded and _world() > 1:
        import torch.distributed as dist
        if dist.get_rank() != 0:
            out_dir = None
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
