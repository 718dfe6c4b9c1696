"""Frame-sharded data parallelism across the GPUs of one node.

The reference runs on one device (main.py:38-39).  Here each rank (one process per GPU,
torch.distributed over RCCL/xGMI) takes a contiguous range of WHOLE det-batches -- MTCNN's
batched_nms offsets depend on batch composition (mtcnn.py:196), so det-batch boundaries
must be the reference's -- detects and encodes it, then one all-gather-v of the embeddings
(counts first, then padded rows) restores the global (frame, face) order that the
order-sensitive grouping steps (dedupe argmin, k-means++) need.
"""
import torch
import torch.distributed as dist


def shard_batches(n_frames, det_bs, rank, world):
    """Contiguous range [lo, hi) of frame indices for `rank`, aligned to det-batches."""
    nb = -(-n_frames // det_bs)
    per, extra = divmod(nb, world)
    b0 = rank * per + min(rank, extra)
    b1 = b0 + per + (1 if rank < extra else 0)
    return min(n_frames, b0 * det_bs), min(n_frames, b1 * det_bs)


def all_gather_rows(local, group=None):
    """All-gather-v of [n_r, D] row blocks in rank order -> [sum n_r, D] on every rank."""
    world = dist.get_world_size(group)
    if world == 1:
        return local
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    mx = max(counts)
    pad = torch.zeros((mx, local.shape[1]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad, group=group)
    return torch.cat([o[:c] for o, c in zip(out, counts)])


def coll_device(group=None):
    """Where this group's collectives take tensors: the current GPU under RCCL ("nccl"), host
    memory under gloo."""
    if dist.get_backend(group) == 'nccl':
        return torch.device('cuda', torch.cuda.current_device())
    return torch.device('cpu')


def all_gather_cpu(t, group=None):
    """all_gather_rows of a host tensor through the group's device (RCCL needs device tensors);
    the result comes back to host memory, in rank order."""
    dev = coll_device(group)
    return all_gather_rows(t.to(dev), group).cpu()


def all_gather_slots(slots, n_slots, shape, dtype, group=None):
    """Gather per-position results dealt round-robin over the ranks (position i on rank
    i % world): `slots` maps this rank's positions to arrays of `shape`; returns the list of all
    n_slots arrays, identical on every rank (one tensor all_gather, no pickles)."""
    import numpy as np
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    per = -(-n_slots // world)
    buf = torch.zeros((per,) + tuple(shape), dtype=dtype)
    for i, v in slots.items():
        assert i % world == rank
        buf[i // world] = torch.as_tensor(np.asarray(v))
    dev = coll_device(group)
    out = [torch.empty_like(buf, device=dev) for _ in range(world)]
    dist.all_gather(out, buf.to(dev), group=group)
    out = [o.cpu() for o in out]
    return [out[i % world][i // world].numpy() for i in range(n_slots)]


def check_replicated(x, what, group=None):
    """Raise unless every rank holds the same array `x` (shape and bytes): the sharded grouping
    steps assume the gathered embeddings are replicated.  One all_gather of (rows, cols, a
    64-bit digest)."""
    import hashlib
    import numpy as np
    x = np.ascontiguousarray(x)
    h = int.from_bytes(hashlib.blake2b(x.tobytes(), digest_size=7).digest(), 'little')
    mine = torch.tensor([[x.shape[0], x.shape[1] if x.ndim > 1 else 1, h]], dtype=torch.int64)
    allv = all_gather_cpu(mine, group)
    if not bool((allv == allv[0]).all()):
        raise ValueError('%s: ranks hold different inputs %s; the sharded step needs the same array on every '
                         'rank' % (what, allv.tolist()))
