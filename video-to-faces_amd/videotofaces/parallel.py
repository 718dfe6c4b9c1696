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
