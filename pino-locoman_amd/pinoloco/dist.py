"""One process per GPU, batch-sharded.

Every MPC problem is independent, so the data path has no collective: rank r
solves problems [first, first + count) of the global batch (synthetic.shard)
with seeds from the global index.  The only collectives are outside the hot
path: the max-over-ranks wall time of the timed region and one all-gather of
the per-problem controller outputs ([u_0, x_state] rows) after it.  Backend
"nccl" is RCCL over xGMI on the GPU node; tests use "gloo" on the CPU.
"""
from __future__ import annotations

import os


def env_ranks():
    """(world, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend="nccl"):
    """Initialise torch.distributed when WORLD_SIZE > 1; returns the module or None."""
    world, _, local_rank = env_ranks()
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
    if not dist.is_initialized():
        dist.init_process_group(backend)
    return dist


def _device(dist):
    import torch
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def max_over_ranks(value: float, dist) -> float:
    """MAX of a scalar (the timed region's wall time) over all ranks."""
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=_device(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(local, dist):
    """All-gather per-problem rows [count, row] from every rank -> [global, row].

    Shards may differ in size by one (synthetic.shard), so rows are padded to the
    largest shard for the collective and trimmed afterwards."""
    if dist is None:
        return local
    import torch
    world = dist.get_world_size()
    dev = local.device
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    top = max(counts)
    pad = torch.zeros((top, local.shape[1]), dtype=local.dtype, device=dev)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], 0)
