"""One process per GPU: rank setup and the few collectives the driver needs.

The gridder/degridder data path has no collective (subgrids shard with no
exchange, idg_amd.shard); torch.distributed is used for the bench's
barrier / max-over-ranks timing, optional gathers of shard outputs, and the
one real exchange step of the pipeline: summing the ranks' partial uv grids
(reduce_grid, SURVEY.md §8e "final grid-sum").
Backend "nccl" is RCCL on ROCm (over xGMI); "gloo" runs the same code on CPU.
IDG_DIST_BACKEND=gloo forces gloo with GPUs present, so a multi-rank run can be
rehearsed with several ranks sharing one device (RCCL refuses that).
"""
import os

import torch
import torch.distributed as torch_dist


def env_rank():
    """(rank, local_rank, world_size) from the torchrun environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init(backend=None):
    """Initialise the process group when WORLD_SIZE > 1.  Returns
    (rank, local_rank, world_size)."""
    rank, local_rank, world = env_rank()
    if torch.cuda.is_available():
        # more ranks than devices only in a gloo rehearsal (IDG_DIST_BACKEND)
        local_rank %= max(1, torch.cuda.device_count())
    if world > 1 and not torch_dist.is_initialized():
        if backend is None:
            backend = os.environ.get("IDG_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            torch_dist.init_process_group(backend, rank=rank, world_size=world,
                                          device_id=torch.device("cuda",
                                                                 local_rank))
        else:
            torch_dist.init_process_group(backend, rank=rank, world_size=world)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    return rank, local_rank, world


def backend_name():
    """What the collectives run on, for reports."""
    if not torch_dist.is_initialized():
        return "none"
    b = torch_dist.get_backend()
    return "RCCL over xGMI" if b == "nccl" else b


def collectives_on_device():
    """True when collectives take device tensors (RCCL); gloo takes host
    tensors for gathers."""
    return torch_dist.is_initialized() and torch_dist.get_backend() == "nccl"


def _device():
    if torch_dist.is_initialized() and \
            torch_dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def barrier():
    if torch_dist.is_initialized():
        if torch_dist.get_backend() == "nccl":
            torch_dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            torch_dist.barrier()


def max_over_ranks(value):
    """Max of a float over all ranks (identity on one process)."""
    if not torch_dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=_device())
    torch_dist.all_reduce(t, op=torch_dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value):
    if not torch_dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=_device())
    torch_dist.all_reduce(t, op=torch_dist.ReduceOp.SUM)
    return float(t.item())


def gather_shards(local, counts):
    """All-gather variable-sized shards along dim 0 (counts[r] rows on rank
    r); returns the concatenation in rank order on every rank."""
    if not torch_dist.is_initialized():
        return local
    world = torch_dist.get_world_size()
    width = max(counts) if counts else 0
    pad = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    pad[:local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    torch_dist.all_gather(bufs, pad)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


def finalize():
    if torch_dist.is_initialized():
        torch_dist.destroy_process_group()


def reduce_grid(grid, to_all=True):
    """Sum the ranks' partial uv grids in place (one RCCL all-reduce, or a
    reduce to rank 0 when to_all is False).  The grid is one contiguous
    [W, 4, G, G, 2] float32 tensor (32 MiB per w-layer at G = 1024), so this
    is a single large collective, ring-bound by the xGMI links."""
    if not torch_dist.is_initialized():
        return grid
    if to_all:
        torch_dist.all_reduce(grid, op=torch_dist.ReduceOp.SUM)
    else:
        torch_dist.reduce(grid, dst=0, op=torch_dist.ReduceOp.SUM)
    return grid
