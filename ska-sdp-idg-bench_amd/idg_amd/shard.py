"""Subgrid sharding across GPUs (one process per GPU).

Subgrids are independent and, in the benchmark's plans, equally expensive
(every subgrid has nr_timesteps = T, reference app/common/init.cpp:134-159),
so the path partitions into contiguous subgrid ranges with no exchange on the
data path.  Each rank uploads only its shard: its metadata, rebased so that
the shard's first referenced visibility row is row 0 (the reference kernels
rebase only baseline_offset, app/CPU/kernels/gridder_reference.cpp:16-25),
plus the uvw/visibility rows that shard references.  Spheroidal, A-terms and
wavenumbers are replicated.  Gridder outputs (subgrids) and degridder outputs
(visibility rows) are disjoint per shard.
"""
import numpy as np

from .api import METADATA_DTYPE, as_metadata


def subgrid_rows(metadata):
    """[start, end) visibility row of every subgrid (reference row index:
    (baseline_offset - md[0].baseline_offset) + time_offset + t)."""
    md = as_metadata(metadata)
    if md.size == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    start = (md["baseline_offset"].astype(np.int64) -
             np.int64(md["baseline_offset"][0]) +
             md["time_offset"].astype(np.int64))
    return start, start + md["nr_timesteps"].astype(np.int64)


def plan_shards(metadata, world_size):
    """Split subgrids into `world_size` contiguous ranges of near-equal cost
    (cost of a subgrid ~ its nr_timesteps).  Returns [(s0, s1), ...]."""
    md = as_metadata(metadata)
    n = md.size
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    cost = np.maximum(md["nr_timesteps"].astype(np.float64), 0.0) + 1e-9
    cum = np.concatenate([[0.0], np.cumsum(cost)])
    total = cum[-1]
    bounds = [0]
    for r in range(1, world_size):
        bounds.append(int(np.searchsorted(cum, total * r / world_size,
                                          side="left")))
    bounds.append(n)
    bounds = np.maximum.accumulate(np.clip(bounds, 0, n))
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(world_size)]


def shard(metadata, s0, s1):
    """Metadata of subgrids [s0, s1) rebased to the shard's own row space,
    and the global visibility-row range [row0, row1) the shard reads."""
    md = as_metadata(metadata)
    start, end = subgrid_rows(md)
    sub = md[s0:s1].copy()
    if sub.size == 0:
        return sub, 0, 0
    row0 = int(start[s0:s1].min())
    row1 = int(end[s0:s1].max())
    sub["time_offset"] = (start[s0:s1] - row0).astype(np.int32)
    sub["baseline_offset"] = 0
    return sub, row0, row1


def merge_shard_outputs(parts):
    """Concatenate per-rank subgrid outputs (in rank order)."""
    return np.concatenate(parts, axis=0) if parts else np.zeros(0)


__all__ = ["subgrid_rows", "plan_shards", "shard", "merge_shard_outputs",
           "METADATA_DTYPE"]
