"""Multi-GPU sharding of a batch: byte-balanced contiguous shards, no
collective on the data path.

Blobs are independent (a PutAccess is reset per blob, access/put.go:25-31),
so N GPUs encode N disjoint contiguous ranges.  Ranges are balanced by BYTES
(prefix sum of the host-known blob sizes), which matters for mixed 64 B-4 KB
batches (config C5).  Each shard's `out_offsets` are shard-relative; stitching
adds the shard's byte base — the only cross-shard step, done on the host.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

from .columns import HostColumns

__all__ = ["blob_sizes_host", "plan_shards", "slice_columns", "stitch_offsets", "config_shard"]


def blob_sizes_host(schema, hc: HostColumns) -> np.ndarray:
    """Encoded size of every blob, computed on the host from var widths and
    validity (packos_schema_blob_size_host); vectorised for fixed schemas."""
    B = schema.fixed_blob_size
    any_valid = any(v is not None for v in hc.valid)
    if B >= 0 and not any_valid:
        return np.full(hc.n, B, dtype=np.int64)
    widths = hc.var_widths()
    ncol = len(hc.specs)
    out = np.empty(hc.n, dtype=np.int64)
    valid = np.ones(ncol, np.uint8)
    for i in range(hc.n):
        for c in range(ncol):
            if hc.valid[c] is not None:
                valid[c] = hc.valid[c][i]
        out[i] = schema.blob_size_host(widths[i], valid)
    return out


def plan_shards(sizes: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) blob ranges, one per rank, with ~equal bytes."""
    n = int(sizes.shape[0])
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    cum = np.concatenate([[0], np.cumsum(sizes.astype(np.int64))])
    total = int(cum[-1])
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        b = int(np.searchsorted(cum, target, side="left"))
        b = min(max(b, bounds[-1]), n)
        bounds.append(b)
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def slice_columns(hc: HostColumns, lo: int, hi: int) -> HostColumns:
    """Rows [lo, hi) of a host column set (var arenas re-based to 0)."""
    out = HostColumns(hc.chain, hi - lo)
    for c, sp in enumerate(hc.specs):
        if sp.fixed:
            w = sp.width
            out.data[c] = hc.data[c][lo * w:hi * w].copy()
        elif sp.var:
            o = hc.offsets[c].astype(np.int64)
            a, b = int(o[lo]), int(o[hi])
            out.data[c] = hc.data[c][a:b].copy()
            out.offsets[c] = (o[lo:hi + 1] - a).astype(np.uint32)
        if hc.valid[c] is not None:
            out.valid[c] = hc.valid[c][lo:hi].copy()
    return out


def stitch_offsets(shard_offsets: Sequence[np.ndarray]) -> np.ndarray:
    """Concatenate per-shard out_offsets (each [n_r+1], starting at 0) into
    the offsets of the concatenated arena."""
    parts, base = [np.zeros(1, dtype=np.uint64)], 0
    for o in shard_offsets:
        o = np.asarray(o, dtype=np.uint64)
        parts.append(o[1:] + np.uint64(base))
        base += int(o[-1])
    return np.concatenate(parts)


def config_shard(cfg, schema, per_gpu: int, world: int, rank: int) -> Tuple[int, int, int]:
    """The [lo, hi) blob range rank `rank` encodes when `world` ranks split
    one global synthetic batch of world x per_gpu blobs of config `cfg`
    byte-balanced (what bench.py --gpus N runs).  Returns (lo, hi, n_global);
    the rank then generates exactly its slice with make_columns(cfg, hi - lo,
    lo=lo)."""
    from .configs import global_blob_sizes
    n_global = per_gpu * world
    B = schema.fixed_blob_size
    if B > 0:
        sizes = np.full(n_global, B, dtype=np.int64)
    else:
        sizes = global_blob_sizes(cfg, n_global, schema.all_present_size())
    lo, hi = plan_shards(sizes, world)[rank]
    return lo, hi, n_global
