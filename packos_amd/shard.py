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

__all__ = ["blob_sizes_host", "plan_shards", "plan_shards_streamed", "slice_columns", "stitch_offsets",
           "config_shard"]


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


def plan_shards_streamed(piece_sizes, n: int, world: int, piece: int) -> List[Tuple[int, int]]:
    """plan_shards over a batch whose blob sizes come in pieces
    (piece_sizes(a, m) -> sizes of blobs [a, a + m)), in two passes of bounded
    memory: piece totals, then the pieces that hold a boundary.  Same result
    as plan_shards(all sizes, world)."""
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    starts = list(range(0, n, piece))
    sums = [int(np.asarray(piece_sizes(a, min(piece, n - a)), dtype=np.int64).sum()) for a in starts]
    total = sum(sums)
    bounds = [0]
    before, k = 0, 0   # bytes before piece k
    for r in range(1, world):
        target = total * r / world
        # searchsorted(cum, target, "left") = first b with cum[b] >= target
        while k < len(starts) and before + sums[k] < target:
            before += sums[k]
            k += 1
        if k == len(starts):
            b = n
        else:
            sz = np.asarray(piece_sizes(starts[k], min(piece, n - starts[k])), dtype=np.int64)
            cum = before + np.concatenate([[0], np.cumsum(sz)])
            b = starts[k] + int(np.searchsorted(cum, target, side="left"))
        b = min(max(b, bounds[-1]), n)
        bounds.append(b)
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def config_shard(cfg, schema, per_gpu: int, world: int, rank: int, piece: int = 1 << 22) -> Tuple[int, int, int]:
    """The [lo, hi) blob range rank `rank` encodes when `world` ranks split
    one global synthetic batch of world x per_gpu blobs of config `cfg`
    byte-balanced (what bench.py --gpus N runs).  Returns (lo, hi, n_global);
    the rank then generates exactly its slice with make_columns(cfg, hi - lo,
    lo=lo).  Sizes are generated `piece` blobs at a time (C5 at 8 ranks is 64M
    blobs: the plan stays within ~100 MB of host memory per rank)."""
    n_global = per_gpu * world
    B = schema.fixed_blob_size
    stat = schema.all_present_size() if B <= 0 else B

    def piece_sizes(a, m):
        if B > 0:
            return np.full(m, B, dtype=np.int64)
        sizes = np.full(m, stat, dtype=np.int64)
        if cfg.var_len:
            for _, l in cfg.var_len(m, cfg.seed, a).items():
                sizes += np.asarray(l, dtype=np.int64)
        return sizes
    lo, hi = plan_shards_streamed(piece_sizes, n_global, world, piece)[rank]
    return lo, hi, n_global
