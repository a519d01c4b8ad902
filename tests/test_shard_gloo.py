"""N>1 path on CPU: byte-balanced shards, no data-path collective, world size 2
over gloo.  Each rank encodes only its shard (the CPU oracle stands in for the
device encode here — there is no GPU in this test); rank 0 stitches the
per-shard arenas/offsets and must reproduce the single-shot encoding
bit-for-bit."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_bridge as ob
from packos_amd.api import CompiledSchema
from packos_amd.configs import CONFIGS, make_columns
from packos_amd.shard import blob_sizes_host, plan_shards, slice_columns, stitch_offsets


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg_name, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = CONFIGS[cfg_name]
    hc = make_columns(cfg, n=n)
    schema = CompiledSchema(cfg.chain, cfg.mode)
    sizes = blob_sizes_host(schema, hc)
    shards = plan_shards(sizes, world)
    lo, hi = shards[rank]
    mine = slice_columns(hc, lo, hi)
    arena, offs, st = ob.encode(cfg.chain, mine, cfg.mode)
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, arena.tobytes(), offs.tolist()))
    if rank == 0:
        full_arena, full_offs, _ = ob.encode(cfg.chain, hc, cfg.mode)
        stitched = b"".join(g[2] for g in gathered)
        offsets = stitch_offsets([np.asarray(g[3], np.uint64) for g in gathered])
        bytes_per = [len(g[2]) for g in gathered]
        q.put((stitched == full_arena.tobytes(), np.array_equal(offsets, full_offs),
               [(g[0], g[1]) for g in gathered], bytes_per, np.array_equal(sizes, np.diff(full_offs.astype(np.int64)))))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg_name,n", [("C5", 3000), ("C3", 4000), ("M", 2048)])
def test_two_rank_shards_stitch(cfg_name, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cfg_name, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    same_bytes, same_offs, ranges, bytes_per, sizes_ok = res
    assert sizes_ok, "host size planning disagrees with the encoder"
    assert same_bytes and same_offs
    assert ranges[0][0] == 0 and ranges[0][1] == ranges[1][0] and ranges[1][1] == n
    # byte-balanced: the two shards differ by at most one blob's worth (+slack)
    assert abs(bytes_per[0] - bytes_per[1]) <= 4200


def test_plan_shards_properties():
    rng = np.random.default_rng(0)
    sizes = rng.integers(64, 4096, 10_000)
    for world in (1, 2, 3, 8):
        sh = plan_shards(sizes, world)
        assert len(sh) == world and sh[0][0] == 0 and sh[-1][1] == len(sizes)
        assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        tot = [int(sizes[lo:hi].sum()) for lo, hi in sh]
        assert max(tot) - min(tot) <= 2 * 4096
    assert plan_shards(np.zeros(0, np.int64), 4) == [(0, 0)] * 4


def _cfg_worker(rank, world, port, cfg_name, per_gpu, q):
    """Exactly bench.py's N>1 data path: config_shard -> make_columns(lo) ->
    encode this rank's slice; no collective but the harness's gather here."""
    from packos_amd.shard import config_shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = CONFIGS[cfg_name]
    schema = CompiledSchema(cfg.chain, cfg.mode)
    lo, hi, n_global = config_shard(cfg, schema, per_gpu, world, rank)
    mine = make_columns(cfg, n=hi - lo, lo=lo)
    arena, offs, st = ob.encode(cfg.chain, mine, cfg.mode)
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, arena.tobytes(), offs.tolist()))
    if rank == 0:
        full_arena, full_offs, _ = ob.encode(cfg.chain, make_columns(cfg, n=n_global), cfg.mode)
        stitched = b"".join(g[2] for g in gathered)
        offsets = stitch_offsets([np.asarray(g[3], np.uint64) for g in gathered])
        spans = [(g[0], g[1]) for g in gathered]
        q.put((stitched == full_arena.tobytes(), np.array_equal(offsets, full_offs), spans,
               [len(g[2]) for g in gathered], n_global))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg_name,per_gpu,world", [("C5", 1500, 2), ("C3", 2000, 2), ("M", 1024, 2), ("C5", 700, 4)])
def test_config_shards_like_bench(cfg_name, per_gpu, world):
    """bench.py --gpus N splits ONE global batch of N x per_gpu blobs by bytes
    (packos_amd.shard.config_shard) and each rank generates only its slice:
    the slices must tile the batch and their encodings stitch to the
    single-shot encoding."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cfg_worker, args=(r, world, port, cfg_name, per_gpu, q)) for r in range(world)]
    for p in procs:
        p.start()
    same_bytes, same_offs, spans, bytes_per, n_global = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert same_bytes and same_offs
    assert spans[0][0] == 0 and spans[-1][1] == n_global
    assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
    assert max(bytes_per) - min(bytes_per) <= 4200 * world   # byte-balanced within a blob or so


@pytest.mark.parametrize("cfg_name,per_gpu,world,piece", [("C5", 3000, 8, 1000), ("C5", 5000, 3, 777), ("C3", 4000, 4, 1 << 22),
                                                          ("M", 1024, 8, 100), ("C5", 10, 8, 3)])
def test_streamed_plan_matches_full_plan(cfg_name, per_gpu, world, piece):
    """config_shard plans C5's 64M-blob batch in bounded pieces: the streamed
    plan must equal plan_shards over the whole size array."""
    from packos_amd.api import CompiledSchema
    from packos_amd.configs import CONFIGS, global_blob_sizes
    from packos_amd.shard import config_shard, plan_shards
    cfg = CONFIGS[cfg_name]
    s = CompiledSchema(cfg.chain, cfg.mode)
    n = per_gpu * world
    B = s.fixed_blob_size
    sizes = np.full(n, B, np.int64) if B > 0 else global_blob_sizes(cfg, n, s.all_present_size())
    full = plan_shards(sizes, world)
    got = [config_shard(cfg, s, per_gpu, world, r, piece=piece)[:2] for r in range(world)]
    assert got == [tuple(x) for x in full]


def _parity_worker(rank, world, port, cfg_name, n, piece, q):
    """bench.shard_parity on each rank's shard (CPU tensors stand in for the
    device arena) and the MIN-reduced flag bench.py builds from it."""
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = CONFIGS[cfg_name]
    schema = CompiledSchema(cfg.chain, cfg.mode)
    hc = make_columns(cfg, n=n)
    lo, hi = plan_shards(blob_sizes_host(schema, hc), world)[rank]
    mine = slice_columns(hc, lo, hi)
    arena, offs, _ = ob.encode(cfg.chain, mine, cfg.mode)
    fixed = schema.fixed_blob_size > 0
    out = torch.from_numpy(arena.copy())
    od = None if fixed else torch.from_numpy(offs.astype(np.int64))
    same, checked, _ = bench.shard_parity(cfg, mine, out, od, schema.fixed_blob_size, 2, piece=piece)
    # one corrupted byte in the rank's last piece must be caught
    out[-1] ^= 0xFF
    bad, _, _ = bench.shard_parity(cfg, mine, out, od, schema.fixed_blob_size, 2, piece=piece)
    flag = torch.tensor([1 if same and checked == hi - lo else 0, checked], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    q.put((rank, same, bad, checked, hi - lo, int(flag[0]), int(flag[1])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg_name,n,piece", [("C5", 3000, 700), ("M", 2048, 1000), ("C3", 4000, 1 << 20)])
def test_two_rank_whole_shard_parity(cfg_name, n, piece):
    """bench.py's N > 1 encode parity covers each rank's WHOLE shard in
    pieces (round 4 capped it at the first 2M blobs)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_parity_worker, args=(r, 2, port, cfg_name, n, piece, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, same, bad, checked, rows, f0, f1 in res:
        assert same and not bad and checked == rows
        assert f0 == 1 and f1 == min(r[4] for r in res)
