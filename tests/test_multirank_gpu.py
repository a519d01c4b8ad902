"""N>1 data path with the real HIP encoder, rehearsed on one GPU: every rank
runs on cuda:0 (the box has one card; the driver's 8-GPU runs put rank r on
cuda:r) and talks gloo for the harness-only gather.  Exactly bench.py's path:
packos_amd.shard.config_shard -> make_columns(lo) -> libpackos encode; the
stitched shards must equal the single-shot encoding and the oracle's."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg_name, per_gpu, q):
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from packos_amd.api import CompiledSchema, DeviceColumns, EncodePlan
    from packos_amd.configs import CONFIGS, make_columns
    from packos_amd.shard import config_shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    cfg = CONFIGS[cfg_name]
    schema = CompiledSchema(cfg.chain, cfg.mode)
    lo, hi, n_global = config_shard(cfg, schema, per_gpu, world, rank)
    hc = make_columns(cfg, n=hi - lo, lo=lo)
    plan = EncodePlan(schema, DeviceColumns.from_host(schema, hc, "cuda:0"))
    plan.run()
    torch.cuda.synchronize()
    arena = plan.out[: plan.total].cpu().numpy().tobytes()
    offs = (plan.offsets.cpu().numpy().astype(np.uint64) if plan.offsets is not None
            else np.arange(hc.n + 1, dtype=np.uint64) * np.uint64(plan.B))
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, arena, offs.tolist()))
    if rank == 0:
        import oracle_bridge as ob
        from packos_amd.shard import stitch_offsets
        full = make_columns(cfg, n=n_global)
        one = EncodePlan(schema, DeviceColumns.from_host(schema, full, "cuda:0"))
        one.run()
        torch.cuda.synchronize()
        single = one.out[: one.total].cpu().numpy().tobytes()
        o_arena, o_offs, _ = ob.encode(cfg.chain, full, cfg.mode, nthreads=8)
        stitched = b"".join(g[2] for g in gathered)
        offsets = stitch_offsets([np.asarray(g[3], np.uint64) for g in gathered])
        q.put((stitched == single, stitched == o_arena.tobytes(), bool(np.array_equal(offsets, o_offs)),
               [(g[0], g[1]) for g in gathered], n_global))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg_name,per_gpu,world", [("C5", 3000, 2), ("C3", 5000, 2), ("M", 4096, 2),
                                                    ("C4", 2048, 3)])
def test_ranks_encode_disjoint_shards(cfg_name, per_gpu, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg_name, per_gpu, q)) for r in range(world)]
    for p in procs:
        p.start()
    same_single, same_oracle, same_offs, spans, n_global = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert same_single and same_oracle and same_offs
    assert spans[0][0] == 0 and spans[-1][1] == n_global


def test_bench_two_ranks_rehearsal():
    """bench.py under torch.distributed.run with 2 ranks (both on cuda:0,
    gloo for the barrier / timing all-reduce): one JSON line, n_gpus = 2,
    the global batch = 2 x per-GPU blobs, per-rank oracle parity."""
    env = dict(os.environ, PACKOS_BENCH_DEVICE="0", PACKOS_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--config", "C5", "--blobs-per-gpu", "20000", "--steps", "3", "--warmup", "1", "--sets", "1",
           "--no-host", "--no-warm", "--parity-piece", "7000"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_blobs"] == 40000 and line["value"] > 0
    # every rank checked its shard against the oracle's encoding of its slice
    assert line["parity"]["result"] == "bit-exact" and line["parity"]["ranks"] == 2
    # ... its WHOLE shard, in 7000-blob pieces (a flag per rank: all pieces, all blobs)
    assert line["parity"]["checked_blobs_per_rank_min"] > 14000
    assert len(line["passes"]["order"]) == 3 and set(line["passes"]["order"]) == {"cold"}


def test_bench_gpus_2_launches_its_own_ranks():
    """`python bench.py --gpus 2` with NO external launcher: bench.py starts the
    two ranks itself (rehearsal env: both on cuda:0, gloo), and the one line
    says n_gpus 2 with every rank's whole shard bit-exact."""
    env = dict(os.environ, PACKOS_BENCH_DEVICE="0", PACKOS_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PACKOS_BENCH_RANK_CHILD"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C3", "--blobs-per-gpu", "30000",
           "--steps", "3", "--warmup", "1", "--sets", "1", "--no-host", "--no-warm", "--parity-piece", "8000"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["world_size"] == 2 and line["config"]["backend"] == "gloo"
    assert [m[0] for m in line["config"]["rank_devices"]] == [0, 1]
    assert line["config"]["global_blobs"] == 60000 and line["value"] > 0
    assert line["parity"]["result"] == "bit-exact" and line["parity"]["ranks"] == 2
    assert line["parity"]["checked_blobs_per_rank_min"] > 25000
