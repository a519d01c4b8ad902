"""bench.py's rank handling on CPU: `--gpus N` with no launcher starts N rank
processes itself (torch.distributed.run as a child, before any GPU call), the
N = 1 path starts nothing, and a rank whose job does not have exactly --gpus
ranks exits non-zero instead of printing a mislabelled line."""
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_one_gpu_runs_in_process():
    assert bench.launch_cmd(1, {}, ["--gpus", "1"]) is None
    assert bench.launch_cmd(1, {"WORLD_SIZE": "1"}, []) is None


def test_gpus_n_without_launcher_starts_n_ranks():
    argv = ["--gpus", "8", "--steps", "7", "--config", "C5"]
    cmd = bench.launch_cmd(8, {}, argv, port=29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-len(argv) - 1] == os.path.join(ROOT, "bench.py") and cmd[-len(argv):] == argv


def test_ranks_under_a_launcher_do_not_relaunch():
    assert bench.launch_cmd(4, {"WORLD_SIZE": "4", "RANK": "2"}, ["--gpus", "4"]) is None
    assert bench.launch_cmd(4, {"PACKOS_BENCH_RANK_CHILD": "1"}, ["--gpus", "4"]) is None


def test_world_checks():
    assert bench.world_error(1, 1, "nccl", 0, 1, 0) is None   # (device count is checked by torch itself at N = 1)
    assert bench.world_error(8, 8, "nccl", 8, 8, 7) is None
    assert "--gpus 8 but the job has 1" in bench.world_error(8, 1, "nccl", 8, 1, 0)
    assert "--gpus 2 but the job has 4" in bench.world_error(2, 4, "gloo", 1, 4, 0)
    assert "device_count() = 1" in bench.world_error(2, 2, "nccl", 1, 2, 0)
    assert "no device" in bench.world_error(2, 2, "nccl", 2, 2, 5)
    # the one-GPU rehearsal (gloo, every rank on cuda:0) only needs the rank count
    assert bench.world_error(2, 2, "gloo", 1, 2, 0) is None


def _run(cmd, env_extra):
    env = dict(os.environ, **env_extra)
    env.pop("WORLD_SIZE", None)
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)


def test_rank_count_mismatch_exits_nonzero():
    """2 ranks started by an external launcher but --gpus 3: every rank refuses
    before touching a GPU, and no JSON line is printed."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(bench._free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "3", "--config", "C1"]
    r = _run(cmd, {"PACKOS_BENCH_BACKEND": "gloo"})
    assert r.returncode != 0
    assert "--gpus 3 but the job has 2 rank(s)" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_self_launch_propagates_rank_failure():
    """`bench.py --gpus 2` with no launcher: the parent starts the 2 ranks; on
    this GPU-less host they fail (nccl needs a device per rank), and the parent
    exits non-zero with their message instead of running a 1-GPU bench."""
    r = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C1"], {})
    assert r.returncode != 0
    assert "needs a GPU per rank" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
