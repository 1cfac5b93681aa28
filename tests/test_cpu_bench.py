"""CPU: ``bench.py --gpus N`` started without a launcher starts N ranks itself (one process per
GPU under torch.distributed.run) from a parent that makes no GPU call — the driver's multi-GPU
scaling command depends on it (the N-GPU line used to time one rank)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_n_spawns_n_ranks():
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3",
                        "--selftest-spawn", "--no-cpu"], capture_output=True, text=True,
                       env=env, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1, 2]
    assert {d["world"] for d in lines} == {3}
    assert sorted(d["local_rank"] for d in lines) == [0, 1, 2]


def test_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--no-cpu"], capture_output=True, text=True, env=env, timeout=300,
                       cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)


def test_torchrun_without_gpus_takes_launcher_world():
    """``torchrun --nproc-per-node 2 bench.py`` (no --gpus): the ranks take WORLD_SIZE from the
    launcher instead of refusing."""
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port",
                        "29613", os.path.join(ROOT, "bench.py"), "--selftest-spawn", "--no-cpu"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert {d["world"] for d in lines} == {2}
