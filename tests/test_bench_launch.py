"""bench.py's multi-GPU launch contract, on CPU: `--gpus N` outside torchrun relaunches
itself as N ranks (torch.distributed.run, 127.0.0.1) and every rank checks the world
size; a world size that disagrees with --gpus fails loudly instead of reporting a
1-GPU number as N (Missing 2)."""
import json
import os
import subprocess
import sys

from conftest import REPO


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_bench_launches_n_ranks_itself():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--backend", "gloo", "--selftest-launch"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2
    ranks = line["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1]
    assert [x["local_rank"] for x in ranks] == [0, 1]
    # agents shard round-robin: C2 keeps 8 per GPU (weak), C3 / C5 split the config's total
    assert sorted(a for x in ranks for a in x["c2_agents"]) == list(range(16))
    assert [len(x["c3_agents"]) for x in ranks] == [8, 8]
    assert [len(x["c5_agents"]) for x in ranks] == [32, 32]


def test_bench_rejects_world_size_mismatch():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--selftest-launch"], capture_output=True, text=True, timeout=120,
                       env=env, cwd=REPO)
    assert r.returncode != 0
    assert "world size 1 != --gpus 2" in r.stderr
