"""bench.py's launch contract (CPU only, no GPU touched): `--gpus N` outside
a torch.distributed launch starts N ranks through torch.distributed.run with
WORLD_SIZE = N; `--gpus 1` stays one plain process; a launch whose
WORLD_SIZE disagrees with --gpus is refused; at 8 GPUs the default shard is
configs[4]'s 1e10 rows / 8."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _run(args, env=None):
    r = subprocess.run([sys.executable, BENCH] + args, env=env or _env(), capture_output=True, text=True,
                       timeout=240)
    return r


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == list(range(n))
    assert all(x["world"] == n and x["master_addr"] == "127.0.0.1" for x in lines)
    assert all(x["rows_per_gpu"] == 1e9 for x in lines)


def test_gpus_1_is_one_plain_process():
    r = _run(["--gpus", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"rank": 0, "local_rank": 0, "world": 1, "rows_per_gpu": 1e9, "master_addr": None}]


def test_world_size_mismatch_is_refused():
    env = _env()
    env.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    r = _run(["--gpus", "4", "--dry-run"], env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_eight_gpus_take_configs4_shards():
    env = _env()
    env.update(RANK="3", LOCAL_RANK="3", WORLD_SIZE="8", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    r = _run(["--gpus", "8", "--dry-run"], env)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["world"] == 8 and line["rows_per_gpu"] * 8 == 1e10
