"""The rank launcher behind `bench.py --gpus N` (ccka/launch.py), on CPU: N
fresh processes with the torchrun rank environment, first failure wins and
stops the peers, and bench.py refuses a rank count that differs from --gpus."""
import json
import os
import subprocess
import sys
import time

from ccka import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
out = sys.argv[1]
rank = int(os.environ["RANK"])
with open(os.path.join(out, f"r{rank}.json"), "w") as f:
    json.dump({k: os.environ.get(k) for k in %r}, f)
mode = sys.argv[2]
if mode == "fail" and rank == 1:
    sys.exit(3)
if mode == "fail":
    time.sleep(60)
"""


def _child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD % (launch.RANK_VARS,))
    return str(p)


def test_spawn_sets_rank_environment(tmp_path):
    rc = launch.spawn_ranks(3, [_child(tmp_path), str(tmp_path), "ok"])
    assert rc == 0
    envs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(3)]
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1"


def test_first_failure_stops_peers(tmp_path):
    t0 = time.time()
    rc = launch.spawn_ranks(2, [_child(tmp_path), str(tmp_path), "fail"])
    assert rc == 3
    assert time.time() - t0 < 30  # rank 0 (sleeping 60 s) was terminated


def test_bench_refuses_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
