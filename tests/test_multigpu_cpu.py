"""The N > 1 path of bench.py on CPU: world_size-2 gloo processes run the same
timed_region() the GPU bench uses (barrier + sync on both sides, MAX over
ranks).  Shards are independent, so the only collective is the timing one."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

WORKER = r'''
import json, os, sys, time
sys.path.insert(0, os.environ["ROOT"])
import bench
world, rank, local = bench.dist_env()
delay = 0.05 * (rank + 1)            # rank 1 is slower: MAX must pick it
steps = 4
calls = {"n": 0}
def step():
    calls["n"] += 1
    time.sleep(delay)
wall = bench.timed_region(step, steps, 2, lambda: None, world)
print(json.dumps({"rank": rank, "wall": wall, "calls": calls["n"], "world": world}), flush=True)
import torch.distributed as dist
dist.destroy_process_group()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(240)
def test_two_rank_gloo_timing_takes_max(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, ROOT=ROOT, WORLD_SIZE="2", RANK=str(rank), LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=200)
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    walls = [o["wall"] for o in outs]
    assert all(o["calls"] == 6 for o in outs)          # 2 warmup + 4 timed
    assert abs(walls[0] - walls[1]) < 1e-9             # both report the max
    assert walls[0] >= 4 * 0.1 * 0.95                  # the slower rank's 4 timed steps


def test_single_rank_timing():
    sys.path.insert(0, ROOT)
    import bench
    n = {"c": 0}

    def step():
        n["c"] += 1

    wall = bench.timed_region(step, 5, 3, lambda: None, 1)
    assert n["c"] == 8 and wall >= 0
