"""Request dispatch and multi-GPU sharding, on CPU.

- mipx_pick_queue is the rule mipx_submit applies (least pending bytes among the
  requested device's queues, or among all queues for device < 0); it needs no GPU.
- workloads.shard_groups splits C5's plan groups over ranks by bytes, largest first,
  each group on as few ranks as possible; a world-size-2 gloo run checks that the
  ranks' byte totals agree to within 5 % on the seed-5 stream of 4096 requests."""
import ctypes as C
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT


def _pick(device, qdev, pend):
    import imaginary_amd as ia
    n = len(qdev)
    return ia.lib.mipx_pick_queue(device, (C.c_int32 * n)(*qdev), (C.c_int64 * n)(*pend), n)


def test_pick_queue_least_loaded():
    # 2 devices x 3 queues
    qdev = [0, 0, 0, 1, 1, 1]
    assert _pick(-1, qdev, [5, 4, 9, 7, 3, 8]) == 4          # global minimum
    assert _pick(0, qdev, [5, 4, 9, 7, 3, 8]) == 1           # minimum among device 0's queues
    assert _pick(1, qdev, [0, 0, 0, 7, 3, 8]) == 4           # device 1 only, even if others are idle
    assert _pick(-1, qdev, [2, 2, 2, 2, 2, 2]) == 0          # ties: the first
    assert _pick(2, qdev, [1] * 6) < 0                       # no queue on that device
    assert _pick(-1, [], []) < 0


def test_pick_queue_spreads_synthetic_stream():
    """Feeding the chooser its own picks spreads a mixed stream evenly by bytes."""
    import numpy as np
    r = np.random.default_rng(5)
    qdev = [d for d in range(8) for _ in range(2)]
    pend = [0] * len(qdev)
    for _ in range(4096):
        q = _pick(-1, qdev, pend)
        pend[q] += int(r.choice([6220800, 24883200, 36000000]))
    per_dev = [pend[2 * d] + pend[2 * d + 1] for d in range(8)]
    assert max(per_dev) - min(per_dev) <= 36000000 * 2   # within two of the largest request


def _bytes_of(wh, opts):
    import imaginary_amd as ia
    w, h = wh
    p = ia.plan_make(ia.make_opts(**opts), ia.make_input(w, h, 3, "png"))
    return w * h * 3 + p.out_w * p.out_h * p.out_bands


@pytest.mark.parametrize("world", [2, 4, 8])
def test_shard_groups_balanced(world):
    sys.path.insert(0, ROOT)
    import imaginary_amd as ia
    import workloads
    reqs = workloads.c5_requests(4096, 5, ia.fit_dimension)
    groups = workloads.c5_groups(reqs)
    shards = workloads.shard_groups(groups, world, _bytes_of)
    assert sum(c for s in shards for _, _, c in s) == 4096
    got = {}
    for s in shards:
        for (w, h), opts, c in s:
            k = (w, h, json.dumps(opts, sort_keys=True))
            got[k] = got.get(k, 0) + c
    want = {(w, h, json.dumps(o, sort_keys=True)): c for (w, h), o, c in groups}
    assert got == want                                        # every request exactly once
    loads = [sum(c * _bytes_of(wh, o) for wh, o, c in s) for s in shards]
    assert (max(loads) - min(loads)) / (sum(loads) / world) <= 0.05
    # groups stay together: at most world - 1 groups are split across ranks
    split = sum(1 for k in want if sum(1 for s in shards for (w, h), o, _ in s
                                       if (w, h, json.dumps(o, sort_keys=True)) == k) > 1)
    assert split <= world - 1


WORKER = r'''
import json, os, sys
sys.path.insert(0, os.environ["ROOT"])
import torch.distributed as dist
import imaginary_amd as ia
import workloads
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
def bytes_of(wh, opts):
    w, h = wh
    p = ia.plan_make(ia.make_opts(**opts), ia.make_input(w, h, 3, "png"))
    return w * h * 3 + p.out_w * p.out_h * p.out_bands
groups = workloads.c5_groups(workloads.c5_requests(4096, 5, ia.fit_dimension))
mine = workloads.shard_groups(groups, world, bytes_of)[rank]
import torch
t = torch.tensor([sum(c * bytes_of(wh, o) for wh, o, c in mine), sum(c for _, _, c in mine)], dtype=torch.float64)
allt = [torch.zeros_like(t) for _ in range(world)]
dist.all_gather(allt, t)
print(json.dumps({"rank": rank, "bytes": [float(x[0]) for x in allt], "reqs": [int(x[1]) for x in allt]}), flush=True)
dist.destroy_process_group()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(240)
def test_two_rank_gloo_c5_byte_balance(tmp_path):
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
    b = outs[0]["bytes"]
    assert outs[0]["bytes"] == outs[1]["bytes"]
    assert sum(outs[0]["reqs"]) == 4096
    assert abs(b[0] - b[1]) / (sum(b) / 2) <= 0.05
