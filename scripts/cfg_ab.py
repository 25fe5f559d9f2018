#!/usr/bin/env python3
"""Same-process A/B of a MIPX_* knob on a bench_configs.py config (C3 / C4 / C5): the
config's plan groups are built once, then timed with each knob value in turn over
several rounds (device time per step, HIP events on the timed stream), output bytes
compared with the first value's.

    python scripts/cfg_ab.py --config C3 --ab MIPX_CHAIN=0,1 --rounds 3
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench_configs as bc  # noqa: E402
from imaginary_amd._abi import check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--ab", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--sampling", choices=["corner", "centre"], default=None)
    a = ap.parse_args()
    if a.sampling:
        check(lib.mipx_set_reduce_sampling({"corner": 0, "centre": 1}[a.sampling]))
    torch.cuda.set_device(0)
    check(lib.mipx_set_device(0))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    import imaginary_amd as ia
    if a.config == "C3":
        plans, w, h = [], 2048, 2048
        for opts in [dict(width=1024, embed=1), dict(width=768, height=512, crop=1), dict(sigma=5.0)]:
            plans.append(bc.plan_for(opts, w, h, 4))
            w, h = plans[-1].out_w, plans[-1].out_h
        groups = [bc.Group(ia.plan_chain(plans), 512, dev, 3)]
        runner = lambda: [g.run(sp) for g in groups]
    elif a.config == "C5":
        # bench_configs.c5 at one rank: 512 requests in their plan groups, 4 streams
        shard = bc.workloads.shard_groups(bc.workloads.c5_groups(bc.c5_requests(512)), 1, bc.c5_request_bytes)[0]
        gl = []
        for (w, h), opts, cnt in shard:
            gl.append((bc.Group(bc.plan_for(opts, w, h, 3), cnt, dev, 5 + len(gl)), opts))
        groups = [g for g, _ in gl]
        runner, _ = bc.stream_runner(gl, 4, dev, sp, stream)
    else:
        raise SystemExit("C3 or C5")
    alg = sum(g.in_bytes + g.out_bytes for g in groups)
    knob, vals = a.ab.split("=", 1)
    first = None
    for rnd in range(a.rounds):
        for v in vals.split(","):
            os.environ[knob] = v
            lib.mipx_tuning_reload()
            run_all = runner
            wall, dev_ms = bc.time_groups(run_all, a.steps, 2, stream)
            same = None
            if rnd == 0:
                for g in groups:
                    g.y.zero_()
                run_all()
                torch.cuda.synchronize()
                out = torch.cat([g.y.flatten() for g in groups])
                first = out.clone() if first is None else first
                same = bool(torch.equal(out, first))
            print(json.dumps({"config": a.config, knob: v, "round": rnd, "device_ms": round(dev_ms, 4),
                              "hbm_frac": round(alg / (dev_ms * 1e-3) / 8e12, 4), "same_as_first": same,
                              "sampling": ["corner", "centre"][lib.mipx_reduce_sampling()]}), flush=True)


if __name__ == "__main__":
    main()
