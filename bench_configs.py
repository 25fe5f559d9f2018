#!/usr/bin/env python3
"""bench_configs.py — the other BASELINE.json configs, device-resident, one JSON
line each (bench.py keeps the headline C2 line).

  C3  /pipeline resize(w=1024) -> crop(768x512) -> blur(sigma=5), 2048^2 RGBA, batch 512
  C4  smartcrop 256x256 + thumbnail 256x256 + 128^2 RGBA watermark on 12 MP
      (4000x3000 and 3000x4000 decoded), batch 64
  C5  mixed request stream (resize/fit/rotate/embed/blur over 1080p/4K/12MP),
      4096 requests drawn with seed 5, grouped by identical plan

Every config runs the bimg plans produced by mipx_plan_make through
mipx_execute_dev; one image of each group is checked bit-exact against the
oracle first.  Algorithmic bytes = inputs + final outputs.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import launch_ranks  # noqa: E402


def _aggregate(texts, nranks):
    """One line per config from the ranks' lines: the whole job's images over the
    slowest rank's step time (the ranks time after a common barrier)."""
    per = {}
    keys = ("images_per_step", "ms_per_step", "device_ms_per_step", "hbm_frac")
    for r, t in enumerate(texts):
        for ln in t.splitlines():
            if ln.startswith("{"):
                d = json.loads(ln)
                if not all(k in d for k in keys):  # E2E / E2EC lines: not step-timed, passed through per rank
                    d["rank"] = r
                    print(json.dumps(d), flush=True)
                    continue
                per.setdefault(d["config"], []).append(d)
    for name, ds in per.items():
        ms = max(d["ms_per_step"] for d in ds)
        imgs = sum(d["images_per_step"] for d in ds)
        out = dict(ds[0])
        out.update({"n_gpus": nranks, "images_per_step": imgs, "ms_per_step": ms,
                    "images_per_sec": round(imgs / (ms * 1e-3), 1),
                    "verified_vs_oracle": all(d["verified_vs_oracle"] for d in ds),
                    "per_rank": [{k: d[k] for k in keys} for d in ds]})
        print(json.dumps(out), flush=True)


if __name__ == "__main__":  # plain `python bench_configs.py --gpus N`: N rank processes, before any GPU call
    _pre = argparse.ArgumentParser(add_help=False)
    _pre.add_argument("--gpus", type=int, default=None)
    _gpus = _pre.parse_known_args()[0].gpus
    if launch_ranks.needs_spawn(_gpus):
        _rc, _outs = launch_ranks.run_ranks(_gpus, os.path.abspath(__file__), sys.argv[1:])
        if _rc == 0:
            _aggregate(_outs, _gpus)
        raise SystemExit(_rc)
    launch_ranks.resolve_world(_gpus)

import torch  # noqa: E402  (before libmipx: one HIP runtime)
import torch.distributed as dist  # noqa: E402

import imaginary_amd as ia  # noqa: E402
import workloads  # noqa: E402
from imaginary_amd._abi import check, lib  # noqa: E402

HBM_PEAK_GBS = 8000.0


class Group:
    """n images sharing one plan, resident on the device."""

    def __init__(self, plan, n, dev, seed, wm=None):
        self.plan, self.n = plan, n
        ib = plan.in_w * plan.in_h * plan.in_bands
        ob = plan.out_w * plan.out_h * plan.out_bands
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        self.x = torch.randint(0, 256, (n, ib), dtype=torch.uint8, device=dev, generator=g)
        self.y = torch.empty((n, ob), dtype=torch.uint8, device=dev)
        self.wsb = lib.mipx_workspace_bytes(C.byref(plan), n)
        self.ws = torch.empty(max(self.wsb, 1), dtype=torch.uint8, device=dev)
        self.wm = None if wm is None else torch.from_numpy(np.ascontiguousarray(wm)).to(dev)
        self.in_bytes, self.out_bytes = n * ib, n * ob

    def run(self, sp):
        check(lib.mipx_execute_dev(C.byref(self.plan), self.n, self.x.data_ptr(), self.y.data_ptr(),
                                   None if self.wm is None else self.wm.data_ptr(), self.ws.data_ptr(),
                                   self.wsb, sp), "mipx_execute_dev")


def stream_runner(groups, nstreams, dev, sp, stream):
    """run_all over plan groups dealt round-robin over nstreams HIP streams (the request
    path's queues_per_device > 1 does the same: independent batches overlap their kernels'
    ramp-up and tail).  Each side stream waits for the timed stream at the start and the
    timed stream waits for all of them at the end, so a step is bracketed as before."""
    side = [torch.cuda.Stream(device=dev) for _ in range(max(0, nstreams - 1))]
    sps = [sp] + [C.c_void_p(x.cuda_stream) for x in side]

    def run_all():
        for x in side:
            x.wait_stream(stream)
        for i, (g, _) in enumerate(groups):
            g.run(sps[i % len(sps)])
        for x in side:
            stream.wait_stream(x)
    return run_all, len(sps)


def plan_for(opts, w, h, b, typ="png", wm_shape=None):
    inp = ia.make_input(w, h, b, typ)
    if wm_shape is not None:
        inp.wm_h, inp.wm_w, inp.wm_bands = wm_shape
    return ia.plan_make(ia.make_opts(**opts), inp)


def verify(group, ref_opts, wm=None):
    from oracle import oracle as o
    p = group.plan
    e, rp = o.plan(ref_opts, dict(w=p.in_w, h=p.in_h, bands=p.in_bands, type=3,
                                  **({} if wm is None else dict(wm_w=wm.shape[1], wm_h=wm.shape[0],
                                                                wm_bands=wm.shape[2]))))
    assert e == 0
    src = group.x[0].cpu().numpy().reshape(p.in_h, p.in_w, p.in_bands)
    got = group.y[0].cpu().numpy().reshape(p.out_h, p.out_w, p.out_bands)
    return bool(np.array_equal(got, o.execute(rp, src, wm)))


WARM_MS = 200.0  # --warm-ms


def time_groups(run_all, steps, warmup, stream):
    """warmup steps, then more until WARM_MS of device time has passed (a fresh process's
    first milliseconds run below the sustained clock: C3's blur averaged 0.60 ms over a
    2-step warm-up against 0.48 ms sustained, profiles/r03/c3_stages.jsonl), then the timed steps"""
    for _ in range(warmup):
        run_all()
    torch.cuda.synchronize()
    w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0.record(stream)
    while WARM_MS > 0:
        run_all()
        w1.record(stream)
        torch.cuda.synchronize()
        if w0.elapsed_time(w1) >= WARM_MS:
            break
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    multi = dist.is_initialized() and dist.get_world_size() > 1
    if multi:  # every rank starts its timed steps together
        dist.barrier()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        run_all()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if multi:
        dist.barrier()
    return wall / steps, e0.elapsed_time(e1) / steps


def line(name, workload, images, wall_s, dev_ms, alg_bytes, verified, extra=None):
    d = {"config": name, "workload": workload, "images_per_sec": round(images / wall_s, 1),
         "images_per_step": images, "n_gpus": int(os.environ.get("WORLD_SIZE", "1")),
         "ms_per_step": round(wall_s * 1e3, 3), "device_ms_per_step": round(dev_ms, 3),
         "achieved_gbs": round(alg_bytes / (dev_ms * 1e-3) / 1e9, 1),
         "hbm_frac": round(alg_bytes / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
         "alg_bytes_per_step": alg_bytes, "verified_vs_oracle": verified,
         "sampling": ["corner", "centre"][lib.mipx_reduce_sampling()]}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def c3(args, dev, sp, stream):
    """/pipeline fused on the device (mipx_plan_chain): the three stage plans run
    as one plan, PNG intermediates lossless and resident in HBM."""
    from oracle import oracle as o
    n = args.c3_batch
    stages = [dict(width=1024, embed=1), dict(width=768, height=512, crop=1), dict(sigma=5.0)]
    plans, w, h = [], 2048, 2048
    for opts in stages:
        plans.append(plan_for(opts, w, h, 4))
        w, h = plans[-1].out_w, plans[-1].out_h
    # --c3-split k: the batch as k sub-batches on k streams (stages of different sub-batches
    # overlap); 1 = one launch per stage over the whole batch
    k = max(1, args.c3_split)
    subs = [Group(ia.plan_chain(plans), n // k + (1 if i < n % k else 0), dev, 3 + i) for i in range(k)]
    g = subs[0]
    run_all, _ = stream_runner([(x, None) for x in subs], k, dev, sp, stream)

    run_all()
    torch.cuda.synchronize()
    px = g.x[0].cpu().numpy().reshape(2048, 2048, 4)
    for opts, p in zip(stages, plans):  # the oracle runs the stages one by one
        e, rp = o.plan(opts, dict(w=p.in_w, h=p.in_h, bands=p.in_bands, type=3))
        assert e == 0
        px = o.execute(rp, px)
    ok = bool(np.array_equal(g.y[0].cpu().numpy().reshape(px.shape), px))
    if ok and (len(subs) > 1 or g.n > 1):  # the batch's last image too (a later chunk under MIPX_PIPE)
        gl = subs[-1]
        px = gl.x[gl.n - 1].cpu().numpy().reshape(2048, 2048, 4)
        for opts, p in zip(stages, plans):
            e, rp = o.plan(opts, dict(w=p.in_w, h=p.in_h, bands=p.in_bands, type=3))
            px = o.execute(rp, px)
        ok = bool(np.array_equal(gl.y[gl.n - 1].cpu().numpy().reshape(px.shape), px))
    wall, dev_ms = time_groups(run_all, args.steps, args.warmup, stream)
    line("C3", "pipeline resize(w=1024)+crop(768x512)+blur(sigma=5), 2048^2 RGBA", n, wall, dev_ms,
         sum(x.in_bytes + x.out_bytes for x in subs), ok, {"batch": n, "split": k, "fused_plan": g.plan.describe()})


def c4(args, dev, sp, stream):
    n = args.c4_batch // 2
    wm = workloads.c4_watermark()
    groups = []
    for (w, h) in workloads.C4_SIZES:
        for opts in workloads.C4_OPTS:
            p = plan_for(opts, w, h, 3, wm_shape=workloads.C4_WM_SHAPE if opts.get("wm_enable") else None)
            groups.append((Group(p, n, dev, 4 + len(groups), wm if opts.get("wm_enable") else None), opts))

    run_all, nst = stream_runner(groups, args.streams, dev, sp, stream)
    run_all()
    torch.cuda.synchronize()
    ok = all(verify(g, opts, wm if opts.get("wm_enable") else None) for g, opts in groups)
    wall, dev_ms = time_groups(run_all, args.steps, args.warmup, stream)
    alg = sum(g.in_bytes + g.out_bytes + (wm.nbytes if g.wm is not None else 0) for g, _ in groups)
    line("C4", "smartcrop 256^2 + thumbnail 256^2 + watermark, 12 MP 4000x3000 / 3000x4000",
         2 * n * 2, wall, dev_ms, alg, ok, {"requests": 4 * n, "streams": nst,
                                            "plans": [g.plan.describe() for g, _ in groups]})


def c5_requests(count, seed=5):
    return workloads.c5_requests(count, seed, ia.fit_dimension)


def c5_request_bytes(wh, opts):
    """Input + output bytes of one C5 request (the planner's output geometry)."""
    w, h = wh
    p = plan_for(opts, w, h, 3)
    return w * h * 3 + p.out_w * p.out_h * p.out_bands


def c5(args, dev, sp, stream):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    allreq = c5_requests(args.c5_requests)
    # byte-balanced shards, each plan group on as few ranks as possible
    shard = workloads.shard_groups(workloads.c5_groups(allreq), world, c5_request_bytes)[rank]
    reqs = [None] * sum(cnt for _, _, cnt in shard)
    groups = []
    for (w, h), opts, cnt in shard:
        groups.append((Group(plan_for(opts, w, h, 3), cnt, dev, 5 + len(groups)), opts))

    run_all, nst = stream_runner(groups, args.streams, dev, sp, stream)

    run_all()
    torch.cuda.synchronize()
    ok = all(verify(g, opts) for g, opts in groups[:: max(1, len(groups) // 8)])
    wall, dev_ms = time_groups(run_all, args.steps, args.warmup, stream)
    alg = sum(g.in_bytes + g.out_bytes for g, _ in groups)
    line("C5", f"mixed stream {len(reqs)} requests (rank {rank}/{world}), {len(groups)} plan groups",
         len(reqs), wall, dev_ms, alg, ok, {"groups": len(groups), "streams": nst})


def e2e(args, dev, sp, stream):
    """Request path, PCIe-inclusive: C2-shaped requests (4K RGB -> 1080p) handed over
    as HOST arrays through mipx_submit/mipx_wait from 8 submitting threads (one per
    "goroutine"), so pinned staging, H2D, kernels, D2H and the copy-out are all in
    the timed region.  Never the headline value."""
    from concurrent.futures import ThreadPoolExecutor
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = args.e2e_requests
    plan = plan_for(dict(width=1920, height=1080, embed=1), 3840, 2160, 3)
    rng = np.random.default_rng(6)
    srcs = [rng.integers(0, 256, (2160, 3840, 3), dtype=np.uint8) for _ in range(8)]  # shared inputs, any thread count
    eng = ia.Engine(devices=[local], max_batch=args.e2e_batch, batch_wait_us=1000,
                    queues_per_device=args.e2e_queues)
    try:
        def one(i):
            t, out = eng.submit(plan, srcs[i % len(srcs)])
            eng.wait(t)
            return out

        with ThreadPoolExecutor(args.e2e_threads) as ex:
            first = list(ex.map(one, range(2 * args.e2e_batch)))  # warm: buffers, pinned pool
            b0, r0 = eng.stats(local)
            t0 = time.perf_counter()
            outs = list(ex.map(one, range(n)))
            dt = time.perf_counter() - t0
        b1, r1 = eng.stats(local)
        qs = eng.queue_stats()
        from oracle import oracle as o
        ok = bool(np.array_equal(outs[0], o.reduce(srcs[0], 2.0, 2.0))) and \
            bool(np.array_equal(first[1], o.reduce(srcs[1], 2.0, 2.0)))
        link = n * (3840 * 2160 * 3 + 1920 * 1080 * 3)
        print(json.dumps({"config": "E2E", "workload": "request path: 4K RGB -> 1080p from host memory, "
                          f"{args.e2e_threads} submitting threads, pinned staging + H2D/compute/D2H streams",
                          "images_per_sec": round(n / dt, 1), "requests": n, "wall_s": round(dt, 3),
                          "host_link_gbs": round(link / dt / 1e9, 2),
                          "batches": int(b1 - b0), "mean_batch": round((r1 - r0) / max(1, b1 - b0), 2),
                          "queues": len(qs), "requests_per_queue": [int(r) for _, _, r, _ in qs],
                          "verified_vs_oracle": ok}), flush=True)
    finally:
        eng.shutdown()


def e2e_c(args, dev, sp, stream):
    """The same request path driven from C (tests/c/mipx_e2e.c: caller threads with
    requests in flight over pre-faulted buffers, no Python between the callers and
    the engine), built with gcc and run as a child process; prints its JSON line."""
    import subprocess
    import tempfile
    root = os.path.dirname(os.path.abspath(__file__))
    exe = os.path.join(tempfile.mkdtemp(), "mipx_e2e")
    subprocess.run(["gcc", "-O2", "-std=c11", "-D_DEFAULT_SOURCE", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "c", "mipx_e2e.c"), "-L", os.path.join(root, "imaginary_amd"),
                    "-lmipx", "-lpthread", "-Wl,-rpath," + os.path.join(root, "imaginary_amd"), "-o", exe], check=True)
    r = subprocess.run([exe, str(args.e2e_threads), str(max(1, args.e2e_requests * 4 // args.e2e_threads)),
                        str(args.e2e_queues), "2", str(args.e2e_batch // 2)],
                       capture_output=True, text=True, timeout=300)
    sys.stdout.write(r.stdout)
    sys.stdout.flush()
    if r.returncode != 0:
        raise RuntimeError(f"mipx_e2e exit {r.returncode}: {r.stderr[-500:]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3,C4,C5")
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks; without torchrun N > 1 starts N processes and prints one aggregate line per config")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--warm-ms", type=float, default=200.0, help="device-time warm-up after --warmup steps; 0: none")
    ap.add_argument("--c3-batch", type=int, default=512)
    ap.add_argument("--c3-split", type=int, default=1, help="C3's batch as k sub-batches on k streams")
    ap.add_argument("--streams", type=int, default=4,
                    help="HIP streams the C4 / C5 plan groups are dealt over (1: one stream, r03's lines; "
                         "4: measured best for C5, profiles/r04/c5_streams.jsonl)")
    ap.add_argument("--c4-batch", type=int, default=64)
    ap.add_argument("--e2e-requests", type=int, default=256)
    ap.add_argument("--e2e-batch", type=int, default=16)
    ap.add_argument("--e2e-threads", type=int, default=16, help="submitting threads (requests in flight)")
    ap.add_argument("--e2e-queues", type=int, default=1, help="request queues (streams + worker) per device")
    ap.add_argument("--c5-requests", type=int, default=512 * int(os.environ.get("WORLD_SIZE", "1")),
                    help="total requests, sharded across ranks (4096 at 8 GPUs)")
    ap.add_argument("--sampling", choices=["corner", "centre"], default=None,
                    help="libvips reduce sampling convention (PARITY_ASSUMPTIONS.md row 1), engine and oracle")
    args = ap.parse_args()
    if args.sampling:
        import imaginary_amd as ia
        from oracle import oracle as o
        ia.set_reduce_sampling(args.sampling)
        o.set_switch("reduce_centre", int(args.sampling == "centre"))
    globals()["WARM_MS"] = args.warm_ms
    world = launch_ranks.resolve_world(args.gpus)
    if world > 1 and not dist.is_initialized():  # barriers around the timed steps only; shards are independent
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=int(os.environ.get("RANK", "0")), world_size=world)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    check(lib.mipx_set_device(local), "mipx_set_device")
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    for c in args.configs.split(","):
        {"C3": c3, "C4": c4, "C5": c5, "E2E": e2e, "E2EC": e2e_c}[c](args, dev, sp, stream)
        torch.cuda.empty_cache()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
