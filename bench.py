#!/usr/bin/env python3
"""bench.py — BASELINE.json metric on config C2: batched 4K RGB -> 1080p Lanczos3
resize (batch 256 uchar per GPU) through libmipx.so, device-resident input.

    python bench.py --gpus N --steps K --warmup W

One process per GPU (torchrun for N > 1, RANK/LOCAL_RANK/WORLD_SIZE from the
env); requests are independent, so every rank runs its own batch with no
collective on the data path ("scaling": "weak").  torch is plumbing only:
device memory, the stream, and a gloo barrier / max-reduce for the timing.

A step = one mipx_execute_dev() of the bimg plan for /resize?width=1920&height=1080
on a 3840x2160x3 decoded image (one Lanczos3 reduce 2x2: the fused k_reduce2x2 at the
corner sampling convention, k_reduce2m at the centre one) over the whole resident batch.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (import before libmipx: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import launch_ranks  # noqa: E402

W_IN, H_IN, BANDS = 3840, 2160, 3
W_OUT, H_OUT = 1920, 1080
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


# the kernel C2 runs under each reduce sampling convention (PARITY_ASSUMPTIONS.md row 1):
# its roofline and PMC traffic record are this kernel's
C2_KERNEL = {"corner": "k_reduce2x2<3, 66>", "centre": "k_reduce2m<3>"}

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) to time; without torchrun, N > 1 starts N rank processes "
                         "(launch_ranks.py); under torchrun it must equal WORLD_SIZE (default: WORLD_SIZE or 1)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU (BASELINE C2: 256)")
    ap.add_argument("--cpu-images", type=int, default=384, help="CPU baseline sample size (images): ~20 CPU-seconds on 16 EPYC cores")
    ap.add_argument("--cpu-distinct", type=int, default=24, help="distinct images in the CPU sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the CPUs allotted to this process")
    ap.add_argument("--c1-seconds", type=float, default=4.0, help="C1 CPU reference: seconds of timing")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--sampling", choices=["corner", "centre"], default=None,
                    help="libvips reduce sampling convention (PARITY_ASSUMPTIONS.md row 1); default: the library's")
    ap.add_argument("--no-centre-leg", action="store_true",
                    help="skip the second, centre-convention leg (the 'centre' object of the line)")
    ap.add_argument("--stub-step-ms", type=float, default=0.0,
                    help="harness test only: each step sleeps (rank + 1) x this many ms, no GPU work")
    return ap.parse_args()


def host_cores():
    """Cores the CPU legs use: the process's allotted CPUs (affinity), capped by
    OMP_NUM_THREADS when the box sets it (the GPU pool allots 16 CPUs per GPU)."""
    try:
        allotted = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        allotted = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(allotted, int(omp))) if omp.isdigit() else allotted


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, sampling, rank_seed=1):
    """The CPU port timed on the host's cores: oracle/vips_fast.c (the oracle's
    reduce in cache-friendly loop order, -O3 x86-64-v3, tested byte-identical to
    the oracle), OpenMP across images, each image single-threaded as libvips'
    per-request concurrency 1, over a bounded sample of distinct 4K images.
    Runs the headline's sampling convention, set explicitly (the oracle switch is
    process-wide and the verification legs move it)."""
    from oracle import oracle as o
    o.set_switch("reduce_centre", int(sampling == "centre"))
    threads = args.cpu_threads or host_cores()
    rng = np.random.default_rng(rank_seed)
    distinct = [rng.integers(0, 256, (H_IN, W_IN, BANDS), dtype=np.uint8) for _ in range(args.cpu_distinct)]
    o.reduce_fast_batch(distinct[:threads], 2.0, 2.0, threads)  # warm: pages, tables
    imgs = [distinct[i % len(distinct)] for i in range(args.cpu_images)]
    t0 = time.perf_counter()
    o.reduce_fast_batch(imgs, 2.0, 2.0, threads)
    dt = time.perf_counter() - t0
    return {"value": round(len(imgs) / dt, 2), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"{len(imgs)} x 3840x2160x3 uniform-random images ({len(distinct)} distinct, "
                      f"{len(distinct) * H_IN * W_IN * BANDS >> 20} MiB), oracle/vips_fast.c ref_reduce_fast "
                      f"(reducev+reduceh Lanczos3 2x2, -O3 x86-64-v3), {threads} OpenMP threads, {dt:.2f} s wall",
            "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "threads_note": "threads = CPUs allotted to this process (affinity, capped by OMP_NUM_THREADS)"}


def c1_cpu_reference(args, sampling):
    """BASELINE.json configs[0] (C1): POST /resize?width=300 on testdata/large.jpg
    through the CPU path, no GPU: host JPEG decode with shrink-on-load (libjpeg DCT
    scaling, 1/4: 480x270), the Lanczos3 reduce of the bimg plan (1.6 x 1.5976,
    oracle/vips_fast.c), JPEG encode (Q75) of the 300x169 result.  ms per image on
    one core and images/s over all allotted cores (one image per thread)."""
    from concurrent.futures import ThreadPoolExecutor
    import imaginary_amd as ia
    from imaginary_amd import codec
    from oracle import oracle as o
    o.set_switch("reduce_centre", int(sampling == "centre"))
    path = os.path.join(ROOT, "tests", "golden", "testdata", "large.jpg")
    with open(path, "rb") as f:
        buf = f.read()
    hdr = codec.header(buf)
    plan = ia.plan_make(ia.make_opts(width=300, embed=1), ia.make_input(hdr.w, hdr.h, hdr.bands, "jpeg"))
    (op, _a, d, _g), = plan.describe()
    assert op == "reduce" and plan.load_shrink == 4, plan.describe()

    def one(_=None):
        px = codec.decode(buf, plan.load_shrink)
        out = o.reduce_fast(px, d[0], d[1])
        return codec.encode(out, "jpeg")

    first = one()
    oh = codec.header(first)
    assert (oh.w, oh.h) == (300, 169), (oh.w, oh.h)
    n1 = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.c1_seconds / 3:
        one()
        n1 += 1
    ms1 = (time.perf_counter() - t0) / n1 * 1e3
    threads = args.cpu_threads or host_cores()
    n = max(threads * 4, int(args.c1_seconds * 1000 / ms1 * threads * 0.6))
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, range(threads)))
        t0 = time.perf_counter()
        list(ex.map(one, range(n)))
        dt = time.perf_counter() - t0
    return {"config": "C1", "workload": "POST /resize?width=300 on testdata/large.jpg (1920x1080 JPEG, "
            f"{len(buf)} B): decode at 1/{plan.load_shrink} + Lanczos3 reduce {d[0]:.4g}x{d[1]:.4g} + JPEG Q75 encode",
            "output": [oh.w, oh.h], "ms_per_image_1core": round(ms1, 3), "images_per_sec": round(n / dt, 1),
            "cores": threads, "images": n, "kind": "port",
            "codec": "Pillow (libjpeg DCT-scaled decode, the mechanism of libvips jpegload shrink) standing in "
                     "for host libvips", "reference_published": "README.md:289-304: 20 req/s, 83 ms mean latency "
                     "end to end over HTTP on an i7 with libvips 7.42 (operation not stated)"}


# the newest committed PMC traffic record of the C2 kernel (profiles/<round>/traffic_*.json:
# one record, or {"records": [...]}, each naming its kernel)
TRAFFIC_JSONS = [os.path.join(ROOT, "profiles", "r06", "traffic_r06.json"),
                 os.path.join(ROOT, "profiles", "r05", "traffic_r05.json"),
                 os.path.join(ROOT, "profiles", "r04", "traffic_r04.json"),
                 os.path.join(ROOT, "profiles", "r03", "traffic_r03.json"),
                 os.path.join(ROOT, "profiles", "r02", "traffic_r02.json"),
                 os.path.join(ROOT, "profiles", "r01", "traffic_v17.json")]


def pmc_traffic(kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC passes of exactly this
    kernel (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 corrections calibrated in
    profiles/r01/calib_*.csv); None when no record names it."""
    for path in TRAFFIC_JSONS:
        try:
            with open(path) as f:
                t = json.load(f)
        except OSError:
            continue
        for rec in t.get("records", [t]):
            if rec.get("kernel") == kernel:
                return rec["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def dist_env():
    """(world, rank, local_rank) from the torchrun environment; gloo group for N > 1.
    The group only carries the barrier and the max-reduce of the timing: the
    shards are independent, there is no data-path collective."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, local


def timed_region(step, steps, warmup, sync, world):
    """W untimed warmup steps, then exactly `steps` steps bracketed by barrier +
    device sync on both sides; returns the MAX wall time over ranks (seconds)."""
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    sync()
    t = torch.tensor([wall], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


METRIC = "images/sec (4K RGB->1080p Lanczos3 batch) + achieved HBM GB/s, 1/2/4/8 GPUs"


def headline(args, world, n, wall_max, sampling, kernel):
    """The JSON line's common part: value = every rank's images / the max-over-ranks wall."""
    return {
        "metric": METRIC,
        "value": round(n * world * args.steps / wall_max, 1),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic uniform-random uchar, device-resident (seed 20241220+rank)",
        "config": {"workload": "C2: batched 3840x2160x3 -> 1920x1080x3 Lanczos3 reduce (bimg "
                               f"/resize?width=1920&height=1080), {sampling} sampling convention "
                               f"(PARITY_ASSUMPTIONS.md row 1), {kernel.split('<')[0]}",
                   "batch_per_gpu": n, "global_batch": n * world, "parallelism": f"dp{world} (independent shards)"},
    }


def stub_main(args, world, rank):
    """The rank harness without a GPU (tests/test_bench_cpu.py): each step sleeps
    (rank + 1) x --stub-step-ms, so the max-over-ranks timing is the slowest rank's."""
    delay = args.stub_step_ms * 1e-3 * (rank + 1)
    wall_max = timed_region(lambda: time.sleep(delay), args.steps, args.warmup, lambda: None, world)
    if rank == 0:
        line = headline(args, world, args.batch, wall_max, "corner", C2_KERNEL["corner"])
        line["data"] = f"STUB: sleep {args.stub_step_ms} ms x (rank + 1) per step, no GPU work (harness test only)"
        print(json.dumps(line), flush=True)


def c2_setup(ia, lib, C, local, rank, n):
    """Plan, resident batch and workspace of C2 under the current sampling setting."""
    plan = ia.plan_make(ia.make_opts(width=W_OUT, height=H_OUT, embed=1), ia.make_input(W_IN, H_IN, BANDS, "png"))
    conv = 1 if ia.reduce_sampling() == "centre" else 0
    assert plan.describe() == [("reduce", (0,) * 7 + (conv,), (2.0, 2.0, 0.0, 0.0), (W_OUT, H_OUT, BANDS))], \
        plan.describe()
    dev = torch.device("cuda", local)
    g = torch.Generator(device=dev)
    g.manual_seed(20241220 + rank)
    d_in = torch.randint(0, 256, (n, W_IN * H_IN * BANDS), dtype=torch.uint8, device=dev, generator=g)
    d_out = torch.empty((n, W_OUT * H_OUT * BANDS), dtype=torch.uint8, device=dev)
    wsb = lib.mipx_workspace_bytes(C.byref(plan), n)
    d_ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    return plan, d_in, d_out, d_ws, wsb


def verify_c2(d_in, d_out, n, sampling):
    """Images 0 and n - 1 byte-compared with the oracle (checker only, after timing)."""
    from oracle import oracle as o
    o.set_switch("reduce_centre", int(sampling == "centre"))
    idx = [0, n - 1]
    got = d_out[idx].cpu().numpy().reshape(len(idx), H_OUT, W_OUT, BANDS)
    src = d_in[idx].cpu().numpy().reshape(len(idx), H_IN, W_IN, BANDS)
    ok = all(np.array_equal(got[i], o.reduce(src[i], 2.0, 2.0)) for i in range(len(idx)))
    if not ok:
        raise SystemExit(f"bench: GPU output differs from the oracle ({sampling} convention)")
    return ok


def roofline(kernel, kern_ms, alg_bytes):
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(kernel)
    return {"kernel": kernel, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
            "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes}


def main():
    args = parse()
    if launch_ranks.needs_spawn(args.gpus):  # plain `python bench.py --gpus N`: N rank processes
        rc, outs = launch_ranks.run_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:])
        sys.stdout.write(outs[0])
        sys.stdout.flush()
        raise SystemExit(rc)
    want_world = launch_ranks.resolve_world(args.gpus)
    world, rank, local = dist_env()
    assert world == want_world, (world, want_world)
    if args.stub_step_ms > 0:
        stub_main(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    torch.cuda.set_device(local)
    import imaginary_amd as ia
    from imaginary_amd._abi import check, lib
    import ctypes as C
    check(lib.mipx_set_device(local), "mipx_set_device")
    if args.sampling:
        ia.set_reduce_sampling(args.sampling)
    sampling = ia.reduce_sampling()
    kernel = C2_KERNEL[sampling]

    n = args.batch
    plan, d_in, d_out, d_ws, wsb = c2_setup(ia, lib, C, local, rank, n)
    in_img = W_IN * H_IN * BANDS
    out_img = W_OUT * H_OUT * BANDS
    stream = torch.cuda.current_stream(torch.device("cuda", local))
    sp = C.c_void_p(stream.cuda_stream)

    def make_step(pl, ws, wsz):
        def step():
            check(lib.mipx_execute_dev(C.byref(pl), n, d_in.data_ptr(), d_out.data_ptr(), None,
                                       ws.data_ptr(), wsz, sp), "mipx_execute_dev")
        return step

    step = make_step(plan, d_ws, wsb)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    count = {"i": 0}

    def timed_step():  # HIP events on the kernel's own stream bracket exactly the K timed steps
        if count["i"] == 0:
            ev0.record(stream)
        step()
        count["i"] += 1
        if count["i"] == args.steps:
            ev1.record(stream)

    for _ in range(args.warmup):
        step()
    wall_max = timed_region(timed_step, args.steps, 0, torch.cuda.synchronize, world)
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # one kernel launch per step, on `stream`

    verify = None
    if not args.no_verify and rank == 0:
        verify = verify_c2(d_in, d_out, n, sampling)

    # the other reduce sampling convention's kernel on the same batch, same process, after
    # the headline leg (PARITY_ASSUMPTIONS.md row 1 is unresolved: the line carries both)
    other = None
    if not args.no_centre_leg and sampling == "corner":
        ia.set_reduce_sampling("centre")
        try:
            cplan = ia.plan_make(ia.make_opts(width=W_OUT, height=H_OUT, embed=1),
                                 ia.make_input(W_IN, H_IN, BANDS, "png"))
        finally:
            ia.set_reduce_sampling(sampling)  # the plan keeps the centre convention (ABI v6)
        cws_b = lib.mipx_workspace_bytes(C.byref(cplan), n)
        cws = torch.empty(max(cws_b, 1), dtype=torch.uint8, device=d_in.device)
        cstep = make_step(cplan, cws, cws_b)
        for _ in range(args.warmup):
            cstep()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            cstep()
        e1.record(stream)
        torch.cuda.synchronize()
        cms = e0.elapsed_time(e1) / args.steps
        other = {"sampling": "centre", "images_per_sec_per_gpu": round(n / (cms * 1e-3), 1),
                 "roofline": roofline(C2_KERNEL["centre"], cms, n * (in_img + out_img)),
                 "verified_vs_oracle": verify_c2(d_in, d_out, n, "centre") if (not args.no_verify and rank == 0)
                 else None}

    if rank == 0:
        line = headline(args, world, n, wall_max, sampling, kernel)
        rl = roofline(kernel, kern_ms, n * (in_img + out_img))
        line["achieved_hbm_gbs"] = rl["achieved"]
        line["roofline"] = rl
        line["verified_vs_oracle"] = verify
        if other:
            line["centre"] = other
        if not args.no_cpu and world == 1:  # the CPU figures are N = 1 figures
            line["cpu_baseline"] = cpu_baseline(args, sampling)
            line["cpu_baseline"]["sampling"] = sampling
            line["c1_cpu_reference"] = c1_cpu_reference(args, sampling)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
