"""The request path (mipx_submit / mipx_wait / mipx_cancel) with several queues per
device, from C and from Python, plus build provenance of the loaded library.

This is the cgo seam that replaces bimg.Resize at reference image.go:96: one
goroutine per HTTP request (middleware.go:76-113) submits, the engine batches
identical plans per queue and dispatches to the least-loaded queue.
"""
import os
import subprocess
import threading

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_loaded_library_is_built_from_these_sources(gpu):
    """Provenance: the libmipx.so this GPU process loaded carries the hash of the
    sources in this tree (imaginary_amd/srchash.py)."""
    from imaginary_amd._abi import LIB_PATH
    from imaginary_amd.srchash import source_hash
    bid = gpu.lib.mipx_build_id().decode()
    assert bid == source_hash(), (bid, source_hash())
    maps = open("/proc/self/maps").read()
    assert os.path.realpath(LIB_PATH) in maps
    print(f"libmipx build {bid} loaded from {LIB_PATH}")


def test_c_client_four_threads_two_queues(gpu, tmp_path):
    """A gcc-compiled C program against include/mipx.h: mipx_plan_make ->
    mipx_submit from 4 pthreads -> mipx_wait -> byte compare with the oracle, on
    two queues of device 0, plus mipx_cancel."""
    from test_abi import build_c_client
    exe = build_c_client(tmp_path)
    r = subprocess.run([exe, "4", "24", "2"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stdout.strip().splitlines()[-1].startswith("ok: 4 threads x 24 requests, 2 queues (2 used)")


def _plans(gpu, oracle):
    specs = [(dict(width=160, height=120, embed=1), (320, 240, 3)),
             (dict(width=97, height=61, crop=1), (301, 203, 4)),
             (dict(sigma=1.5), (90, 70, 3))]
    out = []
    for opts, (w, h, b) in specs:
        p = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, "png"))
        e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3))
        assert e == 0
        out.append((p, rp, (h, w, b)))
    return out


def test_multi_queue_least_loaded_dispatch(gpu, oracle):
    """Three queues on one device under 8 concurrent submitters: every result is
    the oracle's, every queue takes work, per-queue stats add up to the requests,
    and nothing is left pending."""
    from concurrent.futures import ThreadPoolExecutor
    gpu.lib.mipx_shutdown()   # mipx_init keeps a running engine's configuration (imaginary.py's may be up)
    eng = gpu.Engine(devices=[0], max_batch=8, batch_wait_us=300, queues_per_device=3)
    try:
        plans = _plans(gpu, oracle)
        rng = np.random.default_rng(77)
        jobs = []
        for i in range(90):
            p, rp, shape = plans[i % 3]
            jobs.append((p, rp, rng.integers(0, 256, shape, dtype=np.uint8)))

        def one(job):
            p, rp, img = job
            t, out = eng.submit(p, img)
            eng.wait(t)
            return out, oracle.execute(rp, img)

        with ThreadPoolExecutor(8) as ex:
            res = list(ex.map(one, jobs))
        for k, (got, want) in enumerate(res):
            assert np.array_equal(got, want), f"request {k}"
        qs = eng.queue_stats()
        assert len(qs) == 3 and all(d == 0 for d, _, _, _ in qs)
        assert sum(r for _, _, r, _ in qs) == len(jobs)
        assert all(r > 0 for _, _, r, _ in qs), qs           # least-loaded spread the work
        assert all(p == 0 for _, _, _, p in qs), qs
        assert eng.stats(0)[1] == len(jobs)
        # device-pinned submission goes to one of device 0's queues
        p, rp, shape = plans[0]
        img = rng.integers(0, 256, shape, dtype=np.uint8)
        t, out = eng.submit(p, img, device=0)
        eng.wait(t)
        assert np.array_equal(out, oracle.execute(rp, img))
        with pytest.raises(gpu.MipxError):
            eng.submit(p, img, device=7)                      # no queue on that device
    finally:
        eng.shutdown()


def test_cancel_after_timeout_detaches_the_output(gpu):
    """MIPX_ETIMEOUT leaves the request running; mipx_cancel detaches the output so
    the caller may free it, and the ticket is released."""
    import ctypes as C
    gpu.lib.mipx_shutdown()
    eng = gpu.Engine(devices=[0], max_batch=4)
    try:
        p = gpu.plan_make(gpu.make_opts(width=1920, height=1080, embed=1), gpu.make_input(3840, 2160, 3, "png"))
        img = np.zeros((2160, 3840, 3), np.uint8)
        sentinel = 0x5A
        tickets = []
        outs = []
        for _ in range(6):
            # the sentinel goes in before the submit: the request may complete before it returns
            out = np.full((1080, 1920, 3), sentinel, np.uint8)
            t, out = eng.submit(p, img, out=out)
            tickets.append(t)
            outs.append(out)
        code = gpu.lib.mipx_wait(tickets[-1], 0)
        assert code in (0, gpu.MIPX_ETIMEOUT)
        for t in tickets[3:]:
            assert gpu.lib.mipx_cancel(t) in (0, gpu.MIPX_ESTALE)
        for t in tickets[:3]:
            eng.wait(t)
            assert gpu.lib.mipx_cancel(t) == gpu.MIPX_ESTALE    # already waited: released
        assert gpu.lib.mipx_wait(C.c_uint64(tickets[4]), 0) == gpu.MIPX_ESTALE
        for o in outs[:3]:
            assert not (o == sentinel).any()
    finally:
        eng.shutdown()


def test_shutdown_during_traffic_is_safe(gpu):
    """mipx_shutdown racing submitters never frees a queue under a
    submit: each submit either is queued (and then completes) or gets ENOTINIT."""
    p = gpu.plan_make(gpu.make_opts(width=80, height=60, embed=1), gpu.make_input(160, 120, 3, "png"))
    img = np.random.default_rng(3).integers(0, 256, (120, 160, 3), dtype=np.uint8)
    gpu.lib.mipx_shutdown()
    for _round in range(3):
        eng = gpu.Engine(devices=[0], max_batch=4, queues_per_device=2)
        results = {"ok": 0, "notinit": 0, "other": []}
        lock = threading.Lock()
        stop = threading.Event()

        def submitter():
            while not stop.is_set():
                try:
                    t, out = eng.submit(p, img)
                except gpu.MipxError as e:
                    with lock:
                        if e.code == gpu.MIPX_ENOTINIT:
                            results["notinit"] += 1
                        else:
                            results["other"].append(e.code)
                    return
                code = gpu.lib.mipx_wait(t, 20000)
                with lock:
                    if code == 0:
                        results["ok"] += 1
                    else:
                        results["other"].append(code)

        th = [threading.Thread(target=submitter) for _ in range(6)]
        for t in th:
            t.start()
        import time
        time.sleep(0.05)
        eng.shutdown()
        stop.set()
        for t in th:
            t.join(timeout=60)
            assert not t.is_alive(), "submitter hung across shutdown"
        assert results["other"] == [], results
        assert results["ok"] > 0
