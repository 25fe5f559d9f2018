#!/usr/bin/env python3
"""Same-process A/B of the batch device copy (rot 0 through mipx_op_rot): MIPX_COPY=0
(hipMemcpyAsync), 1 (k_copy16, non-temporal), 2 (k_copy16, plain).  One JSON line per
(shape, variant): median ms of 5 groups after a 200 ms warm-up, GB/s read + written."""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imaginary_amd._abi import check, lib  # noqa: E402

SHAPES = [(3840, 2160, 3, 16), (1920, 1080, 3, 64), (4000, 3000, 3, 16), (333, 251, 3, 64)]


def main():
    dev = torch.device("cuda", 0)
    check(lib.mipx_set_device(0))
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    for (w, h, b, n) in SHAPES:
        x = torch.randint(0, 256, (n * w * h * b,), dtype=torch.uint8, device=dev)
        y = torch.empty_like(x)
        for v in ("0", "1", "2"):
            os.environ["MIPX_COPY"] = v
            lib.mipx_tuning_reload()
            run = lambda: check(lib.mipx_op_rot(x.data_ptr(), y.data_ptr(), n, w, h, b, 0, sp))  # noqa: E731
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            while True:
                for _ in range(10):
                    run()
                e1.record(st)
                torch.cuda.synchronize()
                if e0.elapsed_time(e1) > 200:
                    break
            ts = []
            for _ in range(5):
                e0.record(st)
                for _ in range(10):
                    run()
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            ms = statistics.median(ts)
            ok = bool(torch.equal(x, y))
            y.zero_()
            print(json.dumps({"shape": [w, h, b, n], "MIPX_COPY": v, "ms": round(ms, 4),
                              "GBps": round(2 * x.numel() / ms / 1e6, 1), "exact": ok}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
