#!/usr/bin/env python3
"""A/B launch geometry of k_reduce2x2 (band height, XCD remap) in one process."""
import ctypes as C, json, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa
from imaginary_amd._abi import check, lib  # noqa
W, H, B, n = 3840, 2160, 3, 256
dev = torch.device("cuda", 0); lib.mipx_set_device(0)
x = torch.randint(0, 256, (n, H * W * B), dtype=torch.uint8, device=dev)
y = torch.empty((n, (H // 2) * (W // 2) * B), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream(dev); sp = C.c_void_p(st.cuda_stream)
configs = [dict(MIPX_R2_BAND=b, MIPX_R2_ORDER=o) for b in os.environ.get("BANDS_LIST", "1,2,3,4,5,6,8").split(",") for o in ("0", "1")]
times = {i: [] for i in range(len(configs))}
for rnd in range(5):
    for i, cfg in enumerate(configs):
        os.environ.update(cfg)
        lib.mipx_tuning_reload()  # the library snapshots MIPX_* knobs
        check(lib.mipx_op_reduce(x.data_ptr(), y.data_ptr(), n, W, H, B, 2.0, 2.0, None, 0, sp), "r")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(5):
            check(lib.mipx_op_reduce(x.data_ptr(), y.data_ptr(), n, W, H, B, 2.0, 2.0, None, 0, sp), "r")
        e1.record(st); torch.cuda.synchronize()
        times[i].append(e0.elapsed_time(e1) / 5)
alg = n * (H * W * B + (H // 2) * (W // 2) * B)
for i, cfg in enumerate(configs):
    med = statistics.median(times[i])
    print(json.dumps({**cfg, "median_ms": round(med, 4), "frac": round(alg / med / 1e6 / 8000, 4)}))
