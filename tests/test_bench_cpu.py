"""bench.py's bookkeeping on CPU: the PMC traffic record attached to the roofline must
be the record of the kernel the line ran (the centre-convention
line had carried k_reduce2x2's record)."""
import json
import os

import bench


def test_traffic_record_names_the_kernel_that_ran():
    for sampling, kernel in bench.C2_KERNEL.items():
        traffic, src = bench.pmc_traffic(kernel)
        if traffic is None:
            continue
        with open(os.path.join(bench.ROOT, src)) as f:
            t = json.load(f)
        recs = [r for r in t.get("records", [t]) if r.get("kernel") == kernel]
        assert recs and recs[0]["traffic_bytes"] == traffic, (sampling, kernel, src)
    assert bench.pmc_traffic("k_no_such_kernel<3>") == (None, None)
    # the two conventions run different kernels, so they never share a record
    assert len(set(bench.C2_KERNEL.values())) == len(bench.C2_KERNEL)
