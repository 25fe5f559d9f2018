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


def _run_bench(args, env_extra=None, timeout=240):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_two_starts_two_ranks_and_reports_the_max():
    """a plain `python bench.py --gpus 2` (no torchrun) runs two rank
    processes (gloo barrier + max-reduce), and the line says n_gpus 2 with the slower
    rank's time; the stub step sleeps 20 ms on rank 0 and 40 ms on rank 1."""
    r = _run_bench(["--gpus", "2", "--steps", "5", "--warmup", "1", "--stub-step-ms", "20"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * d["config"]["batch_per_gpu"]
    assert d["data"].startswith("STUB")
    assert 40 * 0.95 <= d["ms_per_step"] < 40 * 3            # rank 1's 40 ms steps, not rank 0's 20
    assert abs(d["value"] - d["config"]["global_batch"] / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-3


def test_gpus_one_runs_in_process():
    r = _run_bench(["--gpus", "1", "--steps", "3", "--warmup", "0", "--stub-step-ms", "5"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and 5 * 0.95 <= d["ms_per_step"]


def test_gpus_disagreeing_with_world_size_is_an_error():
    """Under a launcher that set WORLD_SIZE, --gpus must match it: exit non-zero, no line."""
    r = _run_bench(["--gpus", "4", "--steps", "1", "--stub-step-ms", "1"],
                   {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr and not r.stdout.strip()


def test_failing_rank_fails_the_launch(tmp_path):
    """A rank that exits non-zero fails the launch with its status, and the ranks still
    running (which would wait at the barrier forever) are stopped."""
    import time
    import launch_ranks
    script = tmp_path / "rank_fail.py"
    script.write_text("import os, sys, time\nr = int(os.environ['RANK'])\nprint('rank', r, flush=True)\n"
                      "sys.exit(3) if r == 1 else time.sleep(60)\n")
    t0 = time.monotonic()
    rc, outs = launch_ranks.run_ranks(2, str(script), [], timeout_s=90)
    assert rc == 3 and outs[0].strip() == "rank 0" and outs[1].strip() == "rank 1"
    assert time.monotonic() - t0 < 45


def test_bench_configs_aggregates_rank_lines(capsys):
    """bench_configs.py --gpus N: one line per config, the ranks' images over the slowest
    rank's step time."""
    import bench_configs
    mk = lambda imgs, ms, ok=True: json.dumps({"config": "C5", "images_per_step": imgs, "ms_per_step": ms,
                                               "device_ms_per_step": ms, "hbm_frac": 0.5,
                                               "images_per_sec": imgs / ms * 1e3, "verified_vs_oracle": ok})
    bench_configs._aggregate([mk(512, 4.0) + "\nnoise\n", mk(512, 5.0)], 2)
    d = json.loads(capsys.readouterr().out.strip())
    assert d["n_gpus"] == 2 and d["images_per_step"] == 1024 and d["ms_per_step"] == 5.0
    assert abs(d["images_per_sec"] - 1024 / 5e-3) < 0.1 and len(d["per_rank"]) == 2
    # E2E / E2EC lines carry no step timing: passed through per rank, not aggregated
    e2e = json.dumps({"config": "E2E", "requests_per_sec": 100.0, "verified_vs_oracle": True})
    bench_configs._aggregate([e2e, e2e + "\n" + mk(256, 2.0)], 2)
    out = [json.loads(ln) for ln in capsys.readouterr().out.strip().splitlines()]
    assert [(d["config"], d.get("rank")) for d in out] == [("E2E", 0), ("E2E", 1), ("C5", None)]
    assert out[2]["images_per_step"] == 256 and out[2]["n_gpus"] == 2


def test_cpu_baseline_runs_the_headline_convention():
    """the centre leg's verification left the oracle's process-wide switch at
    centre, so the corner headline's CPU baseline timed the centre convention. The CPU
    legs now set the switch to the headline's convention themselves."""
    import argparse
    from oracle import oracle as o
    args = argparse.Namespace(cpu_threads=1, cpu_distinct=1, cpu_images=1)
    for headline, other in (("corner", 1), ("centre", 0)):
        o.set_switch("reduce_centre", other)
        bench.cpu_baseline(args, headline)
        assert o.get_switch("reduce_centre") == int(headline == "centre")
    o.set_switch("reduce_centre", 0)
