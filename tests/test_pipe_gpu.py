"""Stage pipelining across sub-batches (mipx_runtime.cpp execute_pipelined, MIPX_PIPE = k
chunks): the batch runs as k chunks, each chunk's first step on the caller's stream and its
later steps on a second stream, every chunk in its own workspace slice.  The output must be
byte-identical to the plain run (and, for the first and last image, to the oracle run stage by
stage) whatever k, batch size or plan; plans whose first step starts a peephole pair, and
batches smaller than 2 k, take the plain path.  Reference: image.go:379-410 (/pipeline)."""
import numpy as np
import pytest

import imaginary_amd as ia

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("convention")]


def _chain(oracle, w, h, b, stages):
    plans, refs = [], []
    for opts in stages:
        p = ia.plan_make(ia.make_opts(**opts), ia.make_input(w, h, b, "png", 0))
        e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3, orientation=0))
        assert e == 0
        plans.append(p)
        refs.append(rp)
        w, h, b = p.out_w, p.out_h, p.out_bands
    return ia.plan_chain(plans), refs


CHAINS = {
    # C3's shape at 1/4 size: 2 x 2 reduce (split point), window reduce + extract, blur
    "c3_small": (512, 512, 4, [dict(width=256, embed=1), dict(width=192, height=128, crop=1), dict(sigma=5.0)]),
    "c3_rgb": (640, 480, 3, [dict(width=320, embed=1), dict(width=200, height=100, crop=1), dict(sigma=2.0)]),
    # a first step that starts a peephole (reduce 1.6 -> extract): the plain path
    "peephole_first": (480, 320, 3, [dict(width=300, height=100, crop=1), dict(sigma=1.5)]),
    "shrink_rot": (800, 600, 3, [dict(width=100), dict(rotate=90)]),
}


@pytest.mark.parametrize("name", list(CHAINS))
@pytest.mark.parametrize("k,n", [(2, 4), (3, 7), (4, 9), (4, 5)])
def test_pipelined_batch_matches_plain_and_oracle(gpu, oracle, monkeypatch, name, k, n):
    w, h, b, stages = CHAINS[name]
    plan, refs = _chain(oracle, w, h, b, stages)
    px = np.random.default_rng(k * 100 + n).integers(0, 256, (n, h, w, b), dtype=np.uint8)
    monkeypatch.setenv("MIPX_PIPE", "")
    plain = gpu.execute(plan, px, junk=0x3C)
    monkeypatch.setenv("MIPX_PIPE", str(k))
    got = gpu.execute(plan, px, junk=0xA5)
    monkeypatch.delenv("MIPX_PIPE")
    assert np.array_equal(got, plain), f"{plan.describe()}: k={k} n={n} differs from the plain run"
    for i in (0, n - 1):
        want = px[i]
        for rp in refs:
            want = oracle.execute(rp, want)
        assert np.array_equal(got[i], want), f"image {i} differs from the oracle"


def test_pipelined_workspace_covers_every_chunk(gpu, oracle, monkeypatch):
    w, h, b, stages = CHAINS["c3_small"]
    plan, _ = _chain(oracle, w, h, b, stages)
    monkeypatch.setenv("MIPX_PIPE", "")
    ia._abi.sync_tuning()
    plain = ia._abi.lib.mipx_workspace_bytes(ia._abi.C.byref(plan), 9)
    monkeypatch.setenv("MIPX_PIPE", "4")
    ia._abi.sync_tuning()
    piped = ia._abi.lib.mipx_workspace_bytes(ia._abi.C.byref(plan), 9)
    monkeypatch.delenv("MIPX_PIPE")
    ia._abi.sync_tuning()
    assert piped >= plain > 0
