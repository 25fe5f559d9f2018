"""The reduce sampling convention is part of the plan (ABI v6).

PARITY_ASSUMPTIONS.md row 1 leaves libvips' reduce sampling convention open, so the
engine carries both; mipx_plan_make records the process setting in each REDUCE /
SMARTCROP step and the plan runs under it whatever the setting is at execution time.
Every call below goes through the C-ABI (mipx_plan_make, mipx_set_reduce_sampling,
mipx_execute_dev, mipx_submit / mipx_wait)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def restore_sampling(gpu, oracle):
    prev_e, prev_o = gpu.reduce_sampling(), oracle.get_switch("reduce_centre")
    yield
    gpu.set_reduce_sampling(prev_e)
    oracle.set_switch("reduce_centre", prev_o)


def _want(oracle, img, hs, vs, centre):
    oracle.set_switch("reduce_centre", int(centre))
    return oracle.reduce(img, hs, vs)


# 2 x 2 (k_reduce2x2 / k_reduce2m), a generic factor (k_rcol), a crop after a 2 x 2
# reduce (the demand-region walk reads the convention too)
CASES = [(dict(width=160, height=120, embed=1), (320, 240, 3)),
         (dict(width=200, height=150, embed=1), (320, 240, 4)),
         (dict(width=150, height=90, crop=1), (300, 240, 3))]


@pytest.mark.parametrize("made,flipped", [("corner", "centre"), ("centre", "corner")])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_plan_keeps_its_convention_when_the_setting_flips(gpu, oracle, restore_sampling, made, flipped, case, rng):
    opts, (w, h, b) = CASES[case]
    img = rng.integers(0, 256, (2, h, w, b), dtype=np.uint8)
    gpu.set_reduce_sampling(made)
    plan = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, "png"))
    oracle.set_switch("reduce_centre", int(made == "centre"))
    e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3))
    assert e == 0
    want = [oracle.execute(rp, img[i]) for i in range(2)]
    gpu.set_reduce_sampling(flipped)           # after planning, before executing
    got = gpu.execute(plan, img)
    for i in range(2):
        assert np.array_equal(got[i], want[i]), (made, flipped, opts)
    # a plan made now follows the new setting, and the two conventions differ here
    plan2 = gpu.plan_make(gpu.make_opts(**opts), gpu.make_input(w, h, b, "png"))
    assert plan2.steps[0].a[7] == (1 if flipped == "centre" else 0)
    got2 = gpu.execute(plan2, img[:1])
    assert not np.array_equal(got2[0], want[0])


def test_setter_refuses_while_requests_are_in_flight(gpu, oracle, restore_sampling):
    """mipx_set_reduce_sampling returns MIPX_EBUSY while mipx_submit requests are queued
    or running, and succeeds again once they are retired; the requests keep the
    convention their plan recorded."""
    gpu.lib.mipx_shutdown()
    gpu.set_reduce_sampling("corner")
    eng = gpu.Engine(devices=[0], max_batch=4, queues_per_device=1)
    try:
        plan = gpu.plan_make(gpu.make_opts(width=1920, height=1080, embed=1), gpu.make_input(3840, 2160, 3, "png"))
        rng = np.random.default_rng(5)
        imgs = [rng.integers(0, 256, (2160, 3840, 3), dtype=np.uint8) for _ in range(2)]
        tickets = [eng.submit(plan, imgs[i % 2]) for i in range(8)]  # ~200 MB of uploads queued
        busy = gpu.lib.mipx_set_reduce_sampling(1)
        assert busy == gpu.MIPX_EBUSY, busy
        assert gpu.reduce_sampling() == "corner"
        for t, _ in tickets:
            eng.wait(t)
        assert gpu.lib.mipx_set_reduce_sampling(1) == 0          # nothing in flight any more
        oracle.set_switch("reduce_centre", 0)
        for i, (_, out) in enumerate(tickets[:2]):
            assert np.array_equal(out, oracle.reduce(imgs[i % 2], 2.0, 2.0))
    finally:
        eng.shutdown()


def test_per_op_entry_point_reads_the_setting_once(gpu, oracle, restore_sampling, rng):
    """mipx_op_reduce (no plan) runs under the process setting at call time."""
    img = rng.integers(0, 256, (1, 120, 160, 3), dtype=np.uint8)
    for conv in ("corner", "centre"):
        gpu.set_reduce_sampling(conv)
        got = gpu.run_op("reduce", img, hshrink=1.6, vshrink=1.6)
        assert np.array_equal(got[0], _want(oracle, img[0], 1.6, 1.6, conv == "centre")), conv
