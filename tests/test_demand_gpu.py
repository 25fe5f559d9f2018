"""Demand-driven regions (mipx_runtime.cpp plan_demand): a crop after a resize
computes only the rows and columns the crop keeps in the 2 x 2 reduce and the
box shrink upstream, as libvips' demand-driven evaluation does (vips_extract_area
asks its input for its area only).  The results must stay bit-identical to the
oracle run stage by stage and to the same plan computed in full (MIPX_DEMAND=0).
Reference: image.go:379-410 (/pipeline), :171-189 (Crop)."""
import numpy as np
import pytest

import imaginary_amd as ia

# every case under both reduce sampling conventions (the centre one runs k_reduce2m)
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("convention")]


def _chain(oracle, w, h, b, stages):
    plans, refs = [], []
    for opts in stages:
        p = ia.plan_make(ia.make_opts(**opts), ia.make_input(w, h, b, "png", 0))
        e, rp = oracle.plan(opts, dict(w=w, h=h, bands=b, type=3, orientation=0))
        assert e == 0
        assert (rp.out_w, rp.out_h, rp.out_bands) == (p.out_w, p.out_h, p.out_bands)
        plans.append(p)
        refs.append(rp)
        w, h, b = p.out_w, p.out_h, p.out_bands
    return ia.plan_chain(plans), refs


def _ops(p):
    return [p.steps[i].op for i in range(p.n_steps)]


def _check(gpu, oracle, monkeypatch, px, plan, refs):
    # the demand-driven run over a workspace full of junk: a windowed step that
    # read past what its producer computed would pick it up; the full run over another pattern
    got = gpu.execute(plan, px, junk=0xA5)
    monkeypatch.setenv("MIPX_DEMAND", "0")
    full = gpu.execute(plan, px, junk=0x3C)
    monkeypatch.delenv("MIPX_DEMAND")
    for i in range(px.shape[0]):
        want = px[i]
        for rp in refs:
            want = oracle.execute(rp, want)
        d = np.argwhere(got[i] != want)
        assert len(d) == 0, f"{plan.describe()}: {len(d)} bytes differ from the oracle, first at {d[0]}"
    assert np.array_equal(got, full)


CROPS = [(200, 100), (100, 200), (320, 17), (9, 240)]


@pytest.mark.parametrize("bands", [3, 4])
@pytest.mark.parametrize("gravity", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("crop", CROPS, ids=[f"{c[0]}x{c[1]}" for c in CROPS])
def test_reduce2x2_then_crop(gpu, oracle, monkeypatch, bands, gravity, crop):
    r = np.random.default_rng(100 * gravity + crop[0])
    px = r.integers(0, 256, (2, 480, 640, bands), dtype=np.uint8)
    plan, refs = _chain(oracle, 640, 480, bands,
                        [dict(width=320), dict(width=crop[0], height=crop[1], crop=1, gravity=gravity)])
    assert _ops(plan)[0] == ia._abi.OP_REDUCE
    _check(gpu, oracle, monkeypatch, px, plan, refs)


@pytest.mark.parametrize("bands", [3, 4])
@pytest.mark.parametrize("area", [(0, 0, 40, 30), (300, 7, 20, 5), (5, 230, 315, 10), (150, 100, 1, 1)])
def test_reduce2x2_then_extract_area(gpu, oracle, monkeypatch, bands, area):
    left, top, aw, ah = area
    r = np.random.default_rng(left + top)
    px = r.integers(0, 256, (2, 480, 640, bands), dtype=np.uint8)
    plan, refs = _chain(oracle, 640, 480, bands,
                        [dict(width=320), dict(left=left, top=top, area_width=aw, area_height=ah)])
    _check(gpu, oracle, monkeypatch, px, plan, refs)


@pytest.mark.parametrize("gravity", [0, 2, 4])
def test_two_reduce2x2_then_crop(gpu, oracle, monkeypatch, gravity):
    r = np.random.default_rng(gravity)
    px = r.integers(0, 256, (2, 900, 1200, 3), dtype=np.uint8)
    plan, refs = _chain(oracle, 1200, 900, 3,
                        [dict(width=600), dict(width=300), dict(width=120, height=200, crop=1, gravity=gravity)])
    _check(gpu, oracle, monkeypatch, px, plan, refs)


@pytest.mark.parametrize("bands", [3, 4])
@pytest.mark.parametrize("size", [(2000, 1500), (1500, 2000), (2001, 999)])
@pytest.mark.parametrize("gravity", [0, 1, 3])
def test_shrink_reduce_crop(gpu, oracle, monkeypatch, bands, size, gravity):
    """One bimg crop plan: shrink -> reduce -> extract; the shrink computes the window."""
    w, h = size
    r = np.random.default_rng(w + gravity)
    px = r.integers(0, 256, (2, h, w, bands), dtype=np.uint8)
    plan, refs = _chain(oracle, w, h, bands, [dict(width=150, height=150, crop=1, gravity=gravity)])
    assert ia._abi.OP_SHRINK in _ops(plan) and ia._abi.OP_EXTRACT in _ops(plan)
    _check(gpu, oracle, monkeypatch, px, plan, refs)


def test_shrink_then_crop_then_blur(gpu, oracle, monkeypatch):
    """shrink (windowed) -> reduce -> extract -> blur, and a blur before the crop
    (which needs its whole input, so nothing upstream is windowed)."""
    r = np.random.default_rng(5)
    px = r.integers(0, 256, (2, 1600, 2400, 3), dtype=np.uint8)
    plan, refs = _chain(oracle, 2400, 1600, 3,
                        [dict(width=200, height=300, crop=1), dict(sigma=2.0)])
    _check(gpu, oracle, monkeypatch, px, plan, refs)
    plan, refs = _chain(oracle, 2400, 1600, 3,
                        [dict(width=1200), dict(sigma=1.5), dict(width=300, height=100, crop=1, gravity=1)])
    _check(gpu, oracle, monkeypatch, px, plan, refs)


def test_c3_chain_full_size(gpu, oracle, monkeypatch):
    """C3's /pipeline (2048^2 RGBA: resize 1024 -> crop 768x512 -> blur 5): the 2 x 2
    reduce computes the rows the window reduce reads, about 2/3 of its output."""
    r = np.random.default_rng(33)
    px = r.integers(0, 256, (1, 2048, 2048, 4), dtype=np.uint8)
    plan, refs = _chain(oracle, 2048, 2048, 4,
                        [dict(width=1024), dict(width=768, height=512, crop=1), dict(sigma=5.0, min_ampl=0.2)])
    assert _ops(plan) == [ia._abi.OP_REDUCE, ia._abi.OP_REDUCE, ia._abi.OP_EXTRACT, ia._abi.OP_BLUR]
    _check(gpu, oracle, monkeypatch, px, plan, refs)


def test_demand_plan_through_request_path_twice(gpu, oracle):
    """the request path reuses a plan's device buffers across batches, so a
    windowed step reading outside its producer's region would see the previous input's
    values.  The same demand-driven plan, two different inputs in a row, each against
    the oracle."""
    gpu.lib.mipx_shutdown()  # mipx_init refuses another configuration while one runs
    eng = gpu.Engine(devices=[0], max_batch=1)
    try:
        plan, refs = _chain(oracle, 640, 480, 3, [dict(width=320), dict(width=200, height=100, crop=1, gravity=3)])
        assert _ops(plan)[0] == ia._abi.OP_REDUCE
        r = np.random.default_rng(77)
        for k in range(2):
            img = r.integers(0, 256, (480, 640, 3), dtype=np.uint8) if k == 0 else np.full((480, 640, 3), 200, np.uint8)
            t, out = eng.submit(plan, img)
            eng.wait(t)
            want = img
            for rp in refs:
                want = oracle.execute(rp, want)
            assert np.array_equal(out, want), f"request {k}"
    finally:
        eng.shutdown()
