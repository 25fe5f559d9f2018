"""/pipeline GPU-resident fusion (reference image.go:379-410).

imaginary's Pipeline runs up to 10 operations, each on the previous one's output.
Over decoded pixels the engine plans every stage on the previous stage's output
geometry, merges the stage plans (mipx_plan_chain) and runs the chain as ONE plan:
one upload, intermediates in HBM, one download.  CPU tests cover the merge and the
planning; GPU tests check the fused result against the oracle run stage by stage.
"""
import numpy as np
import pytest

import imaginary_amd as ia
from imaginary_amd import _abi
from imaginary_amd import imaginary as im


def _plan(w, h, b, typ="png", orient=0, **opts):
    return ia.plan_make(ia.make_opts(**opts), ia.make_input(w, h, b, typ, orient))


def _steps(p):
    return [(p.steps[i].op, tuple(p.steps[i].a), tuple(p.steps[i].d)) for i in range(p.n_steps)]


# ---------------------------------------------------------------- mipx_plan_chain (CPU)
def test_plan_chain_concatenates_stages():
    a = _plan(2048, 2048, 4, width=1024, embed=1)
    b = _plan(a.out_w, a.out_h, a.out_bands, width=768, height=512, crop=1)
    c = _plan(b.out_w, b.out_h, b.out_bands, sigma=5.0, min_ampl=0.2)
    m = ia.plan_chain([a, b, c])
    assert (m.in_w, m.in_h, m.in_bands, m.load_shrink) == (2048, 2048, 4, 1)
    assert (m.out_w, m.out_h, m.out_bands) == (768, 512, 4)
    assert _steps(m) == _steps(a) + _steps(b) + _steps(c)
    assert [s[0] for s in _steps(m)] == [_abi.OP_REDUCE, _abi.OP_REDUCE, _abi.OP_EXTRACT, _abi.OP_BLUR]


def test_plan_chain_identity_stage_and_single_stage():
    a = _plan(300, 200, 3, width=150, embed=1)
    ident = _plan(a.out_w, a.out_h, a.out_bands)  # no-op stage
    assert ident.n_steps == 0
    m = ia.plan_chain([a, ident])
    assert _steps(m) == _steps(a) and (m.out_w, m.out_h) == (a.out_w, a.out_h)
    assert _steps(ia.plan_chain([a])) == _steps(a)


def test_plan_chain_rejects_bad_chains():
    a = _plan(300, 200, 3, width=150, embed=1)
    wrong = _plan(151, a.out_h, 3, sigma=1.0)
    with pytest.raises(ia.MipxError) as e:
        ia.plan_chain([a, wrong])
    assert e.value.code == _abi.MIPX_EINVAL
    jpeg = _plan(a.out_w * 8, a.out_h * 8, 3, "jpeg", 0, width=a.out_w // 4)
    if jpeg.load_shrink > 1:  # a later stage cannot ask the codec for shrink-on-load
        with pytest.raises(ia.MipxError):
            ia.plan_chain([a, jpeg])
    with pytest.raises(ia.MipxError):
        ia.plan_chain([])


def test_plan_chain_step_limit_and_watermarks():
    s = _plan(64, 64, 3, rotate=90, flip=1, flop=1, sigma=1.0)  # several steps, same geometry
    k = max(1, s.n_steps)
    n = _abi.MAX_STEPS // k + 1
    with pytest.raises(ia.MipxError) as e:
        ia.plan_chain([s] * n)
    assert e.value.code == _abi.MIPX_EUNSUPPORTED
    w = ia.plan_make(ia.make_opts(wm_enable=1, wm_left=2, wm_top=3, wm_opacity=0.5),
                     _wm_input(64, 64, 4, 16, 16, 4))
    assert any(st[0] == _abi.OP_WATERMARK for st in _steps(w))
    ia.plan_chain([w])
    with pytest.raises(ia.MipxError) as e:
        ia.plan_chain([w, w])
    assert e.value.code == _abi.MIPX_EUNSUPPORTED


def _wm_input(w, h, b, ww, wh, wb):
    i = ia.make_input(w, h, b, "png", 0)
    i.wm_w, i.wm_h, i.wm_bands = ww, wh, wb
    return i


# ---------------------------------------------------------------- Pipeline planning (CPU)
def _ops(*pairs):
    return [{"operation": op, "params": params} for op, params in pairs]


C3_OPS = _ops(("resize", {"width": 1024}), ("crop", {"width": 768, "height": 512}), ("blur", {"sigma": 5}))


def test_pipeline_runs_one_merged_plan(monkeypatch):
    calls = []

    def fake_run(plan, px, wm):
        calls.append((plan, px.shape, wm))
        return np.zeros((plan.out_h, plan.out_w, plan.out_bands), np.uint8)

    monkeypatch.setattr(im, "_run", fake_run)
    img = im.Decoded(np.zeros((2048, 2048, 4), np.uint8), type="png")
    out = im.Pipeline(img, im.build_params_from_query({"operations": C3_OPS}))
    assert out.shape == (512, 768, 4)
    assert len(calls) == 1, "the chain must run as one plan"
    plan, shape, wm = calls[0]
    assert shape == (2048, 2048, 4) and wm is None
    assert [s[0] for s in _steps(plan)] == [_abi.OP_REDUCE, _abi.OP_REDUCE, _abi.OP_EXTRACT, _abi.OP_BLUR]


def test_pipeline_ignore_failure_and_watermark_routing(monkeypatch):
    calls = []
    monkeypatch.setattr(im, "_run", lambda plan, px, wm: calls.append((plan, wm)) or
                        np.zeros((plan.out_h, plan.out_w, plan.out_bands), np.uint8))
    img = im.Decoded(np.zeros((120, 160, 3), np.uint8), type="png")
    wm = np.zeros((10, 12, 4), np.uint8)
    ops = _ops(("resize", {"width": 80}), ("watermark", {"text": "x"}),
               ("watermarkImage", {"image": "u", "left": 3, "top": 4, "opacity": 0.5}), ("rotate", {"rotate": 90}))
    ops[1]["ignore_failure"] = True  # text watermark is not an engine op: skipped
    out = im.Pipeline(img, im.build_params_from_query({"operations": ops}), wm=wm)
    assert len(calls) == 1
    plan, got_wm = calls[0]
    ops_run = [s[0] for s in _steps(plan)]
    assert ops_run.count(_abi.OP_WATERMARK) == 1  # only the watermarkImage stage sees the pixels
    assert ops_run[-1] == _abi.OP_ROT and got_wm is wm
    assert out.shape[:2] == (80, 60)
    ops[1]["ignore_failure"] = False
    with pytest.raises(im.ImaginaryError):
        im.Pipeline(img, im.build_params_from_query({"operations": ops}), wm=wm)


def test_pipeline_two_watermarks_run_stage_by_stage(monkeypatch):
    calls = []
    monkeypatch.setattr(im, "_run", lambda plan, px, wm: calls.append(plan) or
                        np.zeros((plan.out_h, plan.out_w, plan.out_bands), np.uint8))
    img = im.Decoded(np.zeros((64, 64, 3), np.uint8), type="png")
    wmop = ("watermarkImage", {"image": "u", "left": 1, "top": 1})
    im.Pipeline(img, im.build_params_from_query({"operations": _ops(wmop, ("flip", {}), wmop)}),
                wm=np.zeros((8, 8, 3), np.uint8))
    assert len(calls) == 3


# ---------------------------------------------------------------- fused chain on the GPU
def _oracle_chain(oracle, rec, px):
    """The oracle run stage by stage on the options each stage handed to Process."""
    for opts, w, h, b, typ, orient, wm in rec:
        o = {k: v for k, v in opts.items() if k not in ("type", "quality", "compression")}
        inp = dict(w=w, h=h, bands=b, type=_abi.TYPES[typ], orientation=orient)
        if wm is not None:
            o["wm_enable"] = 1
            inp.update(wm_w=wm.shape[1], wm_h=wm.shape[0], wm_bands=wm.shape[2])
        e, rp = oracle.plan(o, inp)
        assert e == 0
        px = oracle.execute(rp, px, wm)
    return px


def _fused_with_record(monkeypatch, img, ops, wm=None):
    rec, runs = [], []
    real_process, real_run = im.process, im._run

    def spy(img_, opts, wm=None, redecode=None, chain=None):
        b = img_.pixels.shape[2] if img_.pixels.ndim == 3 else 1
        rec.append((dict(opts), img_.w, img_.h, b, img_.type, img_.orientation,
                    None if wm is None else (wm if wm.ndim == 3 else wm[:, :, None])))
        return real_process(img_, opts, wm=wm, redecode=redecode, chain=chain)

    def run_spy(plan, px, wm_):
        runs.append(plan.n_steps)
        return real_run(plan, px, wm_)

    monkeypatch.setattr(im, "process", spy)
    monkeypatch.setattr(im, "_run", run_spy)
    out = im.Pipeline(img, im.build_params_from_query({"operations": ops}), wm=wm)
    return out, rec, runs


GPU_CHAINS = [
    ("c3-shape", C3_OPS, None),
    ("rot-fit-blur", _ops(("rotate", {"rotate": 270}), ("fit", {"width": 400, "height": 300}),
                          ("blur", {"sigma": 1.5}), ("flop", {})), None),
    ("wm-zoom-bw", _ops(("resize", {"width": 333, "height": 250}),
                        ("watermarkImage", {"image": "u", "left": 20, "top": 9, "opacity": 0.7}),
                        ("zoom", {"factor": 2}), ("convert", {"type": "png", "colorspace": "bw"})), "wm"),
    ("extract-embed-enlarge", _ops(("extract", {"top": 7, "left": 11, "areawidth": 301, "areaheight": 203}),
                                   ("resize", {"width": 400, "height": 400, "extend": "mirror"}),
                                   ("enlarge", {"width": 500, "height": 450})), None),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,ops,use_wm", GPU_CHAINS, ids=[c[0] for c in GPU_CHAINS])
@pytest.mark.parametrize("bands", [3, 4])
def test_fused_pipeline_matches_oracle_stage_by_stage(gpu, oracle, monkeypatch, name, ops, use_wm, bands):
    r = np.random.default_rng(7)
    side = 2048 if name == "c3-shape" else 640
    px = r.integers(0, 256, (side, side if name == "c3-shape" else 480, bands), dtype=np.uint8)
    wm = r.integers(0, 256, (40, 56, 4), dtype=np.uint8) if use_wm else None
    out, rec, runs = _fused_with_record(monkeypatch, im.Decoded(px, type="png"), ops, wm)
    assert len(runs) == 1, "one fused plan"
    want = _oracle_chain(oracle, rec, px)
    assert out.shape == want.shape, (out.shape, want.shape)
    d = np.argwhere(out != want)
    assert len(d) == 0, f"{name}: {len(d)} bytes differ, first at {d[0]}"
