"""params_test.go's tables against the Python mirror of params.go (imaginary_amd/imaginary.py).

Each case below is the reference's own (value, expected) pair, quoted from
/root/reference/params_test.go at the cited lines; the mirror must return Go's result
byte for byte (parseColor, parseColorspace and parseBool
used to differ from strconv's semantics)."""
import json
import math

import pytest

from imaginary_amd import imaginary as im

# bimg constants (bimg v1.1.9 options.go): Extend*, Gravity*
EXTEND_BLACK, EXTEND_COPY, EXTEND_REPEAT, EXTEND_MIRROR, EXTEND_WHITE, EXTEND_BACKGROUND, EXTEND_LAST = range(7)
GRAVITY_CENTRE, GRAVITY_NORTH, GRAVITY_EAST, GRAVITY_SOUTH, GRAVITY_WEST, GRAVITY_SMART = range(6)


def test_read_params():
    """TestReadParams, params_test.go:13-41 (the pixel-relevant fields)."""
    q = {"width": "100", "height": "80", "noreplicate": "1", "opacity": "0.2", "text": "hello",
         "background": "255,10,20", "interlace": "true"}
    p = im.build_params_from_query(q)
    assert p.width == 100 and p.height == 80
    assert p.opacity == float(__import__("numpy").float32(0.2))   # ImageOptions.Opacity is float32
    assert p.text == "hello" and p.background == [255, 10, 20]


@pytest.mark.parametrize("value,expected", [("1", 1), ("0100", 100), ("-100", 100), ("99.02", 99), ("99.9", 100)])
def test_parse_param_int(value, expected):
    """TestParseParam intCases, params_test.go:44-60."""
    assert im.parse_int(value)[0] == expected


@pytest.mark.parametrize("value,expected", [("1.1", 1.1), ("01.1", 1.1), ("-1.10", 1.10), ("99.999999", 99.999999)])
def test_parse_param_float(value, expected):
    """TestParseParam floatCases, params_test.go:62-77 (exact equality, as Go's !=)."""
    assert im.parse_float(value)[0] == expected


@pytest.mark.parametrize("value,expected", [("true", True), ("false", False), ("1", True), ("1.1", False),
                                            ("-1", False), ("0", False), ("0.0", False), ("no", False),
                                            ("yes", False)])
def test_parse_param_bool(value, expected):
    """TestParseParam boolCases, params_test.go:79-99 (the value, errors ignored as there)."""
    assert im.parse_bool(value)[0] is expected


@pytest.mark.parametrize("value,expected", [("200,100,20", [200, 100, 20]), ("0,280,200", [0, 255, 200]),
                                            (" -1, 256 , 50", [0, 255, 50]), (" a, 20 , &hel0", [0, 20, 0]),
                                            ("", [])])
def test_parse_color(value, expected):
    """TestParseColor, params_test.go:102-133."""
    assert im.parse_color(value) == expected


@pytest.mark.parametrize("value,expected", [("white", EXTEND_WHITE), ("black", EXTEND_BLACK), ("copy", EXTEND_COPY),
                                            ("mirror", EXTEND_MIRROR), ("lastpixel", EXTEND_LAST),
                                            ("background", EXTEND_BACKGROUND), (" BACKGROUND  ", EXTEND_BACKGROUND),
                                            ("invalid", EXTEND_MIRROR), ("", EXTEND_MIRROR)])
def test_parse_extend(value, expected):
    """TestParseExtend, params_test.go:135-157."""
    assert im.parse_extend_mode(value) == expected


@pytest.mark.parametrize("value,smart", [("foo", False), ("smart", True)])
def test_gravity(value, smart):
    """TestGravity, params_test.go:159-174."""
    assert (im.build_params_from_query({"gravity": value}).gravity == GRAVITY_SMART) is smart


def test_read_map_params():
    """TestReadMapParams, params_test.go:176-226."""
    o = im.build_params_from_operation({"params": {"width": 100, "opacity": 0.1, "type": "webp", "embed": True,
                                                   "gravity": "west", "color": "255,200,150"}})
    assert o.width == 100 and o.type == "webp" and o.embed is True and o.gravity == GRAVITY_WEST
    assert o.opacity == float(__import__("numpy").float32(0.1)) and o.color == [255, 200, 150]


def test_parse_functions():
    """TestParseFunctions, params_test.go:228-247."""
    assert im.parse_bool("true") == (True, None)
    assert im.parse_bool("false") == (False, None)
    assert im.parse_bool("") == (False, None)
    assert im.parse_bool("foo")[1] is not None


def test_build_params_from_operation():
    """TestBuildParamsFromOperation, params_test.go:249-281."""
    o = im.build_params_from_operation({"params": {"width": 200, "opacity": 2.2, "force": True, "stripmeta": False,
                                                   "type": "jpeg", "background": "255,12,3"}})
    assert o.width == 200 and abs(o.opacity - 2.2) < 1e-4 and o.force is True and o.background[0] == 255


@pytest.mark.parametrize("fn,cases", [
    (im.coerce_type_int, [("200", 200), (200, 200), (200.0, 200), (False, None)]),
    (im.coerce_type_float, [("200", 200.0), (200, 200.0), (200.0, 200.0), (False, None)]),
    (im.coerce_type_bool, [("true", True), (True, True), ("1", True), ("bubblegum", None)]),
    (im.coerce_type_string, [("true", "true"), (False, None), (0.0, None), (0, None)]),
])
def test_coerce_type_fns(fn, cases):
    """TestCoerceTypeFns, params_test.go:283-407 (None = the case expects an error)."""
    for inp, want in cases:
        if want is None:
            with pytest.raises(ValueError):
                fn(inp)
        else:
            got = fn(inp)
            assert got == want and type(got) is type(want), (inp, got, want)


# ---- strconv details beyond the tables (Go semantics, stated) ----------------------------
def test_strconv_edges():
    # ParseUint(.., 10, 8): signs are syntax errors (0), out of range saturates (255)
    assert im.parse_color("+5,007,99999999999999999999,,1 2") == [0, 7, 255, 0, 0]
    # ParseBool: exact spellings only, no trimming or case folding beyond its table
    assert im.parse_bool("TRUE")[0] and im.parse_bool("True")[0] and im.parse_bool("T")[0]
    for bad in ("tRUE", " true", "True ", "yes", "on"):
        assert im.parse_bool(bad)[1] is not None, bad
    # parseColorspace: exactly "bw"
    assert im.parse_colorspace("bw") != im.parse_colorspace("BW") == im.parse_colorspace(" bw")
    # ParseFloat: no surrounding space, no Python-only underscores; inf / nan / hex floats accepted
    for bad in (" 1", "1 ", "1_0", "abc", "1e", "."):
        assert im.parse_float(bad) [1] is not None, bad
    assert im.parse_float("0x1p-2") == (0.25, None)
    assert im.parse_float("-Inf")[0] == math.inf and im.parse_float("1e400")[1] is not None
    assert im.parse_int("2.5") == (3, None) and im.parse_int("-2.5") == (3, None)   # |f| then floor(f + .5)
    # a float JSON number truncates (Go int(float64)), a string rounds
    assert im.coerce_type_int(2.7) == 2 and im.coerce_type_int("2.7") == 3
    # a parse error fails the whole request (HTTP 400), as buildParamsFromQuery returns it
    with pytest.raises(im.ImaginaryError):
        im.build_params_from_query({"width": "abc"})
    with pytest.raises(im.ImaginaryError):
        im.build_params_from_query({"flip": "yes"})


def test_json_operations():
    """parseJSONOperations (params.go:411-419): < 2 bytes is no operations, unknown
    fields are refused, field names match case-insensitively."""
    assert im.parse_json_operations("") == [] and im.parse_json_operations("[") == []
    ops = im.parse_json_operations(json.dumps([{"Operation": "crop", "params": {"width": 10}}]))
    assert ops == [{"operation": "crop", "ignore_failure": False, "params": {"width": 10}}]
    with pytest.raises(ValueError):
        im.parse_json_operations(json.dumps([{"operation": "crop", "bogus": 1}]))
    o = im.build_params_from_query({"operations": json.dumps([{"operation": "blur", "params": {"sigma": 5}}])})
    assert o.operations[0]["operation"] == "blur"
